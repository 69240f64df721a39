#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/batch; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_batched_gpu.py tests/test_batched_refnoise_gpu.py tests/test_sampling_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "Error|assert|FAIL" $O/pytest.log | head -30; exit 1; }
grep -E "passed|failed" $O/pytest.log
timeout -k 10 300 python bench.py --workload batch --qubits 16 --steps 5 --warmup 2 > $O/batch_phys.json 2> $O/batch_phys.err || { cat $O/batch_phys.err; exit 1; }
python3 -c "
import json
d=json.load(open('$O/batch_phys.json')); r=d['roofline']
print(d['value'], d['ms_per_step'], r and (r['kernel'], r['avg_launch_ms'], r['frac']), [(k['name'], round(k['ms'],2), k['launches']) for k in d['kernels']])"
