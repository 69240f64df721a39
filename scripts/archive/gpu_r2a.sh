#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r2a; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_batched_refnoise_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
grep -E "PASS|FAIL" $O/pytest.log
timeout -k 10 300 python bench.py --cpu-budget 0 --steps 10 > $O/bench30.json 2> $O/bench30.err || { cat $O/bench30.err; exit 1; }
cat $O/bench30.json
timeout -k 10 300 python bench.py --workload batch --qubits 16 --steps 5 --warmup 2 > $O/batch_phys.json 2> $O/batch_phys.err || { cat $O/batch_phys.err; exit 1; }
timeout -k 10 300 python bench.py --workload batch --qubits 16 --steps 2 --warmup 1 --batch-noise reference > $O/batch_ref.json 2> $O/batch_ref.err || { cat $O/batch_ref.err; exit 1; }
python3 -c "
import json
for f in ('batch_phys','batch_ref'):
    d=json.load(open('$O/'+f+'.json')); r=d['roofline']
    print(f, d['value'], d['ms_per_step'], r and (r['kernel'], r['avg_launch_ms'], r['frac']), [(k['name'], round(k['ms'],2), k['launches']) for k in d['kernels']])"
