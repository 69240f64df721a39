#!/bin/bash
# Batched relabeling: batched / refnoise / sampling GPU tests, W-BATCH with and without.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/brl; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_batched_gpu.py tests/test_batched_refnoise_gpu.py tests/test_sampling_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python bench.py --workload batch --qubits 16 --steps 10 --warmup 2 > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
QSIM_RELABEL=0 timeout -k 10 200 python bench.py --workload batch --qubits 16 --steps 10 --warmup 2 > $O/b0.json 2> $O/b0.err || { tail $O/b0.err; exit 1; }
for f in b b0; do python3 -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'])"; done
