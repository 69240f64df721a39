#!/bin/bash
# Layout choice (labels for fewer passes + cheaper layouts): relabel / batched / dist GPU tests,
# bench lines at 30q, 28q and W-BATCH.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/lc; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_relabel_gpu.py tests/test_batched_gpu.py tests/test_dist_gpu.py tests/test_bench_path_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --cpu-budget 0 > $O/b30.json 2> $O/b30.err || { tail $O/b30.err; exit 1; }
timeout -k 10 300 python bench.py --qubits 28 --cpu-budget 0 --no-1q28 > $O/b28.json 2> $O/b28.err || { tail $O/b28.err; exit 1; }
timeout -k 10 300 python bench.py --workload batch --qubits 16 --steps 10 --warmup 2 > $O/bb.json 2> $O/bb.err || { tail $O/bb.err; exit 1; }
for f in b30 b28 bb; do python3 -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['launches'])"; done
