#!/bin/bash
# Carried Pauli frames: batched GPU tests + W-BATCH bench (physical noise) + kernel stats.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/frames; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_batched_gpu.py tests/test_batched_refnoise_gpu.py tests/test_sampling_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python bench.py --workload batch --steps 20 --warmup 3 --cpu-budget 0 > $O/batch.json 2> $O/batch.err || { tail $O/batch.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/batch.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'], [(k['name'], k['launches'], round(k['ms']/k['launches'],4)) for k in d['kernels']])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- python3 $R/bench.py --workload batch --steps 10 --warmup 2 --cpu-budget 0 > $O/tr.log 2>&1 || { tail $O/tr.log; exit 1; }
cut -d, -f1-4 $(find $O/tr -name '*kernel_stats.csv' | head -1) | head -8
