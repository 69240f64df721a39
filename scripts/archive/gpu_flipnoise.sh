#!/bin/bash
# Block-geometric flip noise: parity tests (noisy, batched reference noise, shards) + the
# reference-noise W-BATCH bench line and its kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/flip; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_noisy_gpu.py tests/test_batched_refnoise_gpu.py tests/test_batched_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 200 python bench.py --workload batch --batch-noise reference --steps 10 --warmup 2 --cpu-budget 0 > $O/ref.json 2> $O/ref.err || { tail $O/ref.err; exit 1; }
cat $O/ref.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- python3 $R/bench.py --workload batch --batch-noise reference --steps 5 --warmup 1 --cpu-budget 0 > $O/tr.log 2>&1 || { tail $O/tr.log; exit 1; }
find $O/tr -name '*kernel_stats.csv' -exec head -8 {} \;
