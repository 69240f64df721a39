#!/bin/bash
# Round-2 checkpoint: every -m gpu test file, the default bench line, rocprof kernel stats of it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r2c; mkdir -p $O
TLIM=${TLIM:-240} bash scripts/gpu_tests_each.sh || exit 1
cp gpurun_out/each/summary.txt $O/tests_summary.txt
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv \
  -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-budget 0 > $O/prof_bench.json 2> $O/prof.err || { tail $O/prof.err; exit 1; }
cut -d, -f1-4 $(find $O/prof -name "*kernel_stats.csv" | head -1) | head -14
