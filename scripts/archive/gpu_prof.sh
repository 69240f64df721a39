#!/bin/bash
# rocprofv3 kernel-trace summaries of bench.py (per pass kernel) under the given env settings.
# Usage on the GPU box: TAG=x QUBITS=30 bash scripts/gpu_prof.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_${TAG:-run} -o run --output-format csv \
    -- python3 $R/bench.py --qubits ${QUBITS:-30} --steps ${STEPS:-3} --warmup 1 --cpu-budget 0 ${BENCH_ARGS:-} \
    > $OUT/prof_${TAG:-run}.json 2> $OUT/prof_${TAG:-run}.err || { tail -5 $OUT/prof_${TAG:-run}.err; exit 1; }
f=$(find $OUT/prof_${TAG:-run} -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 $f | head -20
