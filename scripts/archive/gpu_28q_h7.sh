#!/bin/bash
# 28q W-HC with the default (13-qubit) tiles: rocprof kernel stats + PMC HBM traffic.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/q28
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof28 -o run --output-format csv \
  -- python3 $R/bench.py --qubits 28 --steps 10 --warmup 2 --cpu-budget 0 > $O/prof28.json 2> $O/prof28.err || exit 1
cut -d, -f1-4 $(find $O/prof28 -name "*kernel_stats.csv" | head -1) | head -12
cd $R && QUBITS=28 TAG=q28_h7 bash scripts/gpu_pmc.sh > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
tail -8 $O/pmc.log
