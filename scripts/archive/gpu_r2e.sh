#!/bin/bash
# Evidence for the relabeled headline: default bench line, rocprof kernel stats of it, PMC HBM
# traffic of the W-HC 30q passes (FETCH_SIZE / WRITE_SIZE passes).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r2e; mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv \
  -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-budget 0 > $O/prof_bench.json 2> $O/prof.err || { tail $O/prof.err; exit 1; }
cut -d, -f1-4 $(find $O/prof -name "*kernel_stats.csv" | head -1) | head -12
cd $R && QUBITS=30 WORKLOAD=hc TAG=hc30r BENCH_ARGS="--no-1q28" bash scripts/gpu_pmc.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
tail -5 $O/pmc.log
