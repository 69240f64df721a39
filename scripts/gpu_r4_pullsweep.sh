#!/bin/bash
# Round 4: pull-pass variants (items per thread, non-temporal traffic) at p = 0 and 0.01, and a
# rocprofv3 kernel-stats run of the default pull step.  Usage: gpu_r4_pullsweep.sh <outdir>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD; O=$PWD/gpurun_out/${1:-r4pull}
mkdir -p $O
for p in 0 0.01; do
  for u in 2 4 8; do
    for nt in 1 0; do
      QSIM_PULL_U=$u QSIM_PULL_NT=$nt timeout -k 10 200 python -u bench.py --workload batch --noise $p --cpu-budget 0 --steps 2 --warmup 1 > $O/p${p}_u${u}_nt${nt}.json 2> $O/p${p}_u${u}_nt${nt}.err || { tail -5 $O/p${p}_u${u}_nt${nt}.err; exit 1; }
      python3 - $O/p${p}_u${u}_nt${nt}.json "p$p u$u nt$nt" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = {x["name"]: round(x["ms"] / max(1, x["launches"]), 4) for x in d["kernels"]}
print(sys.argv[2], d["value"], d["ms_per_step"], k)
PY
    done
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o pull -- python3 $R/bench.py --workload batch --cpu-budget 0 --steps 2 --warmup 1 > $O/prof.json 2> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
head -12 $O/prof/pull_kernel_stats.csv
