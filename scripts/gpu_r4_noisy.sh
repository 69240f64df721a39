#!/bin/bash
# Round 4: NoisySimulator 26q line, pushed vs pulled flips.  Usage: gpu_r4_noisy.sh <outdir>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=$PWD/gpurun_out/${1:-r4noisy}
mkdir -p $O
for pull in 0 1; do
  QSIM_NOISE_PULL=$pull timeout -k 10 300 python -u bench.py --workload noisy --cpu-budget 0 --steps 2 --warmup 1 > $O/pull$pull.json 2> $O/pull$pull.err || { tail -5 $O/pull$pull.err; exit 1; }
  python3 - $O/pull$pull.json "pull=$pull" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = {x["name"]: (round(x["ms"] / max(1, x["launches"]), 4), x["launches"]) for x in d["kernels"]}
print(sys.argv[2], d["value"], d["ms_per_step"], k)
PY
done
