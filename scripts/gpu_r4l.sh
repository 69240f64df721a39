#!/bin/bash
# Round 4: gate + in-tile noise kernel cost by prefix length (0: load / gate / store only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${1:-r4l}
mkdir -p gpurun_out/$O
for pf in 0 4 12; do
  QSIM_NOISE_TILE=1 QSIM_NOISE_TILE_PREFIX=$pf timeout -k 10 200 python -u bench.py --workload batch --cpu-budget 0 --steps 2 --warmup 1 > gpurun_out/$O/pf$pf.json 2> gpurun_out/$O/pf$pf.err || { tail -5 gpurun_out/$O/pf$pf.err; exit 1; }
  python3 - gpurun_out/$O/pf$pf.json prefix=$pf <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = {x["name"]: (round(x["ms"] / max(1, x["launches"]), 4), x["launches"]) for x in d["kernels"]}
print(sys.argv[2], d["value"], d["ms_per_step"], k)
PY
done
