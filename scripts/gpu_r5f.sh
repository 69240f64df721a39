#!/bin/bash
# Round 5: W-BATCH in-tile noise variants (lists on / off, prefix 0 / 12) against the push kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5f}
mkdir -p $O
for v in "1 1 99" "1 0 99" "1 1 0" "1 1 6"; do
  set -- $v
  QSIM_NOISE_TILE=$1 QSIM_NOISE_TILE_LISTS=$2 QSIM_NOISE_TILE_PREFIX=$3 timeout -k 10 300 python -u bench.py --workload batch --cpu-budget 0 --steps 5 --warmup 1 > $O/batch_$1_$2_$3.json 2> $O/batch_$1_$2_$3.err || { tail -5 $O/batch_$1_$2_$3.err; exit 1; }
  python3 - $O/batch_$1_$2_$3.json "tile=$1 lists=$2 prefix=$3" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = {x["name"]: (round(x["ms"] / max(1, x["launches"]), 4), x["launches"]) for x in d["kernels"]}
print(sys.argv[2], d["value"], d["ms_per_step"], k)
PY
done
