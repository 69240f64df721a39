#!/bin/bash
# W-HC 28q seeds 1-4: default tile heights (13-qubit, mixed) vs 12-qubit tiles only (QSIM_TILE_AUTO=0).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/seeds28
mkdir -p $O
cd $R
for S in 1 2 3 4; do
  for A in 1 0; do
    QSIM_TILE_AUTO=$A timeout -k 10 300 python bench.py --qubits 28 --seed $S --cpu-budget 0 > $O/s${S}_auto$A.json 2> $O/s${S}_auto$A.err || exit 1
    python -c "import json; d=json.load(open('$O/s${S}_auto$A.json')); r=d['roofline']; print('28q seed $S auto=$A', d['value'], d['ms_per_step'], r['launches'], r['avg_launch_ms'])"
  done
done
