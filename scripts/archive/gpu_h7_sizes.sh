#!/bin/bash
# W-HC at 26-30 qubits: 12-qubit (h = 6) vs 13-qubit (h = 7, pipelined) tiles.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/h7s
mkdir -p $O
cd $R
for Q in ${QUBITS:-26 27 28 29 30}; do
  for H in 6 7; do
    QSIM_TILE_HMAX=$H timeout -k 10 300 python bench.py --qubits $Q --cpu-budget 0 > $O/b${Q}_h$H.json 2> $O/b${Q}_h$H.err || exit 1
  done
done
python - <<PY
import json, glob
for f in sorted(glob.glob('$O/b*.json')):
    d = json.load(open(f)); r = d['roofline']
    print(f.split('/')[-1], d['value'], d['ms_per_step'], r and round(r['frac'], 4), r and r.get('launches'), r and r.get('avg_launch_ms'))
PY
