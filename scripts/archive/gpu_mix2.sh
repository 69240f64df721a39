#!/bin/bash
# 13-qubit plans with mixed heights and the 13-qubit tile penalty in the layout cost: 28/29/30q.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/mix2
mkdir -p $O
cd $R
for T in 1.25 1.0; do
  for Q in 30 29 28; do
    QSIM_TILE_HMAX=7 QSIM_LAYOUT_T13=$T timeout -k 10 300 python bench.py --qubits $Q --cpu-budget 0 > $O/b${Q}_t$T.json 2> $O/b${Q}_t$T.err || exit 1
    python -c "import json; d=json.load(open('$O/b${Q}_t$T.json')); r=d['roofline']; print('$Q t13=$T', d['value'], d['ms_per_step'], r['launches'], r['avg_launch_ms'], round(r['frac'],4))"
  done
done
for S in 1 3; do
  for H in 7 6; do
    QSIM_TILE_HMAX=$H timeout -k 10 300 python bench.py --qubits 30 --seed $S --cpu-budget 0 > $O/b30_s${S}_h$H.json 2> $O/b30_s${S}_h$H.err || exit 1
    python -c "import json; d=json.load(open('$O/b30_s${S}_h$H.json')); r=d['roofline']; print('30q seed $S h$H', d['value'], d['ms_per_step'], r['launches'], r['avg_launch_ms'])"
  done
done
