#!/bin/bash
# Round 3: variance of the h=7 / T13=1.25 label calibration at 30q seed 42 (candidate timings).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3d
mkdir -p $O
for i in 1 2; do
  for C in 3 6; do
    QSIM_RELABEL_DEBUG=1 QSIM_TILE_HMAX=7 QSIM_LAYOUT_T13=1.25 QSIM_RELABEL_CALIBRATE_CANDIDATES=$C timeout -k 10 300 \
      python bench.py --cpu-budget 0 --no-1q28 --steps 10 > $O/c${C}_$i.json 2> $O/c${C}_$i.err || { tail -5 $O/c${C}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('$O/c${C}_$i.json')); r=d['roofline']; print('cand $C run $i', d['value'], d['ms_per_step'], r['launches'], r['avg_launch_ms'])"
    grep calibrate $O/c${C}_$i.err
  done
done
