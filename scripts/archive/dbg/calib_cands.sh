#!/bin/bash
# Layout calibration: number of timed candidates vs W-HC 30q (seeds 42, 1)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/ccands; mkdir -p $O
for s in 42 1; do for k in 1 3 6; do
  QSIM_RELABEL_DEBUG=1 QSIM_RELABEL_CALIBRATE_CANDIDATES=$k timeout -k 10 200 python bench.py --seed $s --steps 5 --warmup 2 --cpu-budget 0 --no-1q28 > $O/s${s}_k$k.json 2> $O/s${s}_k$k.err || { tail $O/s${s}_k$k.err; exit 1; }
  echo "$(grep -c calibrate $O/s${s}_k$k.err) timed: $(grep calibrate $O/s${s}_k$k.err | awk '{print $5}' | tr '\n' ' ')"
  python3 -c "import json;d=json.load(open('$O/s${s}_k$k.json'));print('seed', $s, 'cands', $k, d['value'], d['ms_per_step'])"
done; done
