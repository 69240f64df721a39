#!/bin/bash
# Round 3: relayout position policy A/B (QSIM_RELAYOUT_RUN6 0 / 1 / 2) on W-HC 30q seeds 42 and 4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/run6; mkdir -p $O
for r in 0 1 2; do for sd in 42 4; do
  QSIM_RELAYOUT_RUN6=$r QSIM_RELABEL_CALIBRATE=0 timeout -k 10 300 python3 bench.py --qubits 30 --seed $sd --cpu-budget 0 --no-1q28 --no-batch16 --steps 10 > $O/b_r${r}_s${sd}.json 2> $O/b_r${r}_s${sd}.err || { tail -5 $O/b_r${r}_s${sd}.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_r${r}_s${sd}.json'));c=d['config'];print($r, $sd, d['value'], c['passes'], c['relayout'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
done; done
