#!/bin/bash
# Round 3: reproduce round 2's h=7 / T13=1.25 30q seed-42 result with that commit's build (54097c9)
# next to the current tree, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=$PWD/gpurun_out/r3f
mkdir -p $O
for i in 1 2; do
  (cd scratch_old54 && QSIM_RELABEL_DEBUG=1 QSIM_TILE_HMAX=7 QSIM_LAYOUT_T13=1.25 timeout -k 10 300 python bench.py --cpu-budget 0 --no-1q28 > $O/old_$i.json 2> $O/old_$i.err) || { tail -5 $O/old_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$O/old_$i.json')); r=d['roofline']; print('old $i', d['value'], d['ms_per_step'], r['launches'], r['avg_launch_ms'])"
  QSIM_RELABEL_DEBUG=1 QSIM_TILE_HMAX=7 QSIM_LAYOUT_T13=1.25 timeout -k 10 300 python bench.py --cpu-budget 0 --no-1q28 > $O/new_$i.json 2> $O/new_$i.err || { tail -5 $O/new_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$O/new_$i.json')); r=d['roofline']; print('new $i', d['value'], d['ms_per_step'], r['launches'], r['avg_launch_ms'])"
done
grep -h calibrate $O/*.err || true
