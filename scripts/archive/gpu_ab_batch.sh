#!/bin/bash
# A/B on one box: W-BATCH 16q x 1024 with the session-start tree (_ab_old, untracked) vs the current one, alternated.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab
mkdir -p $O
cd $R
for i in 1 2; do
  for t in old new; do
    B=bench.py; [ $t = old ] && B=_ab_old/bench.py
    timeout -k 10 300 python $B --workload batch --cpu-budget 0 --steps 10 > $O/${t}_$i.json 2> $O/${t}_$i.err || exit 1
    python -c "import json; d=json.load(open('$O/${t}_$i.json')); r=d['roofline']; print('$t $i', d['value'], d['ms_per_step'], r['avg_launch_ms'])"
  done
done
