#!/bin/bash
# W-HC 30q: layout candidates (QSIM_RELABEL_TRIES) vs measured circuit time on this box
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/htries; mkdir -p $O
for t in 7 0 3 15 31; do
  QSIM_RELABEL_TRIES=$t timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-budget 0 --no-1q28 > $O/t$t.json 2> $O/t$t.err || { tail $O/t$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/t$t.json'));print($t, d['value'], d['ms_per_step'], d['config'].get('tile_passes'), d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
done
