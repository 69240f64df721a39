#!/bin/bash
# W-BATCH: layout candidates (QSIM_RELABEL_TRIES) vs pass time
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/btries; mkdir -p $O
for t in 0 3 7 15 31; do
  QSIM_RELABEL_TRIES=$t timeout -k 10 200 python bench.py --workload batch --steps 20 --warmup 3 --cpu-budget 0 > $O/t$t.json 2> $O/t$t.err || { tail $O/t$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/t$t.json'));print($t, d['value'], d['ms_per_step'], d['config']['tile_passes'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
done
