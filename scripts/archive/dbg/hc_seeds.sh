#!/bin/bash
# W-HC 30q over seeds (default settings: relabeling + calibration)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/hcseeds; mkdir -p $O
for s in 42 1 2 3 4; do
  timeout -k 10 200 python bench.py --seed $s --steps 5 --warmup 2 --cpu-budget 0 --no-1q28 > $O/s$s.json 2> $O/s$s.err || { tail $O/s$s.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/s$s.json'));print('seed', $s, d['value'], d['ms_per_step'], d['roofline']['launches'], d['roofline']['frac'])"
done
