#!/bin/bash
# W-HC 30q: do interpreter pass times rank layout candidates like the JIT ones?
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/htries_i; mkdir -p $O
for j in 0 2; do for t in 7 0 31; do
  QSIM_RELABEL_TRIES=$t timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-budget 0 --no-1q28 --jit $j > $O/t${t}_j$j.json 2> $O/t${t}_j$j.err || { tail $O/t${t}_j$j.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/t${t}_j$j.json'));print('jit', $j, 'tries', $t, d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done; done
