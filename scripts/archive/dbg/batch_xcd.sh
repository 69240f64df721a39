#!/bin/bash
# W-BATCH: JIT tile orders (QSIM_JIT_XCD) and cache policy vs pass time
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/bxcd; mkdir -p $O
for x in 1 0 -1 4 8 12; do
  QSIM_JIT_XCD=$x timeout -k 10 200 python bench.py --workload batch --steps 20 --warmup 3 --cpu-budget 0 > $O/x$x.json 2> $O/x$x.err || { tail $O/x$x.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/x$x.json'));print('xcd', $x, d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
done
QSIM_JIT_NT=0 timeout -k 10 200 python bench.py --workload batch --steps 20 --warmup 3 --cpu-budget 0 > $O/nt0.json 2> $O/nt0.err || { tail $O/nt0.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/nt0.json'));print('nt0', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
