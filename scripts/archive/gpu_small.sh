#!/bin/bash
# Small-state (cache-resident) W-HC: 20q and 24q bench lines, tile height variants, kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/small; mkdir -p $O
for n in 20 22 24; do
  timeout -k 10 120 python bench.py --qubits $n --steps 200 --warmup 5 --cpu-budget 0 --no-1q28 > $O/hc$n.json 2> $O/hc$n.err || { tail $O/hc$n.err; exit 1; }
  QSIM_TILE_HMAX=5 timeout -k 10 120 python bench.py --qubits $n --steps 200 --warmup 5 --cpu-budget 0 --no-1q28 > $O/hc${n}_h5.json 2> $O/hc${n}_h5.err || { tail $O/hc${n}_h5.err; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/tr20 -o run --output-format csv -- python3 $R/bench.py --qubits 20 --steps 50 --warmup 5 --cpu-budget 0 --no-1q28 > $O/tr20.log 2>&1 || { tail $O/tr20.log; exit 1; }
python3 - <<PY
import json, glob
for f in sorted(glob.glob('$O/hc*.json')):
    d=json.load(open(f)); r=d['roofline']
    print(f.split('/')[-1], d['value'], d['ms_per_step'], r['avg_launch_ms'], r['launches'])
PY
