#!/bin/bash
# W-HC bench lines at 20..28 qubits (current defaults) + one kernel trace at 24q
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/sizes; mkdir -p $O
for n in 20 22 24 26 28; do
  timeout -k 10 150 python bench.py --qubits $n --steps 50 --warmup 3 --cpu-budget 0 --no-1q28 > $O/hc$n.json 2> $O/hc$n.err || { tail $O/hc$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/hc$n.json'));r=d['roofline'];c=d['config'];print($n, d['value'], d['ms_per_step'], r['avg_launch_ms'], r['launches'], r['frac'], c.get('tile_passes'), c.get('jit_passes'))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/tr24 -o run --output-format csv -- python3 $R/bench.py --qubits 24 --steps 20 --warmup 3 --cpu-budget 0 --no-1q28 > $O/tr24.log 2>&1 || { tail $O/tr24.log; exit 1; }
find $O/tr24 -name '*kernel_stats.csv' -exec head -6 {} \;
