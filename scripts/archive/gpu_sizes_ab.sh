#!/bin/bash
# W-HC 26/27q: relabeling on vs off (per-pass times)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/sizes_ab; mkdir -p $O
for n in 26 27; do for r in 1 0; do
  QSIM_RELABEL=$r timeout -k 10 150 python bench.py --qubits $n --steps 30 --warmup 3 --cpu-budget 0 --no-1q28 > $O/hc${n}_r$r.json 2> $O/hc${n}_r$r.err || { tail $O/hc${n}_r$r.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/hc${n}_r$r.json'));r=d['roofline'];print($n, $r, d['value'], d['ms_per_step'], r['avg_launch_ms'], r['launches'], r['frac'])"
done; done
