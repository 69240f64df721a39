#!/bin/bash
# Relabeling bench: W-HC 30q and 28q with and without relabeling, seeds 42 and 1.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/rbench; mkdir -p $O
for n in 30 28; do for s in 42 1; do for rl in 1 0; do
  QSIM_RELABEL=$rl timeout -k 10 300 python bench.py --qubits $n --seed $s --cpu-budget 0 --no-1q28 > $O/b${n}_s${s}_r${rl}.json 2> $O/b${n}_s${s}_r${rl}.err || { tail $O/b${n}_s${s}_r${rl}.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/b${n}_s${s}_r${rl}.json')); r=d['roofline']
print('n=$n seed=$s relabel=$rl', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], r['launches'])"
done; done; done
