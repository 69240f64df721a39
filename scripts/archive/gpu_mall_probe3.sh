#!/bin/bash
set -o pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/mall3; mkdir -p $O
for nt in 1 0; do
for n in 22 23 24 26; do
  QSIM_JIT_NT=$nt timeout -k 10 120 python bench.py --workload hc --qubits $n --steps 10 --warmup 2 --cpu-budget 0 --no-1q28 > $O/hc_${nt}_$n.json || exit 1
  python3 -c "
import json; d=json.load(open('$O/hc_${nt}_$n.json')); r=d['roofline']
print('W-HC JIT_NT=$nt', $n, d['value'], d['ms_per_step'], r['avg_launch_ms'], r['achieved'], r['frac'], r['launches'])"
done
done
