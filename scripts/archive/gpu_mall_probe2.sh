#!/bin/bash
set -o pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/mall2; mkdir -p $O
for n in 20 21 22 23 24; do
  QSIM_NT=0 timeout -k 10 120 python bench.py --workload 1q --qubits $n --steps 10 --warmup 2 --cpu-budget 0 > $O/w1q_$n.json || exit 1
  python3 -c "
import json; d=json.load(open('$O/w1q_$n.json')); r=d['roofline']
print('W-1Q NT=0', $n, r['kernel'], r['avg_launch_ms'], r['achieved'], r['frac'])"
done
for n in 22 23 24; do
  QSIM_FUSED_NT=0 timeout -k 10 120 python bench.py --workload hc --qubits $n --steps 10 --warmup 2 --cpu-budget 0 --no-1q28 --jit 0 > $O/hc_$n.json || exit 1
  python3 -c "
import json; d=json.load(open('$O/hc_$n.json')); r=d['roofline']
print('W-HC FUSED_NT=0 interp', $n, d['value'], d['ms_per_step'], r['avg_launch_ms'], r['achieved'], r['frac'], r['launches'])"
done
