#!/bin/bash
# Probe: per-gate H bandwidth vs state size (Infinity Cache residency), fused W-HC per-pass time.
set -o pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/mall; mkdir -p $O
for n in 21 22 23 24 25 26 28; do
  timeout -k 10 120 python bench.py --workload 1q --qubits $n --steps 5 --warmup 2 --cpu-budget 0 > $O/w1q_$n.json || exit 1
  python3 -c "
import json; d=json.load(open('$O/w1q_$n.json')); r=d['roofline']
print('W-1Q', $n, r['kernel'], r['avg_launch_ms'], r['achieved'], r['frac'])"
done
for n in 23 24 26; do
  timeout -k 10 120 python bench.py --workload hc --qubits $n --steps 10 --warmup 2 --cpu-budget 0 --no-1q28 > $O/hc_$n.json || exit 1
  python3 -c "
import json; d=json.load(open('$O/hc_$n.json')); r=d['roofline']
print('W-HC', $n, d['value'], d['ms_per_step'], r['avg_launch_ms'], r['achieved'], r['frac'], r['launches'])"
done
