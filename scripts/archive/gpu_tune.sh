#!/bin/bash
# Sweep the launch knobs on one GPU (one process per configuration):
#   per-gate kernels: QSIM_NT x QSIM_SLICE_U (LANE_U = DIAG_U = 2*SLICE_U)
#   fused passes:     QSIM_FUSED_NT 0/1 on the 28q W-HC bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/tune
mkdir -p $OUT
for nt in ${NTS:-0 1}; do
  for su in ${SUS:-1 2 4}; do
    lu=$((su * 2))
    echo "== NT=$nt SLICE_U=$su LANE_U=$lu DIAG_U=$lu"
    QSIM_NT=$nt QSIM_SLICE_U=$su QSIM_LANE_U=$lu QSIM_DIAG_U=$lu timeout -k 10 200 \
      python scripts/gate_microbench.py --qubits ${QUBITS:-28} --label "nt$nt-su$su" \
      > $OUT/nt${nt}_su${su}.json 2> $OUT/nt${nt}_su${su}.err || { tail -5 $OUT/nt${nt}_su${su}.err; exit 1; }
    python -c "
import json; d=json.load(open('$OUT/nt${nt}_su${su}.json'))
print(' '.join(f\"{r['gate']}{r['qubits']}:{r['GBps']:.0f}\" for r in d['results']))"
  done
done
if [ -n "$FUSED" ]; then
  for fnt in 0 1; do
    echo "== QSIM_FUSED_NT=$fnt (28q W-HC)"
    QSIM_FUSED_NT=$fnt timeout -k 10 300 python bench.py --qubits 28 --steps 5 --warmup 2 --cpu-budget 0 \
      > $OUT/fused_nt$fnt.json 2> $OUT/fused_nt$fnt.err || { tail -5 $OUT/fused_nt$fnt.err; exit 1; }
    python -c "
import json; d=json.loads(open('$OUT/fused_nt$fnt.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline'])"
  done
fi
