#!/bin/bash
# h = 7 pipelined pass kernels: tile order (QSIM_JIT_PIPE_ORDER) and cache policy (QSIM_JIT_NT) at 30q/28q.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/h7k
mkdir -p $O
cd $R
for c in ${ENVS:-0:1 1:1 0:0 1:0}; do
  IFS=: read OR NT <<< "$c"
  for Q in ${QUBITS:-30 28}; do
    QSIM_TILE_HMAX=7 QSIM_JIT_PIPE_ORDER=$OR QSIM_JIT_NT=$NT timeout -k 10 300 python bench.py --qubits $Q --cpu-budget 0 \
      > $O/b${Q}_o${OR}_nt$NT.json 2> $O/b${Q}_o${OR}_nt$NT.err || exit 1
  done
done
python - <<PY
import json, glob
for f in sorted(glob.glob('$O/b*.json')):
    d = json.load(open(f)); r = d['roofline']
    print(f.split('/')[-1], d['value'], d['ms_per_step'], r and round(r['frac'], 4), r and r.get('launches'), r and r.get('avg_launch_ms'))
PY
