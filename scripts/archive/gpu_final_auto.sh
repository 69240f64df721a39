#!/bin/bash
# Round-end evidence (scripts/gpu_final.sh) + W-HC at 26/27/29q with the default (size-based) tile height.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && bash scripts/gpu_final.sh || exit 1
O=$R/gpurun_out/final
for Q in 26 27 29; do
  timeout -k 10 300 python bench.py --qubits $Q --cpu-budget 0 > $O/bench$Q.json 2> $O/bench$Q.err || exit 1
done
python - <<PY
import json
for n in (26, 27, 28, 29, 30):
    d = json.load(open('$O/bench%d.json' % n)); r = d['roofline']
    print(n, d['value'], d['ms_per_step'], round(r['frac'], 4), r['launches'], r['avg_launch_ms'])
PY
for NT in 0 1; do
  QSIM_JIT_NT=$NT timeout -k 10 300 python bench.py --qubits 20 --cpu-budget 0 > $O/bench20_nt$NT.json 2> $O/bench20_nt$NT.err || exit 1
  python -c "import json; d=json.load(open('$O/bench20_nt$NT.json')); print('20q NT=$NT', d['value'], d['roofline']['avg_launch_ms'])"
done
