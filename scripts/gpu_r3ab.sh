#!/bin/bash
# Round 3 final tree: W-HC at 26-29 qubits (calibrated first runs; relayout variants among the candidates).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/sizes_final; mkdir -p $O
for q in 26 27 28 29; do
  timeout -k 10 300 python3 bench.py --qubits $q --cpu-budget 0 --no-1q28 --no-batch16 --steps 20 > $O/b$q.json 2> $O/b$q.err || { tail -5 $O/b$q.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b$q.json'));c=d['config'];print($q, d['value'], d['ms_per_step'], c['passes'], c['relayout'], c['tile_qubits'], c['calibrated'], d['roofline']['frac'])"
done
