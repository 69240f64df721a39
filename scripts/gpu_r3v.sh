#!/bin/bash
# Round 3: W-HC with relayout plans across circuit seeds (30q seeds 1-4, 28q seeds 42/4, 26q).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/seeds_rl; mkdir -p $O
for spec in "30 1" "30 2" "30 3" "30 4" "28 42" "28 4" "26 42"; do
  set -- $spec
  timeout -k 10 300 python3 bench.py --qubits $1 --seed $2 --cpu-budget 0 --no-1q28 --no-batch16 --steps 10 > $O/b$1_s$2.json 2> $O/b$1_s$2.err || { tail -5 $O/b$1_s$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b$1_s$2.json'));c=d['config'];print($1, $2, d['value'], c['passes'], c['relayout'], c['tile_qubits'], d['roofline']['frac'])"
done
