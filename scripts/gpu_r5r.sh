#!/bin/bash
# Round 5: potential of a cheaper pull walk / flip phase under the 2-way split (timing knobs only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5r}
mkdir -p $O
for sk in 0 2 1 3; do
  QSIM_NOISE_TILE_SKIP=$sk timeout -k 10 300 python -u bench.py --workload batch --cpu-budget 0 --steps 5 --warmup 1 > $O/b$sk.json 2> $O/b$sk.err || { tail -5 $O/b$sk.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b$sk.json'));print('skip=$sk', d['value'], d['ms_per_step'])"
done
