#!/bin/bash
# W-1Q per target at 28 qubits with 1 / 2 / 4 / 8 wave-items in flight for the far-partner targets.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3l
mkdir -p $O
for U in 4 2 8 1; do
  QSIM_SLICE_U_FAR=$U timeout -k 10 200 python -u scripts/archive/dbg/h_per_target.py > $O/u$U.jsonl 2>&1 || { tail -3 $O/u$U.jsonl; exit 1; }
  python -c "
import json; r=[json.loads(l) for l in open('$O/u$U.jsonl') if l.startswith('{')]
print('U_far=$U', 'min', min(x['frac'] for x in r), 'mean', round(sum(x['frac'] for x in r)/len(r),4), [x['frac'] for x in r if 18<=x['t']<=27])"
done
