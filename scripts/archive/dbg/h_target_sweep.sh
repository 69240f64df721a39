#!/bin/bash
# Per-target H at 28q under per-gate kernel knobs (slice unroll U, non-temporal loads)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/htarget; mkdir -p $O
for cfg in "1 1" "2 1" "4 1" "1 0"; do set -- $cfg
  QSIM_SLICE_U=$1 QSIM_NT=$2 timeout -k 10 200 python scripts/dbg/h_per_target.py > $O/u$1_nt$2.jsonl 2> $O/u$1_nt$2.err || { tail $O/u$1_nt$2.err; exit 1; }
  python3 -c "
import json
r=[json.loads(l) for l in open('$O/u$1_nt$2.jsonl')]
print('U', $1, 'NT', $2, 'mean frac', round(sum(x['frac'] for x in r)/len(r),4), ' '.join(f\"{x['t']}:{x['frac']:.3f}\" for x in r if x['t']>=6))"
done
