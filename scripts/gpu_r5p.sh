#!/bin/bash
# Round 5: trajectory-split in-tile runs — k = 2 / 3, with the side streams at low priority.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5p}
mkdir -p $O
for v in "2 0" "3 0" "2 1" "2 0"; do
  set -- $v
  QSIM_NOISE_SPLIT=$1 QSIM_NOISE_STREAM_PRIO=$2 timeout -k 10 300 python -u bench.py --workload batch --cpu-budget 0 --steps 5 --warmup 1 > $O/b$1_$2.json 2> $O/b$1_$2.err || { tail -5 $O/b$1_$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b$1_$2.json'));print('split=$1 prio=$2', d['value'], d['ms_per_step'])"
done
