#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3h
mkdir -p $O
DBG_REALLOC=3 QSIM_LAYOUT_T13=1.25 timeout -k 10 200 python -u scripts/dbg_alloc.py 2>&1 | tail -1 | tee -a $O/res.jsonl || exit 1
for off in 4 64 1024 2048 4096 16384 65536 262144 0; do
  QSIM_STATE_OFFSET_KB=$off QSIM_LAYOUT_T13=1.25 timeout -k 10 200 python -u scripts/dbg_alloc.py 2>&1 | tail -1 | tee -a $O/res.jsonl || exit 1
done
