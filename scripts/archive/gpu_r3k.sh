#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3k
mkdir -p $O
QSIM_TILE_HMAX=7 QSIM_LAYOUT_T13=1.25 DBG_STATES=5 timeout -k 10 300 python -u scripts/dbg_multi_alloc.py 2>&1 | tail -1 | tee $O/h7.json || exit 1
QSIM_TILE_HMAX=6 DBG_STATES=5 timeout -k 10 300 python -u scripts/dbg_multi_alloc.py 2>&1 | tail -1 | tee $O/h6.json || exit 1
