#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3g
mkdir -p $O
(rocm-smi --showtemp --showclocks --showpower > $O/smi_before.txt 2>&1 || true)
QSIM_LAYOUT_T13=1.25 DBG_SECONDS=60 timeout -k 10 200 python -u scripts/dbg_h7_time.py > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
(rocm-smi --showtemp --showclocks --showpower > $O/smi_mid.txt 2>&1 || true)
QSIM_LAYOUT_T13=1.25 DBG_SECONDS=30 timeout -k 10 200 python -u scripts/dbg_h7_time.py > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
head -3 $O/p1.log; tail -3 $O/p1.log | head -2; head -3 $O/p2.log; tail -3 $O/p2.log | head -2
