#!/bin/bash
# Kernel trace of the virtual 30q/8-rank run, overlap on / off (per-launch durations).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/dtrace; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/ovl -o run --output-format csv -- python3 $R/scripts/dist_virtual_bench.py 30 8 2 > $O/ovl.log 2>&1 || { tail $O/ovl.log; exit 1; }
QSIM_DIST_OVERLAP=0 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/noovl -o run --output-format csv -- python3 $R/scripts/dist_virtual_bench.py 30 8 2 > $O/noovl.log 2>&1 || { tail $O/noovl.log; exit 1; }
ls -R $O | head
