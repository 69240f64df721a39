#!/bin/bash
# Pass time of fixed tiles under every workgroup -> tile order (QSIM_JIT_XCD).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/op; mkdir -p $O
export PROBE_LIST="0,1,2,3,4,7,16,19,20,23,24,27;0,1,2,3,15,16,18,20,22,26,27,28;0,1,2,3,4,5,14,16,17,21,23,28;0,1,2,3,4,5,6,10,14,18,22,26;0,1,2,3,6,13,16,23,25,26,28,29;0,1,2,3,4,5,24,25,26,27,28,29;0,1,2,3,4,5,12,13,14,15,16,17;0,1,2,3,4,11,21,22,23,24,25,26;0,1,2,3,9,10,14,17,19,21,23,26"
for x in 1 0 -1 2 4 6 8 10 12 14; do
  QSIM_JIT_XCD=$x timeout -k 10 120 python scripts/layout_probe.py 4 > $O/xcd_$x.jsonl 2> $O/xcd_$x.err || exit 1
  echo "xcd $x done"
done
