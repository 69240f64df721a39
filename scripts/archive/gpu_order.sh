#!/bin/bash
# Tile-order variants (QSIM_JIT_XCD) on the W-HC bench: per-pass kernel times via rocprofv3.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for x in ${ORDERS:-0 1 2 5 8 -1}; do
  QSIM_JIT_XCD=$x TAG=ord$x QUBITS=${QUBITS:-30} bash $R/scripts/gpu_prof.sh > $R/gpurun_out/ord$x.txt 2>&1 || { cat $R/gpurun_out/ord$x.txt; exit 1; }
  echo "order $x"; grep '"qk' $R/gpurun_out/ord$x.txt | cut -d, -f1,4 | tr '\n' ' '; echo
done
