#!/bin/bash
# Physically contiguous state allocations (hipDeviceMallocContiguous) vs plain hipMalloc, several
# processes in a row (the first process on a box ran 13-qubit passes 12 % faster than later ones).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3j
mkdir -p $O
b() { local name=$1; shift; env "$@" QSIM_LAYOUT_T13=1.25 timeout -k 10 300 python bench.py --cpu-budget 0 --no-1q28 > $O/$name.json 2> $O/$name.err || { tail -3 $O/$name.err; exit 1; }
      python -c "import json; d=json.load(open('$O/$name.json')); print('$name', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['launches'])"; }
b c1_h7 QSIM_STATE_CONTIGUOUS=1 QSIM_TILE_HMAX=7
b p1_h7 QSIM_TILE_HMAX=7
b c2_h7 QSIM_STATE_CONTIGUOUS=1 QSIM_TILE_HMAX=7
b c3_h6 QSIM_STATE_CONTIGUOUS=1 QSIM_TILE_HMAX=6
b p2_h6 QSIM_TILE_HMAX=6
b c4_h7 QSIM_STATE_CONTIGUOUS=1 QSIM_TILE_HMAX=7
b p3_h7 QSIM_TILE_HMAX=7
