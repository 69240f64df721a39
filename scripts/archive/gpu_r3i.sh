#!/bin/bash
# Is the 13-qubit-tile 30q speed a function of the chip's thermal / power state?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3i
mkdir -p $O
smi() { rocm-smi --showtemp --showclocks --showpower 2>/dev/null | grep -E "junction|memory|mclk|sclk|Power" | tr -s ' ' | tr '\n' ' '; echo; }
b() { QSIM_TILE_HMAX=7 QSIM_LAYOUT_T13=1.25 timeout -k 10 300 python bench.py --cpu-budget 0 --no-1q28 > $O/$1.json 2> $O/$1.err || exit 1
      python -c "import json; d=json.load(open('$O/$1.json')); print('$1', d['value'], d['ms_per_step'], d['ms_per_step_min_max'])"; }
smi; b cold1; smi; b cold2; smi
QSIM_LAYOUT_T13=1.25 DBG_SECONDS=60 timeout -k 10 200 python -u scripts/dbg_h7_time.py > $O/heat.log 2>&1 || exit 1
smi; b hot1; smi; sleep 90; smi; b rest1; smi; sleep 90; b rest2; smi
