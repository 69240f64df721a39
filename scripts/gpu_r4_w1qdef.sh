#!/bin/bash
# Round 4: W-1Q 28q (bench roofline_1q28) under candidate far-target defaults, 3 repeats each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=$PWD/gpurun_out/${1:-r4w1qdef}
mkdir -p $O
run() {  # name, env...
  local name=$1; shift
  for r in 1 2 3; do
    env "$@" STEPS=3 timeout -k 10 120 python -u scripts/w1q28.py > $O/$name.$r.json 2> $O/$name.$r.err || { tail -5 $O/$name.$r.err; return 1; }
  done
  python3 - $name $O/$name.*.json <<'PY'
import json, sys
fr = [json.load(open(f))["frac"] for f in sys.argv[2:]]
print(sys.argv[1], [round(x, 4) for x in fr], "mean", round(sum(fr) / len(fr), 4))
PY
}
run old QSIM_SLICE_FAR_MODE=0 QSIM_SLICE_U_FAR=4 QSIM_SLICE_FAR_LO=20 QSIM_SLICE_FAR_HI=25 || exit 1
run m2u2_20_27 QSIM_SLICE_FAR_MODE=2 QSIM_SLICE_U_FAR=2 QSIM_SLICE_FAR_LO=20 QSIM_SLICE_FAR_HI=27 || exit 1
run m2u2_20_25 QSIM_SLICE_FAR_MODE=2 QSIM_SLICE_U_FAR=2 QSIM_SLICE_FAR_LO=20 QSIM_SLICE_FAR_HI=25 || exit 1
run m2u4_20_27 QSIM_SLICE_FAR_MODE=2 QSIM_SLICE_U_FAR=4 QSIM_SLICE_FAR_LO=20 QSIM_SLICE_FAR_HI=27 || exit 1
run m2u2_20_27_nt0 QSIM_NT=0 QSIM_SLICE_FAR_MODE=2 QSIM_SLICE_U_FAR=2 QSIM_SLICE_FAR_LO=20 QSIM_SLICE_FAR_HI=27 || exit 1
run new_default || exit 1
