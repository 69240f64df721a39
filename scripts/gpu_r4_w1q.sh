#!/bin/bash
# W-1Q per target at 28 qubits for the far-partner slice variants (QSIM_SLICE_FAR_MODE 0/1/2,
# QSIM_SLICE_U_FAR 2/4/8), far range widened to targets 14..27 so every variant covers them.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=$PWD/gpurun_out/${1:-w1q}
export PYTHONPATH=$PWD/cuda-quantum-simulator_amd${PYTHONPATH:+:$PYTHONPATH}
mkdir -p $O
for mode in 0 1 2; do
  for u in 2 4 8; do
    QSIM_SLICE_FAR_LO=14 QSIM_SLICE_FAR_HI=27 QSIM_SLICE_FAR_MODE=$mode QSIM_SLICE_U_FAR=$u \
      timeout -k 10 120 python -u scripts/archive/dbg/h_per_target.py > $O/m${mode}_u${u}.jsonl 2> $O/m${mode}_u${u}.err || { tail -3 $O/m${mode}_u${u}.err; exit 1; }
    python3 - $O/m${mode}_u${u}.jsonl $mode $u <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
far = [r["frac"] for r in rows if 20 <= r["t"] <= 25]
print("mode", sys.argv[2], "u", sys.argv[3], "min20-25", min(far), "all>=14", round(min(r["frac"] for r in rows if r["t"] >= 14), 4))
PY
  done
done
