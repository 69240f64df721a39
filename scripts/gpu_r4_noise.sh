#!/bin/bash
# Round 4: W-BATCH 16q x 1024 reference-noise step, pushed vs pulled noise (kernel breakdown from
# the bench's per-launch timer), pulled at p = 0 / 0.001 / 0.01.  Usage: gpu_r4_noise.sh <outdir>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=$PWD/gpurun_out/${1:-r4noise}
mkdir -p $O
run() {  # name, noise p, env...
  local name=$1 p=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --workload batch --noise $p --cpu-budget 0 --steps 2 --warmup 1 > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; return 1; }
  python3 - $O/$name.json $name <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
ks = d.get("kernels") or d.get("roofline", {}).get("kernels") or []
print(sys.argv[2], d["value"], d["ms_per_step"], json.dumps(ks)[:600])
PY
}
run push 0.01 QSIM_NOISE_PULL=0 || exit 1
run pull 0.01 QSIM_NOISE_PULL=1 || exit 1
run pull_serial 0.01 QSIM_NOISE_PULL=1 QSIM_NOISE_MAP_OVERLAP=0 || exit 1
run pull_p0 0 QSIM_NOISE_PULL=1 || exit 1
run pull_p001 0.001 QSIM_NOISE_PULL=1 || exit 1
run push_p001 0.001 QSIM_NOISE_PULL=0 || exit 1
