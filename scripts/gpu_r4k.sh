#!/bin/bash
# Round 4: gate + in-tile noise kernel: batched reference-noise tests, then W-BATCH 16q x 1024
# with the tile kernel and without.  Usage: gpu_r4k.sh <outdir>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${1:-r4k}
mkdir -p gpurun_out/$O
timeout -k 10 600 python -u -m pytest tests/test_batched_refnoise_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/$O/pytest.log 2>&1 || { tail -30 gpurun_out/$O/pytest.log; exit 1; }
tail -1 gpurun_out/$O/pytest.log
for tile in 1 0; do
  QSIM_NOISE_TILE=$tile timeout -k 10 200 python -u bench.py --workload batch --cpu-budget 0 --steps 3 --warmup 1 > gpurun_out/$O/batch_tile$tile.json 2> gpurun_out/$O/batch_tile$tile.err || { tail -5 gpurun_out/$O/batch_tile$tile.err; exit 1; }
  python3 - gpurun_out/$O/batch_tile$tile.json tile=$tile <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = {x["name"]: (round(x["ms"] / max(1, x["launches"]), 4), x["launches"]) for x in d["kernels"]}
print(sys.argv[2], d["value"], d["ms_per_step"], k)
PY
done
