#!/bin/bash
# Round 4: pulled-noise tests, then the push / pull experiment.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${1:-r4d}
mkdir -p gpurun_out/$O
timeout -k 10 600 python -u -m pytest tests/test_batched_refnoise_gpu.py tests/test_noisy_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/$O/pytest.log 2>&1 || { tail -30 gpurun_out/$O/pytest.log; exit 1; }
tail -2 gpurun_out/$O/pytest.log
bash scripts/gpu_r4_noise.sh $O/noise
