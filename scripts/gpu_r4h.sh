#!/bin/bash
# Round 4: noisy tests (overlapped word maps), W-1Q default candidates, noisy 26q line, virtual
# 30q / 8 sharded run.  Usage: gpu_r4h.sh <outdir>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${1:-r4h}
mkdir -p gpurun_out/$O
timeout -k 10 300 python -u -m pytest tests/test_noisy_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/$O/pytest_noisy.log 2>&1 || { tail -30 gpurun_out/$O/pytest_noisy.log; exit 1; }
tail -1 gpurun_out/$O/pytest_noisy.log
bash scripts/gpu_r4_w1qdef.sh $O/w1qdef || exit 1
bash scripts/gpu_r4_noisy.sh $O/noisy || exit 1
timeout -k 10 400 python -u scripts/dist_virtual_bench.py 30 8 4 > gpurun_out/$O/dist_virtual_30q8.json 2> gpurun_out/$O/dist_virtual.err || { tail -5 gpurun_out/$O/dist_virtual.err; exit 1; }
head -c 1500 gpurun_out/$O/dist_virtual_30q8.json
bash scripts/gpu_r4_dmpmc.sh $O/dmpmc
