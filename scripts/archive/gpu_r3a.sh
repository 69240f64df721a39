#!/bin/bash
# Round 3: multi-process hosted ranks + virtual 30q/8-shard RCCL test + the dist suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r3a
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu \
    tests/test_dist_hosted_gpu.py tests/test_dist_gpu.py > gpurun_out/r3a/pytest.log 2>&1
rc=$?
tail -30 gpurun_out/r3a/pytest.log
exit $rc
