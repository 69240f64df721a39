#!/bin/bash
# Round 3: relayout GPU tests (incl. basis state + readers + per-gate entries).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/rl_tests; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_relayout_gpu.py > $O/pytest.log 2>&1 || { grep -E "FAILED|^E " $O/pytest.log | head -30; tail -3 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
