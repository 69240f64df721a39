#!/bin/bash
# Run a subset (or all) of the -m gpu tests: TESTS="tests/x.py tests/y.py" bash scripts/gpu_tests.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/tests
mkdir -p $O
timeout -k 10 ${TLIM:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_gpu.log | tail -40
exit $rc
