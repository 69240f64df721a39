#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r2b; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_cpp_api.py tests/test_matrix_api_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "Error|assert|FAIL" $O/pytest.log | head -30; exit 1; }
grep -E "passed|failed" $O/pytest.log
timeout -k 10 300 ./tests/cpp/build/bench_scaling 3 22 > $O/wref_scaling.jsonl || exit 1
cat $O/wref_scaling.jsonl
lscpu | grep -E "Model name|^CPU\(s\)" > $O/host_cpu.txt; cat $O/host_cpu.txt
