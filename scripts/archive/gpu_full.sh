#!/bin/bash
# The driver's round-end GPU steps: the whole -m gpu suite in one process, then smoke().
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/full; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
