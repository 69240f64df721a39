#!/bin/bash
# Dump every hipRTC source the dist GPU tests generate (QSIM_JIT_DUMP), to find compiler crashes.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/jitdump; mkdir -p $O
QSIM_JIT_DUMP=$O timeout -k 10 150 python -u -m pytest tests/test_dist_gpu.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
echo "rc=$?"; ls $O | wc -l; tail -3 $O/pytest.log
