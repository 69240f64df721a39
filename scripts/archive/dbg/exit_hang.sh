#!/bin/bash
set -o pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/dbg; mkdir -p $O
for f in tests/test_dist_gpu.py tests/test_jit.py tests/test_bench_path_gpu.py; do
  s=$(date +%s.%N)
  timeout -k 5 150 python -u -m pytest $f -m gpu -x -q --timeout 120 --timeout-method thread > $O/$(basename $f).log 2>&1; rc=$?
  e=$(date +%s.%N)
  echo "$f rc=$rc wall=$(python3 -c "print(round($e-$s,1))") $(tail -1 $O/$(basename $f).log)"
  [ $rc -eq 0 ] || exit $rc
done
