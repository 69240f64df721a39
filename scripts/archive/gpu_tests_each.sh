#!/bin/bash
# Every -m gpu test file in its own pytest process (per-file wall time, exit hangs visible).
set -o pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/each; mkdir -p $O
for f in ${TESTS:-tests/test_*.py}; do
  grep -q "gpu" $f || continue
  s=$(date +%s.%N)
  timeout -k 5 ${TLIM:-170} python -u -m pytest $f -m gpu -x -q --timeout 150 --timeout-method thread > $O/$(basename $f).log 2>&1; rc=$?
  e=$(date +%s.%N)
  echo "$f rc=$rc wall=$(python3 -c "print(round($e-$s,1))") $(tail -1 $O/$(basename $f).log)" | tee -a $O/summary.txt
  [ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
done
