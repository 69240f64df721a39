#!/bin/bash
# Which group of tests/test_dist_gpu.py leaves the process hanging at exit?  Each group runs in
# its own pytest process; when the process outlives its test summary by 25 s, the thread names
# and kernel wait channels are dumped and the process is killed (no GPU work is outstanding then).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/exitp; mkdir -p $O
run() {
  local tag=$1; shift
  python -u -m pytest tests/test_dist_gpu.py -m gpu -q --timeout 120 --timeout-method thread "$@" > $O/$tag.log 2>&1 &
  local pid=$! t=0 done_t=-1
  while kill -0 $pid 2>/dev/null; do
    sleep 1; t=$((t+1))
    if [ $done_t -lt 0 ] && grep -qE "passed|failed|error" $O/$tag.log; then done_t=$t; fi
    if [ $done_t -ge 0 ] && [ $((t-done_t)) -ge 25 ]; then
      echo "$tag: HANG at exit" | tee -a $O/summary.txt
      for d in /proc/$pid/task/*; do echo "$(basename $d) $(cat $d/comm) $(cat $d/wchan 2>/dev/null) $(cut -d' ' -f3 $d/stat)"; done > $O/$tag.threads
      cat /proc/$pid/maps | awk '{print $6}' | sort -u | grep -E "\.so" > $O/$tag.maps
      kill -9 $pid; wait $pid; return 1
    fi
    [ $t -ge 170 ] && { echo "$tag: timeout" | tee -a $O/summary.txt; kill -9 $pid; return 1; }
  done
  wait $pid; local rc=$?
  echo "$tag: rc=$rc exit $((t-done_t))s after summary: $(tail -1 $O/$tag.log)" | tee -a $O/summary.txt
  return 0
}
run virt -k "virtual_ranks or pipelined" && run rccl -k "single_rank" && run ovl -k "overlapped" && run all
