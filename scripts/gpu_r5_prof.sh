#!/bin/bash
# Round 5: timed-region profiles (roctx range, --marker-trace) of the noisy26 (serial run) and dm14
# objects, with the roofline recomputed from rocprof (scripts/roofline_check.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/${1:-r5prof}
mkdir -p $O
prof() {  # region, extra bench args...
  local rg=$1; shift
  cd /tmp && timeout -k 10 400 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv \
    -d $O/prof_$rg -o $rg -- python3 $R/bench.py --cpu-budget 0 --profile-region $rg "$@" \
    > $O/bench_$rg.json 2> $O/bench_$rg.err || { tail -5 $O/bench_$rg.err; return 1; }
  cd $R
  python3 scripts/roofline_check.py $rg $O/bench_$rg.json $O/prof_$rg/${rg}_kernel_trace.csv $O/check_$rg.json \
    --markers=$O/prof_$rg/${rg}_marker_api_trace.csv | grep -E "frac|launches"
}
prof noisy26 --workload noisy --steps 3 || exit 1
prof dm14 --workload dm --steps 5 || exit 1
