#!/bin/bash
# Round 5, first GPU call: the new parity tests (large-n vs the oracle, pinned pointers, carry),
# then timed-region-only rocprofv3 profiles of the three roofline objects
# (--profile-region + --selected-regions) and their recomputation (scripts/roofline_check.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/${1:-r5a}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_headline_gpu.py::test_pinned_state_is_never_relabeled \
  tests/test_noisy_gpu.py::test_pulled_noise_on_a_pinned_pointer \
  tests/test_dist_gpu.py::test_cross_run_carry_matches_oracle \
  tests/test_large_oracle_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -15 $O/pytest.log
prof() {  # region, extra bench args...
  local rg=$1; shift
  cd /tmp && timeout -k 10 400 rocprofv3 --selected-regions --kernel-trace --stats --output-format csv \
    -d $O/prof_$rg -o $rg -- python3 $R/bench.py --cpu-budget 0 --profile-region $rg "$@" \
    > $O/bench_$rg.json 2> $O/bench_$rg.err || { tail -5 $O/bench_$rg.err; return 1; }
  cd $R
  local tr=$(find $O/prof_$rg -name "*kernel_trace.csv" | head -1)
  python3 scripts/roofline_check.py $rg $O/bench_$rg.json $tr $O/check_$rg.json
}
prof hc --steps 20 --warmup 2 --no-1q28 --no-batch16 --no-extras || exit 1
prof 1q28 --steps 3 --warmup 1 --no-batch16 --no-extras || exit 1
prof batch16ref --steps 3 --warmup 1 --no-1q28 --no-extras || exit 1
