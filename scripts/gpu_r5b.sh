#!/bin/bash
# Round 5: the new in-tile noise kernel (tests + W-BATCH against the push kernels), the large-n
# oracle tests, the carry test, and the timed-region-only profiles of the roofline objects.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/${1:-r5b}
mkdir -p $O
PT="python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 600 $PT -x tests/test_batched_refnoise_gpu.py > $O/pytest_batch.log 2>&1 || { tail -30 $O/pytest_batch.log; exit 1; }
tail -3 $O/pytest_batch.log
for t in 1 0; do
  QSIM_NOISE_TILE=$t timeout -k 10 300 python -u bench.py --workload batch --cpu-budget 0 --steps 5 --warmup 1 > $O/batch_tile$t.json 2> $O/batch_tile$t.err || { tail -5 $O/batch_tile$t.err; exit 1; }
  python3 - $O/batch_tile$t.json tile=$t <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = {x["name"]: (round(x["ms"] / max(1, x["launches"]), 4), x["launches"]) for x in d["kernels"]}
print(sys.argv[2], d["value"], d["ms_per_step"], k)
PY
done
timeout -k 10 300 $PT -s tests/test_dist_gpu.py::test_cross_run_carry_matches_oracle > $O/pytest_carry.log 2>&1; echo "carry rc $?"
grep -E "carry merges|passed|failed" $O/pytest_carry.log | tail -8
timeout -k 10 900 $PT -x tests/test_large_oracle_gpu.py > $O/pytest_large.log 2>&1 || { tail -30 $O/pytest_large.log; exit 1; }
tail -6 $O/pytest_large.log
prof() {  # region, extra bench args...
  local rg=$1; shift
  cd /tmp && timeout -k 10 400 rocprofv3 --selected-regions --kernel-trace --stats --output-format csv \
    -d $O/prof_$rg -o $rg -- python3 $R/bench.py --cpu-budget 0 --profile-region $rg "$@" \
    > $O/bench_$rg.json 2> $O/bench_$rg.err || { tail -5 $O/bench_$rg.err; return 1; }
  cd $R
  local tr=$(find $O/prof_$rg -name "*kernel_trace.csv" | head -1)
  python3 scripts/roofline_check.py $rg $O/bench_$rg.json $tr $O/check_$rg.json | grep -E "frac|launches|avg|median"
}
prof hc --steps 20 --warmup 2 --no-1q28 --no-batch16 --no-extras || exit 1
prof 1q28 --steps 3 --warmup 1 --no-batch16 --no-extras || exit 1
prof batch16ref --steps 3 --warmup 1 --no-1q28 --no-extras || exit 1
