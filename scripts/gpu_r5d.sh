#!/bin/bash
# Round 5: in-tile noise with precomputed flip lists (tests, W-BATCH variants), the sharded
# engine with coarse parts (virtual / RCCL-world-1 / hosted tests), headline profile at 30q with
# the roctx marker range.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/${1:-r5d}
mkdir -p $O
PT="python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 600 $PT -x tests/test_batched_refnoise_gpu.py > $O/pytest_batch.log 2>&1 || { tail -30 $O/pytest_batch.log; exit 1; }
tail -2 $O/pytest_batch.log
for v in "1 1" "1 0" "0 1"; do
  set -- $v
  QSIM_NOISE_TILE=$1 QSIM_NOISE_TILE_LISTS=$2 timeout -k 10 300 python -u bench.py --workload batch --cpu-budget 0 --steps 5 --warmup 1 > $O/batch_$1_$2.json 2> $O/batch_$1_$2.err || { tail -5 $O/batch_$1_$2.err; exit 1; }
  python3 - $O/batch_$1_$2.json "tile=$1 lists=$2" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = {x["name"]: (round(x["ms"] / max(1, x["launches"]), 4), x["launches"]) for x in d["kernels"]}
print(sys.argv[2], d["value"], d["ms_per_step"], k)
PY
done
timeout -k 10 900 $PT -x tests/test_dist_gpu.py tests/test_dist_hosted_gpu.py > $O/pytest_dist.log 2>&1 || { tail -30 $O/pytest_dist.log; exit 1; }
tail -2 $O/pytest_dist.log
grep "carry merges" $O/pytest_dist.log
cd /tmp && timeout -k 10 400 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d $O/prof_hc -o hc -- python3 $R/bench.py --cpu-budget 0 --profile-region hc --steps 20 --warmup 2 --no-1q28 --no-batch16 --no-extras > $O/bench_hc.json 2> $O/bench_hc.err || { tail -5 $O/bench_hc.err; exit 1; }
cd $R
python3 scripts/roofline_check.py hc $O/bench_hc.json $O/prof_hc/hc_kernel_trace.csv $O/check_hc.json --markers=$O/prof_hc/hc_marker_api_trace.csv | grep -E "frac|launches|avg|median"
timeout -k 10 600 $PT -x tests/test_density.py tests/test_jit.py > $O/pytest_dm.log 2>&1 || { tail -30 $O/pytest_dm.log; exit 1; }
tail -2 $O/pytest_dm.log
timeout -k 10 300 python -u bench.py --workload dm --cpu-budget 0 --steps 5 > $O/dm.json 2> $O/dm.err || { tail -5 $O/dm.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/dm.json'));print('dm', d['value'], d['ms_per_step'], d['roofline'])"
