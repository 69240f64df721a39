#!/bin/bash
# Round 5: where the in-tile noise kernel's time goes (QSIM_NOISE_TILE_SKIP knobs, lists on/off).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5h}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu -x tests/test_batched_refnoise_gpu.py > $O/pytest_batch.log 2>&1 || { tail -30 $O/pytest_batch.log; exit 1; }
tail -1 $O/pytest_batch.log
for v in "1 0" "1 1" "1 2" "1 3" "0 0" "0 3"; do
  set -- $v
  QSIM_NOISE_TILE_LISTS=$1 QSIM_NOISE_TILE_SKIP=$2 timeout -k 10 300 python -u bench.py --workload batch --cpu-budget 0 --steps 3 --warmup 1 > $O/b_$1_$2.json 2> $O/b_$1_$2.err || { tail -5 $O/b_$1_$2.err; exit 1; }
  python3 - $O/b_$1_$2.json "lists=$1 skip=$2" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = {x["name"]: (round(x["ms"] / max(1, x["launches"]), 4), x["launches"]) for x in d["kernels"]}
print(sys.argv[2], d["value"], d["ms_per_step"], k)
PY
done
for h in 6 7; do
  QSIM_TILE_HMAX=$h timeout -k 10 300 python -u bench.py --workload dm --cpu-budget 0 --steps 5 > $O/dm_h$h.json 2> $O/dm_h$h.err || { tail -5 $O/dm_h$h.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/dm_h$h.json'));print('dm h=$h', d['value'], d['ms_per_step'], d['passes'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
done
