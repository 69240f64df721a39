#!/bin/bash
# Round 5: threshold-table flip sampler — every noise parity suite, then W-BATCH / noisy / DM.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5j}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu -x tests/test_batched_refnoise_gpu.py tests/test_noisy_gpu.py tests/test_batched_gpu.py tests/test_density.py > $O/pytest_noise.log 2>&1 || { tail -30 $O/pytest_noise.log; exit 1; }
tail -1 $O/pytest_noise.log
for v in "1 0" "0 0" "1 3"; do
  set -- $v
  QSIM_NOISE_TILE_LISTS=$1 QSIM_NOISE_TILE_SKIP=$2 timeout -k 10 300 python -u bench.py --workload batch --cpu-budget 0 --steps 3 --warmup 1 > $O/b_$1_$2.json 2> $O/b_$1_$2.err || { tail -5 $O/b_$1_$2.err; exit 1; }
  python3 - $O/b_$1_$2.json "lists=$1 skip=$2" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = {x["name"]: (round(x["ms"] / max(1, x["launches"]), 4), x["launches"]) for x in d["kernels"]}
print(sys.argv[2], d["value"], d["ms_per_step"], k)
PY
done
QSIM_NOISE_TILE=0 timeout -k 10 300 python -u bench.py --workload batch --cpu-budget 0 --steps 3 --warmup 1 > $O/b_push.json 2> $O/b_push.err || { tail -5 $O/b_push.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b_push.json'));print('push', d['value'], d['ms_per_step'], [(k['name'], round(k['ms']/max(1,k['launches']),4)) for k in d['kernels']])"
timeout -k 10 300 python -u bench.py --workload noisy --cpu-budget 0 --steps 3 > $O/noisy.json 2> $O/noisy.err || { tail -5 $O/noisy.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/noisy.json'));print('noisy', d['value'], d['ms_per_step'], [(k['name'], round(k['ms']/max(1,k['launches']),4)) for k in d['kernels']])"
timeout -k 10 300 python -u bench.py --workload dm --cpu-budget 0 --steps 5 > $O/dm.json 2> $O/dm.err || { tail -5 $O/dm.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/dm.json'));print('dm', d['value'], d['ms_per_step'], d['passes'], d['roofline']['frac'])"
