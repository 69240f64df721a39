#!/bin/bash
# Round 5: tile kernel fast path (isolated flips pushed, compacted pulls) — tests, W-BATCH, SQ counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/${1:-r5s}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu -x tests/test_batched_refnoise_gpu.py tests/test_batched_gpu.py tests/test_noisy_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for sk in 0 2; do
  QSIM_NOISE_TILE_SKIP=$sk timeout -k 10 300 python -u bench.py --workload batch --cpu-budget 0 --steps 5 --warmup 1 > $O/b$sk.json 2> $O/b$sk.err || { tail -5 $O/b$sk.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b$sk.json'));print('skip=$sk', d['value'], d['ms_per_step'])"
done
QSIM_NOISE_SPLIT=1 timeout -k 10 300 python -u bench.py --workload batch --cpu-budget 0 --steps 5 --warmup 1 > $O/b1part.json 2> $O/b1part.err || { tail -5 $O/b1part.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b1part.json'));print('split=1', d['value'], d['ms_per_step'], [(k['name'], round(k['ms']/max(1,k['launches']),4)) for k in d['kernels']])"
