#!/bin/bash
# Round 5: W-BATCH (split 2 default) with smaller suffix units; full batched test files.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5q}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu -x tests/test_batched_refnoise_gpu.py tests/test_batched_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in "16" "15" "17"; do
  QSIM_NOISE_UNIT_LOG=$v timeout -k 10 300 python -u bench.py --workload batch --cpu-budget 0 --steps 5 --warmup 1 > $O/b$v.json 2> $O/b$v.err || { tail -5 $O/b$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b$v.json'));print('unit_log=$v', d['value'], d['ms_per_step'])"
done
