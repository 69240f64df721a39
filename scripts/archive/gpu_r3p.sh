#!/bin/bash
# Round 3: W-BATCH reference noise process with the ensemble split over two streams.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r3p
mkdir -p $out
QSIM_BATCH_REF_STREAMS=2 timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_batched_refnoise_gpu.py > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
grep -E "passed|failed" $out/pytest.log | tail -2
for S in 1 2 1 2; do
  QSIM_BATCH_REF_STREAMS=$S timeout -k 10 300 python -u bench.py --workload batch --batch-noise reference \
      --steps 10 --warmup 2 > $out/s$S.json 2> $out/s$S.err || { tail -5 $out/s$S.err; exit 1; }
  python -c "import json;d=json.load(open('$out/s$S.json'));print($S, d['value'], d['ms_per_step'])"
done
