#!/bin/bash
# Round 3: two-phase k_noise_units (walk -> LDS list -> whole-work-group apply): parity + W-BATCH ref.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r3n
mkdir -p $out
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_batched_refnoise_gpu.py tests/test_noisy_gpu.py tests/test_batched_gpu.py > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
grep -E "passed|failed" $out/pytest.log | tail -2
for B in 1024; do
  timeout -k 10 300 python -u bench.py --workload batch --batch-noise reference --trajectories $B \
      --steps 10 --warmup 2 > $out/b$B.json 2> $out/b$B.err || { tail -5 $out/b$B.err; exit 1; }
  python -c "import json;d=json.load(open('$out/b$B.json'));print($B, d['value'], d['ms_per_step'], [(k['name'],round(k['ms']/max(1,k['launches']),4),k['launches']) for k in d['kernels']])"
done
