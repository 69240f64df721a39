#!/bin/bash
# Round 3: fused gate+noise (reference batched noise process) — tests + bench per mode.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r3b
mkdir -p $out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_batched_refnoise_gpu.py > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
grep -E "passed|failed" $out/pytest.log | tail -2
for m in 512 1024 256 0; do
  QSIM_BATCH_GATE_NOISE=$m timeout -k 10 300 python -u bench.py --workload batch --batch-noise reference \
      --steps 10 --warmup 2 > $out/bench_$m.json 2> $out/bench_$m.err || { tail -5 $out/bench_$m.err; exit 1; }
  python -c "import json;d=json.load(open('$out/bench_$m.json'));print('$m', d['value'], d['ms_per_step'], [(k['name'],round(k['ms']/max(1,k['launches']),4),k['launches']) for k in d['kernels']])"
done
