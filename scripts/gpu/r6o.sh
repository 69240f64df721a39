set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6o; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_cache_gpu.py tests/test_headline_gpu.py tests/test_relayout_gpu.py tests/test_relabel_gpu.py tests/test_bench_path_gpu.py tests/test_density.py -m gpu -x -q --timeout 500 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 1 0; do
  QSIM_JIT_PREFETCH=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-1q28 --no-batch16 --no-extras --cpu-budget 0 > $O/hc_p$v.json 2> $O/hc_p$v.err || { tail -5 $O/hc_p$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/hc_p$v.json')); print('prefetch $v', d['value'], d['first_run_ms'], d['config']['passes'])"
done
