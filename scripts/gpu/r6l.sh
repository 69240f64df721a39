set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_cache_gpu.py -m gpu -x -q --timeout 500 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-1q28 --no-batch16 --extras first_run_cache --cpu-budget 0 > $O/bench_frc.json 2> $O/bench_frc.err || { tail -5 $O/bench_frc.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench_frc.json')); print(d['value'], d['first_run_ms']); print(json.dumps(d['first_run_cache']))"
