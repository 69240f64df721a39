set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-1q28 --no-batch16 --extras w_hc_28q,h_single --cpu-budget 0 > $O/bench_extras.json 2> $O/bench_extras.err || { tail -10 $O/bench_extras.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench_extras.json'))
print('hc30', d['value'], d['roofline']['frac']); w=d['w_hc_28q']; print('hc28', w['value'], w['passes'], w['roofline']['frac'], w['first_run_ms'])
print(d['h_single_synced']['rows'])"
bash scripts/gpu/profiles.sh r6a_prof hc28 pmchc28 || exit 1
