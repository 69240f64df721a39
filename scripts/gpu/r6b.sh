# round 6: register-stage search A/B (DM 14q, W-HC 30q) + the parity suites it touches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_density.py tests/test_bench_path_gpu.py tests/test_relayout_gpu.py tests/test_tile13_gpu.py tests/test_headline_gpu.py tests/test_parity_gpu.py tests/test_dist_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in 1 0; do
  QSIM_STAGE_SEARCH=$v timeout -k 10 300 python -u bench.py --workload dm --steps 5 --warmup 1 > $O/dm_s$v.json 2> $O/dm_s$v.err || { tail -5 $O/dm_s$v.err; exit 1; }
  QSIM_STAGE_SEARCH=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-1q28 --no-batch16 --no-extras --cpu-budget 0 > $O/hc_s$v.json 2> $O/hc_s$v.err || { tail -5 $O/hc_s$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/dm_s$v.json')); h=json.load(open('$O/hc_s$v.json'))
print('search $v dm', d['value'], d['ms_per_step'], d['passes'], d['roofline']['frac'], '| hc', h['value'], h['ms_per_step'], h['config']['passes'], h['roofline']['frac'])"
done
