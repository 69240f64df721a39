set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_noisy_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 12 11 10; do
  QSIM_NOISE_REGION_LOG=$r timeout -k 10 300 python -u bench.py --workload noisy --steps 5 --warmup 1 > $O/noisy_$r.json 2> $O/noisy_$r.err || { tail -5 $O/noisy_$r.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/noisy_$r.json'))
print('region log $r:', d['value'], [ (k['name'], round(k['ms']/max(1,k['launches']),4)) for k in d['kernels']])"
done
