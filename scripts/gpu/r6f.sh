set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_noisy_gpu.py tests/test_batched_refnoise_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 1 0 1; do
  QSIM_NOISE_SPARSE=$v timeout -k 10 300 python -u bench.py --workload noisy --steps 5 --warmup 1 > $O/noisy_s$v.json 2> $O/noisy_s$v.err || { tail -5 $O/noisy_s$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/noisy_s$v.json')); r=d['noise_roofline']
print('sparse $v noisy', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac'], [ (k['name'], round(k['ms']/max(1,k['launches']),4)) for k in d['kernels']])"
done
