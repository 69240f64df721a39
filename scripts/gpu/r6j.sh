set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6j; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_noisy_gpu.py tests/test_batched_refnoise_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for u in 1 2 def; do
  if [ $u = def ]; then E=""; else E="QSIM_PULL_U=$u"; fi
  env $E timeout -k 10 300 python -u bench.py --workload noisy --steps 5 --warmup 1 > $O/noisy_$u.json 2> $O/noisy_$u.err || { tail -5 $O/noisy_$u.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/noisy_$u.json'))
print('U $u:', d['value'], [ (k['name'], round(k['ms']/max(1,k['launches']),4)) for k in d['kernels']])"
done
