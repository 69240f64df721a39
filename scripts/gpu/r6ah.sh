set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6ah; mkdir -p $O
QSIM_NOISE_BMAP=1 QSIM_PULL_BMAP=1 timeout -k 10 900 python -u -m pytest tests/test_batched_refnoise_gpu.py tests/test_noisy_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
i=0
for E in "QSIM_NOISE_BMAP=0" "QSIM_NOISE_BMAP=1" "QSIM_NOISE_BMAP=0 X=2" "QSIM_NOISE_BMAP=1 X=2"; do
  i=$((i+1))
  env $E timeout -k 10 300 python -u bench.py --workload batch --steps 8 --warmup 1 --cpu-budget 0 > $O/b$i.json 2> $O/b$i.err || { tail -5 $O/b$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/b$i.json')); print('$E batch', d['value'], d['ms_per_step'])"
done
for E in "QSIM_PULL_BMAP=0" "QSIM_PULL_BMAP=1"; do
  i=$((i+1))
  env $E timeout -k 10 300 python -u bench.py --workload noisy --steps 5 --warmup 1 > $O/n$i.json 2> $O/n$i.err || { tail -5 $O/n$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/n$i.json')); print('$E noisy', d['value'], [ (k['name'], round(k['ms']/max(1,k['launches']),4)) for k in d['kernels']])"
done
