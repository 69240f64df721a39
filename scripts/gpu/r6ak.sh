set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6ak; mkdir -p $O
QSIM_MAP_BMAP=1 QSIM_PULL_BMAP=2 timeout -k 10 600 python -u -m pytest tests/test_noisy_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
i=0
for E in "X=1" "QSIM_MAP_BMAP=1" "QSIM_PULL_BMAP=2" "QSIM_MAP_BMAP=1 QSIM_PULL_BMAP=2" "X=2" "QSIM_MAP_BMAP=1 X=2"; do
  i=$((i+1))
  env $E timeout -k 10 300 python -u bench.py --workload noisy --steps 5 --warmup 1 > $O/n$i.json 2> $O/n$i.err || { tail -5 $O/n$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/n$i.json')); print('$E noisy', d['value'], [ (k['name'], round(k['ms']/max(1,k['launches']),4)) for k in d['kernels']])"
done
