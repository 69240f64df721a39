set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6i; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_noisy_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in "4 1" "2 1" "8 1" "4 0" "2 0"; do set -- $cfg
  QSIM_PULL_U=$1 QSIM_PULL_NT=$2 timeout -k 10 300 python -u bench.py --workload noisy --steps 5 --warmup 1 > $O/noisy_$1_$2.json 2> $O/noisy_$1_$2.err || { tail -5 $O/noisy_$1_$2.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/noisy_$1_$2.json'))
print('U $1 NT $2:', d['value'], [ (k['name'], round(k['ms']/max(1,k['launches']),4)) for k in d['kernels']])"
done
