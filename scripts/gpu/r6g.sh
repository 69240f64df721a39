set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6g; mkdir -p $O
for cfg in "1 0" "1 1" "1 2" "0 0" "0 1" "0 2"; do set -- $cfg
  QSIM_NOISE_SPARSE=$1 QSIM_MAP_SKIP=$2 QSIM_NOISE_MAP_OVERLAP=0 timeout -k 10 300 python -u bench.py --workload noisy --steps 3 --warmup 1 > $O/noisy_$1_$2.json 2> $O/noisy_$1_$2.err || { tail -5 $O/noisy_$1_$2.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/noisy_$1_$2.json'))
print('sparse $1 skip $2:', d['value'], [ (k['name'], round(k['ms']/max(1,k['launches']),4)) for k in d['kernels']])"
done
QSIM_NOISE_SPARSE=1 timeout -k 10 300 python -u bench.py --workload noisy --steps 5 --warmup 1 > $O/noisy_def.json 2> $O/noisy_def.err || exit 1
python3 -c "
import json; d=json.load(open('$O/noisy_def.json')); print('default', d['value'], [ (k['name'], round(k['ms']/max(1,k['launches']),4)) for k in d['kernels']])"
