set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6ap; mkdir -p $O
i=0
for E in "X=1" "QSIM_CU_MASK_MAIN=w:55555555 QSIM_CU_MASK_NOISE=w:aaaaaaaa" "QSIM_CU_MASK_MAIN=w:77777777 QSIM_CU_MASK_NOISE=w:88888888" "QSIM_CU_MASK_MAIN=w:ffffffff QSIM_CU_MASK_NOISE=w:88888888" "QSIM_CU_MASK_MAIN=r:0-127 QSIM_CU_MASK_NOISE=r:128-255" "QSIM_CU_MASK_MAIN=w:3f3f3f3f QSIM_CU_MASK_NOISE=w:c0c0c0c0"; do
  i=$((i+1))
  env $E timeout -k 10 300 python -u bench.py --workload noisy --steps 5 --warmup 1 > $O/n$i.json 2> $O/n$i.err || { tail -5 $O/n$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/n$i.json')); print('$E noisy', d['value'], [ (k['name'], round(k['ms']/max(1,k['launches']),4)) for k in d['kernels']])"
done
