set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6x; mkdir -p $O
i=0
for E in "X=1" "QSIM_TILE_HMAX=6" "QSIM_JIT_PIPE=0" "X=2" "QSIM_TILE_HMAX=6 X=2"; do
  i=$((i+1))
  env $E timeout -k 10 300 python -u bench.py --workload dm --steps 5 --warmup 1 > $O/dm$i.json 2> $O/dm$i.err || { tail -5 $O/dm$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/dm$i.json')); r=d.get('roofline',{}); print('$E dm', d['value'], d['ms_per_step'], r.get('frac'), [(k['name'], k['launches'], round(k['ms']/max(1,k['launches']),4)) for k in d.get('kernels',[])][:8])"
done
