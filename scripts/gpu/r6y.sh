set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6y; mkdir -p $O
i=0
for E in "QSIM_TILE_HMAX=6 QSIM_DM_RELABEL_TRIES=1024" "QSIM_TILE_HMAX=6 QSIM_DM_RELABEL_TRIES=4096" "QSIM_TILE_HMAX=6 QSIM_DM_RELABEL_TRIES=1024 QSIM_DM_RELABEL_CANDIDATES=16" "QSIM_TILE_HMAX=6 QSIM_DM_STAGE_US=0"; do
  i=$((i+1))
  env $E timeout -k 10 400 python -u bench.py --workload dm --steps 5 --warmup 1 > $O/dm$i.json 2> $O/dm$i.err || { tail -5 $O/dm$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/dm$i.json')); r=d.get('roofline',{}); print('$E dm', d['value'], d['ms_per_step'], r.get('frac'), d.get('first_run_ms'), [(k['name'], k['launches'], round(k['ms']/max(1,k['launches']),4)) for k in d.get('kernels',[])][:8])"
done
