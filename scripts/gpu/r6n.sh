set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6n; mkdir -p $O
i=0
for E in "X=1" "QSIM_TILE_HMAX=6" "QSIM_TILE_RB7=3" "QSIM_DM_RELABEL_CANDIDATES=16" "QSIM_STAGE_BEAM=16 QSIM_DM_RELABEL_TRIES=1024 QSIM_DM_RELABEL_CANDIDATES=16"; do
  i=$((i+1))
  env $E timeout -k 10 300 python -u bench.py --workload dm --steps 5 --warmup 1 > $O/d$i.json 2> $O/d$i.err || { tail -5 $O/d$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/d$i.json')); print('$E', d['value'], d['ms_per_step'], d['passes'], d['roofline']['frac'])"
done
