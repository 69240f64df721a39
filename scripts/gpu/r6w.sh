set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6w; mkdir -p $O
i=0
for E in "X=1" "QSIM_STAGE_SELECT=0" "X=2" "QSIM_STAGE_SELECT=0 X=3"; do
  i=$((i+1))
  env $E timeout -k 10 300 python -u bench.py --workload dm --steps 5 --warmup 1 > $O/dm$i.json 2> $O/dm$i.err || { tail -5 $O/dm$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/dm$i.json')); r=d.get('roofline',{}); print('$E dm', d['value'], d['ms_per_step'], r.get('frac'), d.get('config',{}).get('passes'), d.get('config',{}).get('stages'))"
done
for E in "X=1" "QSIM_STAGE_SELECT=0"; do
  i=$((i+1))
  env $E timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-extras > $O/hc$i.json 2> $O/hc$i.err || { tail -5 $O/hc$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/hc$i.json')); print('$E hc', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
