set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6ac; mkdir -p $O
i=0
for E in "QSIM_RELAYOUT_VARIANTS=16 QSIM_RELAYOUT_LAYOUT_VARIANTS=6" "X=1" "QSIM_RELAYOUT_VARIANTS=32 QSIM_RELAYOUT_LAYOUT_VARIANTS=8" "QSIM_RELAYOUT_VARIANTS=16 QSIM_RELAYOUT_LAYOUT_VARIANTS=6 X=2"; do
  i=$((i+1))
  env $E timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 --no-extras --no-1q28 --no-batch16 --cpu-budget 0 > $O/hc$i.json 2> $O/hc$i.err || { tail -5 $O/hc$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/hc$i.json')); print('$E', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('first_run_ms'), [(k['name'], round(k['ms']/max(1,k['launches']),3)) for k in d['kernels']][:6])"
done
