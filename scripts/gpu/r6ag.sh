set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6ag; mkdir -p $O
: > $O/sweep.jsonl
for E in "QSIM_SLICE_BMAP=0" "QSIM_SLICE_BMAP=1 QSIM_SLICE_FAR_BMAP=1" "QSIM_SLICE_BMAP=1 QSIM_SLICE_FAR_BMAP=2"; do
  env $E TARGETS=0,1,2,3,4,5,6,8,10,12,14,16,17,18,19,20,21,22,23,24,25,26,27 timeout -k 10 120 python -u scripts/w1q_far_sweep.py >> $O/sweep.jsonl 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  env $E timeout -k 10 200 python -u scripts/w1q28.py > $O/w1q_$(echo $E | tr ' =' '__').json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
done
python3 - <<'PY'
import json, glob
rows=[json.loads(l) for l in open('gpurun_out/r6ag/sweep.jsonl')]
for r in rows:
    f=r['frac']; allv=list(f.values())
    print(r['knobs'], 'min all', min(allv), 'mean all', round(sum(allv)/len(allv),4), 'low', [f[str(k)] for k in range(6)], 'far', [f[str(k)] for k in range(20,26)])
for p in sorted(glob.glob('gpurun_out/r6ag/w1q_*.json')):
    d=json.load(open(p)); print(p, d['frac'], d['avg_launch_ms'])
PY
