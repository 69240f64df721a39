set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6af; mkdir -p $O
: > $O/sweep.jsonl
for E in "QSIM_SLICE_FAR_BMAP=0" "QSIM_SLICE_FAR_BMAP=1" "QSIM_SLICE_FAR_BMAP=2" "QSIM_SLICE_FAR_BMAP=1 QSIM_SLICE_BMAP=1" "QSIM_SLICE_FAR_BMAP=2 QSIM_SLICE_BMAP=2" "QSIM_SLICE_FAR_BMAP=1 QSIM_SLICE_U_FAR=1" "QSIM_SLICE_FAR_BMAP=1 QSIM_SLICE_FAR_MODE=0" "QSIM_SLICE_FAR_BMAP=1 QSIM_SLICE_FAR_LO=14 QSIM_SLICE_FAR_HI=27"; do
  env $E TARGETS=6,8,10,12,14,16,17,18,19,20,21,22,23,24,25,26,27 timeout -k 10 120 python -u scripts/w1q_far_sweep.py >> $O/sweep.jsonl 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
done
python3 - <<'PY'
import json
rows=[json.loads(l) for l in open('gpurun_out/r6af/sweep.jsonl')]
for r in rows:
    f=r['frac']; far=[f[str(t)] for t in range(20,26)]; allv=list(f.values())
    print(r['knobs'], 'min20-25', min(far), 'mean20-25', round(sum(far)/6,4), 'min all', min(allv), 'mean all', round(sum(allv)/len(allv),4), [f[k] for k in ('6','8','12','16','18','26','27')])
PY
