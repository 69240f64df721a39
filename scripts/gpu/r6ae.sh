set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6ae; mkdir -p $O
: > $O/sweep.jsonl
for B in 0 1 2; do
for U in 2 4; do
  QSIM_SLICE_FAR_BMAP=$B QSIM_SLICE_U_FAR=$U timeout -k 10 120 python -u scripts/w1q_far_sweep.py >> $O/sweep.jsonl 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
done; done
python3 - <<'PY'
import json
rows=[json.loads(l) for l in open('gpurun_out/r6ae/sweep.jsonl')]
for r in rows:
    f=r['frac']; far=[f[str(t)] for t in range(20,26)]
    print(r['knobs'], 'min20-25', min(far), 'mean20-25', round(sum(far)/6,4), 'far', far)
PY
