set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6ad; mkdir -p $O
: > $O/sweep.jsonl
for NT in 1 0; do
for M in 2 0 1; do
for U in 1 2 4 8; do
  QSIM_NT=$NT QSIM_SLICE_FAR_MODE=$M QSIM_SLICE_U_FAR=$U timeout -k 10 120 python -u scripts/w1q_far_sweep.py >> $O/sweep.jsonl 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
done; done; done
python3 - <<'PY'
import json
rows=[json.loads(l) for l in open('gpurun_out/r6ad/sweep.jsonl')]
for r in rows:
    f=r['frac']; far=[f[str(t)] for t in range(20,26)]
    print(r['knobs'].get('QSIM_NT'), r['knobs'].get('QSIM_SLICE_FAR_MODE'), r['knobs'].get('QSIM_SLICE_U_FAR'), 'min20-25', min(far), 'mean20-25', round(sum(far)/6,4), 'others', [f[k] for k in ('8','16','18','19','26','27')])
PY
