set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6ao; mkdir -p $O
i=0
for E in "X=1" "QSIM_NOISE_SPLIT=1" "QSIM_NOISE_SPLIT=3" "QSIM_NOISE_UNIT_LOG=15" "QSIM_NOISE_UNIT_LOG=17" "QSIM_NOISE_LISTS8=0" "X=2"; do
  i=$((i+1))
  env $E timeout -k 10 300 python -u bench.py --workload batch --steps 8 --warmup 1 --cpu-budget 0 > $O/b$i.json 2> $O/b$i.err || { tail -5 $O/b$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/b$i.json')); print('$E batch', d['value'], d['ms_per_step'])"
done
