set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6ai; mkdir -p $O
i=0
for E in "QSIM_FUSED_XCD=0" "QSIM_FUSED_XCD=1" "QSIM_FUSED_XCD=0 X=2" "QSIM_FUSED_XCD=1 X=2"; do
  i=$((i+1))
  env $E timeout -k 10 300 python -u bench.py --workload batch --batch-noise physical --steps 8 --warmup 1 --cpu-budget 0 > $O/p$i.json 2> $O/p$i.err || { tail -5 $O/p$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/p$i.json')); print('$E physical', d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'))"
done
for E in "QSIM_FUSED_XCD=0 QSIM_JIT=0" "QSIM_FUSED_XCD=1 QSIM_JIT=0"; do
  i=$((i+1))
  env $E timeout -k 10 300 python -u bench.py --qubits 26 --steps 10 --warmup 2 --no-extras --no-1q28 --no-batch16 --cpu-budget 0 > $O/h$i.json 2> $O/h$i.err || { tail -5 $O/h$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/h$i.json')); print('$E hc26 interp', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
