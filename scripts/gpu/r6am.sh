set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6am; mkdir -p $O
i=0
for E in "QSIM_JIT_PIPE_ORDER=1" "QSIM_JIT_PIPE_ORDER=2" "QSIM_JIT_PIPE_ORDER=1 X=2" "QSIM_JIT_PIPE_ORDER=2 X=2"; do
  i=$((i+1))
  env $E timeout -k 10 300 python -u bench.py --workload dm --steps 5 --warmup 1 > $O/dm$i.json 2> $O/dm$i.err || { tail -5 $O/dm$i.err; exit 1; }
  env $E timeout -k 10 300 python -u bench.py --qubits 28 --steps 8 --warmup 2 --no-extras --no-1q28 --no-batch16 --cpu-budget 0 > $O/hc$i.json 2> $O/hc$i.err || { tail -5 $O/hc$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/dm$i.json')); h=json.load(open('$O/hc$i.json')); print('$E dm', d['value'], d['roofline']['frac'], 'hc28', h['value'], h['roofline']['frac'], h['config'].get('passes'))"
done
