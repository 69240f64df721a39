set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6an; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_density.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
i=0
for E in "X=1" "X=2" "QSIM_CALIBRATE_HEIGHTS=0"; do
  i=$((i+1))
  env $E timeout -k 10 400 python -u bench.py --workload dm --steps 5 --warmup 1 > $O/dm$i.json 2> $O/dm$i.err || { tail -5 $O/dm$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/dm$i.json')); print('$E dm', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('passes'), d.get('first_run_ms'), [(k['name'], k['launches'], round(k['ms']/max(1,k['launches']),4)) for k in d.get('kernels',[])][:3])"
done
