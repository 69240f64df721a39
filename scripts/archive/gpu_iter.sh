set -o pipefail
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu2.log 2>&1; rc=$?; tail -3 $O/pytest_gpu2.log; [ $rc -eq 0 ] || exit $rc
for x in 0 1; do
  QSIM_JIT_XCD=$x timeout -k 10 300 python bench.py --cpu-budget 0 > $O/bench30_xcd$x.json 2> $O/bench30_xcd$x.err || exit 1
  python -c "import json;d=json.load(open('$O/bench30_xcd$x.json'));print('xcd',$x,d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['roofline']['launches'])"
  QSIM_JIT_XCD=$x timeout -k 10 300 python bench.py --qubits 28 --cpu-budget 0 > $O/bench28_xcd$x.json 2> $O/bench28_xcd$x.err || exit 1
  python -c "import json;d=json.load(open('$O/bench28_xcd$x.json'));print('xcd28',$x,d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['roofline']['launches'])"
done
QSIM_JIT_XCD=1 timeout -k 10 300 python scripts/pass_probe.py 30 5 > $O/pass_probe30_xcd.jsonl 2>&1 || exit 1
echo done
