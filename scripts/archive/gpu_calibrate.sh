#!/bin/bash
# Layout calibration with the real kernels (first run, QSIM_JIT=2): W-HC 30q / 28q on vs off.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/calib2; mkdir -p $O
for n in 30 28; do for c in 1 0; do
  QSIM_RELABEL_DEBUG=1 QSIM_RELABEL_CALIBRATE=$c timeout -k 10 200 python bench.py --qubits $n --steps 5 --warmup 2 --cpu-budget 0 --no-1q28 > $O/n${n}_c$c.json 2> $O/n${n}_c$c.err || { tail $O/n${n}_c$c.err; exit 1; }
  grep calibrate $O/n${n}_c$c.err || true
  python3 -c "import json;d=json.load(open('$O/n${n}_c$c.json'));print('n', $n, 'calib', $c, d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done; done
timeout -k 10 300 python -u -m pytest tests/test_relabel_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/relabel_tests.log 2>&1 || { tail -20 $O/relabel_tests.log; exit 1; }
tail -1 $O/relabel_tests.log
