#!/bin/bash
# Round 3: cross-height first-run calibration (12- vs 13-qubit tile candidates timed on the device).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_relabel_gpu.py tests/test_tile13_gpu.py tests/test_bench_path_gpu.py > $O/pytest.log 2>&1 \
    || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for a in "30 42" "30 1" "30 3" "28 42" "29 42"; do
  set -- $a
  QSIM_RELABEL_DEBUG=1 timeout -k 10 300 python bench.py --cpu-budget 0 --no-1q28 --qubits $1 --seed $2 \
      > $O/q$1_s$2.json 2> $O/q$1_s$2.err || { tail -5 $O/q$1_s$2.err; exit 1; }
  python -c "import json; d=json.load(open('$O/q$1_s$2.json')); r=d['roofline']; c=d['config']; print('q$1 s$2', d['value'], d['value_mean'], d['ms_per_step'], r['launches'], r['avg_launch_ms'], round(r['frac'],4), c['tile_qubits'], c['calibrated'], d['restore_ms'], d['restore_passes'])"
  grep calibrate $O/q$1_s$2.err
done
