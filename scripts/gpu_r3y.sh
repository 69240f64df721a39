#!/bin/bash
# Round 3: relayout variants timed at the first run — GPU tests + W-HC 30q seeds 42 / 4 / 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/variants2; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_relayout_gpu.py tests/test_headline_gpu.py tests/test_bench_path_gpu.py > $O/pytest.log 2>&1 || { grep -E "FAILED|^E " $O/pytest.log | head -30; tail -3 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for sd in 42 4 2 1; do
  QSIM_RELABEL_DEBUG=1 timeout -k 10 300 python3 bench.py --qubits 30 --seed $sd --cpu-budget 0 --no-1q28 --no-batch16 --steps 10 > $O/b30_s$sd.json 2> $O/b30_s$sd.err || { tail -5 $O/b30_s$sd.err; exit 1; }
  grep calibrate $O/b30_s$sd.err | tail -12
  python3 -c "import json;d=json.load(open('$O/b30_s$sd.json'));c=d['config'];print(30, $sd, d['value'], c['passes'], c['relayout'], c['tile_qubits'], d['roofline']['frac'])"
done
