#!/bin/bash
# Round 3: timed relayout variants for 20-27 qubit first runs (bench mode) — tests + W-HC benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/small_timed; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_bench_path_gpu.py tests/test_relayout_gpu.py tests/test_relabel_gpu.py tests/test_api_gpu.py > $O/pytest.log 2>&1 || { grep -E "FAILED|^E " $O/pytest.log | head -30; tail -3 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for q in 20 22 24 26; do
  QSIM_RELABEL_DEBUG=1 timeout -k 10 300 python3 bench.py --qubits $q --cpu-budget 0 --no-1q28 --no-batch16 --steps 50 > $O/b$q.json 2> $O/b$q.err || { tail -5 $O/b$q.err; exit 1; }
  grep -c calibrate $O/b$q.err
  python3 -c "import json;d=json.load(open('$O/b$q.json'));c=d['config'];print($q, d['value'], d['ms_per_step'], c['passes'], c['relayout'], c['calibrated'])"
done
