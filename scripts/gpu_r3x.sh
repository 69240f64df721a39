#!/bin/bash
# Round 3: relayout below the relabeling threshold (first runs of 16-25 qubit states) — GPU tests
# that run such states by default, and W-HC A/B at 18-24 qubits (relayout from 16 vs off).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/small_rl; mkdir -p $O
QSIM_RELAYOUT_MIN_QUBITS=16 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_relayout_gpu.py tests/test_bench_path_gpu.py tests/test_relabel_gpu.py tests/test_api_gpu.py tests/test_parity_gpu.py tests/test_tile13_gpu.py tests/test_matrix_api_gpu.py > $O/pytest.log 2>&1 || { grep -E "FAILED|^E " $O/pytest.log | head -30; tail -3 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for q in 18 20 22 24; do for m in 16 0; do
  if [ $m = 0 ]; then E="QSIM_RELAYOUT=0"; else E="QSIM_RELAYOUT_MIN_QUBITS=$m"; fi
  env $E timeout -k 10 300 python3 bench.py --qubits $q --cpu-budget 0 --no-1q28 --no-batch16 --steps 50 > $O/b${q}_m$m.json 2> $O/b${q}_m$m.err || { tail -5 $O/b${q}_m$m.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b${q}_m$m.json'));c=d['config'];print($q, '$E', d['value'], d['ms_per_step'], c['passes'], c['relayout'])"
done; done
