#!/bin/bash
# Pipelined 13-qubit pass kernels: prefetch before (EARLY=1) or after (0) the first barrier.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/h7e
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_tile13_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for E in 1 0; do
  for Q in 26 28 30; do
    QSIM_TILE_HMAX=7 QSIM_JIT_PIPE_EARLY=$E timeout -k 10 300 python bench.py --qubits $Q --cpu-budget 0 > $O/b${Q}_e$E.json 2> $O/b${Q}_e$E.err || exit 1
  done
done
python - <<PY
import json, glob
for f in sorted(glob.glob('$O/b*.json')):
    d = json.load(open(f)); r = d['roofline']
    print(f.split('/')[-1], d['value'], d['ms_per_step'], r and round(r['frac'], 4), r and r.get('launches'), r and r.get('avg_launch_ms'))
PY
