#!/bin/bash
# 13-qubit tiles (h = 7, 128 KiB LDS, 512 threads) and persistent pipelined pass kernels:
# parity subset + 30q/28q benches.  ENVS: list of "HMAX:PIPE:TRIES" configurations to bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/h7
mkdir -p $O
cd $R
if [ -z "$SKIP_TESTS" ]; then
QSIM_TILE_HMAX=7 timeout -k 10 400 python -u -m pytest tests/test_bench_path_gpu.py tests/test_jit.py tests/test_relabel_gpu.py \
  -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_h7.log 2>&1; rc=$?
tail -3 $O/pytest_h7.log; [ $rc -eq 0 ] || exit $rc
QSIM_JIT_PIPE=2 timeout -k 10 400 python -u -m pytest tests/test_bench_path_gpu.py tests/test_jit.py \
  -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_pipe6.log 2>&1; rc=$?
tail -3 $O/pytest_pipe6.log; [ $rc -eq 0 ] || exit $rc
fi
for c in ${ENVS:-6:1:7 7:1:31 6:2:7 7:0:31}; do
  IFS=: read H P T <<< "$c"
  for Q in ${QUBITS:-30 28}; do
    QSIM_TILE_HMAX=$H QSIM_JIT_PIPE=$P QSIM_RELABEL_TRIES=$T timeout -k 10 300 python bench.py --qubits $Q --cpu-budget 0 \
      > $O/b${Q}_h${H}_p${P}_t$T.json 2> $O/b${Q}_h${H}_p${P}_t$T.err || exit 1
  done
done
python - <<PY
import json, glob
for f in sorted(glob.glob('$O/b*.json')):
    d = json.load(open(f)); r = d['roofline']
    print(f.split('/')[-1], d['value'], d['ms_per_step'], r and round(r['frac'], 4), r and r.get('launches'), r and r.get('avg_launch_ms'))
PY
