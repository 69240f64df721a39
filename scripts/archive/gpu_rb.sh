#!/bin/bash
# 20q passes with 8 / 4 amplitudes per thread (QSIM_TILE_RB = 3 / 2) vs 16 (4): parity + benches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/rb
mkdir -p $O
cd $R
for RB in 3 2; do
  QSIM_TILE_RB=$RB timeout -k 10 400 python -u -m pytest tests/test_bench_path_gpu.py tests/test_jit.py tests/test_api_gpu.py \
    -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_rb$RB.log 2>&1; rc=$?
  tail -2 $O/pytest_rb$RB.log; [ $rc -eq 0 ] || exit $rc
done
for RB in 4 3 2; do
  for Q in 20 18; do
    QSIM_TILE_RB=$RB timeout -k 10 300 python bench.py --qubits $Q --cpu-budget 0 > $O/b${Q}_rb$RB.json 2> $O/b${Q}_rb$RB.err || exit 1
  done
done
for RB in 4 3; do
  QSIM_TILE_RB=$RB QSIM_JIT=0 timeout -k 10 300 python bench.py --qubits 20 --cpu-budget 0 > $O/b20_rb${RB}_interp.json 2> $O/b20_rb${RB}_interp.err || exit 1
done
python - <<PY
import json, glob
for f in sorted(glob.glob('$O/b*.json')):
    d = json.load(open(f)); r = d['roofline']
    print(f.split('/')[-1], d['value'], d['ms_per_step'], r and round(r['frac'], 4), r and r.get('launches'), r and r.get('avg_launch_ms'))
PY
