#!/bin/bash
# Mixed tile heights (13-qubit plans whose passes that fit 12 qubits run as 12-qubit tiles):
# parity at h = 7, benches 26-30q at h = 7 with and without mixing.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/mix
mkdir -p $O
cd $R
QSIM_TILE_HMAX=7 timeout -k 10 400 python -u -m pytest tests/test_tile13_gpu.py tests/test_bench_path_gpu.py tests/test_relabel_gpu.py \
  -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for M in 1 0; do
  for Q in 30 29 28 27 26; do
    QSIM_TILE_HMAX=7 QSIM_TILE_MIX=$M timeout -k 10 300 python bench.py --qubits $Q --cpu-budget 0 > $O/b${Q}_m$M.json 2> $O/b${Q}_m$M.err || exit 1
    python -c "import json; d=json.load(open('$O/b${Q}_m$M.json')); r=d['roofline']; print('$Q mix=$M', d['value'], d['ms_per_step'], r['launches'], r['avg_launch_ms'], round(r['frac'],4))"
  done
done
