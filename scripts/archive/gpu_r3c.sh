#!/bin/bash
# Round 3: 13-qubit tiles with 8 amplitudes per thread (QSIM_TILE_RB7=3, 1024-thread workgroups)
# vs the default 16 (512 threads), mixed-height label search (QSIM_LAYOUT_T13=1.25), and 12-qubit
# tiles; W-HC 30q seeds 42/1/3 and 28q.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3c
mkdir -p $O
QSIM_TILE_RB7=3 timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_tile13_gpu.py > $O/pytest_rb3.log 2>&1 || { tail -30 $O/pytest_rb3.log; exit 1; }
tail -1 $O/pytest_rb3.log
run() {  # name "ENV=.. ENV=.." bench-args...
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python bench.py --cpu-budget 0 --no-1q28 --steps 10 "$@" > $O/$name.json 2> $O/$name.err \
    || { tail -5 $O/$name.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$name.json')); r=d['roofline']; print('$name', d['value'], d['ms_per_step'], r['launches'], r['avg_launch_ms'], round(r['frac'],4))"
}
for S in 42 1 3; do
  run q30_s${S}_h6 "QSIM_TILE_HMAX=6" --seed $S
  run q30_s${S}_h7t125_rb4 "QSIM_TILE_HMAX=7 QSIM_LAYOUT_T13=1.25 QSIM_TILE_RB7=4" --seed $S
  run q30_s${S}_h7t125_rb3 "QSIM_TILE_HMAX=7 QSIM_LAYOUT_T13=1.25 QSIM_TILE_RB7=3" --seed $S
done
run q28_s42_h7_rb4 "QSIM_TILE_RB7=4" --qubits 28
run q28_s42_h7_rb3 "QSIM_TILE_RB7=3" --qubits 28
run q28_s42_h6 "QSIM_TILE_HMAX=6" --qubits 28
