#!/bin/bash
# Round 3: 13-qubit passes with chunked LDS transitions (QSIM_JIT_CHUNK7=1: 64 KiB LDS, two
# workgroups per CU) — parity at h = 7, then forced-h7 and default (calibrated) benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r3r
mkdir -p $O
QSIM_JIT_CHUNK7=1 timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_tile13_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for a in "28 42 0" "28 42 1" "30 42 0" "30 42 1" "30 3 1" "30 1 1"; do
  set -- $a
  QSIM_JIT_CHUNK7=$3 QSIM_TILE_HMAX=7 QSIM_RELABEL_CALIBRATE=0 timeout -k 10 300 python bench.py --cpu-budget 0 --no-1q28 --no-batch16 --qubits $1 --seed $2 \
      > $O/h7_q$1_s$2_c$3.json 2> $O/h7_q$1_s$2_c$3.err || { tail -5 $O/h7_q$1_s$2_c$3.err; exit 1; }
  python -c "import json; d=json.load(open('$O/h7_q$1_s$2_c$3.json')); r=d['roofline']; c=d['config']; print('h7 q$1 s$2 c$3', d['value'], d['ms_per_step'], r['launches'], r['avg_launch_ms'], round(r['frac'],4), c['tile_qubits'], [(k['name'], round(k['ms']/k['launches'],3)) for k in d['kernels']][:8])"
done
for a in "30 42" "30 1" "30 3" "28 42"; do
  set -- $a
  QSIM_JIT_CHUNK7=1 QSIM_RELABEL_DEBUG=1 timeout -k 10 300 python bench.py --cpu-budget 0 --no-1q28 --no-batch16 --qubits $1 --seed $2 \
      > $O/def_q$1_s$2.json 2> $O/def_q$1_s$2.err || { tail -5 $O/def_q$1_s$2.err; exit 1; }
  python -c "import json; d=json.load(open('$O/def_q$1_s$2.json')); r=d['roofline']; c=d['config']; print('def q$1 s$2', d['value'], d['ms_per_step'], r['launches'], round(r['frac'],4), c['tile_qubits'], c['calibrated'])"
  grep calibrate $O/def_q$1_s$2.err
done
