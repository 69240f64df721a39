#!/bin/bash
# GPU validation + measurement pass (run on the MI355X box via gpurun from the repo root).
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
TAG=${TAG:-run}
step() { echo "== $*"; }

step pytest
timeout -k 10 900 python -m pytest tests -m gpu -q -x > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc

for n in ${QUBITS:-20 28 30}; do
  step bench $n
  timeout -k 10 400 python bench.py --qubits $n --steps ${STEPS:-5} --warmup 2 --cpu-budget ${CPU_BUDGET:-10} \
      > $OUT/bench${n}_$TAG.json 2> $OUT/bench${n}_$TAG.err || { cat $OUT/bench${n}_$TAG.err | tail; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench${n}_$TAG.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['achieved'],d['roofline']['frac'])"
done

if [ -n "$ONEQ" ]; then
  step bench 1q 28
  timeout -k 10 300 python bench.py --qubits 28 --workload 1q --steps 2 --warmup 1 --cpu-budget 0 \
      > $OUT/bench28_1q_$TAG.json 2> $OUT/bench28_1q_$TAG.err || exit 1
  python -c "import json;d=json.load(open('$OUT/bench28_1q_$TAG.json'));print(d['value'],d['roofline'])"
fi

if [ -n "$PROF" ]; then
  step rocprof
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv \
      -- python3 $R/bench.py --qubits ${PROF_QUBITS:-30} --steps 3 --warmup 1 --cpu-budget 0 \
      > $OUT/prof_$TAG.log 2>&1 || { tail -20 $OUT/prof_$TAG.log; exit 1; }
  find $OUT/prof_$TAG -name "*stats*" | head
fi
echo done
