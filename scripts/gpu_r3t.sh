#!/bin/bash
# Round 3: relayout plans — GPU parity (interpreter + JIT, calibration) and the W-HC benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/relayout; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_relayout_gpu.py tests/test_relabel_gpu.py tests/test_headline_gpu.py > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for q in 30 28; do
  timeout -k 10 300 python3 bench.py --qubits $q --cpu-budget 0 --no-1q28 --no-batch16 --steps 20 > $O/b${q}.json 2> $O/b${q}.err || { tail -5 $O/b${q}.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b${q}.json'));print($q, d['value'], d['config']['passes'], d['config']['relayout'], d['config']['tile_qubits'], d['roofline']['frac'], d['restore_ms'])"
done
QSIM_RELAYOUT=0 timeout -k 10 300 python3 bench.py --qubits 30 --cpu-budget 0 --no-1q28 --no-batch16 --steps 20 > $O/b30_off.json 2> $O/b30_off.err || { tail -5 $O/b30_off.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b30_off.json'));print('off', d['value'], d['config']['passes'], d['config']['relayout'], d['roofline']['frac'])"
