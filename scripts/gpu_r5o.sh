#!/bin/bash
# Round 5: trajectory-split in-tile runs (QSIM_NOISE_SPLIT) — test, then W-BATCH k = 1 / 2 / 4; DM box check.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5o}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu -x tests/test_batched_refnoise_gpu.py -k "split or lists" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for k in 1 2 4; do
  QSIM_NOISE_SPLIT=$k timeout -k 10 300 python -u bench.py --workload batch --cpu-budget 0 --steps 3 --warmup 1 > $O/b$k.json 2> $O/b$k.err || { tail -5 $O/b$k.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b$k.json'));print('split=$k', d['value'], d['ms_per_step'], [(k['name'], round(k['ms']/max(1,k['launches']),4), k['launches']) for k in d['kernels']])"
done
timeout -k 10 300 python -u bench.py --workload dm --cpu-budget 0 --steps 5 > $O/dm.json 2> $O/dm.err || { tail -5 $O/dm.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/dm.json'));print('dm', d['value'], d['ms_per_step'], d['passes'], d['roofline']['frac'])"
