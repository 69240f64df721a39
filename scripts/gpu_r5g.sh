#!/bin/bash
# Round 5: batched tile-noise tests, then W-BATCH variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5g}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu -x tests/test_batched_refnoise_gpu.py > $O/pytest_batch.log 2>&1 || { tail -30 $O/pytest_batch.log; exit 1; }
tail -1 $O/pytest_batch.log
bash scripts/gpu_r5f.sh ${1:-r5g}
for h in 6 7; do
  QSIM_TILE_HMAX=$h timeout -k 10 300 python -u bench.py --workload dm --cpu-budget 0 --steps 5 > $O/dm_h$h.json 2> $O/dm_h$h.err || { tail -5 $O/dm_h$h.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/dm_h$h.json'));print('dm h=$h', d['value'], d['ms_per_step'], d['passes'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
done
