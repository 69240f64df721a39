#!/bin/bash
# Round 5: per-(tile, channel) list builder restored — W-BATCH check, then the noisy26 / dm14
# timed-region profiles.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5l}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu -x tests/test_batched_refnoise_gpu.py > $O/pytest_batch.log 2>&1 || { tail -30 $O/pytest_batch.log; exit 1; }
tail -1 $O/pytest_batch.log
for st in 3 5; do
  timeout -k 10 300 python -u bench.py --workload batch --cpu-budget 0 --steps $st --warmup 1 > $O/b$st.json 2> $O/b$st.err || { tail -5 $O/b$st.err; exit 1; }
  python3 - $O/b$st.json "steps=$st" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = {x["name"]: (round(x["ms"] / max(1, x["launches"]), 4), x["launches"]) for x in d["kernels"]}
print(sys.argv[2], d["value"], d["ms_per_step"], k)
PY
done
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-extras --no-1q28 --cpu-budget 0 > $O/line.json 2> $O/line.err || { tail -5 $O/line.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/line.json'));r=d['roofline_batch16'];print('line batch ref', r['reference']['value'], r['reference']['ms_per_step'], 'phys', r['physical']['value'])"
bash scripts/gpu_r5_prof.sh ${1:-r5l}
