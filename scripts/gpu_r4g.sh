#!/bin/bash
# Round 4: GPU suite + smoke (gpu_r4b.sh), then the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${1:-r4g}
bash scripts/gpu_r4b.sh $O || exit 1
timeout -k 10 420 python -u bench.py > gpurun_out/$O/bench.json 2> gpurun_out/$O/bench.err || { tail -5 gpurun_out/$O/bench.err; exit 1; }
python3 - gpurun_out/$O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("bench", d["value"], d["ms_per_step"], d["first_run_ms"], d["config"]["passes"], d["config"]["relayout"], d["roofline"]["frac"])
for k in ("roofline_batch16", "roofline_1q28", "dm_14q", "noisy_26q"):
    v = d.get(k)
    if isinstance(v, dict):
        v = {kk: vv for kk, vv in v.items() if kk != "kernels"}
    print(k, json.dumps(v)[:500])
PY
