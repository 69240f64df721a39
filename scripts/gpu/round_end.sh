#!/bin/bash
# The driver's round-end sequence on one MI355X (run through gpurun): the GPU suite in one process,
# smoke(), the default bench line; results under gpurun_out/<tag>/ (copied to profiles/rNN/).
#     gpurun --timeout 1200 -- bash scripts/gpu/round_end.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/${1:-round_end}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 2 > $O/bench.json 2> $O/bench.err || { tail -10 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("value", d["value"], "ms", d["ms_per_step"], "frac", d["roofline"]["frac"], "passes", d["config"]["passes"])
print("1q28", d["roofline_1q28"]["frac"], "batch ref", d["roofline_batch16"]["reference"]["value"], "phys", d["roofline_batch16"]["physical"]["value"])
print("dm", d["dm_14q"]["value"], "noisy", d["noisy_26q"]["value"], "cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["w_hc_28q"]["value"])
PY
