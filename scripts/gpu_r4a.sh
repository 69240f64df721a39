#!/bin/bash
# Round 4: new parity tests (headline pinning, relayout fallback, pulled noise), then the default
# bench line with its new objects.  Usage: gpu_r4a.sh <outdir-name>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/${1:-r4a}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_batched_refnoise_gpu.py tests/test_noisy_gpu.py tests/test_headline_gpu.py tests/test_relayout_gpu.py \
  > $O/pytest.log 2>&1
rc=$?
grep -E "passed|failed" $O/pytest.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAILED|^E " $O/pytest.log | head -30; exit $rc; }
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("bench", d["value"], d["ms_per_step"], d["first_run_ms"], d["config"]["passes"], d["roofline"]["frac"])
for k in ("seeds", "default_mode", "w_ref", "gate_table_20q", "dm_14q", "noisy_26q", "roofline_batch16"):
    v = d.get(k)
    print(k, json.dumps(v)[:600])
PY
