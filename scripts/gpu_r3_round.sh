#!/bin/bash
# Round 3 evidence: GPU suite in one process, smoke, default bench line, rocprofv3 kernel stats of
# the bench command.  Usage: gpu_r3_round.sh <outdir-name>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/${1:-round}
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "passed|failed" $O/pytest.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAILED|^E " $O/pytest.log | head -30; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench30.json 2> $O/bench30.err || { tail -5 $O/bench30.err; exit 1; }
python - "$O/bench30.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d["roofline"]; c = d["config"]
print("bench", d["value"], d["value_mean"], d["ms_per_step"], c["tile_qubits"], c["calibrated"], d["restore_ms"],
      r["launches"], r["avg_launch_ms"], r["frac"], d["roofline_1q28"]["frac"], d["cpu_baseline"]["value"],
      (d["cpu_baseline"].get("w_hc_20q") or {}).get("value"))
PY
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench30 -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-budget 0 > $O/prof_bench.json 2> $O/prof_bench.err || { tail -5 $O/prof_bench.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
