#!/bin/bash
# Round 3 evidence with relayout plans: GPU suite in one process, smoke, default bench line,
# rocprofv3 kernel stats of the headline region, PMC traffic (FETCH_SIZE / WRITE_SIZE passes) of
# the W-HC 30q relayout passes.  Usage: gpu_r3u.sh <outdir-name>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/${1:-r3u}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "passed|failed" $O/pytest.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAILED|^E " $O/pytest.log | head -30; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench30.json 2> $O/bench30.err || { tail -5 $O/bench30.err; exit 1; }
python - "$O/bench30.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d["roofline"]; c = d["config"]
print("bench", d["value"], d["value_mean"], d["ms_per_step"], c["passes"], c["relayout"], c["tile_qubits"], c["calibrated"], d["restore_ms"],
      r["launches"], r["avg_launch_ms"], r["frac"], d["roofline_1q28"]["frac"], d["cpu_baseline"]["value"],
      (d["cpu_baseline"].get("w_hc_20q") or {}).get("value"))
PY
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o hc30 -- python3 $R/bench.py --cpu-budget 0 --no-1q28 --no-batch16 > $O/prof_hc.json 2> $O/prof_hc.err || { tail -5 $O/prof_hc.err; exit 1; }
head -8 $O/prof/hc30_kernel_stats.csv
for i in 1 2; do
  C=FETCH_SIZE; [ $i = 2 ] && C=WRITE_SIZE
  QSIM_RELABEL_CALIBRATE=0 timeout -s KILL 180 rocprofv3 --pmc $C -d $O/pmc/p$i -o run --output-format csv -- python3 $R/bench.py --cpu-budget 0 --no-1q28 --no-batch16 --steps 2 --warmup 1 > $O/pmc_p$i.log 2>&1 || { tail -5 $O/pmc_p$i.log; exit 1; }
done
python3 $R/scripts/pmc_summary.py $O/pmc $O/pmc_hc_30q.json
