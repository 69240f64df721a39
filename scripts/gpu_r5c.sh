#!/bin/bash
# Round 5: packed-word in-tile noise (prefix 0 / 4 / 12 vs push) and the roctx timed-region
# profile modes (--selected-regions vs --marker-trace) on a short 24q headline run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/${1:-r5c}
mkdir -p $O
for v in "1 99" "1 0" "1 4" "0 99"; do
  set -- $v
  QSIM_NOISE_TILE=$1 QSIM_NOISE_TILE_PREFIX=$2 timeout -k 10 300 python -u bench.py --workload batch --cpu-budget 0 --steps 5 --warmup 1 > $O/batch_$1_$2.json 2> $O/batch_$1_$2.err || { tail -5 $O/batch_$1_$2.err; exit 1; }
  python3 - $O/batch_$1_$2.json "tile=$1 prefix=$2" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = {x["name"]: (round(x["ms"] / max(1, x["launches"]), 4), x["launches"]) for x in d["kernels"]}
print(sys.argv[2], d["value"], d["ms_per_step"], k)
PY
done
B="python3 $R/bench.py --cpu-budget 0 --profile-region hc --qubits 24 --steps 10 --warmup 2 --no-1q28 --no-batch16 --no-extras"
cd /tmp && timeout -k 10 200 rocprofv3 --selected-regions --kernel-trace --stats --output-format csv -d $O/sel -o sel -- $B > $O/sel.json 2> $O/sel.err; echo "selected-regions rc $?"
cd /tmp && timeout -k 10 200 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d $O/mk -o mk -- $B > $O/mk.json 2> $O/mk.err; echo "marker rc $?"
cd $R; find $O/sel $O/mk -type f | head -20
M=$(find $O/mk -name "*marker_api_trace.csv" | head -1); K=$(find $O/mk -name "*kernel_trace.csv" | head -1)
head -3 $M
python3 scripts/roofline_check.py hc $O/mk.json $K $O/check_mk.json --markers=$M | grep -E "frac|launches|selection"
S=$(find $O/sel -name "*kernel_trace.csv" | head -1)
[ -n "$S" ] && python3 scripts/roofline_check.py hc $O/sel.json $S $O/check_sel.json | grep -E "frac|launches|selection"
exit 0
