#!/bin/bash
# Round 3: rocprofv3 kernel stats of the headline region alone (W-HC 30q, no 1q28 / batch16 objects,
# so the qk<pass> names are the 30q passes only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/final
mkdir -p $O
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_hc -o hc30 -- python3 $R/bench.py --cpu-budget 0 --no-1q28 --no-batch16 > $O/prof_hc.json 2> $O/prof_hc.err || { tail -5 $O/prof_hc.err; exit 1; }
head -8 $O/prof_hc/hc30_kernel_stats.csv
python3 -c "import json;d=json.load(open('$O/prof_hc.json'));print(d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
