#!/bin/bash
# 20q W-HC: kernel durations and the gaps between consecutive passes (launch overhead)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/gaps20; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 $R/bench.py --qubits 20 --steps 200 --warmup 5 --cpu-budget 0 --no-1q28 > $O/log.txt 2>&1 || { tail $O/log.txt; exit 1; }
python3 - <<PY
import csv, glob
f = glob.glob('$O/tr/**/*kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
qk = [r for r in rows if r['Kernel_Name'].startswith('qk')]
d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in qk]
g = [(int(qk[i]['Start_Timestamp']) - int(qk[i-1]['End_Timestamp'])) / 1e3 for i in range(1, len(qk))]
import statistics as st
print('passes', len(qk), 'median dur us', st.median(d), 'median gap us', st.median(g), 'p90 gap', sorted(g)[int(len(g)*.9)])
# per step: 4 passes; gap after every 4th
gi = [g[i] for i in range(len(g)) if (i+1) % 4 == 0]
print('inter-run gap median', st.median(gi))
PY
