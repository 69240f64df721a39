#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/allocvar; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 $R/scripts/dbg/alloc_variance.py > $O/log.txt 2>&1 || { tail $O/log.txt; exit 1; }
cat $O/log.txt | grep ms
python3 - <<PY
import csv, glob
f = glob.glob('$O/tr/**/*kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
qk = [(r['Kernel_Name'], (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6) for r in rows if r['Kernel_Name'].startswith('qk')]
for i in range(0, len(qk), 5):
    print(' '.join(f'{n}:{d:.3f}' for n, d in qk[i:i+5]))
PY
