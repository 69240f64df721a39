#!/bin/bash
# Self-timed launches: overhead of profiling at small n, and HIP-event kernel times vs rocprof.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/evc; mkdir -p $O
timeout -k 10 200 python scripts/dbg/event_overhead.py > $O/overhead.jsonl 2> $O/overhead.err || { tail $O/overhead.err; exit 1; }
cat $O/overhead.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --cpu-budget 0 > $O/bench30.json 2> $O/bench30.err || { tail $O/bench30.err; exit 1; }
python3 - <<PY
import json, glob, csv
d=json.load(open('$O/bench30.json')); print('bench', d['value'], d['roofline']['avg_launch_ms'], d['roofline_1q28']['avg_launch_ms'])
f=glob.glob('$O/prof/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if r['Name'].startswith('qk') or 'm1_' in r['Name']: print(r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e6)
PY
