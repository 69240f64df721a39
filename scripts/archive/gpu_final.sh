#!/bin/bash
# Round-end evidence: GPU parity suite, default bench (30q W-HC), 28q + 20q bench, rocprof kernel
# stats of the default bench, PMC HBM traffic of the fused passes at 30q.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/final
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench30.json 2> $O/bench30.err || exit 1
timeout -k 10 300 python bench.py --qubits 28 --cpu-budget 10 > $O/bench28.json 2> $O/bench28.err || exit 1
timeout -k 10 300 python bench.py --qubits 20 --cpu-budget 10 > $O/bench20.json 2> $O/bench20.err || exit 1
python -c "
import json
for n in (30,28,20):
    d=json.load(open('$O/bench%d.json'%n)); r=d['roofline']
    print(n, d['value'], d['ms_per_step'], r['kernel'], r['achieved'], r['frac'], r['launches'], d['cpu_baseline'] and d['cpu_baseline']['value'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof30 -o run --output-format csv \
  -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-budget 0 > $O/prof30.json 2> $O/prof30.err || exit 1
cut -d, -f1-4 $(find $O/prof30 -name "*kernel_stats.csv" | head -1) | head -12
cd $R && QUBITS=30 TAG=final30 bash scripts/gpu_pmc.sh > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
tail -8 $O/pmc.log
