#!/bin/bash
# Relabeling: GPU tests, default bench line, 28q bench, whole GPU suite in one process.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/relabel; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_relabel_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_relabel.log 2>&1 || { tail -40 $O/pytest_relabel.log; exit 1; }
tail -1 $O/pytest_relabel.log
timeout -k 10 300 python bench.py > $O/bench30.json 2> $O/bench30.err || { tail $O/bench30.err; exit 1; }
timeout -k 10 300 python bench.py --qubits 28 --cpu-budget 0 --no-1q28 > $O/bench28.json 2> $O/bench28.err || { tail $O/bench28.err; exit 1; }
QSIM_RELABEL=0 timeout -k 10 300 python bench.py --cpu-budget 0 --no-1q28 > $O/bench30_norelabel.json 2> $O/bench30n.err || { tail $O/bench30n.err; exit 1; }
python3 -c "
import json
for f in ('bench30','bench28','bench30_norelabel'):
    d=json.load(open('$O/'+f+'.json')); r=d['roofline']
    print(f, d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], [(k['name'],round(k['ms']/k['launches'],3)) for k in d['kernels']])"
timeout -k 10 700 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
