#!/bin/bash
# Sharded engine, pivot chosen by planned passes vs the gate-level score: dist GPU tests +
# virtual 30q/8 (per-rank pass time, launches, overlapped remaps).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/dpiv; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_dist_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 1 0; do
  QSIM_DIST_PIVOT_PLAN=$v timeout -k 10 240 python scripts/dist_virtual_bench.py 30 8 4 > $O/virt_p$v.json 2> $O/virt_p$v.err || { tail $O/virt_p$v.err; exit 1; }
done
python3 -c "
import json
for f in ('virt_p1','virt_p0'):
    d=json.load(open('$O/'+f+'.json')); print(f, {k:(round(v['per_rank_ms_per_run'],3), v['launches_per_run']) for k,v in d.items() if isinstance(v,dict)}, {k:v for k,v in d.items() if not isinstance(v,dict)})"
