#!/bin/bash
# Sharded engine check: dist GPU tests + virtual 30q/8-rank run (per-rank pass time), overlap on
# and off.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/dist; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_dist_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python scripts/dist_virtual_bench.py 30 8 4 > $O/virt_ovl.json 2> $O/virt_ovl.err || { tail $O/virt_ovl.err; exit 1; }
QSIM_DIST_OVERLAP=0 timeout -k 10 200 python scripts/dist_virtual_bench.py 30 8 4 > $O/virt_noovl.json 2> $O/virt_noovl.err || { tail $O/virt_noovl.err; exit 1; }
python3 -c "
import json
for f in ('virt_ovl','virt_noovl'):
    d=json.load(open('$O/'+f+'.json')); print(f, {k:(round(v['per_rank_ms_per_run'],3), v['launches_per_run']) for k,v in d.items() if isinstance(v,dict)})"
