#!/bin/bash
# Sharded engine with local-position relabeling: dist GPU tests + virtual 30q/8 with/without.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/drl; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_dist_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python scripts/dist_virtual_bench.py 30 8 4 > $O/virt.json 2> $O/virt.err || { tail $O/virt.err; exit 1; }
QSIM_RELABEL=0 timeout -k 10 200 python scripts/dist_virtual_bench.py 30 8 4 > $O/virt_norl.json 2> $O/virt_norl.err || { tail $O/virt_norl.err; exit 1; }
python3 -c "
import json
for f in ('virt','virt_norl'):
    d=json.load(open('$O/'+f+'.json')); print(f, {k:(round(v['per_rank_ms_per_run'],3), v['launches_per_run']) for k,v in d.items() if isinstance(v,dict)})"
