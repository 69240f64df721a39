#!/bin/bash
# smoke() + W-BATCH under both noise processes + virtual 30q/8 shards on the final tree.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/sb
mkdir -p $O
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py --workload batch --cpu-budget 0 > $O/batch_phys.json 2> $O/batch_phys.err || exit 1
timeout -k 10 300 python bench.py --workload batch --batch-noise reference --steps 2 --warmup 1 --cpu-budget 0 > $O/batch_ref.json 2> $O/batch_ref.err || exit 1
python - <<PY
import json
for f in ('batch_phys', 'batch_ref'):
    d = json.load(open('$O/%s.json' % f)); r = d['roofline']
    print(f, d['value'], d['unit'], d['ms_per_step'], r and round(r['frac'], 4), r and r.get('avg_launch_ms'))
PY
