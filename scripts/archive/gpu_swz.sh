#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/swz; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_jit.py tests/test_parity_gpu.py tests/test_bench_path_gpu.py tests/test_batched_gpu.py tests/test_density.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "Error|assert|FAIL" $O/pytest.log | head -30; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --cpu-budget 0 --steps 10 > $O/bench30.json 2> $O/bench30.err || { cat $O/bench30.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench30.json')); r=d['roofline']
print('30q', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], d['roofline_1q28']['frac'])"
timeout -k 10 300 python bench.py --workload batch --qubits 16 --steps 5 --warmup 2 > $O/batch.json 2>&1 || exit 1
python3 -c "
import json; d=json.load(open('$O/batch.json')); r=d['roofline']
print('batch', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof30 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-budget 0 --no-1q28 > $O/prof30.json 2> $O/prof30.err || exit 1
cut -d, -f1-4 $(find $O/prof30 -name "*kernel_stats.csv" | head -1) | head -12
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES -d $O/pmc_lds -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-budget 0 --no-1q28 > $O/pmc_lds.log 2>&1 || exit 1
python3 - <<PY
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for p in glob.glob("$O/pmc_lds/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if r["Kernel_Name"].startswith("qk"):
            acc[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(acc.items()): print(k, dict(v))
PY
