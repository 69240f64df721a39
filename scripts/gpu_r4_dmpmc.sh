#!/bin/bash
# Round 4: why DensityMatrixSimulator passes stream at ~58 %: SQ issue / wait counters of the DM
# 14q line's pass kernels (one --pmc pass, 8 SQ counters).  Usage: gpu_r4_dmpmc.sh <outdir>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD; O=$PWD/gpurun_out/${1:-r4dmpmc}
mkdir -p $O
cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS -d $O/sq -o run --output-format csv -- python3 $R/bench.py --workload dm --cpu-budget 0 --steps 1 --warmup 1 > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 1; }
python3 - $O/sq <<'PY'
import csv, glob, sys, collections
rows = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    k = r.get("Kernel_Name", r.get("Kernel-Name", "?"))[:40]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    wc = v.get("SQ_WAVE_CYCLES", 1) or 1
    print(k, {c: round(x / wc, 3) for c, x in v.items() if c != "SQ_WAVE_CYCLES"}, "wave_cycles", wc)
PY
