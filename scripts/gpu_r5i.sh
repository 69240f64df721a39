#!/bin/bash
# Round 5: SQ counters of the in-tile noise kernel, full vs no-flip (QSIM_NOISE_TILE_SKIP=3).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/${1:-r5i}
mkdir -p $O
for sk in 0 3; do
  cd /tmp && QSIM_NOISE_TILE_SKIP=$sk timeout -s KILL 240 rocprofv3 --kernel-include-regex gate_noise --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d $O/sq$sk -o run --output-format csv -- python3 $R/bench.py --workload batch --cpu-budget 0 --steps 1 --warmup 1 > $O/sq$sk.log 2>&1 || { cd $R; tail -5 $O/sq$sk.log; exit 1; }
  cd $R
  python3 - $O/sq$sk "skip=$sk" <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(float); n = collections.Counter()
for p in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
print(sys.argv[2], {k: round(v / max(1, n[k]) , 1) for k, v in sorted(tot.items())})
PY
done
