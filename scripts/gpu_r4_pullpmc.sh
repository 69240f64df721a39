#!/bin/bash
# Round 4: PMC HBM traffic of the opt-in pulled reference-noise step (W-BATCH 16q x 1024):
# FETCH_SIZE / WRITE_SIZE in separate passes.  Usage: gpu_r4_pullpmc.sh <outdir>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD; O=$PWD/gpurun_out/${1:-r4pullpmc}
mkdir -p $O
export QSIM_NOISE_PULL=1
cd /tmp
for i in 1 2; do
  C=FETCH_SIZE; [ $i = 2 ] && C=WRITE_SIZE
  timeout -s KILL 240 rocprofv3 --pmc $C -d $O/pmc/p$i -o run --output-format csv -- python3 $R/bench.py --workload batch --cpu-budget 0 --steps 1 --warmup 1 > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
done
python3 $R/scripts/pmc_summary.py $O/pmc $O/pmc_batch_ref_pull_16q.json > $O/pmc.txt || exit 1
cat $O/pmc.txt
