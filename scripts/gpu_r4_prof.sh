#!/bin/bash
# Round 4 profiles: rocprofv3 kernel stats of the headline region, and PMC HBM traffic
# (FETCH_SIZE / WRITE_SIZE in separate passes) of the headline W-HC 30q passes, W-1Q 28q and
# W-BATCH 16q x 1024 under the reference noise process.  Usage: gpu_r4_prof.sh <outdir-name>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/${1:-r4prof}
mkdir -p $O
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o hc30 -- python3 $R/bench.py --cpu-budget 0 --no-1q28 --no-batch16 --no-extras > $O/prof_hc.json 2> $O/prof_hc.err || { tail -5 $O/prof_hc.err; exit 1; }
head -8 $O/prof/hc30_kernel_stats.csv
run_pmc() {  # name, command...
  local name=$1; shift
  for i in 1 2; do
    C=FETCH_SIZE; [ $i = 2 ] && C=WRITE_SIZE
    timeout -s KILL 240 rocprofv3 --pmc $C -d $O/pmc_$name/p$i -o run --output-format csv -- "$@" > $O/pmc_${name}_p$i.log 2>&1 || { tail -5 $O/pmc_${name}_p$i.log; return 1; }
  done
  python3 $R/scripts/pmc_summary.py $O/pmc_$name $O/pmc_$name.json > $O/pmc_$name.txt || return 1
  cat $O/pmc_$name.txt
}
QSIM_RELABEL_CALIBRATE=0 run_pmc hc_30q python3 $R/bench.py --cpu-budget 0 --no-1q28 --no-batch16 --no-extras --steps 2 --warmup 1 || exit 1
run_pmc 1q_28q python3 $R/scripts/w1q28.py || exit 1
run_pmc batch_ref_16q python3 $R/bench.py --workload batch --cpu-budget 0 --steps 2 --warmup 1 || exit 1
for w in dm noisy; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o $w -- python3 $R/bench.py --workload $w --cpu-budget 0 > $O/prof_$w.json 2> $O/prof_$w.err || { tail -5 $O/prof_$w.err; exit 1; }
  head -6 $O/prof/${w}_kernel_stats.csv
done
