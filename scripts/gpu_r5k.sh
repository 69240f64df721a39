#!/bin/bash
# Round 5: PMC HBM traffic of the batched tile kernel and the NoisySimulator pull pass; timed-region
# profiles of the noisy26 (serial run) and dm14 objects.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/${1:-r5k}
mkdir -p $O
run_pmc() {  # name, command...
  local name=$1; shift
  for i in 1 2; do
    C=FETCH_SIZE; [ $i = 2 ] && C=WRITE_SIZE
    cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $C -d $O/pmc_$name/p$i -o run --output-format csv -- "$@" > $O/pmc_${name}_p$i.log 2>&1 || { cd $R; tail -5 $O/pmc_${name}_p$i.log; return 1; }
    cd $R
  done
  python3 scripts/pmc_summary.py $O/pmc_$name $O/pmc_$name.json > $O/pmc_$name.txt || return 1
  cat $O/pmc_$name.txt | head -30
}
run_pmc batch_ref_16q python3 $R/bench.py --workload batch --cpu-budget 0 --steps 2 --warmup 1 || exit 1
run_pmc noisy_26q python3 $R/bench.py --workload noisy --cpu-budget 0 --steps 2 --warmup 1 || exit 1
prof() {  # region, extra bench args...
  local rg=$1; shift
  cd /tmp && timeout -k 10 400 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv \
    -d $O/prof_$rg -o $rg -- python3 $R/bench.py --cpu-budget 0 --profile-region $rg "$@" \
    > $O/bench_$rg.json 2> $O/bench_$rg.err || { tail -5 $O/bench_$rg.err; return 1; }
  cd $R
  python3 scripts/roofline_check.py $rg $O/bench_$rg.json $O/prof_$rg/${rg}_kernel_trace.csv $O/check_$rg.json \
    --markers=$O/prof_$rg/${rg}_marker_api_trace.csv | grep -E "frac|launches"
}
prof noisy26 --workload noisy --steps 3 || exit 1
prof dm14 --workload dm --steps 5 || exit 1
