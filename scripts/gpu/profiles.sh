#!/bin/bash
# Timed-region rocprof profiles of every roofline object of the bench line (roctx range
# "timed_<region>", --marker-trace), each line's frac recomputed from the rocprof durations
# (scripts/roofline_check.py), then PMC HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes,
# scripts/pmc_summary.py) of the batched tile kernel and the NoisySimulator pull pass.
#     gpurun --timeout 1200 -- bash scripts/gpu/profiles.sh <tag> [region ...]
# regions: hc 1q28 batch16ref noisy26 dm14 pmc (default: all)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/${1:-profiles}
shift
REGIONS=${*:-hc 1q28 batch16ref noisy26 dm14 pmc}
mkdir -p $O
prof() {  # region, extra bench args...
  local rg=$1; shift
  cd /tmp && timeout -k 10 400 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv \
    -d $O/prof_$rg -o $rg -- python3 $R/bench.py --cpu-budget 0 --profile-region $rg "$@" \
    > $O/bench_$rg.json 2> $O/bench_$rg.err || { tail -5 $O/bench_$rg.err; return 1; }
  cd $R
  python3 scripts/roofline_check.py $rg $O/bench_$rg.json $O/prof_$rg/${rg}_kernel_trace.csv $O/check_$rg.json \
    --markers=$O/prof_$rg/${rg}_marker_api_trace.csv | grep -E "frac|launches"
}
run_pmc() {  # name, command...
  local name=$1; shift
  for i in 1 2; do
    C=FETCH_SIZE; [ $i = 2 ] && C=WRITE_SIZE
    cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $C -d $O/pmc_$name/p$i -o run --output-format csv -- "$@" > $O/pmc_${name}_p$i.log 2>&1 || { cd $R; tail -5 $O/pmc_${name}_p$i.log; return 1; }
    cd $R
  done
  python3 scripts/pmc_summary.py $O/pmc_$name $O/pmc_$name.json > $O/pmc_$name.txt || return 1
  head -30 $O/pmc_$name.txt
}
for rg in $REGIONS; do
  case $rg in
    hc) prof hc --steps 20 --warmup 2 --no-1q28 --no-batch16 --no-extras || exit 1 ;;
    hc28) prof hc28 --steps 3 --warmup 1 --no-1q28 --no-batch16 --extras w_hc_28q || exit 1 ;;
    pmchc28)
      run_pmc hc_28q python3 $R/bench.py --qubits 28 --cpu-budget 0 --steps 3 --warmup 1 --no-1q28 --no-batch16 --no-extras || exit 1 ;;
    1q28) prof 1q28 --steps 3 --warmup 1 --no-batch16 --no-extras || exit 1 ;;
    batch16ref) prof batch16ref --steps 3 --warmup 1 --no-1q28 --no-extras || exit 1 ;;
    noisy26) prof noisy26 --workload noisy --steps 3 || exit 1 ;;
    dm14) prof dm14 --workload dm --steps 5 || exit 1 ;;
    pmcnoisy)
      run_pmc noisy_26q python3 $R/bench.py --workload noisy --cpu-budget 0 --steps 2 --warmup 1 || exit 1 ;;
    pmc1q)
      run_pmc 1q_28q python3 $R/scripts/w1q28.py || exit 1 ;;
    pmcbatch)
      ( export QSIM_NOISE_SPLIT=1; run_pmc batch_ref_16q python3 $R/bench.py --workload batch --cpu-budget 0 --steps 2 --warmup 1 ) || exit 1 ;;
    pmc)
      # (one part on one stream: every tile launch covers the whole ensemble, as the line's
      # per-kernel table, which looks this traffic up per launch)
      ( export QSIM_NOISE_SPLIT=1; run_pmc batch_ref_16q python3 $R/bench.py --workload batch --cpu-budget 0 --steps 2 --warmup 1 ) || exit 1
      run_pmc noisy_26q python3 $R/bench.py --workload noisy --cpu-budget 0 --steps 2 --warmup 1 || exit 1 ;;
    *) echo "unknown region $rg"; exit 2 ;;
  esac
done
