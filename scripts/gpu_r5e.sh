#!/bin/bash
# Round 5: timed-region profiles (roctx range, --marker-trace) of the 1q28 / batch16ref / noisy26 /
# dm14 objects with their recomputed rooflines, and PMC HBM traffic (FETCH_SIZE / WRITE_SIZE in
# separate passes) of the batched tile kernel and the NoisySimulator pull pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/${1:-r5e}
mkdir -p $O
prof() {  # region, extra bench args...
  local rg=$1; shift
  cd /tmp && timeout -k 10 400 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv \
    -d $O/prof_$rg -o $rg -- python3 $R/bench.py --cpu-budget 0 --profile-region $rg "$@" \
    > $O/bench_$rg.json 2> $O/bench_$rg.err || { tail -5 $O/bench_$rg.err; return 1; }
  cd $R
  python3 scripts/roofline_check.py $rg $O/bench_$rg.json $O/prof_$rg/${rg}_kernel_trace.csv $O/check_$rg.json \
    --markers=$O/prof_$rg/${rg}_marker_api_trace.csv | grep -E "frac|\"launches|avg_ms|median_ms"
}
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu -x tests/test_batched_refnoise_gpu.py tests/test_noisy_gpu.py > $O/pytest_noise.log 2>&1 || { tail -30 $O/pytest_noise.log; exit 1; }
tail -1 $O/pytest_noise.log
prof 1q28 --steps 3 --warmup 1 --no-batch16 --no-extras || exit 1
prof batch16ref --steps 3 --warmup 1 --no-1q28 --no-extras || exit 1
run_pmc() {  # name, command...
  local name=$1; shift
  for i in 1 2; do
    C=FETCH_SIZE; [ $i = 2 ] && C=WRITE_SIZE
    cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $C -d $O/pmc_$name/p$i -o run --output-format csv -- "$@" > $O/pmc_${name}_p$i.log 2>&1 || { cd $R; tail -5 $O/pmc_${name}_p$i.log; return 1; }
    cd $R
  done
  python3 scripts/pmc_summary.py $O/pmc_$name $O/pmc_$name.json > $O/pmc_$name.txt || return 1
  grep -E "gate_noise|noise_lists|\"noise\"|pull_gate|noise_map" -A4 $O/pmc_$name.json | grep -E "^  \"|hbm_bytes" | head -20
}
run_pmc batch_ref_16q python3 $R/bench.py --workload batch --cpu-budget 0 --steps 2 --warmup 1 || exit 1
run_pmc noisy_26q python3 $R/bench.py --workload noisy --cpu-budget 0 --steps 2 --warmup 1 || exit 1
cp $O/pmc_noisy_26q.json profiles/pmc_noisy_26q.json
timeout -k 10 300 python -u bench.py --workload noisy --cpu-budget 0 --steps 3 > $O/noisy.json 2> $O/noisy.err || { tail -5 $O/noisy.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/noisy.json'));print('noisy', d['value'], d['ms_per_step'], d['noise_roofline']); print([(k['name'], round(k['ms']/max(1,k['launches']),4)) for k in d['kernels']])"
cd /tmp && timeout -k 10 400 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d $O/prof_noisy26 -o noisy26 -- python3 $R/bench.py --workload noisy --cpu-budget 0 --steps 3 --profile-region noisy26 > $O/bench_noisy26.json 2> $O/bench_noisy26.err || { tail -5 $O/bench_noisy26.err; exit 1; }
cd /tmp && timeout -k 10 400 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d $O/prof_dm14 -o dm14 -- python3 $R/bench.py --workload dm --cpu-budget 0 --steps 5 --profile-region dm14 > $O/bench_dm14.json 2> $O/bench_dm14.err || { tail -5 $O/bench_dm14.err; exit 1; }
cd $R
python3 scripts/roofline_check.py dm14 $O/bench_dm14.json $O/prof_dm14/dm14_kernel_trace.csv $O/check_dm14.json --markers=$O/prof_dm14/dm14_marker_api_trace.csv | grep -E "frac|\"launches"
