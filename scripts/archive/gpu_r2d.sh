#!/bin/bash
# Round-2 evidence: whole GPU suite in one process (the driver's way), smoke, W-BATCH under both
# noise processes, virtual 30q/8-rank sharded run (remap overlap), W-REF GPU-vs-CPUSimulator
# table, PMC passes for the batched and the W-HC 30q pass kernels.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r2d; mkdir -p $O
cd $R
echo "== suite"; timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
echo "== smoke"; timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
cat $O/smoke.log
echo "== batch"
timeout -k 10 300 python bench.py --workload batch --qubits 16 --steps 5 --warmup 2 --cpu-budget 5 > $O/batch_phys.json 2> $O/batch_phys.err || { tail $O/batch_phys.err; exit 1; }
timeout -k 10 300 python bench.py --workload batch --batch-noise reference --qubits 16 --steps 3 --warmup 1 --cpu-budget 0 > $O/batch_ref.json 2> $O/batch_ref.err || { tail $O/batch_ref.err; exit 1; }
echo "== virtual dist"
timeout -k 10 300 python scripts/dist_virtual_bench.py 30 8 4 > $O/dist_virtual_30_8.json 2> $O/dist_virtual.err || { tail $O/dist_virtual.err; exit 1; }
cat $O/dist_virtual_30_8.json
echo "== wref"
timeout -k 10 300 ./tests/cpp/build/bench_scaling 3 22 > $O/wref_scaling.jsonl 2> $O/wref.err || { tail $O/wref.err; exit 1; }
lscpu | grep -E "Model name|^CPU\(s\)" > $O/host_cpu.txt
echo "== pmc"
QUBITS=16 WORKLOAD=batch TAG=batch16 FULL=1 BENCH_ARGS="--trajectories 1024" bash scripts/gpu_pmc.sh > $O/pmc_batch16.log 2>&1 || { tail -20 $O/pmc_batch16.log; exit 1; }
QUBITS=30 WORKLOAD=hc TAG=hc30 FULL=1 BENCH_ARGS="--no-1q28" bash scripts/gpu_pmc.sh > $O/pmc_hc30.log 2>&1 || { tail -20 $O/pmc_hc30.log; exit 1; }
echo "== done"
