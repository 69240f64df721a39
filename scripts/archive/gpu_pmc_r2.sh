#!/bin/bash
# PMC evidence for round 2: batched 16q x 1024 frame passes and W-HC 30q passes (traffic + VALU).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
QUBITS=16 WORKLOAD=batch TAG=batch16 FULL=1 BENCH_ARGS="--trajectories 1024" bash scripts/gpu_pmc.sh > gpurun_out/pmc_batch16.log 2>&1 || { tail -20 gpurun_out/pmc_batch16.log; exit 1; }
tail -40 gpurun_out/pmc_batch16.log
QUBITS=30 WORKLOAD=hc TAG=hc30 FULL=1 BENCH_ARGS="--no-1q28" bash scripts/gpu_pmc.sh > gpurun_out/pmc_hc30.log 2>&1 || { tail -20 gpurun_out/pmc_hc30.log; exit 1; }
tail -60 gpurun_out/pmc_hc30.log
