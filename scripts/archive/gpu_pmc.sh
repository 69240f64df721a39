#!/bin/bash
# PMC counter passes (rocprofv3 --pmc, one counter group per pass, no tracing domains mixed in).
# Usage on the GPU box: QUBITS=28 TAG=x bash scripts/gpu_pmc.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_${TAG:-run}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
N=${QUBITS:-28}
ARGS="--qubits $N --workload ${WORKLOAD:-hc} --steps 1 --warmup 0 --cpu-budget 0 ${BENCH_ARGS:-}"
timeout -k 10 120 rocprofv3 -L > $OUT/counters_available.txt 2>&1 || true
i=0
PGROUPS=("FETCH_SIZE" "WRITE_SIZE")
[ -n "$FULL" ] && PGROUPS+=("SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" \
    "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES" \
    "SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM")
for grp in "${PGROUPS[@]}"; do
  i=$((i+1))
  echo "== pmc pass $i: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp -d $OUT/p$i -o run --output-format csv \
      -- python3 $R/bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 $R/scripts/pmc_summary.py $OUT $R/gpurun_out/pmc_${WORKLOAD:-hc}_${N}q.json
