#!/bin/bash
# Compare fused-pass variants on one GPU: parity subset + pass microbench + W-HC benches per variant.
# Variants are env settings (QSIM_TILE_HMAX, QSIM_TILE_R0, QSIM_FUSED_NT).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/fsweep
mkdir -p $OUT
VARIANTS=${VARIANTS:-"base R05 R04"}
for v in $VARIANTS; do
  case $v in
    base) E="" ;;
    HMAX5) E="QSIM_TILE_HMAX=5" ;;
    NT0) E="QSIM_FUSED_NT=0" ;;
    R05) E="QSIM_TILE_R0=5" ;;
    R04) E="QSIM_TILE_R0=4" ;;
    R06) E="QSIM_TILE_R0=6" ;;
    *) echo "unknown variant $v"; exit 2 ;;
  esac
  echo "== $v ($E)"
  env $E timeout -k 10 300 python -m pytest tests/test_parity_gpu.py tests/test_dist_gpu.py -q -x \
    > $OUT/$v.pytest 2>&1 || { tail -15 $OUT/$v.pytest; exit 1; }
  tail -1 $OUT/$v.pytest
  if [ -z "$NOMICRO" ]; then
    env $E timeout -k 10 300 python scripts/fused_microbench.py --qubits 28 \
      > $OUT/$v.micro 2> $OUT/$v.micro.err || { tail -5 $OUT/$v.micro.err; exit 1; }
    cat $OUT/$v.micro
  fi
  for n in ${BENCH_QUBITS:-28 30}; do
    env $E timeout -k 10 300 python bench.py --qubits $n --steps 3 --warmup 1 --cpu-budget 0 \
      > $OUT/$v.bench$n 2> $OUT/$v.bench$n.err || { tail -5 $OUT/$v.bench$n.err; exit 1; }
    python -c "
import json; d=json.loads(open('$OUT/$v.bench$n').read().strip().splitlines()[-1])
r=d['roofline']; print('bench $n', d['value'], d['ms_per_step'], r['achieved'], r['avg_launch_ms'], r['launches'])"
  done
done
