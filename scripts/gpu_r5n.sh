#!/bin/bash
# Round 5: DensityMatrixSimulator 14q variants (tile height, stage width, pipelined kernels).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5n}
mkdir -p $O
for v in "x=0" "QSIM_TILE_RB7=3" "QSIM_JIT_PIPE=0" "QSIM_TILE_HMAX=6" "QSIM_TILE_HMAX=6 QSIM_TILE_RB=3" "QSIM_JIT_NT=0"; do
  tag=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 300 python -u bench.py --workload dm --cpu-budget 0 --steps 5 > $O/dm_$tag.json 2> $O/dm_$tag.err || { tail -5 $O/dm_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/dm_$tag.json'));print('$v', d['value'], d['ms_per_step'], d['passes'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
done
for pr in 0 1; do
  QSIM_NOISE_STREAM_PRIO=$pr timeout -k 10 300 python -u bench.py --workload batch --cpu-budget 0 --steps 3 --warmup 1 > $O/b_prio$pr.json 2> $O/b_prio$pr.err || { tail -5 $O/b_prio$pr.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_prio$pr.json'));print('batch prio=$pr', d['value'], d['ms_per_step'], [(k['name'], round(k['ms']/max(1,k['launches']),4)) for k in d['kernels']])"
done
