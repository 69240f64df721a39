#!/bin/bash
# reference-noise unit kernel: per-trajectory noise time vs ensemble size (state in / out of the
# Infinity Cache)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/mall; mkdir -p $O
for B in 128 256 512 1024 2048; do
  QSIM_NOISE_UNIT_MIN=1 timeout -k 10 200 python bench.py --workload batch --batch-noise reference --trajectories $B --steps 3 --warmup 1 --cpu-budget 0 > $O/b$B.json 2> $O/b$B.err || { tail $O/b$B.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b$B.json'));print($B, d['value'], d['ms_per_step'], [(k['name'], round(k['ms']/k['launches'],4)) for k in d['kernels']])"
done
