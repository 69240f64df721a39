#!/bin/bash
# Round 3: W-BATCH reference noise process — per-step time vs ensemble size (does a smaller,
# cache-resident ensemble run proportionally faster?)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r3m
mkdir -p $out
for B in 1024 256 128 64 32; do
  timeout -k 10 300 python -u bench.py --workload batch --batch-noise reference --trajectories $B \
      --steps 5 --warmup 1 > $out/b$B.json 2> $out/b$B.err || { tail -5 $out/b$B.err; exit 1; }
  python -c "import json;d=json.load(open('$out/b$B.json'));print($B, d['value'], d['ms_per_step'], [(k['name'],round(k['ms']/max(1,k['launches']),4),k['launches']) for k in d['kernels']])"
done
