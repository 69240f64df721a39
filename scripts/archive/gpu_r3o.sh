#!/bin/bash
# Round 3: phase timing of k_noise_traj (QSIM_NOISE_DBG skips phases; results not valid)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r3o
mkdir -p $out
for d in 0 1 2 4 7 3 5 6; do
  QSIM_NOISE_DBG=$d timeout -k 10 300 python -u bench.py --workload batch --batch-noise reference --trajectories 1024 \
      --steps 3 --warmup 1 > $out/d$d.json 2> $out/d$d.err || { tail -5 $out/d$d.err; exit 1; }
  python -c "import json;d=json.load(open('$out/d$d.json'));print($d, d['value'], d['ms_per_step'], [(k['name'],round(k['ms']/max(1,k['launches']),4),k['launches']) for k in d['kernels']])"
done
