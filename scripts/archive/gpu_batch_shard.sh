#!/bin/bash
# Trajectory sharding: GPU parity test + the 1-rank and 2-rank (sharing the box's one GPU) W-BATCH
# bench legs.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/bshard; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_batched_gpu.py tests/test_batched_refnoise_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python bench.py --workload batch --qubits 16 --steps 5 --warmup 2 > $O/b1.json 2> $O/b1.err || { tail $O/b1.err; exit 1; }
timeout -k 10 300 python bench.py --workload batch --qubits 16 --steps 5 --warmup 2 --gpus 2 > $O/b2.json 2> $O/b2.err || { tail $O/b2.err; exit 1; }
python3 -c "
import json
for f in ('b1','b2'):
    d=json.load(open('$O/'+f+'.json')); print(f, d['n_gpus'], d['value'], d['ms_per_step'], d['config'].get('trajectories_per_rank'), d['config'].get('ensemble_probability_sum'))"
