#!/usr/bin/env python3
"""Single-GPU estimate of the sharded path's per-rank work: W virtual ranks on one GPU (the same
planner, per-rank lowering, fused passes and pack/unpack kernels as the RCCL path; exchanges are
device copies).  Prints passes and remaps per run and the per-rank local compute time (all shards'
pass time / W), which is what one GPU of a W-GPU node spends outside the xGMI transfers.

usage: python scripts/dist_virtual_bench.py [n] [world] [steps]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))

import qsim_amd as q  # noqa: E402
from qsim_amd.dist import DistributedSimulator  # noqa: E402
from qsim_amd.plan import set_jit  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
set_jit(2, -1)
c = q.createRandomHCCircuit(n, 100, 42)
d = DistributedSimulator.virtual(n, world)
seen = {tuple(d.perm())}
for i in range(12):
    d.run(c)
    p = tuple(d.perm())
    if p in seen:
        break
    seen.add(p)
d.synchronize()
d.profile(True)
t0 = time.perf_counter()
for _ in range(steps):
    d.run(c)
d.synchronize()
wall = time.perf_counter() - t0
st = d.profileStats()
out = {"n": n, "world": world, "steps": steps, "wall_ms_per_run_all_shards": wall / steps * 1e3,
       "fused_remaps_last_run": d.fusedRemaps()}
for s in st:
    out[s["name"]] = {"ms_per_run": s["ms"] / steps, "launches_per_run": s["launches"] / steps,
                      "per_rank_ms_per_run": s["ms"] / steps / world,
                      "GBps": s["alg_bytes"] / (s["ms"] / 1e3) / 1e9 if s["ms"] else None}
print(json.dumps(out, indent=1))
