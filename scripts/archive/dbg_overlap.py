"""Debug: per-run overlapped remaps of the engine vs the host planner (virtual ranks, one GPU)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cuda-quantum-simulator_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import qsim_amd as q
import dist_hosted
from qsim_amd.dist import DistributedSimulator, plan
for world, n in [(2, 14), (4, 16)]:
    c = dist_hosted.circuits(q, n)[0][1]
    d = DistributedSimulator.virtual(n, world)
    for i in range(3):
        p = d.perm()
        steps, po = plan(c, world, 0, list(p))
        d.run(c)
        print(world, n, i, "engine", d.overlappedRemaps(), "plan",
              sum(1 for s in steps if s["kind"] == "exchange" and s["pivots"]),
              [(s["kind"][0], s.get("k"), s.get("pmask"), s.get("role")) for s in steps], flush=True)
    d.close()
