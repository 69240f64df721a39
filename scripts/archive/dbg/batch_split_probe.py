"""W-BATCH 16q x 1024 in one process as K objects of 1024/K trajectories (own streams, trajectory
offsets): does running sub-batches concurrently beat one object?"""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))
import qsim_amd as q
from qsim_amd.plan import set_jit
set_jit(2, -1)
n, B = 16, 1024
c = q.createRandomHCCircuit(n, 100, 42)
nm = q.NoiseModel(); nm.addDepolarizingAll(n, 0.01)
for K in (1, 2, 4, 8, 1, 2):
    sims = []
    for k in range(K):
        s = q.BatchedSimulator(n, B // K, nm); s.setSeed(42); s.setTrajectoryOffset(k * (B // K)); sims.append(s)
    for _ in range(2):
        for s in sims: s.run(c)
    for s in sims: s.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        for s in sims: s.run(c)
    for s in sims: s.synchronize()
    ms = (time.perf_counter() - t0) / 10 * 1e3
    print(json.dumps({"K": K, "ms_per_step": round(ms, 3), "traj_gates_per_s": round(100 * B / ms * 1e3)}), flush=True)
    del sims
