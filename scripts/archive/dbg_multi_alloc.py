"""Debug: several 16 GiB W-HC 30q states alive at once in one (fresh) process, same plan (layout
memo), per-run time of each — does the 13-qubit-tile pass speed depend on which memory the state
got?"""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))
import qsim_amd as q
from qsim_amd.plan import set_jit
set_jit(2, -1)
n, k = 30, int(os.environ.get("DBG_STATES", "4"))
c = q.createRandomHCCircuit(n, 100, 42)
sims = [q.Simulator(n) for _ in range(k)]
for s in sims:
    s.run(c); s.synchronize()
res = []
for rep in range(2):
    for i, s in enumerate(sims):
        ts = []
        for _ in range(3):
            t0 = time.perf_counter(); s.run(c); s.synchronize(); ts.append((time.perf_counter() - t0) * 1e3)
        res.append((rep, i, round(min(ts), 3)))
print(json.dumps({"tile": os.environ.get("QSIM_TILE_HMAX"), "runs": res}), flush=True)
