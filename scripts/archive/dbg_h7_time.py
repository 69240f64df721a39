"""Debug: per-step times of W-HC 30q under 13-qubit tiles (h=7, T13 1.25) and 12-qubit tiles, two
states in one process, alternating, over ~1 minute — is the slow/fast 13-qubit behaviour a per-process
(allocation) effect or a drift over time?"""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))
import qsim_amd as q
from qsim_amd.plan import set_jit, set_tile_height
set_jit(2, -1)
n = 30
c = q.createRandomHCCircuit(n, 100, 42)
sims = {}
for h in (7, 6):
    set_tile_height(h)
    s = q.Simulator(n)
    s.run(c); s.synchronize()
    sims[h] = s
set_tile_height(-1)
t_end = time.time() + float(os.environ.get("DBG_SECONDS", "60"))
rows = []
while time.time() < t_end:
    for h in (7, 6):
        ts = time.perf_counter()
        for _ in range(3):
            sims[h].run(c)
        sims[h].synchronize()
        rows.append((round(time.time(), 2), h, round((time.perf_counter() - ts) / 3 * 1e3, 3)))
    print(rows[-2], rows[-1], flush=True)
print(json.dumps({"h7": [r[2] for r in rows if r[1] == 7], "h6": [r[2] for r in rows if r[1] == 6]}))
