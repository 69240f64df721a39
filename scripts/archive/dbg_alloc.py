"""Debug: W-HC 30q per-run time with 13-qubit (h=7) and 12-qubit (h=6) tiles for one state
allocation each (QSIM_STATE_OFFSET_KB shifts the amplitudes inside their allocation); with
DBG_REALLOC=k the h=7 state is freed and allocated again k times in this process."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))
import qsim_amd as q
from qsim_amd.plan import set_jit, set_tile_height
set_jit(2, -1)
n = 30
c = q.createRandomHCCircuit(n, 100, 42)
def timed(h):
    set_tile_height(h)
    s = q.Simulator(n)
    s.run(c); s.synchronize()
    ts = []
    for _ in range(4):
        t0 = time.perf_counter(); s.run(c); s.synchronize(); ts.append((time.perf_counter() - t0) * 1e3)
    del s
    return round(sorted(ts)[1], 3)
out = {"offset_kb": os.environ.get("QSIM_STATE_OFFSET_KB", "0"), "h7": [], "h6": timed(6)}
for _ in range(1 + int(os.environ.get("DBG_REALLOC", "0"))):
    out["h7"].append(timed(7))
print(json.dumps(out), flush=True)
