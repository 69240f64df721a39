"""Host cost of the first fused run (planning, layout choice, JIT) vs later runs, 28q W-HC:
a fresh Simulator, then a second fresh Simulator with the same circuit (layout memo hit)."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))
import qsim_amd as q
from qsim_amd.plan import set_jit
set_jit(1, -1)  # the library default: background compile
n = 28
c = q.createRandomHCCircuit(n, 100, 42)
out = {}
for obj in ("first", "second"):
    sim = q.Simulator(n)
    t0 = time.perf_counter(); sim.run(c); sim.synchronize(); out[obj + "_run_s"] = round(time.perf_counter() - t0, 3)
    t0 = time.perf_counter(); sim.run(c); sim.synchronize(); out[obj + "_rerun_s"] = round(time.perf_counter() - t0, 4)
    del sim
print(json.dumps({"relabel": os.environ.get("QSIM_RELABEL", "1"), **out}))
