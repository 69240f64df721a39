"""W-HC at small n: wall time per circuit with and without per-launch HIP events (profiling)."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))
import qsim_amd as q
from qsim_amd.plan import set_jit
set_jit(2, -1)
for n in (20, 22, 24, 26):
    c = q.createRandomHCCircuit(n, 100, 42)
    sim = q.Simulator(n)
    for _ in range(5): sim.run(c)
    sim.synchronize()
    res = {}
    for prof in (False, True, False, True):
        sim.state.profile(prof)
        t0 = time.perf_counter()
        for _ in range(200): sim.run(c)
        sim.synchronize()
        res.setdefault(prof, []).append(round((time.perf_counter() - t0) / 200 * 1e6, 2))
    sim.state.profile(False)
    print(json.dumps({"n": n, "us_per_circuit_no_events": res[False], "us_per_circuit_events": res[True]}), flush=True)
