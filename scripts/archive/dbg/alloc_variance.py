"""W-HC 30q: per-pass times across several state allocations in one process (run under
rocprofv3 --kernel-trace; the trace's dispatch order gives pass j of run r of allocation a)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "cuda-quantum-simulator_amd"))
import qsim_amd as q
from qsim_amd.plan import set_jit

set_jit(2, -1)
c = q.createRandomHCCircuit(30, 100, 42)
for a in range(int(os.environ.get("ALLOCS", 3))):
    sim = q.Simulator(30)
    for r in range(3):
        sim.reset() if r else None
        t = time.perf_counter()
        sim.run(c)
        sim.synchronize()
        print(a, r, round((time.perf_counter() - t) * 1e3, 2), "ms", flush=True)
    del sim
