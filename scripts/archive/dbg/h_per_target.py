"""Per-target H at 28 qubits (unfused, PerGate): average kernel time per target (HIP events)."""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "cuda-quantum-simulator_amd"))
import qsim_amd as q

n = int(os.environ.get("QUBITS", 28))
sim = q.Simulator(n, mode=q.RunMode.PerGate)
for t in range(n):
    c = q.Circuit(n)
    for _ in range(10):
        c.h(t)
    sim.run(c)
    sim.synchronize()
    sim.state.profileReset()
    sim.state.profile(True)
    sim.run(c)
    sim.synchronize()
    st = sim.state.profileStats()
    sim.state.profile(False)
    ms = sum(s["ms"] for s in st) / sum(s["launches"] for s in st)
    frac = 32 * 2 ** n / (ms / 1e3) / 8e12
    print(json.dumps({"t": t, "kernel": [s["name"] for s in st], "ms": round(ms, 4), "frac": round(frac, 4)}), flush=True)
