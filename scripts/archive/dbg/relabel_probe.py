"""W-HC 30q original vs qubit-relabeled (gate qubits mapped q -> pi[q]): same computation up to a
relabeling; does the relabeled circuit's pass layout stream faster?  usage: relabel_probe.py pi.json"""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))
import qsim_amd as q
from qsim_amd.plan import set_jit
set_jit(2, -1)
n = 30
pi = json.load(open(sys.argv[1]))
c0 = q.createRandomHCCircuit(n, 100, 42)
c1 = q.Circuit(n)
for g in c0.getGates():
    c1.append(q.GateOp(g.type, [pi[x] for x in g.qubits], g.parameter))
sim = q.Simulator(n)
for name, c in (("original", c0), ("relabeled", c1), ("original", c0), ("relabeled", c1)):
    for _ in range(2):
        sim.run(c)
    sim.synchronize()
    sim.state.profile(True)
    sim.state.profileReset()
    t0 = time.perf_counter()
    for _ in range(5):
        sim.run(c)
    sim.synchronize()
    ms = (time.perf_counter() - t0) / 5 * 1e3
    st = sim.state.profileStats()
    sim.state.profile(False)
    print(json.dumps({"circuit": name, "ms_per_step": round(ms, 3), "passes_per_step": sum(s["launches"] for s in st) / 5,
                      "gates_per_s": round(100 / ms * 1e3, 1)}), flush=True)
