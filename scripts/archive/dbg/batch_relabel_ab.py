"""W-BATCH 16q x 1024: original vs qubit-relabeled W-HC circuit (depolarizing on every qubit, so
the noise model is relabeling-invariant); the map is the engine's choice for the 16q plan."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))
import qsim_amd as q
from qsim_amd.plan import set_jit, plan_relabel
set_jit(2, -1)
n, B = 16, 1024
c0 = q.createRandomHCCircuit(n, 100, 42)
pi, before, after = plan_relabel(c0)
c1 = q.Circuit(n)
for g in c0.getGates():
    c1.append(q.GateOp(g.type, [pi[x] for x in g.qubits], g.parameter))
nm = q.NoiseModel(); nm.addDepolarizingAll(n, 0.01)
print(json.dumps({"pi": pi, "pred_before_us": before, "pred_after_us": after}), flush=True)
res = {"original": [], "relabeled": []}
for rnd in range(3):
    for name, c in (("original", c0), ("relabeled", c1)):
        s = q.BatchedSimulator(n, B, nm); s.setSeed(42)
        for _ in range(2): s.run(c)
        s.synchronize()
        t0 = time.perf_counter()
        for _ in range(10): s.run(c)
        s.synchronize()
        res[name].append(round((time.perf_counter() - t0) / 10 * 1e3, 3))
        del s
print(json.dumps(res), flush=True)
