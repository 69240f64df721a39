"""A/B of explicit qubit relabelings of W-HC 30q seed 42 in one process (engine relabeling off):
each permutation file's circuit (gate qubits mapped q -> pi[q]) is timed in interleaved rounds.
usage: QSIM_RELABEL=0 relabel_ab.py pi_a.json pi_b.json ..."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))
import qsim_amd as q
from qsim_amd.plan import set_jit
set_jit(2, -1)
n = int(os.environ.get("N", "30"))
c0 = q.createRandomHCCircuit(n, 100, int(os.environ.get("SEED", "42")))
circs = {"identity": c0}
for f in sys.argv[1:]:
    pi = json.load(open(f))
    c = q.Circuit(n)
    for g in c0.getGates():
        c.append(q.GateOp(g.type, [pi[x] for x in g.qubits], g.parameter))
    circs[os.path.basename(f)] = c
sim = q.Simulator(n)
res = {k: [] for k in circs}
for rnd in range(3):
    for name, c in circs.items():
        for _ in range(2):
            sim.run(c)
        sim.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            sim.run(c)
        sim.synchronize()
        res[name].append(round((time.perf_counter() - t0) / 5 * 1e3, 3))
for k, v in res.items():
    print(json.dumps({"perm": k, "ms_per_step": v, "best_gates_per_s": round(100 / min(v) * 1e3, 1)}), flush=True)
