#!/usr/bin/env python3
"""One-pass probes: circuits the planner turns into exactly ONE fused tile pass, timed on the GPU
(circuit-specialised kernels, HIP events).  Separates what a pass costs from which tile qubits it
spans (run width r0, positions of the high tile bits) and from how many gates it holds.

usage: python scripts/pass_probe.py [n] [reps]     (prints one JSON line per probe)
"""
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))
import qsim_amd as q  # noqa: E402
from qsim_amd.plan import plan_fused, set_jit  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
G = q.GateType


def light(qs):
    c = q.Circuit(n)
    for t in qs:
        c.append(q.GateOp(G.H, [t]))
    return c


def hc(qs, ngates, seed=3):
    """one H per tile qubit, then random H / CNOT inside the tile"""
    rng = random.Random(seed)
    c = light(qs)
    for _ in range(ngates):
        if rng.random() < 0.5:
            c.append(q.GateOp(G.H, [rng.choice(qs)]))
        else:
            a, b = rng.sample(qs, 2)
            c.append(q.GateOp(G.CNOT, [a, b]))
    return c


W = [list(range(4)) + [6, 12, 15, 16, 19, 22, 27, 28],   # W-HC 30q pass 1 tile (r0 = 4)
     list(range(4)) + [6, 8, 13, 18, 23, 25, 26, 29],    # pass 0 tile (r0 = 4)
     list(range(4)) + [6, 8, 10, 12, 14, 16, 18, 20],
     list(range(4)) + [6, 7, 8, 9, 10, 11, 12, 13],
     list(range(4)) + [22, 23, 24, 25, 26, 27, 28, 29],
     list(range(6)) + [6 + i for i in range(6)],
     list(range(6)) + [24, 25, 26, 27, 28, 29],
     list(range(6)) + [10, 14, 17, 19, 21, 24],           # pass 2 tile (r0 = 6)
     list(range(5)) + [6, 9, 12, 15, 18, 21, 24]]
probes = []
for qs in W:
    probes.append(("light", qs, light(qs)))
    probes.append(("hc20", qs, hc(qs, 20)))
    probes.append(("hc40", qs, hc(qs, 40)))
set_jit(2, -1)
sv = q.StateVector(n)
sv.applyGate(q.GateOp(G.H, [0]))
for kind, qs, c in probes:
    _, _, npass = plan_fused(c)
    sv.run(c)
    sv.synchronize()
    sv.profile(True)
    sv.profileReset()
    for _ in range(reps):
        sv.run(c)
    sv.synchronize()
    st = {k["name"]: k for k in sv.profileStats()}
    sv.profile(False)
    k = st.get("fused_tile")
    ms = k["ms"] / k["launches"] if k else None
    print(json.dumps({"kind": kind, "tile": qs, "gates": c.getGateCount(), "plan_passes": npass,
                      "ms_per_pass": round(ms * (k["launches"] / reps) / max(npass, 1), 4) if ms else None,
                      "GBps_per_pass": round(32.0 * 2 ** n / (ms / 1e3) / 1e9, 1) if ms else None}),
          flush=True)
