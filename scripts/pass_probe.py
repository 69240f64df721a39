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


W = [list(range(4)) + [6, 12, 15, 16, 19, 22, 27, 28],   # old W-HC 30q pass 1 tile (r0 = 4)
     list(range(4)) + [6, 13, 16, 23, 25, 26, 28, 29],   # 5-pass plan: pass 0 tile
     list(range(4)) + [9, 10, 14, 17, 19, 21, 23, 26],   # pass 3 tile
     list(range(4)) + [5, 9, 11, 12, 15, 18, 20, 21],    # pass 1 tile
     list(range(6)) + [6 + i for i in range(6)],
     list(range(6)) + [24, 25, 26, 27, 28, 29]]
if os.environ.get("PROBE_LANES"):  # r0 = 4 with lane bits (a, b), registers on 20..25
    W = [list(range(4)) + [a, b] + list(range(20, 26))
         for a, b in ((6, 7), (6, 13), (9, 10), (5, 9), (12, 13), (16, 17), (6, 9), (7, 8))]
probes = []
for qs in W:
    probes.append(("light", qs, light(qs)))
    if not os.environ.get("PROBE_LANES"):
        probes.append(("hc20", qs, hc(qs, 20)))
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
