#!/usr/bin/env python3
"""Fused tile-pass microbenchmark: one pass per circuit, chosen tile qubits, light vs heavy op lists.

Each circuit touches qubits 0..5 plus six chosen high qubits only, so the planner emits exactly one
fused pass whose tile is those 12 qubits.  "light" = one H per qubit (12 ops), "heavy" = the light
list plus 60 random Rx/Ry/Rz/CNOT/CZ gates inside the tile.  Reports per-launch ms and GB/s
(32 B per amplitude per pass).
"""
import argparse
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))

import qsim_amd as q  # noqa: E402
from qsim_amd.plan import plan_fused  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--qubits", type=int, default=28)
p.add_argument("--reps", type=int, default=10)
args = p.parse_args()
n = args.qubits
G = q.GateType
sets = [list(range(6, 12)), list(range(12, 18)), list(range(n - 12, n - 6)), list(range(n - 6, n)),
        [6, 10, 14, 18, 22, n - 1], [6, 7, 8, n - 3, n - 2, n - 1]]


def circuit(hs, heavy):
    rng = random.Random(7)
    qs = list(range(6)) + hs
    c = q.Circuit(n)
    for t in qs:
        c.append(q.GateOp(G.H, [t]))
    if heavy:
        for _ in range(60):
            k = rng.randrange(5)
            if k < 3:
                c.append(q.GateOp([G.Rx, G.Ry, G.Rz][k], [rng.choice(qs)], rng.uniform(0, 6.28)))
            else:
                a, b = rng.sample(qs, 2)
                c.append(q.GateOp(G.CNOT if k == 3 else G.CZ, [a, b]))
    return c


sim = q.StateVector(n)
sim.applyGate(q.GateOp(G.H, [0]))
out = []
for hs in sets:
    for heavy in (False, True):
        c = circuit(hs, heavy)
        plan = plan_fused(c, 6)
        sim.run(c)
        sim.synchronize()
        sim.profile(True)
        sim.profileReset()
        for _ in range(args.reps):
            sim.run(c)
        sim.synchronize()
        st = {k["name"]: k for k in sim.profileStats()}
        sim.profile(False)
        k = st["fused_tile"]
        ms = k["ms"] / k["launches"]
        out.append({"hpos": hs, "heavy": heavy, "passes": k["launches"] // args.reps,
                    "ops": c.getGateCount(), "ms": round(ms, 4),
                    "GBps": round(32.0 * 2 ** n / (ms / 1e3) / 1e9, 1),
                    "plan_passes": plan[2]})
        print(json.dumps(out[-1]), flush=True)
