#!/usr/bin/env python3
"""One gate, three execution paths at n qubits: the per-gate kernel (RunMode.PerGate), a one-op
fused pass run by the pass interpreter, and the same pass as a specialised (hipRTC) kernel.
Prints per-launch ms and algorithmic GB/s (SURVEY §8(d) bytes of the gate)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))

import qsim_amd as q  # noqa: E402
from qsim_amd.plan import set_jit  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--qubits", type=int, default=28)
p.add_argument("--reps", type=int, default=10)
args = p.parse_args()
n = args.qubits
G = q.GateType
cases = [("H", [t]) for t in (6, 10, 20, n - 1)] + [("CNOT", [n - 1, 8]), ("CNOT", [3, 20]), ("Rx", [15])]
sv = q.StateVector(n)
out = []
for name, qs in cases:
    c = q.Circuit(n)
    c.append(q.GateOp(getattr(G, name), qs, 0.3))
    row = {"gate": name, "qubits": qs}
    for path, mode, jit in (("per_gate", q.RunMode.PerGate, 0), ("pass", q.RunMode.Fused, 0),
                            ("pass_jit", q.RunMode.Fused, 2)):
        set_jit(jit, 0)
        sv.run(c, mode)
        sv.run(c, mode)
        sv.synchronize()
        sv.profile(True)
        sv.profileReset()
        for _ in range(args.reps):
            sv.run(c, mode)
        sv.synchronize()
        st = sv.profileStats()
        sv.profile(False)
        ms = sum(k["ms"] for k in st) / args.reps
        by = 32.0 * 2 ** n if name in ("H", "Rx") else 16.0 * 2 ** n
        row[path] = {"ms": round(ms, 4), "GBps": round(by / (ms / 1e3) / 1e9, 1),
                     "kernels": sorted({k["name"] for k in st})}
    out.append(row)
    print(json.dumps(row), flush=True)
