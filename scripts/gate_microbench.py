#!/usr/bin/env python3
"""Per-gate kernel microbenchmark (W-1Q and friends, one kernel launch per gate, unfused).

For each gate/target: `--reps` launches timed with per-launch HIP events (qsim_state_profile);
reports algorithmic GB/s (SURVEY §8(d) byte table) and the fraction of the 8 TB/s HBM peak.
Run one configuration per process (the launch knobs QSIM_SLICE_U/QSIM_LANE_U/QSIM_DIAG_U/QSIM_NT are
read once per process).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))

import qsim_amd as q  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--qubits", type=int, default=28)
p.add_argument("--reps", type=int, default=10)
p.add_argument("--label", default="")
args = p.parse_args()
n = args.qubits
G = q.GateType
cases = [("H", G.H, [t]) for t in (0, 1, 3, 5, 6, 7, 10, 15, 20, 27)]
cases += [("CNOT", G.CNOT, [27, 0]), ("CNOT", G.CNOT, [3, 20]), ("CNOT", G.CNOT, [10, 20]),
          ("Z", G.Z, [27]), ("Z", G.Z, [3]), ("CZ", G.CZ, [4, 20]), ("Rz", G.Rz, [12]),
          ("Toffoli", G.Toffoli, [1, 2, 27])]
sv = q.StateVector(n)
sv.applyGate(q.GateOp(G.H, [0]))
out = []
for name, t, qs in cases:
    op = q.GateOp(t, qs, 0.3)
    for _ in range(2):
        sv.applyGate(op)
    sv.synchronize()
    sv.profile(True)
    sv.profileReset()
    for _ in range(args.reps):
        sv.applyGate(op)
    sv.synchronize()
    st = sv.profileStats()
    sv.profile(False)
    k = st[0]
    gbps = k["alg_bytes"] / (k["ms"] / 1e3) / 1e9
    out.append({"gate": name, "qubits": qs, "kernel": k["name"], "ms": round(k["ms"] / k["launches"], 4),
                "GBps": round(gbps, 1), "frac": round(gbps / 8000.0, 4)})
cfg = {k: os.environ.get(k) for k in ("QSIM_SLICE_U", "QSIM_LANE_U", "QSIM_DIAG_U", "QSIM_NT")}
print(json.dumps({"label": args.label, "n": n, "knobs": cfg, "results": out}))
