"""W-1Q far targets: H on one target at 28 qubits, 20 launches per target,
per-launch HIP-event times -> fraction of 8 TB/s (32 B x 2^28 per launch).  Run once per knob
setting (the slice tables read QSIM_SLICE_* / QSIM_NT at first use); prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))
import qsim_amd as q  # noqa: E402

n = 28
targets = [int(x) for x in os.environ.get("TARGETS", "8,16,18,19,20,21,22,23,24,25,26,27").split(",")]
reps = int(os.environ.get("REPS", 20))
sim = q.Simulator(n, mode=q.RunMode.PerGate)
out = {"knobs": {k: v for k, v in os.environ.items() if k.startswith(("QSIM_SLICE", "QSIM_NT"))}, "frac": {}}
for t in targets:
    c = q.Circuit(n)
    for _ in range(reps):
        c.h(t)
    sim.run(c)
    sim.synchronize()
    sim.state.profile(True)
    sim.state.profileReset()
    sim.run(c)
    sim.synchronize()
    st = sim.state.profileStats()
    sim.state.profile(False)
    ms = sum(s["ms"] for s in st) / max(1, sum(s["launches"] for s in st))
    out["frac"][t] = round(32.0 * 2 ** n / (ms / 1e3) / 8e12, 4)
print(json.dumps(out))
