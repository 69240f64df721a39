"""W-1Q far targets at 28 qubits: one H per run through the per-gate slice kernel vs through a
one-op tile pass (the interpreter and the compiled pass kernel), ms per gate and fraction of
8 TB/s (32 B x 2^28 per gate)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))
import qsim_amd as q  # noqa: E402
from qsim_amd.plan import set_jit, set_relabel, set_relayout  # noqa: E402

n = 28
set_relabel(0, -1)
set_relayout(0, -1)
bytes_ = 32.0 * (1 << n)
for t in (18, 20, 22, 23, 25, 26):
    c = q.Circuit(n)
    c.h(t)
    row = {"t": t}
    for name, mode, jit in (("per_gate", q.RunMode.PerGate, 0), ("pass_interp", q.RunMode.Fused, 0),
                            ("pass_jit", q.RunMode.Fused, 2)):
        set_jit(jit, -1)
        sim = q.Simulator(n, mode=mode)
        for _ in range(3):
            sim.run(c)
        sim.synchronize()
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            sim.run(c)
        sim.synchronize()
        ms = (time.perf_counter() - t0) / reps * 1e3
        row[name] = {"ms": round(ms, 4), "frac": round(bytes_ / (ms / 1e3) / 8e12, 4)}
        sim.state.close()
    print(json.dumps(row), flush=True)
