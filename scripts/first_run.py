#!/usr/bin/env python3
"""One process's first run of the W-HC circuit (bench.py's mode: inline compilation, calibrated
first run), for the on-disk cache measurement (csrc/hip/cache.hip): prints one JSON line with the
first run's wall time, the steady-state step time, the cache counters of this process and a
checksum of the final probabilities (equal across processes: the cache must not change results).

    QSIM_CACHE_DIR=<dir> python scripts/first_run.py [n] [seed]
"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "cuda-quantum-simulator_amd"))
import qsim_amd as q  # noqa: E402
from qsim_amd import _lib  # noqa: E402
from qsim_amd.plan import set_jit  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 42
set_jit(2, -1)
c = q.createRandomHCCircuit(n, 100, seed)
sim = q.Simulator(n)
t0 = time.perf_counter()
sim.run(c)
sim.synchronize()
first = time.perf_counter() - t0
ts = []
for _ in range(3):
    t0 = time.perf_counter()
    sim.run(c)
    sim.synchronize()
    ts.append(time.perf_counter() - t0)
st = [ctypes.c_uint64() for _ in range(4)]
_lib.check(_lib.hip.qsim_cache_stats(*[ctypes.byref(x) for x in st]))
p0 = [round(sim.state.probBitZero(b), 12) for b in range(n)]
print(json.dumps({"qubits": n, "seed": seed, "first_run_ms": round(first * 1e3, 1),
                  "step_ms": round(sorted(ts)[1] * 1e3, 3), "passes": sim.state.lastRunInfo()[0],
                  "jit_hits": st[0].value, "jit_stores": st[1].value, "layout_hits": st[2].value,
                  "layout_stores": st[3].value, "p0": p0}))
