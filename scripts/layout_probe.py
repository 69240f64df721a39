#!/usr/bin/env python3
"""Layout probes at 30q: one-pass circuits (one H per tile qubit) whose tile is given explicitly,
timed with the circuit-specialised kernels.  Families: lane bits of r0 = 4 tiles over low / high
register bits, r0 = 6 tiles with their 6 free bits in different address ranges, and the W-HC 30q
plan's tiles.  One JSON line per probe (ms per pass, GB/s).
usage: python scripts/layout_probe.py [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))
import qsim_amd as q  # noqa: E402
from qsim_amd.plan import plan_fused, set_jit  # noqa: E402

n = 30
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
G = q.GateType
R4 = [0, 1, 2, 3]
R6 = list(range(6))
P = []
for hi in ([14, 15, 16, 17, 18, 19], [24, 25, 26, 27, 28, 29]):
    for a, b in ((4, 5), (6, 7), (6, 13), (9, 10), (12, 13), (20, 21)):
        if a in hi or b in hi:
            continue
        P.append(("lanes", R4 + [a, b] + hi))
for hi in ([6, 7, 8, 9, 10, 11], [12, 13, 14, 15, 16, 17], [18, 19, 20, 21, 22, 23],
           [24, 25, 26, 27, 28, 29], [6, 7, 8, 27, 28, 29], [6, 10, 14, 18, 22, 26],
           [8, 12, 16, 20, 24, 28], [20, 21, 22, 23, 24, 25], [9, 11, 13, 15, 17, 19]):
    P.append(("r6", R6 + hi))
for t in ([0, 1, 2, 3, 6, 13, 16, 23, 25, 26, 28, 29], [0, 1, 2, 3, 5, 9, 11, 12, 15, 18, 20, 21],
          [0, 1, 2, 3, 4, 8, 17, 18, 21, 22, 24, 25], [0, 1, 2, 3, 9, 10, 14, 17, 19, 21, 23, 26],
          [0, 1, 2, 3, 4, 7, 9, 11, 12, 14, 16, 27]):
    P.append(("whc", t))
if os.environ.get("PROBE_RANDOM"):  # random tiles for a layout cost model
    import random
    rng = random.Random(int(os.environ["PROBE_RANDOM"]))
    P = []
    for i in range(int(os.environ.get("PROBE_COUNT", "160"))):
        r0 = rng.choice([4, 5, 6])
        k = 12 - r0
        mode = i % 3
        if mode == 0:
            hi = rng.sample(range(r0, n), k)
        elif mode == 1:  # clustered: a contiguous block plus a few stragglers
            s0 = rng.randrange(r0, n - k + 1)
            blk = list(range(s0, s0 + k - 2))
            rest = [x for x in range(r0, n) if x not in blk]
            hi = blk + rng.sample(rest, 2)
        else:  # biased high
            hi = rng.sample(range(max(r0, 14), n), k)
        P.append(("rand", list(range(r0)) + sorted(hi)))
if os.environ.get("PROBE_LIST"):  # explicit tiles: "0,1,2,...;0,1,..."
    P = [("list", [int(x) for x in t.split(",")]) for t in os.environ["PROBE_LIST"].split(";")]
set_jit(2, -1)
sv = q.StateVector(n)
sv.applyGate(q.GateOp(G.H, [0]))
for kind, qs in P:
    c = q.Circuit(n)
    for t in qs:
        c.append(q.GateOp(G.H, [t]))
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
    print(json.dumps({"kind": kind, "tile": qs, "passes": npass, "launches": k and k["launches"],
                      "ms_per_pass": ms and round(ms, 4),
                      "GBps": ms and round(32.0 * 2 ** n / (ms / 1e3) / 1e9, 1)}), flush=True)
