#!/usr/bin/env python3
"""Is there a K-pass tile plan for a W-HC circuit?  An exact answer by integer programming (scipy
milp / HiGHS), host-only, for VERDICT r5 item 5 ("settle 3 versus 4 passes for seed 42").

Model (a RELAXATION of every plan the engine can build, so "infeasible" is a proof for all of them):
  * gate g runs in exactly one pass p in 1..K; a gate may run in an earlier pass than a gate before
    it only if they share no qubit (the planner's only reordering rule): for every pair
    of consecutive gates on a qubit, pass(first) <= pass(second);
  * pass p has a tile T_p of at most H qubits (H = 13: 8192 amplitudes = 128 KiB, the LDS limit;
    14-qubit tiles need 256 KiB); a gate's TARGET must lie in its pass's tile — its control need not
    (tile-constant controls), which only relaxes the model further;
  * tile shape constraints are then added per layout family:
      free     no other constraint (any relabeling, any relayout, any mix of heights);
      fixed    every tile holds the same r0 >= 4 run qubits (fixed-layout plans: physical qubits
               0..r0-1 are the contiguous HBM run of every pass, whatever the labels);
      relayout consecutive tiles (cyclically: the last pass stores under the first layout) share
               >= 4 qubits, tiles of at most 12 qubits (relayout plans).
The circuit is the engine's own createRandomHCCircuit (the reference's factory, src/Circuit.cpp).

    python scripts/pass_lower_bound.py [--qubits 30] [--seeds 42,1,2,3,4] [--passes 3] [--height 13]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
from scipy.optimize import Bounds, LinearConstraint, milp
from scipy.sparse import lil_matrix

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "cuda-quantum-simulator_amd"))


SHARE = [4]  # relayout: qubits consecutive tiles share (the next pass's run: 2^share amplitudes)
RUN = [4]    # fixed: run qubits every tile holds (r0: runs of 2^r0 amplitudes)


def circuit_gates(n, depth, seed):
    from qsim_amd import circuit as qc
    out = []
    for g in qc.createRandomHCCircuit(n, depth, seed).getGates():
        qs = list(g.qubits)
        out.append((qs[-1], qs))  # (target, all qubits)
    return out


def feasible(n, gates, K, H, family, time_limit=600.0, n_high=None):
    G = len(gates)
    # variables: x[g,p] (G*K), y[q,p] (n*K), then family extras
    nx, ny = G * K, n * K
    X = lambda g, p: g * K + p
    Y = lambda q, p: nx + q * K + p
    extra = 0
    if family == "fixed":
        R0 = nx + ny  # r[q]: q is a run qubit (in every tile)
        extra = n
    elif family == "relayout":
        S0 = nx + ny  # s[q,p]: q in T_p and T_{p+1 mod K}
        extra = n * K
    # n_high: at most this many passes may use H-qubit tiles, the others H - 1 (mixed heights:
    # z[p] = 1 when pass p is a tall one)
    Z0 = nx + ny + extra
    if n_high is not None:
        extra += K
    nv = nx + ny + extra
    rows = []  # (coeffs dict, lo, hi)
    for g in range(G):
        rows.append(({X(g, p): 1 for p in range(K)}, 1, 1))
        t = gates[g][0]
        for p in range(K):
            rows.append(({X(g, p): 1, Y(t, p): -1}, -np.inf, 0))
    last = {}
    for g, (_, qs) in enumerate(gates):
        for q in qs:
            if q in last:  # pass(last[q]) <= pass(g)
                f = last[q]
                c = {}
                for p in range(K):
                    c[X(f, p)] = c.get(X(f, p), 0) + (p + 1)
                    c[X(g, p)] = c.get(X(g, p), 0) - (p + 1)
                rows.append((c, -np.inf, 0))
            last[q] = g
    hp = 12 if family == "relayout" else H
    for p in range(K):
        if n_high is None:
            rows.append(({Y(q, p): 1 for q in range(n)}, 0, hp))
        else:  # |T_p| <= H - 1 + z[p]
            c = {Y(q, p): 1 for q in range(n)}
            c[Z0 + p] = -1
            rows.append((c, 0, hp - 1))
    if n_high is not None:
        rows.append(({Z0 + p: 1 for p in range(K)}, 0, n_high))
    if family == "fixed":
        rows.append(({R0 + q: 1 for q in range(n)}, RUN[0], np.inf))
        for q in range(n):
            for p in range(K):
                rows.append(({R0 + q: 1, Y(q, p): -1}, -np.inf, 0))
    elif family == "relayout":
        for p in range(K):
            pn = (p + 1) % K
            rows.append(({S0 + q * K + p: 1 for q in range(n)}, SHARE[0], np.inf))
            for q in range(n):
                rows.append(({S0 + q * K + p: 1, Y(q, p): -1}, -np.inf, 0))
                rows.append(({S0 + q * K + p: 1, Y(q, pn): -1}, -np.inf, 0))
    A = lil_matrix((len(rows), nv))
    lo, hi = np.empty(len(rows)), np.empty(len(rows))
    for i, (c, a, b) in enumerate(rows):
        for j, v in c.items():
            A[i, j] = v
        lo[i], hi[i] = a, b
    t0 = time.time()
    res = milp(c=np.zeros(nv), constraints=LinearConstraint(A.tocsr(), lo, hi),
               integrality=np.ones(nv), bounds=Bounds(0, 1),
               options={"time_limit": time_limit, "presolve": True})
    dt = time.time() - t0
    # status 0: optimal (a feasible plan exists), 2: infeasible (proof), else undecided
    verdict = {0: "feasible", 2: "infeasible"}.get(res.status, f"undecided ({res.message})")
    plan = None
    if res.status == 0:
        x = np.round(res.x[:nx]).reshape(G, K)
        y = np.round(res.x[nx:nx + ny]).reshape(n, K)
        plan = {"pass_of_gate": [int(np.argmax(x[g])) + 1 for g in range(G)],
                "tiles": [[q for q in range(n) if y[q, p] > 0.5] for p in range(K)]}
    return verdict, round(dt, 2), plan


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=30)
    ap.add_argument("--depth", type=int, default=100)
    ap.add_argument("--seeds", default="42,1,2,3,4")
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--height", type=int, default=13)
    ap.add_argument("--families", default="free,fixed,relayout")
    ap.add_argument("--tall", type=int, default=None,
                    help="mixed heights: at most this many passes of --height qubits, the rest one less")
    ap.add_argument("--share", type=int, default=4,
                    help="relayout family: qubits consecutive tiles share (run of 2^share amplitudes)")
    ap.add_argument("--run", type=int, default=4, help="fixed family: run qubits shared by every tile (r0)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    SHARE[0] = a.share
    RUN[0] = a.run
    results = []
    for sd in [int(s) for s in a.seeds.split(",")]:
        gates = circuit_gates(a.qubits, a.depth, sd)
        targets = len({t for t, _ in gates})
        for fam in a.families.split(","):
            v, dt, plan = feasible(a.qubits, gates, a.passes, a.height, fam, n_high=a.tall)
            r = {"seed": sd, "qubits": a.qubits, "passes": a.passes, "max_tile_qubits": a.height if fam != "relayout" else 12,
                 "tall_passes_max": a.tall, "relayout_share": a.share if fam == "relayout" else None,
                 "fixed_run": a.run if fam == "fixed" else None,
                 "family": fam, "target_qubits": targets, "verdict": v, "seconds": dt}
            if plan:
                r["tiles"] = plan["tiles"]
            print(json.dumps(r), flush=True)
            results.append(r)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
