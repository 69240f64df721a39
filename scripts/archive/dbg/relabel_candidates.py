"""Tiles worth probing for the layout model: the physical pass tiles of relabeled W-HC plans
(engine choice + annealing variants under the current model) at 30 and 28 qubits.  Prints one
PROBE_LIST string (tiles separated by ';')."""
import json, os, random, re, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))
import qsim_amd as q
from qsim_amd.plan import plan_relabel, jit_source

text = open(os.path.join(ROOT, "cuda-quantum-simulator_amd/csrc/hip/layout_cost.hpp")).read()
base = float(re.search(r"kBase = ([-\d.]+)f", text).group(1))
w1 = [float(x) for x in re.search(r"kW1\[kN\] = \{([^}]*)\}", text).group(1).replace("f", "").split(",")]
blk = text.split("kW2[kN][kN] = {")[1].split("};")[0]
w2 = np.array([float(x) for x in re.findall(r"-?\d+\.\d+", blk)]).reshape(30, 30)
def cost(t):
    t = sorted(x for x in t if x >= 4)
    return base + sum(w1[x] for x in t) + sum(w2[a][b] for i, a in enumerate(t) for b in t[i + 1:])

def tiles_of(c):
    out = []
    for k in jit_source(c).split('extern "C"')[1:]:
        r0 = int(re.search(r'<< (\d+);\n', k).group(1))
        gb = re.search(r'const unsigned long long gb = (.*);', k).group(1)
        out.append(tuple(list(range(r0)) + [int(x) for x in re.findall(r'<< (\d+)\)', gb)]))
    return out

def relabeled(c, n, pi):
    c1 = q.Circuit(n)
    for g in c.getGates():
        c1.append(q.GateOp(g.type, [pi[x] for x in g.qubits], g.parameter))
    return c1

seen = set()
for n, seeds in ((30, (42, 1, 2, 3, 4)), (28, (42, 1, 2, 3)), (27, (42, 5))):
    for s in seeds:
        c = q.createRandomHCCircuit(n, 100, s)
        ltiles = tiles_of(c)
        cands = [plan_relabel(c)[0]]
        for v in range(int(os.environ.get("VARIANTS", "6"))):  # annealing variants
            rng = random.Random(1000 * s + v)
            pi = list(range(n)); free = list(range(4, n)); rng.shuffle(free)
            for a, b in zip(range(4, n), free): pi[a] = b
            cur = sum(cost({pi[x] for x in t}) for t in ltiles); T = 300.0
            for it in range(8000):
                a, b = rng.sample(range(4, n), 2)
                pi[a], pi[b] = pi[b], pi[a]
                c2 = sum(cost({pi[x] for x in t}) for t in ltiles)
                if c2 < cur or rng.random() < np.exp((cur - c2) / T): cur = c2
                else: pi[a], pi[b] = pi[b], pi[a]
                T *= 0.999
            cands.append(pi)
        for pi in cands:
            for t in tiles_of(relabeled(c, n, pi)):
                if max(t) < 30 and t not in seen:
                    seen.add(t)
print(";".join(",".join(map(str, t)) for t in sorted(seen)))
print(len(seen), file=sys.stderr)
