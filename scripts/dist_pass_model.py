"""Host-only model of the sharded engine's local work: fused passes per step for W-HC at n
qubits on `world` ranks, over consecutive runs (each run starts from the map the last one ended
with, as a benchmark loop does).  No GPU: the planner is host code (qsim_dist_plan_passes)."""
import ctypes, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "cuda-quantum-simulator_amd"))
import qsim_amd as q
from qsim_amd import _lib

n = int(os.environ.get("QUBITS", 30)); world = int(os.environ.get("WORLD", 8))
runs = int(os.environ.get("RUNS", 4)); seed = int(os.environ.get("SEED", 42))
c = q.createRandomHCCircuit(n, 100, seed)
arr, cnt = c.to_abi()
perm = (ctypes.c_int32 * n)(*range(n))
tot = 0
rows = []
for r in range(runs):
    passes = (ctypes.c_int32 * (3 * 64))()
    ns = ctypes.c_size_t(0)
    _lib.check(_lib.hip.qsim_dist_plan_passes(n, world, 0, arr, cnt, perm, passes, 64, ctypes.byref(ns)))
    steps = [tuple(passes[3 * i:3 * i + 3]) for i in range(ns.value)]
    p = sum(x[0] for x in steps if x[0] > 0)
    tot += p
    rows.append(steps)
    print(f"run {r}: steps (passes, head, tail) {steps} passes {p}")
print("mean passes per run", tot / runs)

# exchange sizes: k globals swapped per remap -> fraction (1 - 2^-k) of the shard leaves each rank
perm = (ctypes.c_int32 * n)(*range(n))
vol = 0.0
for r in range(runs):
    steps = (_lib.qsim_dist_step * 64)()
    ns, no = ctypes.c_size_t(0), ctypes.c_size_t(0)
    _lib.check(_lib.hip.qsim_dist_plan(n, world, 0, arr, cnt, perm, steps, 64, ctypes.byref(ns), None, 0,
                                       ctypes.byref(no)))
    ks = [steps[i].k for i in range(ns.value) if steps[i].kind == 1]
    vol += sum(1 - 2.0 ** -k for k in ks)
    print(f"run {r}: remap k {ks} pivots {[steps[i].pivot for i in range(ns.value) if steps[i].kind == 1]}")
print("mean shard fraction sent per run", vol / runs)

# The time model of DESIGN §5 per run (one remap between ops steps A and B):
#   T = max(T_x + (nA - t + nB - h) * P + (t + h) * P / K,  (nA + nB) * P + T_x / K)
# P: one local pass over the 2 GiB shard (32 B x 2^27 at 6.4 TB/s), K = 2^(pivots).
P = float(os.environ.get("PASS_MS", 32 * 2 ** (n - 3) / 6.4e12 * 1e3))
perm = (ctypes.c_int32 * n)(*range(n))
for r in range(runs):
    steps = (_lib.qsim_dist_step * 64)()
    ns, no = ctypes.c_size_t(0), ctypes.c_size_t(0)
    _lib.check(_lib.hip.qsim_dist_plan(n, world, 0, arr, cnt, perm, steps, 64, ctypes.byref(ns), None, 0,
                                       ctypes.byref(no)))
    ps = rows[r]
    for i in range(ns.value):
        if steps[i].kind != 1 or i == 0 or i + 1 >= ns.value:
            continue
        K = 2 ** bin(steps[i].pmask).count("1")
        nA, _, t = ps[i - 1]
        nB, h, _ = ps[i + 1]
        for tx in (4.4, 3.5):
            T = max(tx + (nA - t + nB - h) * P + (t + h) * P / K, (nA + nB) * P + tx / K)
            print(f"run {r}: nA {nA} t {t} nB {nB} h {h} K {K}: T_x {tx} ms -> {T:.2f} ms per run "
                  f"(pass {P:.3f} ms; pack/unpack not counted)")
