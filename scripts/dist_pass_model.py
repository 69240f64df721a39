"""Host-only model of the sharded engine's local work and run time: fused passes per step for
W-HC at n qubits on `world` ranks over consecutive runs (each run starts from the map the last
one ended with, and from the remap it left in flight, as a benchmark loop does).  No GPU: the
planner is host code (qsim_dist_plan_passes_carry, qsim_dist_plan).

Time model per run: one remap X per run between ops steps A and B, K = 2^pivots
parts; the cycle from X_{i-1}'s first part leaving to X_i's first part leaving is
    T_i = max(T_x + (h_{i-1} + hA_i) * P / K_{i-1} + (nA_i - hA_i - t_i - c_i) * PW + c_i * P / Kc_i
                   + t_i * P / K_i + (nB_{i-1} - h_{i-1}) * PW,
              (whole passes) * PW + (per-part passes) * P + T_x / K_i)
t: A's trailing passes that avoid X's pivots (run per part, feeding the transfer), h: B's leading
passes that avoid them (run per part as each part lands), hA: A's leading passes that avoid the
pivots of the PREVIOUS run's remap (run per part, interleaved with that run's carried B, after its
last part landed), c: A's passes just ahead of t that run per COARSE part (Kc = 2^coarse bits: the
pivots they leave untouched; round 5), P: one local pass over the shard, 32 B x 2^L at the rate
PASS_TBPS (default 5.15 TB/s: what the per-part sub-space launches of the virtual 30q / 8 run
streamed at, profiles/r04/dist_virtual/, rather than the 6.4 TB/s of whole-shard passes).  The remap's pack /
unpack run inside the passes (fused remap), so they add no HBM time.  Without a carry (hA = 0) and
with h = nB this is the round-3 formula max(T_x + (nA - t) P + (t + h) P / K, (nA + nB) P + T_x / K).
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "cuda-quantum-simulator_amd"))
import qsim_amd as q  # noqa: E402
from qsim_amd import _lib  # noqa: E402

n = int(os.environ.get("QUBITS", 30))
world = int(os.environ.get("WORLD", 8))
runs = int(os.environ.get("RUNS", 8))
seed = int(os.environ.get("SEED", 42))
carry_on = os.environ.get("QSIM_DIST_CARRY", "0") != "0"  # (the engine's default: off)
L = n - (world.bit_length() - 1)
# per-part (sub-space) launches at the measured 5.15 TB/s, whole-shard passes at 6.4 TB/s
P = float(os.environ.get("PASS_MS", 32 * 2 ** L / (float(os.environ.get("PASS_TBPS", "5.15")) * 1e12) * 1e3))
PW = float(os.environ.get("PASS_WHOLE_MS", 32 * 2 ** L / (float(os.environ.get("PASS_WHOLE_TBPS", "6.4")) * 1e12) * 1e3))
ONE_GPU_MS = float(os.environ.get("ONE_GPU_MS", "21.408"))  # BENCH_r04.json ms_per_step (W-HC 30q, 1 GPU)
c = q.createRandomHCCircuit(n, 100, seed)
arr, cnt = c.to_abi()
perm = (ctypes.c_int32 * n)(*range(n))
carry = ctypes.c_uint64(0)
tot, Ts = 0, []
prev = None  # (K, nB, h) of the previous run's remap
for r in range(runs):
    perm_in = list(perm)
    carry_in = carry.value if carry_on else 0
    carry.value = carry_in
    passes = (ctypes.c_int32 * (5 * 64))()
    ns = ctypes.c_size_t(0)
    _lib.check(_lib.hip.qsim_dist_plan_passes_coarse(n, world, 0, arr, cnt, perm, ctypes.byref(carry), passes, 64,
                                                     ctypes.byref(ns)))
    steps5 = [tuple(passes[5 * i:5 * i + 5]) for i in range(ns.value)]
    steps = [x[:3] for x in steps5]
    p = sum(x[0] for x in steps if x[0] > 0)
    tot += p
    # the exchange skeleton (pivots) of the same run
    pp = (ctypes.c_int32 * n)(*perm_in)
    st = (_lib.qsim_dist_step * 64)()
    ns2, no = ctypes.c_size_t(0), ctypes.c_size_t(0)
    _lib.check(_lib.hip.qsim_dist_plan(n, world, 0, arr, cnt, pp, st, 64, ctypes.byref(ns2), None, 0,
                                       ctypes.byref(no)))
    ks = [st[i].k for i in range(ns2.value) if st[i].kind == 1]
    line = f"run {r}: steps (passes, head, tail) {steps} passes {p} carry_in {carry_in:#x} remap k {ks}"
    xs = [i for i in range(1, len(steps) - 1) if steps[i][0] == -1]
    if len(xs) == 1:
        i = xs[0]
        K = 2 ** bin(st[i].pmask).count("1")
        nA, hA, t = steps[i - 1]
        c, cbits = steps5[i - 1][3], steps5[i - 1][4]
        Kc = 2 ** cbits
        nB, h, _ = steps[i + 1]
        if not carry_in:
            hA = 0  # (no earlier remap in flight before A)
        Kp, nBp, hp = prev if prev else (K, nB, h)
        for tx in (4.4, 3.5):
            T = max(tx + (hp + hA) * P / Kp + (nA - hA - t - c) * PW + c * P / Kc + t * P / K + (nBp - hp) * PW,
                    (nA - hA - t - c + nBp - hp) * PW + (hA + t + c + hp) * P + tx / K)
            if tx == 4.4:
                Ts.append(T)
            line += (f"\n    nA {nA} hA {hA} t {t} c {c} (Kc {Kc}) | nB {nB} h {h} | K {K} (previous K {Kp}): "
                     f"T_x {tx} ms -> {T:.2f} ms per run")
        prev = (K, nB, h)
    print(line)
print(f"mean passes per run {tot / runs:.2f}; pass {PW:.3f} ms whole shard, {P:.3f} ms per shard in parts")
if Ts:
    steady = Ts[len(Ts) // 2:]
    Tm = sum(steady) / len(steady)
    print(f"steady-state model at T_x = 4.4 ms: {Tm:.2f} ms per run = {ONE_GPU_MS / Tm:.2f}x the 1-GPU "
          f"{ONE_GPU_MS} ms")
