"""PARITY ORACLE (test infrastructure only) — independent numpy formulation + ctypes access to the
C++ CPUSimulator restatement (cpu_simulator.hpp).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker / timed CPU baseline.  The product never imports it.

Two implementations, written differently on purpose:
  * `run_numpy`: each gate is a small unitary contracted into the state viewed as a rank-n tensor
    (np.tensordot over the gate's axes).  Gate matrices come from their textbook definitions
    (Nielsen & Chuang ch.4); qubit q is index bit q (reference SURVEY F1), i.e. tensor axis n-1-q.
    CRY/CRZ/Toffoli follow the reference GPU kernels src/Gates.cu:322-410.
  * `run_cpu`: the C++ restatement of the reference CPUSimulator (src/Simulator.cu:191-345),
    loaded from oracle/build/libqsim_oracle.so.
The two are cross-checked in tests/test_oracle.py and both against the reference's known-answer
vectors in tests/golden/.
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import Iterable, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_LIB = os.path.join(HERE, "build", "libqsim_oracle.so")

INV_SQRT2 = 0.70710678118654752440

# (type, qubits, parameter) tuples; type numbering == reference GateType.
Gate = Tuple[int, Sequence[int], float]


def _mat1(t: int, th: float) -> np.ndarray:
    c, s = np.cos(th / 2.0), np.sin(th / 2.0)
    r = INV_SQRT2
    return {
        0: np.array([[0, 1], [1, 0]], complex),
        1: np.array([[0, -1j], [1j, 0]], complex),
        2: np.array([[1, 0], [0, -1]], complex),
        3: np.array([[r, r], [r, -r]], complex),
        4: np.array([[1, 0], [0, 1j]], complex),
        5: np.array([[1, 0], [0, r + 1j * r]], complex),
        6: np.array([[1, 0], [0, -1j]], complex),
        7: np.array([[1, 0], [0, r - 1j * r]], complex),
        8: np.array([[c, -1j * s], [-1j * s, c]], complex),
        9: np.array([[c, -s], [s, c]], complex),
        10: np.array([[c - 1j * s, 0], [0, c + 1j * s]], complex),
    }[t]


def _controlled(u: np.ndarray, ncontrols: int) -> np.ndarray:
    """Matrix on (controls..., target) with controls as the most significant tensor axes."""
    d = 2 ** (ncontrols + 1)
    m = np.eye(d, dtype=complex)
    m[d - 2:, d - 2:] = u
    return m


def gate_matrix(t: int, qubits: Sequence[int], th: float):
    """Return (matrix, qubit order) where the matrix acts on tensor axes in that order
    (first listed qubit = most significant axis of the small matrix)."""
    if t <= 10:
        return _mat1(t, th), [qubits[0]]
    if t == 11:  # CNOT(control, target)
        return _controlled(_mat1(0, 0.0), 1), [qubits[0], qubits[1]]
    if t == 12:  # CZ
        return _controlled(_mat1(2, 0.0), 1), [qubits[0], qubits[1]]
    if t == 13:  # CRY
        return _controlled(_mat1(9, th), 1), [qubits[0], qubits[1]]
    if t == 14:  # CRZ
        return _controlled(_mat1(10, th), 1), [qubits[0], qubits[1]]
    if t == 15:  # SWAP
        m = np.eye(4, dtype=complex)[[0, 2, 1, 3]]
        return m, [qubits[0], qubits[1]]
    if t == 16:  # Toffoli(c1, c2, target)
        return _controlled(_mat1(0, 0.0), 2), [qubits[0], qubits[1], qubits[2]]
    raise ValueError(f"unknown gate type {t}")


def apply_numpy(state: np.ndarray, n: int, gate: Gate) -> np.ndarray:
    t, qubits, th = gate
    m, order = gate_matrix(t, list(qubits), th)
    k = len(order)
    psi = state.reshape((2,) * n)
    axes = [n - 1 - q for q in order]
    mt = m.reshape((2,) * (2 * k))
    out = np.tensordot(mt, psi, axes=(list(range(k, 2 * k)), axes))
    # tensordot puts the gate's output axes first; move them back to their positions
    out = np.moveaxis(out, list(range(k)), axes)
    return out.reshape(-1)


def zero_state(n: int) -> np.ndarray:
    s = np.zeros(1 << n, complex)
    s[0] = 1.0
    return s


def run_numpy(n: int, gates: Iterable[Gate], state: np.ndarray | None = None) -> np.ndarray:
    s = zero_state(n) if state is None else np.array(state, dtype=complex)
    for g in gates:
        s = apply_numpy(s, n, g)
    return s


def gates_of(circuit) -> list:
    """(type, qubits, parameter) tuples from a qsim_amd.Circuit (or any getGates() provider)."""
    return [(int(g.type), list(g.qubits), float(g.parameter)) for g in circuit.getGates()]


# ---- C++ restatement of CPUSimulator -----------------------------------------------------
class _Gate(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("nqubits", ctypes.c_int32),
                ("qubits", ctypes.c_int32 * 3), ("_pad", ctypes.c_int32),
                ("parameter", ctypes.c_double)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_LIB):
            raise RuntimeError(f"oracle library missing: {ORACLE_LIB} (run make -C oracle)")
        _lib = ctypes.CDLL(ORACLE_LIB)
        _lib.qsim_oracle_run.argtypes = [ctypes.c_int, ctypes.POINTER(_Gate), ctypes.c_size_t,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        _lib.qsim_oracle_sample.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_int, ctypes.c_void_p]
        _lib.qsim_oracle_time_prefix.argtypes = [ctypes.c_int, ctypes.POINTER(_Gate),
                                                 ctypes.c_size_t, ctypes.c_double,
                                                 ctypes.POINTER(ctypes.c_size_t),
                                                 ctypes.POINTER(ctypes.c_double)]
        _lib.qsim_oracle_run_mt.argtypes = [ctypes.c_int, ctypes.POINTER(_Gate), ctypes.c_size_t,
                                            ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    return _lib


def _to_abi(gates: Sequence[Gate]):
    arr = (_Gate * max(1, len(gates)))()
    for i, (t, qs, th) in enumerate(gates):
        arr[i].type = int(t)
        arr[i].nqubits = len(qs)
        for j, q in enumerate(qs):
            arr[i].qubits[j] = int(q)
        arr[i].parameter = float(th)
    return arr


def run_cpu(n: int, gates: Sequence[Gate], state: np.ndarray | None = None,
            strict_cpu: bool = False) -> np.ndarray:
    """C++ CPUSimulator restatement. strict_cpu=True keeps the reference's CRY/CRZ/CCX no-ops (F4)."""
    gates = list(gates)
    out = np.zeros(1 << n, complex) if state is None else np.array(state, dtype=complex)
    rc = lib().qsim_oracle_run(n, _to_abi(gates), len(gates), 1 if strict_cpu else 0,
                               0 if state is None else 1, out.ctypes.data_as(ctypes.c_void_p))
    if rc != 0:
        raise ValueError("oracle rejected input")
    return out


def run_cpu_mt(n: int, gates: Sequence[Gate], state: np.ndarray | None = None, threads: int = 16,
               strict_cpu: bool = False) -> np.ndarray:
    """run_cpu with each gate's loop split over `threads` threads: bit-identical to run_cpu (the
    same operations per amplitude, disjoint pair ranges); for the 26-30 qubit parity tests."""
    gates = list(gates)
    out = np.zeros(1 << n, complex) if state is None else np.array(state, dtype=complex)
    rc = lib().qsim_oracle_run_mt(n, _to_abi(gates), len(gates), 1 if strict_cpu else 0,
                                  0 if state is None else 1, out.ctypes.data_as(ctypes.c_void_p), int(threads))
    if rc != 0:
        raise ValueError("oracle rejected input")
    return out


def sample_cpu(n: int, state: np.ndarray, uniforms: np.ndarray) -> np.ndarray:
    st = np.ascontiguousarray(state, dtype=complex)
    u = np.ascontiguousarray(uniforms, dtype=np.float64)
    out = np.empty(u.size, dtype=np.int64)
    lib().qsim_oracle_sample(n, st.ctypes.data_as(ctypes.c_void_p),
                             u.ctypes.data_as(ctypes.c_void_p), int(u.size),
                             out.ctypes.data_as(ctypes.c_void_p))
    return out


def time_prefix(n: int, gates: Sequence[Gate], budget_s: float):
    """Single-threaded CPU baseline: gates of `gates` applied in order until budget_s elapses."""
    gates = list(gates)
    done = ctypes.c_size_t(0)
    secs = ctypes.c_double(0.0)
    lib().qsim_oracle_time_prefix(n, _to_abi(gates), len(gates), budget_s, ctypes.byref(done),
                                  ctypes.byref(secs))
    return done.value, secs.value


# ---- NoisySimulator per-pair noise (test infrastructure) ---------------------------------
# Restates the reference kernels src/NoiseModel.cu:115-314 (per-pair draws, per-pair damping
# renormalisation) driven by the engine's documented counter hash (csrc/hip/noise.hip), so the
# GPU pass can be checked exactly; the reference's cuRAND stream itself is parity-unpinned.
_M64 = (1 << 64) - 1


def _mix(z):
    z = (z + 0x9e3779b97f4a7c15) & _M64
    z = ((z ^ (z >> 30)) * 0xbf58476d1ce4e5b9) & _M64
    z = ((z ^ (z >> 27)) * 0x94d049bb133111eb) & _M64
    return z ^ (z >> 31)


def _mix_np(z):
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9e3779b97f4a7c15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
        return z ^ (z >> np.uint64(31))


def noise_key(seed, counter):
    return _mix(_mix(seed & _M64) ^ ((counter * 0x9e3779b97f4a7c15 + 0x632be59bd9b4e019) & _M64))


def _uniform(h):
    return ((h >> np.uint64(40)).astype(np.uint32).astype(np.float32) + np.float32(1.0)) * \
        np.float32(1.0 / 16777216.0)


# Flip channels (X / Z / Y / depolarizing) draw their flips per block of 256 global pair
# indices with geometric gaps (csrc/hip/noise.hip k_noise_flips): every pair still flips
# independently with P = P(float uniform in (0, 1] < p), the reference's per-pair law
# (src/NoiseModel.cu:195, :857-861), but the engine does work per flip rather than per pair.
_FLIP_BLOCK_LOG = 8
_BLOCK_SALT = 0xb10c5a17b10c5a17


def flip_probability(p):
    """P(curand_uniform < p) for curand_uniform = (k + 1) / 2^24, k uniform in [0, 2^24)."""
    if not p > 0.0:
        return 0.0
    c = math.ceil(p * 16777216.0) - 1.0
    return min(16777216.0, max(0.0, c)) / 16777216.0


def flip_events(key, idx0, pairs, p, depolarizing):
    """(global pair indices, Pauli codes 1 X / 2 Y / 3 Z or None) of one flip pass over the
    global pairs [idx0, idx0 + pairs), in the engine's draw order."""
    P = flip_probability(p)
    if P <= 0.0 or pairs == 0:
        return np.zeros(0, np.uint64), np.zeros(0, np.int64)
    always = P >= 1.0
    lq = -1.0 if always else math.log1p(-P)
    B = 1 << _FLIP_BLOCK_LOG
    blocks = np.arange(idx0 >> _FLIP_BLOCK_LOG, ((idx0 + pairs - 1) >> _FLIP_BLOCK_LOG) + 1,
                       dtype=np.uint64)
    stream = _mix_np(np.uint64(key) ^ _mix_np(blocks ^ np.uint64(_BLOCK_SALT)))
    pos = np.full(blocks.size, -1, np.int64)
    live = np.ones(blocks.size, bool)
    out_g, out_h = [], []
    k = 0
    with np.errstate(over="ignore", divide="ignore"):
        while live.any():
            h = _mix_np(stream + np.uint64(k) * np.uint64(0x9e3779b97f4a7c15))
            if always:
                step = np.ones(blocks.size, np.int64)
            else:
                u = ((h >> np.uint64(11)) + np.uint64(1)).astype(np.float64) * 2.0 ** -53
                gap = np.floor(np.log(u) / lq)
                live &= gap < B
                step = np.where(live, np.minimum(gap, B), 0).astype(np.int64) + 1
            pos = np.where(live, pos + step, pos)
            live &= pos < B
            g = (blocks << np.uint64(_FLIP_BLOCK_LOG)) + pos.astype(np.uint64)
            keep = live & (g >= np.uint64(idx0)) & (g < np.uint64(idx0 + pairs))
            out_g.append(g[keep])
            out_h.append(h[keep])
            k += 1
    g = np.concatenate(out_g)
    h = np.concatenate(out_h)
    if not depolarizing:
        return g, None
    r2 = _uniform(_mix_np(h ^ np.uint64(0x5bd1e9955bd1e995)))
    pauli = np.where(r2 < np.float32(1.0) / np.float32(3.0), 1,
                     np.where(r2 < np.float32(2.0) / np.float32(3.0), 2, 3))
    return g, pauli


def noise_pass(state, n, ntype, q, p, seed, counter):
    """One reference noise kernel (type numbering == NoiseType) on `state` (modified copy)."""
    s = np.array(state, dtype=complex)
    idx = np.arange(1 << (n - 1), dtype=np.uint64)
    h = _mix_np(np.uint64(noise_key(seed, counter)) ^ _mix_np(idx))
    r1 = _uniform(h)
    mask = np.uint64((1 << q) - 1)
    i0 = ((idx & mask) | ((idx & ~mask) << np.uint64(1))).astype(np.int64)
    i1 = i0 | (1 << q)
    a0, a1 = s[i0].copy(), s[i1].copy()
    if ntype in (0, 3, 4, 5):
        # each pair flips with P(float draw < p), the draw promoted to double (NoiseModel.cu:195)
        g, dp = flip_events(noise_key(seed, counter), 0, 1 << (n - 1), p, ntype == 0)
        fire = np.zeros(idx.size, bool)
        fire[g.astype(np.int64)] = True
        pauli = np.full(idx.size, {0: 0, 3: 1, 4: 3, 5: 2}[ntype])
        if ntype == 0:
            pauli[g.astype(np.int64)] = dp
        x, y, z = fire & (pauli == 1), fire & (pauli == 2), fire & (pauli == 3)
        s[i0[x]], s[i1[x]] = a1[x], a0[x]
        s[i0[y]], s[i1[y]] = -1j * a1[y], 1j * a0[y]
        s[i1[z]] = -a1[z]
        return s
    g = p
    p1 = np.abs(a1) ** 2
    n0 = np.abs(a0) ** 2
    if ntype == 1:
        dec = r1 < p1 * g
        nd = np.sqrt(n0 + g * p1)
        nk = np.sqrt(n0 + (1.0 - g) * p1)
        ok_d, ok_k = dec & (nd > 1e-15), ~dec & (nk > 1e-15)
        s[i0[ok_d]] = (a0[ok_d] + np.sqrt(g) * a1[ok_d]) / nd[ok_d]
        s[i1[ok_d]] = 0
        s[i0[ok_k]] = a0[ok_k] / nk[ok_k]
        s[i1[ok_k]] = np.sqrt(1.0 - g) * a1[ok_k] / nk[ok_k]
        return s
    k1 = r1 < g * p1
    s[i0[k1]] = 0
    pos = k1 & (p1 > 1e-15)
    s[i1[pos]] = a1[pos] / np.sqrt(p1[pos])
    ns = n0 + (1.0 - g) * p1
    ok = ~k1 & (ns > 1e-15)
    s[i0[ok]] = a0[ok] / np.sqrt(ns[ok])
    s[i1[ok]] = np.sqrt(1.0 - g) * a1[ok] / np.sqrt(ns[ok])
    return s


def noisy_run(n, gates, channels, seed, counter=0, state=None):
    """NoisySimulator::run (src/NoiseModel.cu:369-382): gate, then every (type, qubit, p) entry."""
    s = zero_state(n) if state is None else np.array(state, dtype=complex)
    for g in gates:
        s = apply_numpy(s, n, g)
        for (t, q, p) in channels:
            s = noise_pass(s, n, t, q, p, seed, counter)
            counter += 1
    return s, counter


# ---- DensityMatrixSimulator (test infrastructure) ----------------------------------------
# rho' = U rho U^dag with textbook matrices, channels per the reference kernels
# src/DensityMatrix.cu:978-1122 (depolarizing: off-diagonal x (1 - 4p/3) only; bit-phase flip =
# phase flip, :343-356; amplitude damping with the pre-channel rho11).
# ---- BatchedSimulator, reference noise process (test infrastructure) ---------------------
# Restates run() + applyBatchedNoise() + applyBatchedDepolarizingKernel
# (src/NoiseModel.cu:815-892): after EVERY circuit gate (also gates the reference gate set
# skips), one pass per Depolarizing channel entry in order; pass idx covers all B x 2^(n-1)
# pairs (traj = idx / n_pairs, pair = idx % n_pairs, :843-856); a pair fires when its float
# uniform < p (promoted to double), then a second float uniform picks X (< 1/3f), Y (< 2/3f),
# else Z, applied to that pair of that trajectory only.  Draws: the engine's documented counter
# hash keyed by (seed, pass counter, idx) in place of curandState[idx] (parity unpinned vs cuRAND).
_REF_BATCH_GATES = {0, 1, 2, 3, 11}  # src/NoiseModel.cu:742-763 (X/Y/Z/H), :808-812 (CNOT)


def batched_depolarizing_pass(states, n, q, p, seed, counter):
    """states: (B, 2^n) complex, modified copy returned."""
    s = np.array(states, dtype=complex)
    B = s.shape[0]
    npairs = 1 << (n - 1)
    idx = np.arange(B * npairs, dtype=np.uint64)
    g, dp = flip_events(noise_key(seed, counter), 0, B * npairs, p, True)
    fire = np.zeros(idx.size, bool)
    fire[g.astype(np.int64)] = True
    pauli = np.zeros(idx.size, np.int64)
    pauli[g.astype(np.int64)] = dp
    traj = (idx // np.uint64(npairs)).astype(np.int64)
    pr = (idx % np.uint64(npairs)).astype(np.int64)
    mask = (1 << q) - 1
    i0 = (pr & mask) | ((pr & ~mask) << 1)
    i1 = i0 | (1 << q)
    flat = s.reshape(-1)
    o0, o1 = traj * (1 << n) + i0, traj * (1 << n) + i1
    a0, a1 = flat[o0].copy(), flat[o1].copy()
    x, y, z = fire & (pauli == 1), fire & (pauli == 2), fire & (pauli == 3)
    flat[o0[x]], flat[o1[x]] = a1[x], a0[x]
    flat[o0[y]], flat[o1[y]] = -1j * a1[y], 1j * a0[y]
    flat[o1[z]] = -a1[z]
    return s


def batched_reference_run(n, B, gates, channels, seed, reference_gateset=False, states=None,
                          counter=0):
    """channels: (type, qubit, p) entries in order; returns (states (B, 2^n), next counter)."""
    st = np.zeros((B, 1 << n), complex) if states is None else np.array(states, dtype=complex)
    if states is None:
        st[:, 0] = 1.0
    dep = [(q, p) for (t, q, p) in channels if t == 0]
    for g in gates:
        if not reference_gateset or g[0] in _REF_BATCH_GATES:
            for b in range(B):
                st[b] = run_cpu(n, [g], st[b])
        for q, p in dep:
            st = batched_depolarizing_pass(st, n, q, p, seed, counter)
            counter += 1
    return st, counter


def dm_apply_gate(rho, n, gate):
    t, qubits, th = gate
    if t in (13, 14, 16):
        raise RuntimeError("Gate not supported in density matrix simulation")
    d = 1 << n
    cols = np.stack([apply_numpy(rho[:, j], n, gate) for j in range(d)], axis=1)  # U rho
    return np.stack([apply_numpy(cols[i, :].conj(), n, gate).conj() for i in range(d)], axis=0)


def dm_channel(rho, n, ntype, q, p):
    d = 1 << n
    r = (np.arange(d) >> q) & 1
    R, C = np.meshgrid(r, r, indexing="ij")
    off = R != C
    out = rho.copy()
    flip = np.arange(d) ^ (1 << q)
    if ntype == 0:
        out[off] *= 1.0 - 4.0 * p / 3.0
    elif ntype == 1:
        partner = rho[np.ix_(flip, flip)]
        d00 = (R == 0) & (C == 0)
        out[d00] = rho[d00] + p * partner[d00]
        out[(R == 1) & (C == 1)] *= 1.0 - p
        out[off] *= np.sqrt(1.0 - p)
    elif ntype == 2:
        out[off] *= np.sqrt(1.0 - p)
    elif ntype == 3:
        out = (1.0 - p) * rho + p * rho[np.ix_(flip, flip)]
    else:
        out[off] *= 1.0 - 2.0 * p
    return out


def dm_run(n, gates, channels=(), rho=None, reference_y=False):
    """DensityMatrixSimulator::run (src/DensityMatrix.cu:201-212); channel qubit -1 = global.
    reference_y: Y as dmApplyY computes it, -Y rho Y^dag (src/DensityMatrix.cu:540-544: the
    element (r, c) <- phase2 * rho[r^1][c^1] with phase2 = +-1 opposite to Y rho Y^dag's)."""
    d = 1 << n
    if rho is None:
        rho = np.zeros((d, d), complex)
        rho[0, 0] = 1.0
    for g in gates:
        rho = dm_apply_gate(rho, n, g)
        if reference_y and g[0] == 1:
            rho = -rho
        for q in g[1]:
            for (t, cq, p) in channels:
                if cq < 0 or cq == q:
                    rho = dm_channel(rho, n, t, q, p)
    return rho
