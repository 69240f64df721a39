"""general matrix APIs beyond the reference's 2x2 applyGate1Q_opt
(include/OptimizedGates.cuh:91-93) and the diagonal layer applyFusedSingleQubitLayer
(src/OptimizedGates.cu:344-382), checked against dense numpy application on random states
(re/im ~ normal(0,1), normalised, like tests/test_optimized_gates.cu:45-61)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rand_state(n, seed):
    rng = np.random.default_rng(seed)
    s = rng.normal(size=1 << n) + 1j * rng.normal(size=1 << n)
    return s / np.linalg.norm(s)


def _apply2(state, n, m, q0, q1, controls=()):
    out = state.copy()
    idx = np.arange(1 << n)
    base = idx[((idx >> q0) & 1 == 0) & ((idx >> q1) & 1 == 0)]
    for c in controls:
        base = base[(base >> c) & 1 == 1]
    grp = [base, base | (1 << q0), base | (1 << q1), base | (1 << q0) | (1 << q1)]
    v = np.stack([state[g] for g in grp])
    w = m @ v
    for k in range(4):
        out[grp[k]] = w[k]
    return out


@pytest.mark.parametrize("n,q0,q1,controls", [(2, 0, 1, ()), (5, 3, 1, ()), (10, 7, 2, (0,)),
                                              (12, 0, 11, (5, 9)), (14, 13, 6, ())])
def test_matrix2q_matches_numpy(qsim, gpu_ready, n, q0, q1, controls):
    rng = np.random.default_rng(n + q0)
    m = rng.normal(size=(4, 4)) + 1j * rng.normal(size=(4, 4))  # any matrix (not only unitary)
    s0 = _rand_state(n, n)
    sv = qsim.StateVector(n)
    sv.fromHost(s0)
    sv.applyMatrix2Q(q0, q1, m, controls)
    np.testing.assert_allclose(sv.toHost(), _apply2(s0, n, m, q0, q1, controls), atol=1e-12, rtol=0)


def test_matrix2q_cnot_and_errors(qsim, oracle, gpu_ready):
    n = 6
    s0 = _rand_state(n, 1)
    cnot = np.eye(4)[[0, 3, 2, 1]]  # control q0, target q1 in the (b1 b0) basis
    sv = qsim.StateVector(n)
    sv.fromHost(s0)
    sv.applyMatrix2Q(2, 4, cnot)
    np.testing.assert_allclose(sv.toHost(), oracle.run_numpy(n, [(11, [2, 4], 0.0)], s0), atol=1e-12)
    with pytest.raises(IndexError):
        sv.applyMatrix2Q(0, n, cnot)
    with pytest.raises(ValueError):
        sv.applyMatrix2Q(1, 1, cnot)
    with pytest.raises(ValueError):
        sv.applyMatrix2Q(0, 1, cnot, [1])


@pytest.mark.parametrize("n", [3, 12, 22])
def test_diagonal_layer_matches_numpy(qsim, gpu_ready, n):
    rng = np.random.default_rng(n)
    params = rng.normal(size=(n, 4)) + 1j * rng.normal(size=(n, 4))
    active = int(rng.integers(1, 1 << n))
    s0 = _rand_state(n, n + 1)
    sv = qsim.StateVector(n)
    sv.fromHost(s0)
    sv.applyDiagonalLayer(params, active)
    idx = np.arange(1 << n)
    want = s0.copy()
    for q in range(n):
        if (active >> q) & 1:
            want = want * np.where((idx >> q) & 1, params[q, 3], params[q, 0])
    np.testing.assert_allclose(sv.toHost(), want, atol=1e-12 * np.max(np.abs(want)) * 10, rtol=1e-12)


def _numpy_controlled_1q(state, n, target, m, controls):
    out = state.copy()
    idx = np.arange(1 << n)
    sel = np.ones(1 << n, bool)
    for c in controls:
        sel &= ((idx >> c) & 1) == 1
    i0 = idx[sel & (((idx >> target) & 1) == 0)]
    i1 = i0 | (1 << target)
    a0, a1 = state[i0], state[i1]
    out[i0] = m[0, 0] * a0 + m[0, 1] * a1
    out[i1] = m[1, 0] * a0 + m[1, 1] * a1
    return out


@pytest.mark.parametrize("target,controls", [(7, [6, 8, 9]), (2, [6, 7, 8, 9]), (9, [0, 6, 7, 8]),
                                             (11, [6, 7, 8, 9, 10]), (3, [0, 1, 6, 7, 8, 10, 11])])
def test_matrix1q_many_high_controls(qsim, gpu_ready, target, controls):
    """more fixed high positions than the wave-item kernels hold (3) -> general
    kernel; checked against numpy on a random state."""
    n = 12
    rng = np.random.default_rng(target * 31 + len(controls))
    psi = rng.normal(size=1 << n) + 1j * rng.normal(size=1 << n)
    psi /= np.linalg.norm(psi)
    a = rng.normal(size=(2, 2)) + 1j * rng.normal(size=(2, 2))
    u, _ = np.linalg.qr(a)
    sv = qsim.StateVector(n)
    sv.fromHost(psi)
    sv.applyMatrix1Q(target, u, controls)
    np.testing.assert_allclose(sv.toHost(), _numpy_controlled_1q(psi, n, target, u, controls),
                               atol=1e-12, rtol=0)


def _numpy_apply_k(state, n, targets, m, controls=()):
    """Dense reference: out[i] = sum_c M[r(i)][c] psi[i with target bits = c] on control == 1."""
    out = state.copy()
    k = len(targets)
    idx = np.arange(1 << n)
    sel = np.ones(1 << n, bool)
    for c in controls:
        sel &= ((idx >> c) & 1) == 1
    for t in targets:
        sel &= ((idx >> t) & 1) == 0
    base = idx[sel]
    cols = []
    for c in range(1 << k):
        off = 0
        for j, t in enumerate(targets):
            if (c >> j) & 1:
                off |= 1 << t
        cols.append(base | off)
    vec = np.stack([state[ci] for ci in cols])  # (2^k, groups)
    res = m @ vec
    for r, ci in enumerate(cols):
        out[ci] = res[r]
    return out


@pytest.mark.parametrize("targets,controls", [([3], []), ([0, 7], [2]), ([1, 5, 9], []),
                                              ([11, 2, 6], [0, 8]), ([0, 1, 2, 3], [10]),
                                              ([4, 9, 1, 7, 11], []), ([2, 3, 4, 5, 6, 7, 8, 9], [11])])
def test_matrix_k_qubits(qsim, gpu_ready, targets, controls):
    """General k-qubit matrix (qsim_apply_matrix, k <= 8) vs dense numpy on a random state."""
    n = 12
    rng = np.random.default_rng(len(targets) * 13 + len(controls))
    psi = _rand_state(n, 40 + len(targets))
    d = 1 << len(targets)
    a = rng.normal(size=(d, d)) + 1j * rng.normal(size=(d, d))
    u, _ = np.linalg.qr(a)
    sv = qsim.StateVector(n)
    sv.fromHost(psi)
    sv.applyMatrix(targets, u, controls)
    np.testing.assert_allclose(sv.toHost(), _numpy_apply_k(psi, n, targets, u, controls),
                               atol=1e-12, rtol=0)


def test_matrix_k_rejects_bad_input(qsim, gpu_ready):
    sv = qsim.StateVector(6)
    with pytest.raises(ValueError):
        sv.applyMatrix([1, 1], np.eye(4))
    with pytest.raises(IndexError):
        sv.applyMatrix([6], np.eye(2))
    with pytest.raises(ValueError):
        sv.applyMatrix([0, 1], np.eye(4), controls=[1])


def test_named_optimized_dispatchers(qsim, oracle, gpu_ready):
    """applyHadamardOptimized / applyCNOTOptimized / applyGate1Q_opt (src/OptimizedGates.cu:
    388-413) on a raw device pointer == the same gates through the simulator."""
    import ctypes
    from qsim_amd import _lib
    n = 10
    psi = _rand_state(n, 77)
    sv = qsim.StateVector(n)
    sv.fromHost(psi)
    ptr, stream = sv.devicePtr(), ctypes.c_void_p(sv.stream())
    _lib.check(_lib.hip.qsim_apply_hadamard_optimized(ptr, n, 3, stream))
    _lib.check(_lib.hip.qsim_apply_cnot_optimized(ptr, n, 3, 8, stream))
    ry = oracle.gate_matrix(9, [0], 0.7)[0]
    buf = (ctypes.c_double * 8)(*[v for z in ry.reshape(4) for v in (z.real, z.imag)])
    _lib.check(_lib.hip.qsim_apply_matrix1q_raw(ptr, n, 6, buf, stream))
    ref = oracle.run_cpu(n, [(3, [3], 0.0), (11, [3, 8], 0.0), (9, [6], 0.7)], state=psi)
    np.testing.assert_allclose(sv.toHost(), ref, atol=1e-12, rtol=0)
