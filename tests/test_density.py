"""DensityMatrix / DensityMatrixSimulator (reference include/DensityMatrix.cuh:63-224,
src/DensityMatrix.cu): rho as a 2n-index-bit state of the HIP engine (csrc/hip/density.hip).

CPU: the oracle's density-matrix restatement (oracle/numpy_oracle.py dm_run) reproduces the
reference's own expectations (tests/test_density_matrix.cu:83-366).
GPU: the engine equals the oracle at 1e-12 on random circuits with every channel type (fused and
per-gate), plus the reference suite, init/measure/validity and the error conventions.
"""
import numpy as np
import pytest

# (gates, channels, check) from tests/test_density_matrix.cu; channel qubit -1 = global form
REF_CASES = [
    ("XGate :93-103", 1, [(0, [0], 0)], [], lambda p, r: abs(p[1] - 1) < 1e-10),
    ("HGate :105-115", 1, [(3, [0], 0)], [], lambda p, r: abs(p[0] - .5) < 1e-10),
    ("HH :117-127", 1, [(3, [0], 0), (3, [0], 0)], [], lambda p, r: abs(p[0] - 1) < 1e-10),
    ("Bell :142-157", 2, [(3, [0], 0), (11, [0, 1], 0)], [],
     lambda p, r: abs(p[0] - .5) < 1e-10 and abs(p[3] - .5) < 1e-10 and abs(r - 1) < 1e-10),
    ("SWAP :159-172", 2, [(0, [0], 0), (15, [0, 1], 0)], [], lambda p, r: abs(p[2] - 1) < 1e-10),
    ("Depolarizing purity :190-204", 1, [(3, [0], 0)], [(0, -1, 0.1)], lambda p, r: 0 < r < 1),
    ("AmplitudeDamping :206-220", 1, [(0, [0], 0)], [(1, -1, 0.5)], lambda p, r: p[0] > 0),
    ("PhaseDamping :222-237", 1, [(3, [0], 0)], [(2, -1, 0.3)], lambda p, r: abs(p[0] - .5) < .1),
    ("BitFlip :251-265", 1, [(0, [0], 0)], [(3, -1, 0.5)], lambda p, r: abs(p[0] - .5) < .1),
    ("GHZ noisy :271-290", 3, [(3, [0], 0), (11, [0, 1], 0), (11, [1, 2], 0)], [(0, -1, 0.01)],
     lambda p, r: p[0] + p[7] > .8 and r < 1),
    ("Rx(pi) :320-331", 1, [(8, [0], np.pi)], [], lambda p, r: abs(p[1] - 1) < 1e-6),
    ("Ry(pi/2) :333-344", 1, [(9, [0], np.pi / 2)], [], lambda p, r: abs(p[0] - .5) < 1e-6),
]


@pytest.mark.parametrize("case", REF_CASES, ids=[c[0] for c in REF_CASES])
def test_oracle_pinned_by_reference_suite(oracle, case):
    _, n, gates, ch, check = case
    rho = oracle.dm_run(n, gates, ch)
    assert check(np.real(np.diag(rho)), float(np.sum(np.abs(rho) ** 2)))
    assert abs(np.trace(rho).real - 1.0) < 1e-10  # TracePreservedUnderNoise :306-318


def _circuit(q, n, depth, seed):
    rng = np.random.default_rng(seed)
    c = q.Circuit(n)
    for _ in range(depth):
        k = int(rng.integers(0, 14))
        a, b = (int(x) for x in rng.choice(n, 2, replace=False)) if n > 1 else (0, 0)
        th = float(rng.uniform(-3, 3))
        if k < 8:
            getattr(c, ("x", "y", "z", "h", "s", "t", "sdag", "tdag")[k])(a)
        elif k < 11:
            getattr(c, ("rx", "ry", "rz")[k - 8])(a, th)
        elif n > 1:
            (c.cnot, c.cz, c.swap)[k - 11](a, b)
    return c


def _noise(q, channels):
    nm = q.NoiseModel()
    adders = [nm.addDepolarizing, nm.addAmplitudeDamping, nm.addPhaseDamping, nm.addBitFlip,
              nm.addPhaseFlip, nm.addBitPhaseFlip]
    for t, qb, p in channels:
        adders[t](p) if qb < 0 else adders[t]([qb], p)
    return nm


@pytest.mark.gpu
@pytest.mark.parametrize("n,seed", [(1, 1), (3, 2), (5, 3), (7, 4)])
def test_engine_matches_oracle(qsim, oracle, gpu_ready, n, seed):
    c = _circuit(qsim, n, 25, seed)
    channels = [(0, -1, 0.05), (1, 0, 0.2), (2, n - 1, 0.3), (3, -1, 0.1), (4, n // 2, 0.15),
                (5, 0, 0.05)]
    want = oracle.dm_run(n, oracle.gates_of(c), channels)
    for mode in (qsim.RunMode.Fused, qsim.RunMode.PerGate):
        sim = qsim.DensityMatrixSimulator(n, _noise(qsim, channels), mode=mode)
        sim.run(c)
        np.testing.assert_allclose(sim.getDensityMatrix(), want, atol=1e-12, rtol=0)
        assert abs(sim.getTrace() - np.trace(want).real) < 1e-12
        assert abs(sim.getPurity() - np.sum(np.abs(want) ** 2)) < 1e-12


@pytest.mark.gpu
def test_large_fused_equals_per_gate(qsim, gpu_ready):
    """n = 11: a 22-bit state, so the fused passes, beam planner and specialised kernels run."""
    n = 11
    c = _circuit(qsim, n, 60, 9)
    nm = _noise(qsim, [(0, -1, 0.02), (1, 3, 0.1), (3, 7, 0.05)])
    a = qsim.DensityMatrixSimulator(n, nm, mode=qsim.RunMode.Fused)
    b = qsim.DensityMatrixSimulator(n, nm, mode=qsim.RunMode.PerGate)
    a.run(c)
    b.run(c)
    np.testing.assert_allclose(a.getProbabilities(), b.getProbabilities(), atol=1e-12, rtol=0)
    assert abs(a.getTrace() - 1.0) < 1e-10


@pytest.mark.gpu
@pytest.mark.parametrize("case", REF_CASES, ids=[c[0] for c in REF_CASES])
def test_reference_suite_on_gpu(qsim, gpu_ready, case):
    _, n, gates, ch, check = case
    c = qsim.Circuit(n)
    for t, qs, th in gates:
        c.append(qsim.GateOp(t, qs, th))
    sim = qsim.DensityMatrixSimulator(n, _noise(qsim, ch))
    sim.run(c)
    assert check(sim.getProbabilities(), sim.getPurity())
    assert abs(sim.getTrace() - 1.0) < 1e-10


@pytest.mark.gpu
def test_density_matrix_api(qsim, gpu_ready):
    rng = np.random.default_rng(3)
    psi = rng.normal(size=8) + 1j * rng.normal(size=8)
    psi /= np.linalg.norm(psi)
    dm = qsim.DensityMatrix(3, psi)
    np.testing.assert_allclose(dm.getMatrix(), np.outer(psi, psi.conj()), atol=1e-14)
    assert abs(dm.purity() - 1) < 1e-12 and dm.isValid()
    dm.initMaximallyMixed()
    assert abs(dm.purity() - 1 / 8) < 1e-15 and abs(dm.trace() - 1) < 1e-15
    dm.reset()
    assert abs(dm.getProbabilities()[0] - 1) < 1e-15
    assert dm.getMemoryBytes() == 16 * 64 and dm.getNumElements() == 64
    for bad in (0, 16):
        with pytest.raises(ValueError):
            qsim.DensityMatrix(bad)
    with pytest.raises(ValueError):
        qsim.DensityMatrix(2, np.ones(3))
    sim = qsim.DensityMatrixSimulator(2)
    c = qsim.Circuit(2)
    c.cry(0, 1, 0.3)
    with pytest.raises(RuntimeError):
        sim.run(c)
    # measurement (src/DensityMatrix.cu:374-406): Bell -> both qubits agree, rho pure again
    sim = qsim.DensityMatrixSimulator(2)
    sim.setSeed(5)
    sim.run(qsim.createBellCircuit())
    m0 = sim.measureQubit(0)
    assert sim.measureQubit(1) == m0
    p = sim.getProbabilities()
    assert abs(p[3 * m0] - 1) < 1e-12 and abs(sim.getPurity() - 1) < 1e-12


def _dm_apply_y_reference_loop(rho, n, target):
    """Element loop of dmApplyY (src/DensityMatrix.cu:507-546) on a host array: the pair
    (row, col) <-> (row ^ m, col ^ m), written once from the lower index."""
    out = rho.copy()
    dim = 1 << n
    m = 1 << target
    for row in range(dim):
        for col in range(dim):
            nr, nc = row ^ m, col ^ m
            if row < nr or (row == nr and col < nc):
                rb, cb = (row >> target) & 1, (col >> target) & 1
                ph1 = (1 if rb else -1) * (-1 if cb else 1)
                ph2 = (1 if not rb else -1) * (-1 if not cb else 1)
                v1, v2 = rho[row, col], rho[nr, nc]
                out[row, col] = ph2 * v2
                out[nr, nc] = ph1 * v1
    return out


@pytest.mark.parametrize("n,target", [(1, 0), (2, 1), (3, 0)])
def test_oracle_reference_y_is_the_kernel_formula(oracle, n, target):
    """The oracle's reference_y (-Y rho Y^dag) equals dmApplyY's element formula."""
    rng = np.random.default_rng(n + target)
    d = 1 << n
    a = rng.normal(size=(d, d)) + 1j * rng.normal(size=(d, d))
    rho = a @ a.conj().T
    rho /= np.trace(rho)
    want = _dm_apply_y_reference_loop(rho, n, target)
    got = oracle.dm_run(n, [(1, [target], 0.0)], rho=rho, reference_y=True)
    np.testing.assert_allclose(got, want, atol=1e-14)
    phys = oracle.dm_run(n, [(1, [target], 0.0)], rho=rho)
    np.testing.assert_allclose(phys, -want, atol=1e-14)


@pytest.mark.gpu
@pytest.mark.parametrize("n,seed", [(2, 5), (5, 6)])
def test_reference_compatible_y(qsim, oracle, gpu_ready, n, seed):
    """setReferenceCompatible(): Y as the reference computes it (-Y rho Y^dag); every other gate
    and channel unchanged.  Fused and per-gate."""
    c = _circuit(qsim, n, 30, seed)
    c.y(0)
    channels = [(0, -1, 0.05), (3, 0, 0.1)]
    want = oracle.dm_run(n, oracle.gates_of(c), channels, reference_y=True)
    for mode in (qsim.RunMode.Fused, qsim.RunMode.PerGate):
        sim = qsim.DensityMatrixSimulator(n, _noise(qsim, channels), mode=mode)
        sim.setReferenceCompatible()
        sim.run(c)
        np.testing.assert_allclose(sim.getDensityMatrix(), want, atol=1e-12, rtol=0)
    ny = sum(1 for g in c.getGates() if g.type == qsim.GateType.Y)
    assert abs(np.trace(want).real - (-1) ** ny) < 1e-10


def _dm_jit_source(qsim, n, circuit, channels):
    import ctypes
    from qsim_amd import _lib
    g, ng = circuit.to_abi()
    arr = (_lib.qsim_noise_channel * max(1, len(channels)))()
    for i, (t, qb, p) in enumerate(channels):
        arr[i].type, arr[i].qubit, arr[i].probability = t, qb, p
    size = ctypes.c_size_t()
    _lib.check(_lib.hip.qsim_dm_jit_source(n, g, ng, arr, len(channels), 1, None, 0, ctypes.byref(size)))
    buf = ctypes.create_string_buffer(size.value + 1)
    _lib.check(_lib.hip.qsim_dm_jit_source(n, g, ng, arr, len(channels), 1, buf, size.value + 1,
                                           ctypes.byref(size)))
    return buf.value.decode()


def test_channel_triples_emitted_as_one_scale(qsim):
    """Host-only: the depolarizing / phase-damping / phase-flip lowering CX · diag(1, g) · CX
    (density.hip dm_channel) is generated as one per-register scale by g where the row and column
    bits differ (jit.hip Gen::xor_diag), so the circuit-specialised DM kernels carry far fewer
    per-lane selects than three ops would."""
    n = 14
    c = qsim.createRandomHCCircuit(n, 100, 42)
    src = _dm_jit_source(qsim, n, c, [(0, -1, 0.01)])
    assert src.count("__global__") >= 6
    g = repr(1.0 - 4.0 * 0.01 / 3.0)
    fused = sum(1 for line in src.splitlines() if line.lstrip().startswith("const double f") and "1.0" in line)
    assert fused > 0 or g in src  # per-lane factor pairs (thread-bit rows) or compile-time scales
    assert src.count("qsel(") < 1200  # (2 657 with the three ops emitted one by one)


@pytest.mark.gpu
@pytest.mark.parametrize("n,seed", [(6, 11), (7, 12)])
def test_specialised_kernels_match_oracle(qsim, oracle, gpu_ready, n, seed):
    """The DM passes as circuit-specialised kernels (JIT forced below its 20-bit threshold), every
    channel type: the full rho equals the oracle at 1e-12 (the fused channel scales included)."""
    from qsim_amd.plan import set_jit
    c = _circuit(qsim, n, 40, seed)
    channels = [(0, -1, 0.05), (2, 1, 0.2), (4, n - 1, 0.15), (5, 0, 0.1), (1, 2, 0.3), (3, 3, 0.1)]
    want = oracle.dm_run(n, oracle.gates_of(c), channels)
    set_jit(2, 0)
    try:
        sim = qsim.DensityMatrixSimulator(n, _noise(qsim, channels))
        sim.run(c)
        got = sim.getDensityMatrix()
    finally:
        set_jit(1, 20)
    np.testing.assert_allclose(got, want, atol=1e-12, rtol=0)


def test_relabeled_plan_has_fewer_passes(qsim):
    """Host-only (qsim_dm_plan_info with QSIM_DM_PLAN_RELABELED): the first-run index-bit labels
    (capi.hip dm_choose_layout) plan the bench's DM circuit into fewer passes than the identity."""
    import ctypes
    from qsim_amd import _lib
    n = 14
    c = qsim.createRandomHCCircuit(n, 100, 42)
    g, ng = c.to_abi()
    arr = (_lib.qsim_noise_channel * 1)()
    arr[0].type, arr[0].qubit, arr[0].probability = 0, -1, 0.01
    passes = []
    for flags in (1, 1 | 0x100):
        info = (ctypes.c_int32 * 400)()
        npass = ctypes.c_size_t()
        _lib.check(_lib.hip.qsim_dm_plan_info(n, g, ng, arr, 1, flags, info, 100, ctypes.byref(npass)))
        passes.append(npass.value)
    assert passes[1] < passes[0], passes


@pytest.mark.gpu
@pytest.mark.parametrize("n,depth,seed,timed", [(8, 30, 21, False), (9, 16, 22, False), (8, 24, 23, True)])
def test_relabeled_runs_match_oracle(qsim, oracle, gpu_ready, n, depth, seed, timed):
    """16 / 18 index bits: the first fused run of a reset rho takes relabeled index bits
    (capi.hip qsim_dm_run; timed: the candidates timed on the device, specialised kernels); a
    second run keeps them (its ops mapped through the labels); readers restore the identity first.
    Every step equals the oracle at 1e-12, and a reset + rerun (the memoised labels) gives the
    same rho."""
    if timed:
        from qsim_amd.plan import set_calibrate, set_jit
        set_jit(2, 0)
        set_calibrate(1, 16)
        try:
            _relabeled_runs(qsim, oracle, n, depth, seed)
        finally:
            set_calibrate(1, 26)
            set_jit(1, 20)
    else:
        _relabeled_runs(qsim, oracle, n, depth, seed)


def _relabeled_runs(qsim, oracle, n, depth, seed):
    channels = [(0, -1, 0.03), (2, 1, 0.2), (1, 2, 0.1), (3, n - 1, 0.05), (4, 0, 0.1)]
    c1 = _circuit(qsim, n, depth, seed)
    c2 = _circuit(qsim, n, depth // 2, seed + 100)
    want1 = oracle.dm_run(n, oracle.gates_of(c1), channels)
    want2 = oracle.dm_run(n, oracle.gates_of(c2), channels, rho=want1)
    want3 = oracle.dm_channel(want2, n, 1, 3, 0.25)
    sim = qsim.DensityMatrixSimulator(n, _noise(qsim, channels))
    sim.run(c1)
    sim.run(c2)  # (no reader in between: still under the first run's labels)
    sim.run(qsim.Circuit(n))  # (an empty run keeps the state as it is)
    np.testing.assert_allclose(sim.getDensityMatrix(), want2, atol=1e-12, rtol=0)
    sim.applyChannel(qsim.NoiseType.AmplitudeDamping, 3, 0.25)
    np.testing.assert_allclose(sim.getDensityMatrix(), want3, atol=1e-12, rtol=0)
    sim.reset()
    sim.run(c1)
    np.testing.assert_allclose(sim.getProbabilities(), np.real(np.diag(want1)), atol=1e-12, rtol=0)
    np.testing.assert_allclose(sim.getDensityMatrix(), want1, atol=1e-12, rtol=0)
    assert abs(sim.getPurity() - np.sum(np.abs(want1) ** 2)) < 1e-12


@pytest.mark.gpu
def test_relabel_policy_governs_dm_relabeling(qsim, oracle, gpu_ready):
    """the DM first-run relabeling follows qsim_set_relabel — mode 0 keeps the
    identity labels (no host search); the default relabels from 16 index bits; a parameter sweep
    (same structure, new angles) reuses the memoised labels; every result equals the oracle."""
    from qsim_amd.plan import set_relabel
    n = 8
    channels = [(0, -1, 0.02)]

    def circ(theta):
        c = _circuit(qsim, n, 20, 41)
        c.rz(2, theta)
        c.ry(5, 0.5 * theta)
        return c
    set_relabel(0, -1)
    try:
        sim = qsim.DensityMatrixSimulator(n, _noise(qsim, channels))
        sim.run(circ(0.3))
        assert not sim.density.state.layoutInfo()["relabeled"]
        np.testing.assert_allclose(sim.getDensityMatrix(), oracle.dm_run(n, oracle.gates_of(circ(0.3)), channels),
                                   atol=1e-12, rtol=0)
    finally:
        set_relabel(1, 26)
    sim = qsim.DensityMatrixSimulator(n, _noise(qsim, channels))
    sim.run(circ(0.3))
    assert sim.density.state.layoutInfo()["relabeled"]
    perm0 = sim.density.state.perm()
    for theta in (0.7, 1.1):
        sim.reset()
        sim.run(circ(theta))
        assert sim.density.state.perm() == perm0  # (memo keyed on structure, not angles)
        np.testing.assert_allclose(sim.getDensityMatrix(), oracle.dm_run(n, oracle.gates_of(circ(theta)), channels),
                                   atol=1e-12, rtol=0)


@pytest.mark.gpu
def test_relabeled_run_reference_y_and_pinned_pointer(qsim, oracle, gpu_ready):
    """18 index bits: the relabeled first run with the reference's Y sign (its global -1 op moves
    with the labels), and a rho whose device pointer was handed out before the run (never
    relabeled: the pointer holds row-major rho right after the run, no reader in between)."""
    import ctypes
    n = 9
    c = _circuit(qsim, n, 14, 31)
    c.y(3)
    channels = [(0, -1, 0.02), (4, 2, 0.1)]
    want = oracle.dm_run(n, oracle.gates_of(c), channels, reference_y=True)
    sim = qsim.DensityMatrixSimulator(n, _noise(qsim, channels))
    sim.setReferenceCompatible()
    sim.run(c)
    np.testing.assert_allclose(sim.getDensityMatrix(), want, atol=1e-12, rtol=0)
    want2 = oracle.dm_run(n, oracle.gates_of(c), channels)
    sim2 = qsim.DensityMatrixSimulator(n, _noise(qsim, channels))
    ptr = sim2.density.state.devicePtr()
    sim2.run(c)
    sim2.density.state.synchronize()
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    raw = np.empty(1 << (2 * n), dtype=np.complex128)
    assert hip.hipMemcpy(raw.ctypes.data, ctypes.c_void_p(ptr), raw.nbytes, 2) == 0  # D2H
    np.testing.assert_allclose(raw.reshape(1 << n, 1 << n), want2, atol=1e-12, rtol=0)
