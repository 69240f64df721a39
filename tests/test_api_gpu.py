"""GPU: StateVector / Simulator / BatchedSimulator API semantics.

Mirrors tests/test_statevector.cu, tests/test_boundary.cu and the batched part of
tests/test_noise.cu (:233-339, :449-462) of the reference, plus size-independent properties at
the benchmark sizes (norm preservation, inverse-circuit round trips, fused == per-gate).
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
TOL = 1e-12


def test_statevector_init_and_basis(qsim, gpu_ready):
    sv = qsim.StateVector(3)
    assert sv.getNumQubits() == 3 and sv.getSize() == 8
    s = sv.toHost()
    assert abs(abs(s[0]) - 1) < 1e-10 and np.all(np.abs(s[1:]) < 1e-10)
    sv4 = qsim.StateVector(4)
    for b in range(16):
        sv4.initializeBasis(b)
        s = sv4.toHost()
        assert abs(abs(s[b]) - 1) < TOL and np.sum(np.abs(s) > TOL) == 1
    with pytest.raises(ValueError):
        sv4.initializeBasis(16)
    with pytest.raises(ValueError):
        sv4.initializeBasis(100)
    for n in range(1, 11):
        assert abs(qsim.StateVector(n).getTotalProbability() - 1.0) <= TOL
    assert abs(qsim.StateVector(20).getTotalProbability() - 1.0) <= 1e-8


def test_probabilities_and_normalization(qsim, gpu_ready):
    sv = qsim.StateVector(2)
    p = sv.getProbabilities()
    assert list(p) == [1.0, 0.0, 0.0, 0.0]
    sv.assertNormalized()
    sv.fromHost(np.array([1, 1, 0, 0], complex))
    assert not sv.isNormalized()
    with pytest.raises(RuntimeError):
        sv.assertNormalized()


def test_prob_bit_zero_matches_sum(qsim, oracle, gpu_ready):
    n = 14
    c = qsim.createRandomCircuit(n, 120, 5)
    sim = qsim.Simulator(n)
    sim.run(c)
    st = oracle.run_cpu(n, oracle.gates_of(c))
    p = np.abs(st) ** 2
    for bit in range(n):
        mask = ((np.arange(1 << n) >> bit) & 1) == 0
        assert abs(sim.state.probBitZero(bit) - p[mask].sum()) < 1e-12


def test_measure_semantics(qsim, gpu_ready):
    sv = qsim.StateVector(2)
    assert sv.measure(0) == 0 and sv.isNormalized(1e-10)
    sv1 = qsim.StateVector(1)
    sv1.initializeBasis(1)
    assert sv1.measure(0) == 1 and sv1.isNormalized(1e-10)
    for q in (-1, 3, 100):
        with pytest.raises(ValueError):
            qsim.StateVector(3).measure(q)
    # Bell correlations (tests/test_statevector.cu:143-171)
    for seed in range(20):
        sim = qsim.Simulator(2)
        sim.setSeed(seed)
        sim.run(qsim.createBellCircuit())
        r0 = sim.measureQubit(0)
        r1 = sim.measureQubit(1)
        assert r0 == r1
        assert sim.state.isNormalized(1e-10)


def test_measure_is_big_endian_reference_quirk(qsim, gpu_ready):
    """Reference StateVector::measure(q) reads index bit n-1-q."""
    sim = qsim.Simulator(3)
    c = qsim.Circuit(3)
    c.x(0)                      # index 1: gate-qubit 0 is 1
    sim.run(c)
    assert sim.measureQubit(2) == 1   # bit n-1-2 = 0
    assert sim.measureQubit(0) == 0   # bit 2
    sv = qsim.StateVector(3)
    sv.initializeBasis(1)
    assert sv.measureBit(0) == 1


def test_sampling(qsim, oracle, gpu_ready):
    sv = qsim.StateVector(2)
    assert np.all(sv.sample(100) == 0)
    sv.initializeBasis(3)
    assert np.all(sv.sample(100) == 3)
    for bad in (0, -1):
        with pytest.raises(ValueError):
            sv.sample(bad)
    s1 = qsim.StateVector(1)
    s1.applyGate(qsim.GateOp(qsim.GateType.H, [0]))
    s1.setSeed(3)
    r = s1.sample(10000)
    assert abs(np.mean(r == 0) - 0.5) < 0.05
    sim = qsim.Simulator(2)
    sim.run(qsim.createBellCircuit())
    counts = np.bincount(sim.sample(1000), minlength=4)
    assert counts[1] == 0 and counts[2] == 0 and counts[0] > 0 and counts[3] > 0
    assert len(sim.sample(0)) == 0


def test_sampling_matches_reference_lower_bound(qsim, oracle, gpu_ready):
    """Device CDF sampling == lower_bound over the sequential CDF for the same uniforms."""
    for n in (5, 12, 15):
        c = qsim.createRandomCircuit(n, 60, n)
        sim = qsim.Simulator(n)
        sim.run(c)
        st = oracle.run_cpu(n, oracle.gates_of(c))
        u = np.random.default_rng(n).random(4000)
        got = sim.state.sampleWith(u)
        exp = oracle.sample_cpu(n, st, u)
        assert np.mean(got == exp) > 0.999


def test_boundary_errors(qsim, gpu_ready):
    for bad in (0, -1, 31, 40):
        with pytest.raises(ValueError):
            qsim.Simulator(bad)
    sim = qsim.Simulator(4)
    c = qsim.Circuit(3)
    c.h(0)
    with pytest.raises(ValueError):
        sim.run(c)
    with pytest.raises(IndexError):
        sim.applyGate(qsim.GateOp(qsim.GateType.H, [4]))
    with pytest.raises(ValueError):
        sim.applyGate(qsim.GateOp(qsim.GateType.CNOT, [1, 1]))


def test_reset_and_coexisting_simulators(qsim, gpu_ready):
    sim = qsim.Simulator(4)
    sim.run(qsim.createRandomCircuit(4, 50, 123))
    assert abs(sim.getProbabilities()[0] - 1.0) > TOL
    sim.reset()
    p = sim.getProbabilities()
    assert abs(p[0] - 1) < TOL and np.all(p[1:] < TOL)
    sims = [qsim.Simulator(n) for n in (4, 6, 8)]
    for s in sims:
        s.run(qsim.createGHZCircuit(s.getNumQubits()))
    for s in sims:
        p = s.getProbabilities()
        assert abs(p[0] - .5) < TOL and abs(p[-1] - .5) < TOL


def test_normalization_deep_circuit(qsim, gpu_ready):
    for mode in (qsim.RunMode.PerGate, qsim.RunMode.Fused):
        sim = qsim.Simulator(4, mode=mode)
        sim.run(qsim.createRandomCircuit(4, 1000, 42))
        assert abs(sim.getProbabilities().sum() - 1.0) < 1e-10


def test_raw_kernel_entry(qsim, gpu_ready):
    """Kernel-level entry on a device pointer (reference tests launch applyH<<<>>> directly)."""
    import ctypes
    from qsim_amd import _lib
    sv = qsim.StateVector(2)
    for t, qs in ((3, [0]), (11, [0, 1])):
        g = _lib.qsim_gate()
        g.type, g.nqubits = t, len(qs)
        for j, q in enumerate(qs):
            g.qubits[j] = q
        # launched on the state's own stream, so toHost() (same stream) is ordered after it
        _lib.check(_lib.hip.qsim_apply_gate_raw(sv.devicePtr(), 2, ctypes.byref(g),
                                                ctypes.c_void_p(sv.stream())))
    s = sv.toHost()
    np.testing.assert_allclose(np.abs(s) ** 2, [0.5, 0, 0, 0.5], atol=1e-12)


# ---------------------------------------------------------------- size-independent properties
@pytest.mark.parametrize("n", [22, 26])
def test_fused_matches_per_gate_large(qsim, gpu_ready, n):
    c = qsim.createRandomHCCircuit(n, 100, 42)
    c2 = qsim.createRandomCircuit(n, 100, 7)
    for circ in (c, c2):
        a = qsim.Simulator(n, mode=qsim.RunMode.PerGate)
        b = qsim.Simulator(n, mode=qsim.RunMode.Fused)
        a.run(circ)
        b.run(circ)
        sa, sb = a.getStateVector(), b.getStateVector()
        assert np.max(np.abs(sa - sb)) < 1e-12


@pytest.mark.parametrize("n", [24, 28])
def test_inverse_round_trip_large(qsim, gpu_ready, n):
    """W-HC circuit followed by its inverse (H, CNOT self-inverse) returns to |0..0>."""
    c = qsim.createRandomHCCircuit(n, 100, 42)
    inv = qsim.Circuit(n)
    for g in reversed(c.getGates()):
        inv.append(g)
    for mode in (qsim.RunMode.Fused, qsim.RunMode.PerGate):
        sim = qsim.Simulator(n, mode=mode)
        sim.run(c)
        assert abs(sim.state.getTotalProbability() - 1.0) < 1e-10
        sim.run(inv)
        p0 = 1.0 - sim.state.probBitZero(n - 1)
        assert sim.state.probBitZero(0) > 1 - 1e-10 and p0 < 1e-10
        amp0 = sim.state.sampleWith(np.array([0.5]))
        assert amp0[0] == 0


# ---------------------------------------------------------------- batched trajectories
def test_batched_init_and_bell(qsim, gpu_ready):
    b = qsim.BatchedSimulator(2, 10)
    for t in range(10):
        p = b.getProbabilities(t)
        assert abs(p[0] - 1) < 1e-10 and np.all(p[1:] < 1e-10)
    b5 = qsim.BatchedSimulator(2, 5)
    c = qsim.Circuit(2)
    c.h(0).cnot(0, 1)
    b5.run(c)
    for t in range(5):
        p = b5.getProbabilities(t)
        assert abs(p[0] - .5) < 1e-10 and abs(p[3] - .5) < 1e-10
    with pytest.raises(IndexError):
        b5.getProbabilities(5)


def test_batched_average_and_histogram(qsim, gpu_ready):
    b = qsim.BatchedSimulator(2, 100)
    c = qsim.Circuit(2)
    c.h(0)
    b.run(c)
    np.testing.assert_allclose(b.getAverageProbabilities(), [.5, .5, 0, 0], atol=1e-10)
    b10 = qsim.BatchedSimulator(2, 10)
    b10.run(c)
    assert b10.getHistogram(100).sum() == 1000
    assert qsim.BatchedSimulator(10, 100).getTotalMemoryBytes() == 100 * 1024 * 16


def test_batched_noise_free_equals_single(qsim, oracle, gpu_ready):
    n = 9
    c = qsim.createRandomCircuit(n, 80, 3)
    b = qsim.BatchedSimulator(n, 7)
    b.run(c)
    ref = oracle.run_cpu(n, oracle.gates_of(c))
    for t in range(7):
        np.testing.assert_allclose(b.getStateVector(t), ref, atol=1e-12, rtol=0)


def test_batched_reference_gateset_skips(qsim, oracle, gpu_ready):
    c = qsim.Circuit(3)
    c.h(0).h(1).h(2).cnot(0, 1).cnot(1, 2).x(0).y(1).z(2).s(0).rz(1, 0.3).toffoli(0, 1, 2)
    b = qsim.BatchedSimulator(3, 4, gate_set=qsim.BatchedGateSet.Reference)
    b.run(c)
    kept = [g for g in oracle.gates_of(c) if g[0] <= 3 or g[0] == 11]
    ref = oracle.run_cpu(3, kept)
    np.testing.assert_allclose(b.getStateVector(0), ref, atol=1e-12)
    assert abs(b.getAverageProbabilities().sum() - 1) < 1e-10


def test_batched_depolarizing_statistics(qsim, gpu_ready):
    """Physical depolarizing: one X/Y/Z on a trajectory with prob p (per channel, per gate)."""
    n, B, p = 1, 20000, 0.3
    nm = qsim.NoiseModel()
    nm.addDepolarizing([0], p)
    b = qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Physical)
    b.setSeed(42)
    c = qsim.Circuit(1)
    c.x(0)                      # |1>; after noise: X flips to |0> (p/3), Y -> |0> (p/3), Z keeps |1>
    b.run(c)
    avg = b.getAverageProbabilities()
    assert abs(avg[0] - 2 * p / 3) < 0.02
    # global-form noise applies to no qubit (F6)
    nm2 = qsim.NoiseModel()
    nm2.addDepolarizing(0.5)
    b2 = qsim.BatchedSimulator(1, 100, nm2)
    b2.run(c)
    np.testing.assert_allclose(b2.getAverageProbabilities(), [0, 1], atol=1e-12)


def test_batched_noise_reproducible_and_normalized(qsim, gpu_ready):
    nm = qsim.NoiseModel()
    nm.addDepolarizingAll(5, 0.05)
    c = qsim.createRandomHCCircuit(5, 40, 1)
    outs = []
    for _ in range(2):
        b = qsim.BatchedSimulator(5, 64, nm)
        b.setSeed(7)
        b.run(c)
        outs.append(np.stack([b.getStateVector(t) for t in range(64)]))
        for t in range(0, 64, 9):
            assert abs(np.sum(np.abs(outs[-1][t]) ** 2) - 1) < 1e-12
    np.testing.assert_array_equal(outs[0], outs[1])
    # noise realizations differ across trajectories
    assert np.max(np.abs(outs[0][0] - outs[0][1:]).reshape(63, -1).max(axis=1)) > 1e-6
