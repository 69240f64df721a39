"""Layout-aware qubit relabeling (csrc/hip/relabel.hip, qsim_run in capi.hip).

The first fused run of a basis state may run the whole circuit under a logical -> physical qubit
permutation chosen for the plan's tile layouts; every entry that reads or writes amplitudes by
index first restores the identity layout with a fused SWAP network.  The bench runs it at 30q
(default threshold 26 qubits); here the threshold is lowered so the same code runs at sizes the
oracle checks exactly (1e-12 per component), through every kind of entry that must see the
canonical layout: readback, probabilities, measurement, sampling, per-gate and matrix entries,
re-runs under the permutation, non-zero basis states and the per-gate run mode.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture
def relabel_low():
    from qsim_amd.plan import set_relabel
    set_relabel(1, 14)
    yield
    set_relabel(1, 26)


def _err(a, b):
    d = a - b
    return float(np.max(np.abs(np.concatenate([d.real, d.imag]))))


@pytest.mark.parametrize("n,seed", [(16, 1), (18, 2), (20, 3)])
def test_relabeled_runs_match_oracle(qsim, oracle, gpu_ready, relabel_low, n, seed):
    c = qsim.createRandomHCCircuit(n, 100, seed)
    g = oracle.gates_of(c)
    sim = qsim.Simulator(n)
    sim.run(c)
    assert sim.state.perm() != list(range(n)), "expected the planner to relabel this circuit"
    sim.run(c)  # second run under the permutation (no readback in between)
    assert _err(sim.getStateVector(), oracle.run_cpu(n, g + g)) < 1e-12
    assert sim.state.perm() == list(range(n))  # readback restored the identity layout


def test_relabel_then_every_reader(qsim, oracle, gpu_ready, relabel_low):
    n = 18
    c = qsim.createRandomCircuit(n, 120, 5)  # all gate types
    g = oracle.gates_of(c)
    ref = oracle.run_cpu(n, g)
    probs = np.abs(ref) ** 2

    def fresh():
        sim = qsim.Simulator(n)
        sim.run(c)
        assert sim.state.perm() != list(range(n))
        return sim

    np.testing.assert_allclose(fresh().getProbabilities(), probs, atol=1e-12, rtol=0)

    idx = np.arange(1 << n)
    assert abs(fresh().state.probBitZero(7) - probs[((idx >> 7) & 1) == 0].sum()) < 1e-12

    # sampling: the engine's CDF of the same amplitudes; an index may differ from the oracle's
    # only where the uniform lies within rounding of a CDF step
    u = np.random.default_rng(3).random(4000)
    got = fresh().state.sampleWith(u)
    exp = oracle.sample_cpu(n, ref, u)
    cdf = np.cumsum(probs)
    for i in np.nonzero(got != exp)[0]:
        assert abs(cdf[min(got[i], exp[i])] - u[i]) < 1e-12

    sim = fresh()  # relabeled, then per-gate entries map their qubits
    sim.applyGate(qsim.GateOp(qsim.GateType.H, [n - 1]))
    sim.applyGate(qsim.GateOp(qsim.GateType.CNOT, [2, n - 3]))
    c2 = qsim.Circuit(n)
    c2.h(n - 1)
    c2.cnot(2, n - 3)
    assert _err(sim.getStateVector(), oracle.run_cpu(n, g + oracle.gates_of(c2))) < 1e-12

    sim = fresh()  # relabeled, then a matrix entry (canonicalises first)
    m = np.array([[0.6, 0.8j], [0.8j, 0.6]], dtype=np.complex128)
    sim.state.applyMatrix1Q(5, m)
    t = ref.reshape([2] * n)
    ax = n - 1 - 5  # qubit q is index bit q; numpy axis 0 is bit n-1
    t = np.moveaxis(np.tensordot(m, np.moveaxis(t, ax, 0), axes=([1], [0])), 0, ax).reshape(-1)
    assert _err(sim.getStateVector(), t) < 1e-12

    sim = fresh()  # measurement (prob + collapse) on the canonical layout
    r = sim.measureQubit(3)
    bit = n - 1 - 3  # measure(q) reads index bit n-1-q (reference F2)
    keep = ((idx >> bit) & 1) == r
    post = np.where(keep, ref, 0)
    post /= np.linalg.norm(post)
    assert _err(sim.getStateVector(), post) < 1e-12


def test_relabel_nonzero_basis_and_per_gate_mode(qsim, oracle, gpu_ready, relabel_low):
    n = 18
    c = qsim.createRandomHCCircuit(n, 100, 2)  # relabeled (as in test_relabeled_runs_match_oracle)
    g = oracle.gates_of(c)
    k = 0b101100100111001011
    start = np.zeros(1 << n, dtype=np.complex128)
    start[k] = 1.0
    ref = oracle.run_cpu(n, g, state=start)
    sv = qsim.StateVector(n)
    sv.initializeBasis(k)
    sv.run(c, qsim.RunMode.Fused)
    assert sv.perm() != list(range(n))
    sv.run(c, qsim.RunMode.PerGate)  # per-gate run under the same permutation
    assert _err(sv.toHost(), oracle.run_cpu(n, g, state=ref)) < 1e-12


def test_relabel_off_is_identity(qsim, gpu_ready):
    from qsim_amd.plan import set_relabel
    set_relabel(0, 14)
    try:
        n = 18
        sim = qsim.Simulator(n)
        sim.run(qsim.createRandomHCCircuit(n, 100, 1))
        assert sim.state.perm() == list(range(n))
    finally:
        set_relabel(1, 26)


def test_calibrated_choice_matches_oracle(qsim, oracle, gpu_ready, relabel_low):
    """Layout calibration (inline compilation): the first run times the model's choice and its
    alternatives on the device — running each candidate's plan on the basis state and restoring
    it — then runs the circuit under the fastest.  The result is exact, also from a non-zero
    basis state."""
    from qsim_amd.plan import set_calibrate, set_jit
    set_jit(2, -1)
    set_calibrate(1, 14)
    try:
        n = 18
        c = qsim.createRandomHCCircuit(n, 100, 2)
        g = oracle.gates_of(c)
        sim = qsim.Simulator(n)
        sim.run(c)
        assert sim.state.perm() != list(range(n))
        assert _err(sim.getStateVector(), oracle.run_cpu(n, g)) < 1e-12
        k = 0b110010101100111010
        start = np.zeros(1 << n, dtype=np.complex128)
        start[k] = 1.0
        sv = qsim.StateVector(n)
        sv.initializeBasis(k)
        sv.run(c, qsim.RunMode.Fused)
        sv.run(c, qsim.RunMode.Fused)
        assert _err(sv.toHost(), oracle.run_cpu(n, g + g, state=start)) < 1e-12
    finally:
        set_calibrate(1, 28)
        set_jit(1, -1)
