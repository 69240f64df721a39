"""Relayout plans on the GPU (csrc/hip/relayout.hip; the pass kernels' store layouts in fused.hip
k_fused_staged and the generated kernels of jit.hip).  The first fused run of a basis state may
pick a relayout plan (every pass stores its tile under the next pass's qubit layout, the last one
restores the first layout); the bench takes it at 30q, here the thresholds are lowered so the
same code runs at sizes the oracle checks exactly (1e-12 per component) — through the pass
interpreter and through the circuit-specialised kernels, re-run under the layout, and with the
device calibration choosing between it and the fixed-layout candidates."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _err(a, b):
    d = a - b
    return float(np.max(np.abs(np.concatenate([d.real, d.imag]))))


@pytest.fixture
def relayout_low():
    from qsim_amd.plan import set_calibrate, set_jit, set_relabel, set_relayout
    set_relabel(1, 14)
    set_relayout(2, 22)  # forced: a relayout plan whenever one exists
    set_calibrate(0, -1)
    yield
    from qsim_amd.plan import restore_defaults
    restore_defaults()  # (the shipped thresholds: later tests must run the default paths)


@pytest.mark.parametrize("jit", [0, 2])
@pytest.mark.parametrize("n,seed", [(22, 42), (24, 3)])
def test_relayout_runs_match_oracle(qsim, oracle, gpu_ready, relayout_low, jit, n, seed):
    from qsim_amd.plan import set_jit
    set_jit(jit, 20)
    c = qsim.createRandomHCCircuit(n, 100, seed)
    g = oracle.gates_of(c)
    sim = qsim.Simulator(n)
    sim.run(c)
    info = sim.state.layoutInfo()
    assert info["relayout"] and info["tile_qubits"] == 12, info
    sim.run(c)  # the second run starts from the layout the first one restored
    assert _err(sim.getStateVector(), oracle.run_cpu(n, g + g)) < 1e-12


def test_relayout_all_gate_types(qsim, oracle, gpu_ready, relayout_low):
    from qsim_amd.plan import plan_relayout, set_jit
    n = 22
    c = qsim.createRandomCircuit(n, 150, 7)
    c.cz(3, 17).swap(2, 20).toffoli(1, 9, 21).cry(4, 18, 0.3).crz(19, 0, 1.1).s(13).tdag(14)
    assert plan_relayout(c)[1] > 0
    ref = oracle.run_cpu(n, oracle.gates_of(c))
    for jit in (0, 2):
        set_jit(jit, 20)
        sim = qsim.Simulator(n)
        sim.run(c)
        relayout = sim.state.layoutInfo()["relayout"]
        np.testing.assert_allclose(sim.getProbabilities(), np.abs(ref) ** 2, atol=1e-12, rtol=0)
        assert _err(sim.getStateVector(), ref) < 1e-12
        assert relayout


def test_relayout_calibrated_choice_matches_oracle(qsim, oracle, gpu_ready, relayout_low):
    """With inline compilation and calibration on (the bench's mode) the relayout plan is timed
    against the fixed-layout candidates; whichever wins, forward + inverse returns to |0>."""
    from qsim_amd.plan import set_calibrate, set_jit, set_relayout
    set_jit(2, 20)
    set_calibrate(1, 22)
    set_relayout(1, 22)  # a candidate among the timed ones
    n = 24
    c = qsim.createRandomHCCircuit(n, 100, 42)
    inv = qsim.Circuit(n)
    for gt in reversed(c.getGates()):
        inv.append(gt)  # H and CNOT are self-inverse
    sim = qsim.Simulator(n)
    sim.run(c)
    assert sim.state.layoutInfo()["calibrated"]
    sim.run(inv)
    sv = sim.getStateVector()
    assert abs(sv[0] - 1.0) < 1e-10 and float(np.sum(np.abs(sv[1:]) ** 2)) < 1e-20


def test_relayout_from_basis_state_then_readers_and_gates(qsim, oracle, gpu_ready, relayout_low):
    """A relayout run from a non-zero basis state, then per-gate entries under the layout, then
    the readers (each restores the identity layout with one gate-free relayout pass first)."""
    from qsim_amd.plan import set_jit
    set_jit(0, 20)
    n = 22
    c = qsim.createRandomCircuit(n, 120, 9)
    g = oracle.gates_of(c)
    k = (1 << 21) | (1 << 13) | 5
    start = np.zeros(1 << n, complex)
    start[k] = 1.0
    sv = qsim.StateVector(n)
    sv.initializeBasis(k)
    sv.run(c, qsim.RunMode.Fused)
    assert sv.perm() != list(range(n))
    extra = qsim.Circuit(n)
    extra.h(n - 1).cnot(3, 17).t(9)
    for gt in extra.getGates():
        sv.applyGate(gt)  # mapped through the layout (no restore needed)
    assert sv.perm() != list(range(n))
    ref = oracle.run_cpu(n, oracle.gates_of(extra), state=oracle.run_cpu(n, g, state=start))
    probs = np.abs(ref) ** 2
    idx = np.arange(1 << n)
    assert abs(sv.probBitZero(11) - probs[((idx >> 11) & 1) == 0].sum()) < 1e-12
    assert sv.perm() == list(range(n))
    assert _err(sv.toHost(), ref) < 1e-12


@pytest.mark.parametrize("n", [22, 24])
def test_run_sequence_matches_runs_and_oracle(qsim, oracle, gpu_ready, relayout_low, n):
    """Simulator.runSequence: consecutive circuits planned as one engine run (a pass may hold the end
    of one circuit and the start of the next — fewer passes than the runs one by one) give the
    oracle's state of the circuits applied in turn, from a basis state (relayout plan) and again
    on the evolved state; the same circuits run one by one agree."""
    from qsim_amd.plan import plan_relayout
    cs = [qsim.createRandomHCCircuit(n, 100, sd) for sd in (42, 43, 44)]
    seq = qsim.Circuit(n)
    for c in cs:
        seq.extend(c)
    assert seq.getGateCount() == 300
    assert plan_relayout(seq)[1] < sum(plan_relayout(c)[1] for c in cs)
    g = oracle.gates_of(seq)
    a = qsim.Simulator(n)
    a.runSequence(cs)
    assert a.state.layoutInfo()["relayout"]
    want = oracle.run_cpu(n, g)
    assert _err(a.getStateVector(), want) < 1e-12
    a.runSequence(cs)
    want2 = oracle.run_cpu(n, g, want)
    assert _err(a.getStateVector(), want2) < 1e-12
    b = qsim.Simulator(n)
    for _ in range(2):
        for c in cs:
            b.run(c)
    assert _err(b.getStateVector(), want2) < 1e-12
    with pytest.raises(ValueError):
        a.runSequence([qsim.Circuit(n), qsim.Circuit(n - 1)])
