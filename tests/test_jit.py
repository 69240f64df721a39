"""Circuit-specialised pass kernels (jit.hip): generated source compiles for gfx950 (CPU), and on
the GPU the compiled kernels give the oracle's state for every gate kind, control placement and
run width the planner produces, and agree with the pass interpreter at larger sizes."""
import numpy as np
import pytest

GATES_2Q = ("cnot", "cz", "cry", "crz", "swap")


def _mixed_circuit(q, n, depth, seed):
    """All 17 gate types, targets/controls spread over run, lane and high tile bits."""
    rng = np.random.default_rng(seed)
    c = q.Circuit(n)
    for _ in range(depth):
        k = int(rng.integers(0, 17))
        a, b, d = (int(x) for x in rng.choice(n, 3, replace=False))
        th = float(rng.uniform(-3.1, 3.1))
        if k < 8:
            getattr(c, ("x", "y", "z", "h", "s", "t", "sdag", "tdag")[k])(a)
        elif k < 11:
            getattr(c, ("rx", "ry", "rz")[k - 8])(a, th)
        elif k < 16:
            name = GATES_2Q[k - 11]
            if name in ("cry", "crz"):
                getattr(c, name)(a, b, th)
            else:
                getattr(c, name)(a, b)
        else:
            c.toffoli(a, b, d)
    return c


def test_generated_source_compiles(qsim):
    from qsim_amd.plan import jit_build, jit_source
    for c in (qsim.createRandomHCCircuit(24, 100, 42), _mixed_circuit(qsim, 14, 120, 3)):
        src = jit_source(c)
        assert "extern \"C\" __global__" in src and "qk" in src
        assert jit_build(c) > 0
    assert jit_source(qsim.createBellCircuit()) == ""  # no staged pass: nothing to specialise


@pytest.fixture
def jit_inline(qsim, gpu_ready):
    from qsim_amd.plan import set_jit
    set_jit(2, 0)
    yield
    set_jit(1, 20)


@pytest.mark.gpu
@pytest.mark.parametrize("n,depth,seed", [(10, 150, 1), (12, 200, 2), (14, 250, 3), (16, 300, 4)])
def test_jit_matches_oracle(qsim, oracle, jit_inline, n, depth, seed):
    c = _mixed_circuit(qsim, n, depth, seed)
    ref = oracle.run_cpu(n, oracle.gates_of(c))
    sim = qsim.Simulator(n)
    for _ in range(2):  # first run compiles inline; both runs use the compiled kernels
        sim.reset()
        sim.run(c)
        np.testing.assert_allclose(sim.getStateVector(), ref, atol=1e-12, rtol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_jit_random_reference_circuits(qsim, oracle, jit_inline, seed):
    n = 11 + seed % 4
    c = qsim.createRandomCircuit(n, 200, seed)
    sim = qsim.Simulator(n)
    sim.run(c)
    np.testing.assert_allclose(sim.getStateVector(), oracle.run_cpu(n, oracle.gates_of(c)),
                               atol=1e-12, rtol=0)


@pytest.mark.gpu
def test_jit_equals_interpreter_at_22q(qsim, gpu_ready):
    from qsim_amd.plan import set_jit
    n = 22
    c = _mixed_circuit(qsim, n, 200, 9)
    out = []
    for mode in (0, 2):
        set_jit(mode, 0)
        sim = qsim.Simulator(n)
        sim.run(c)
        out.append(sim.getStateVector())
    set_jit(1, 20)
    np.testing.assert_allclose(out[1], out[0], atol=1e-12, rtol=0)
    assert abs(np.vdot(out[1], out[1]).real - 1.0) < 1e-10


@pytest.mark.gpu
def test_jit_background_switches_over(qsim, oracle, gpu_ready):
    """Mode 1: early runs use the interpreter while hipRTC compiles; results never change."""
    import time
    from qsim_amd.plan import set_jit
    set_jit(1, 0)
    try:
        n = 13
        c = _mixed_circuit(qsim, n, 150, 21)
        ref = oracle.run_cpu(n, oracle.gates_of(c))
        sim = qsim.Simulator(n)
        for _ in range(8):
            sim.reset()
            sim.run(c)
            np.testing.assert_allclose(sim.getStateVector(), ref, atol=1e-12, rtol=0)
            time.sleep(0.3)
    finally:
        set_jit(1, 20)


@pytest.mark.gpu
def test_jit_sharded_virtual(qsim, oracle, jit_inline):
    from qsim_amd.dist import DistributedSimulator
    n = 14
    c = _mixed_circuit(qsim, n, 150, 5)
    ref = oracle.run_cpu(n, oracle.gates_of(c))
    d = DistributedSimulator.virtual(n, 4)
    d.run(c)
    np.testing.assert_allclose(d.getStateVector(), ref, atol=1e-12, rtol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [26, 28])
def test_full_size_paths_agree(qsim, gpu_ready, n):
    """At BASELINE sizes (beyond the oracle): W-HC through the per-gate kernels, the pass
    interpreter and the specialised kernels gives the same state, and the norm stays 1."""
    from qsim_amd.plan import set_jit
    c = qsim.createRandomHCCircuit(n, 100, 42)
    states = []
    try:
        for mode, jit in ((qsim.RunMode.PerGate, 0), (qsim.RunMode.Fused, 0), (qsim.RunMode.Fused, 2)):
            set_jit(jit, 0)
            sim = qsim.Simulator(n, mode=mode)
            sim.run(c)
            assert abs(sim.state.getTotalProbability() - 1.0) < 1e-10
            states.append(sim.getStateVector())
            del sim
    finally:
        set_jit(1, 20)
    np.testing.assert_allclose(states[1], states[0], atol=1e-12, rtol=0)
    np.testing.assert_allclose(states[2], states[0], atol=1e-12, rtol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("jit", [0, 2])
def test_many_h_in_one_pass_stay_finite(qsim, gpu_ready, jit):
    """a pass runs uncontrolled H as unnormalised butterflies (norm x sqrt2 each) and
    rescales at the store; the planner caps them per pass (the rest run as the normalised
    matrix), so 4000 H on a 12-qubit state (one tile, one pass) stay finite: H.H pairs = identity.
    (With jit = 2 this pass exceeds the specialised kernels' op limit and runs on the
    interpreter; specialised passes hold at most 192 ops, far below the cap.)"""
    from qsim_amd.plan import set_jit
    n = 12
    rng = np.random.default_rng(4)
    c = qsim.Circuit(n)
    for _ in range(2000):
        q = int(rng.integers(0, n))
        c.h(q).h(q)
    psi = rng.normal(size=1 << n) + 1j * rng.normal(size=1 << n)
    psi /= np.linalg.norm(psi)
    try:
        set_jit(jit, 0)
        sim = qsim.Simulator(n, mode=qsim.RunMode.Fused)
        sim.state.fromHost(psi)
        sim.run(c)
        got = sim.getStateVector()
    finally:
        set_jit(1, 20)
    assert np.all(np.isfinite(got))
    np.testing.assert_allclose(got, psi, atol=1e-11, rtol=0)
    zero = qsim.Simulator(n, mode=qsim.RunMode.Fused)
    zero.run(c)
    p = zero.getProbabilities()
    assert abs(p[0] - 1.0) < 1e-10
