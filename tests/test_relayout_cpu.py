"""CPU: relayout plans (csrc/hip/relayout.hip) — every fused pass stores its tile under the next
pass's qubit layout, so each pass chooses all of its tile qubits except the four of the contiguous
run.  qsim_plan_exec_host runs a plan on the host exactly as the staged pass kernels address the
state (register stages, LDS slots through the stage layouts, the store layout of every pass), so
these tests pin the planner's and the stages' index math without a GPU: the result must equal the
oracle for W-HC and for circuits over the whole gate set from random states.  No reference
counterpart (the reference launches one kernel per gate, src/Simulator.cu:28-154)."""
import numpy as np
import pytest


def _err(a, b):
    d = a - b
    return float(np.max(np.abs(np.concatenate([d.real, d.imag]))))


@pytest.mark.parametrize("n,seed", [(22, 42), (23, 1)])
def test_relayout_plan_executes_whc_exactly(qsim, oracle, n, seed):
    from qsim_amd.plan import plan_exec_host
    c = qsim.createRandomHCCircuit(n, 100, seed)
    ref = oracle.run_cpu(n, oracle.gates_of(c))
    st1, perm1, p1 = plan_exec_host(c, 1)
    st0, perm0, p0 = plan_exec_host(c, 0)
    assert sorted(perm1) == list(range(n)) and perm0 == list(range(n))
    assert p1 <= p0  # (the run-sharing constraint leaves room for fewer passes or as many)
    assert _err(st1, ref) < 1e-12 and _err(st0, ref) < 1e-12


def test_relayout_plan_executes_all_gates_from_random_state(qsim, oracle):
    from qsim_amd.plan import plan_exec_host
    n = 22
    c = qsim.createRandomCircuit(n, 150, 7)
    c.cz(3, 17).swap(2, 20).toffoli(1, 9, 21).cry(4, 18, 0.3).crz(19, 0, 1.1).s(13).tdag(14)
    c.ry(16, 0.7).rx(5, 0.2).y(11).sdag(12).t(20).x(21).z(0).rz(15, 2.2)
    rng = np.random.default_rng(11)
    s0 = rng.normal(size=1 << n) + 1j * rng.normal(size=1 << n)
    s0 /= np.linalg.norm(s0)
    ref = oracle.run_cpu(n, oracle.gates_of(c), state=s0)
    st, perm, passes = plan_exec_host(c, 1, state=s0)
    assert passes >= 2
    assert _err(st, ref) < 1e-12


@pytest.mark.parametrize("seed,ctrl_out,want", [(42, 0, 4), (1, 0, 5), (2, 0, 5), (4, 0, 4),
                                                (42, 1, 4), (1, 1, 4), (2, 1, 4), (4, 1, 3)])
def test_relayout_needs_fewer_passes_at_30_qubits(qsim, seed, ctrl_out, want):
    """W-HC 30q, every control a tile qubit: 5 passes (seed 42) / 6 (seeds 1, 2, 4) with the
    fixed-layout planner under the chosen labels; relayout plans need one fewer,
    deterministically.  With tile-constant controls (the default; a CNOT needs only its target in
    the tile) relayout plans need 4 / 4 / 4 / 3, never more than the fixed-layout plan."""
    from qsim_amd.plan import plan_fused, plan_relabel, plan_relayout, set_tile_ctrl_out
    n = 30
    c = qsim.createRandomHCCircuit(n, 100, seed)
    set_tile_ctrl_out(ctrl_out)
    try:
        perm, passes, pred = plan_relayout(c)
        assert sorted(perm) == list(range(n))
        lab, _, _ = plan_relabel(c)
        c2 = qsim.Circuit(n)
        for g in c.getGates():
            c2.append(qsim.GateOp(g.type, [lab[x] for x in g.qubits], g.parameter))
        fixed = plan_fused(c2)[2]
        assert passes == want and (passes < fixed if not ctrl_out else passes <= fixed)
        assert plan_relayout(c) == (perm, passes, pred)
    finally:
        set_tile_ctrl_out(1)


def test_relayout_kernels_compile_for_gfx950(qsim):
    from qsim_amd.plan import jit_build_relayout
    assert jit_build_relayout(qsim.createRandomHCCircuit(30, 100, 42)) > 0


@pytest.mark.parametrize("n,seed", [(16, 1), (20, 2)])
def test_one_pass_identity_restore(qsim, n, seed):
    """The identity-layout restore before index-based readers is one gate-free relayout pass
    (capi.hip canonicalize): every amplitude lands at its logical index."""
    import ctypes
    from qsim_amd import _lib
    rng = np.random.default_rng(seed)
    perm = rng.permutation(n).astype(np.int32)
    psi = rng.normal(size=1 << n) + 1j * rng.normal(size=1 << n)
    idx = np.arange(1 << n, dtype=np.int64)
    phys = np.zeros_like(idx)
    for q in range(n):
        phys |= ((idx >> q) & 1) << int(perm[q])
    st = np.zeros(1 << n, np.complex128)
    st[phys] = psi
    p = (ctypes.c_int32 * n)(*perm.tolist())
    passes = ctypes.c_int(0)
    arr, cnt = qsim.Circuit(n).to_abi()
    _lib.check(_lib.hip.qsim_plan_exec_host(n, arr, 0, 2, st.ctypes.data_as(ctypes.c_void_p), p,
                                            ctypes.byref(passes)))
    assert passes.value == 1
    assert np.array_equal(st, psi)


@pytest.mark.parametrize("ctrl_out", [0, 1])
@pytest.mark.parametrize("n,seed", [(22, 3), (24, 4)])
def test_tile_constant_controls_execute_exactly(qsim, oracle, ctrl_out, n, seed):
    """Tile-constant controls (qsim_set_tile_ctrl_out): a CNOT's control need not be a tile
    qubit — the op runs on the tiles whose fixed bits read 1.  Both planners, executed on the host
    as the kernels address the state (incl. the uniform per-tile control test), equal the oracle;
    W-HC needs no more passes with them than without."""
    from qsim_amd.plan import plan_exec_host, set_tile_ctrl_out
    c = qsim.createRandomHCCircuit(n, 100, seed)
    ref = oracle.run_cpu(n, oracle.gates_of(c))
    set_tile_ctrl_out(ctrl_out)
    got = {}
    for mode in (0, 1):
        st, perm, p = plan_exec_host(c, mode)
        assert _err(st, ref) < 1e-12, (mode, ctrl_out)
        got[mode] = p
    set_tile_ctrl_out(1 - ctrl_out)
    other = {mode: plan_exec_host(c, mode)[2] for mode in (0, 1)}
    set_tile_ctrl_out(1)
    on, off = (got, other) if ctrl_out else (other, got)
    assert on[0] <= off[0] and on[1] <= off[1]


def test_sequence_circuit_and_joint_plan(qsim):
    """Simulator.runSequence's circuit (qsim_amd.simulator.sequence_circuit: the gates in order) and
    why it pays: four consecutive 100-gate W-HC circuits at 30 qubits plan into at most 11 relayout
    passes together against 4 each alone (host planner, no GPU)."""
    from qsim_amd.plan import plan_relayout
    from qsim_amd.simulator import sequence_circuit
    cs = [qsim.createRandomHCCircuit(30, 100, sd) for sd in (42, 43, 44, 45)]
    seq = sequence_circuit(cs, 30)
    assert [(g.type, g.qubits) for g in seq.getGates()] == [(g.type, g.qubits) for c in cs for g in c.getGates()]
    alone = [plan_relayout(c)[1] for c in cs]
    assert alone == [4, 4, 4, 4]
    assert 0 < plan_relayout(seq)[1] <= 11
    with pytest.raises(ValueError):
        sequence_circuit([cs[0], qsim.Circuit(29)], 30)
    with pytest.raises(ValueError):
        qsim.Circuit(30).extend(qsim.Circuit(29))


def test_joint_plan_of_a_sequence_executes_exactly(qsim, oracle):
    """The relayout plan of three consecutive W-HC circuits (what runSequence runs), executed on the
    host as the pass kernels address the state, equals the oracle of the circuits in turn."""
    from qsim_amd.plan import plan_exec_host, plan_relayout
    from qsim_amd.simulator import sequence_circuit
    n = 20
    cs = [qsim.createRandomHCCircuit(n, 100, sd) for sd in (7, 8, 9)]
    seq = sequence_circuit(cs, n)
    assert plan_relayout(seq)[1] < sum(plan_relayout(c)[1] for c in cs)
    st, perm, passes = plan_exec_host(seq, 1)
    assert _err(st, oracle.run_cpu(n, oracle.gates_of(seq))) < 1e-12
