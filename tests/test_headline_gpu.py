"""GPU: the bench's exact headline configuration at full size, pinned permutation-sensitively.

W-HC depth 100 at 30 qubits (16 GiB), inline compilation (jit = 2, as bench.py runs it), so the
first run on |0..0> chooses the qubit labels, the tile height and between fixed-layout and
relayout plans by timing candidates on the device (layout + cross-height calibration), then runs
the chosen plan with the specialised pass kernels.  Relabeling and relayout are qubit
permutations, so a round trip (circuit, then its inverse under the same labels) cannot see a bug
that applies the circuit on consistently permuted qubits.  The forward state itself is therefore
compared with RunMode::PerGate on a second state, which never relabels, never fuses and never
relayouts (its kernels are oracle-checked gate by gate in test_parity_gpu.py):
  * every amplitude at 1e-12 per component (reference tests/test_gpu_cpu_equivalence.cu:26),
    on the device (qsim_state_max_abs_diff: no 2 x 16 GiB host copy);
  * probBitZero of all n qubits, and sampleWith on 64 fixed uniforms (identical indices);
  * after ONE run (the first run: calibration, then the chosen plan) and after TWO runs (the
    second starts from the layout the first ends in: the bench's timed steady state).
Also: config 3 (28 qubits, its calibrated plan), W-HC seed 2 under its 5-pass relayout plan, a
state whose raw device pointer was handed out (never relabeled: the pointer stays canonical), and the
fallback when the relayout plan's second buffer does not fit in device memory.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture
def jit2(qsim):
    from qsim_amd.plan import set_jit
    set_jit(2, -1)
    yield
    # (conftest puts every policy back to the shipped defaults)


def _same_distribution(qsim, fused, ref, n, label):
    """probBitZero on every qubit and 64 fixed-uniform samples: equal."""
    for q in range(n):
        a, b = fused.probBitZero(q), ref.probBitZero(q)
        assert abs(a - b) < 1e-12, (label, q, a, b)
    u = np.random.default_rng(7).random(64)
    assert np.array_equal(fused.sampleWith(u), ref.sampleWith(u)), label


def _pin_against_per_gate(qsim, n, seed, expect_relayout=None, expect_passes=None, expect_relabeled=True):
    c = qsim.createRandomHCCircuit(n, 100, seed)
    ref = qsim.Simulator(n, mode=qsim.RunMode.PerGate)
    ref.run(c)
    for runs in (1, 2):
        sim = qsim.Simulator(n)  # (the second object takes the memoised first-run decision)
        for _ in range(runs):
            sim.run(c)
        info = sim.state.layoutInfo()
        passes = sim.state.lastRunInfo()[0]
        if expect_relabeled:
            assert info["relabeled"], info  # the bench's path: a non-identity layout
        if expect_relayout is not None:
            assert info["relayout"] == expect_relayout, info
        if expect_passes is not None:
            assert passes == expect_passes, passes
        if runs == 2:
            ref.run(c)  # the reference state after two runs too
        err = sim.state.maxAbsDiff(ref.state)
        assert err < 1e-12, (n, seed, runs, err)
        assert not sim.state.layoutInfo()["relabeled"]  # the reader restored the identity layout
        _same_distribution(qsim, sim.state, ref.state, n, (n, seed, runs))
        assert abs(sim.state.getTotalProbability() - 1.0) < 1e-10
        sim.state.close()
    return info, passes


def test_w_hc_30q_headline_path_equals_per_gate(qsim, gpu_ready, jit2):
    """The bench's line: W-HC 30q seed 42, calibrated first run (fixed-layout and relayout
    candidates timed on the device, 4 passes either way with tile-constant controls)."""
    info, passes = _pin_against_per_gate(qsim, 30, 42, expect_passes=4)
    assert info["calibrated"] and info["tile_qubits"] == 12


def test_w_hc_28q_config3_equals_per_gate(qsim, gpu_ready, jit2):
    """BASELINE config 3 (28 qubits) under whatever plan its calibrated first run keeps."""
    info, passes = _pin_against_per_gate(qsim, 28, 42, expect_relabeled=False)
    assert info["calibrated"] and passes <= 5


@pytest.mark.parametrize("seed,ctrl_out,passes", [(2, 1, 4), (42, 1, 4), (2, 0, 5)])
def test_w_hc_30q_relayout_plans_equal_per_gate(qsim, gpu_ready, jit2, seed, ctrl_out, passes):
    """W-HC 30q under its relayout plan (forced, so the timing cannot pick another plan and leave
    the relayout cycle untested): seeds 2 and 42 with tile-constant controls (4 passes), and seed 2
    with every control a tile qubit (the 5-pass relayout plan of round 3)."""
    from qsim_amd.plan import set_relayout, set_tile_ctrl_out
    set_relayout(2, -1)
    set_tile_ctrl_out(ctrl_out)
    _pin_against_per_gate(qsim, 30, seed, expect_relayout=True, expect_passes=passes)


def test_w_hc_30q_headline_path_round_trip(qsim, gpu_ready, jit2):
    """Kept as an extra check: the circuit then its inverse under the same labels is |0..0>."""
    n = 30
    c = qsim.createRandomHCCircuit(n, 100, 42)
    inv = qsim.Circuit(n)
    for g in reversed(c.getGates()):
        inv.append(g)
    sim = qsim.Simulator(n)
    sim.run(c)
    info = sim.state.layoutInfo()
    assert info["calibrated"] and info["relabeled"]
    sim.run(inv)
    for q in (0, 15, n - 1):
        assert sim.state.probBitZero(q) > 1 - 1e-10, q
    assert not sim.state.layoutInfo()["relabeled"]
    assert abs(sim.state.getTotalProbability() - 1.0) < 1e-10


def _read_device(ptr, n):
    """The 2^n amplitudes at a raw device pointer (D2H through the loaded HIP runtime)."""
    hip = _hip()
    out = np.empty(1 << n, dtype=np.complex128)
    assert hip.hipDeviceSynchronize() == 0
    assert hip.hipMemcpy(out.ctypes.data, ctypes.c_void_p(ptr), out.nbytes, 2) == 0  # D2H
    return out


def test_pinned_state_is_never_relabeled(qsim, oracle, gpu_ready):
    """a pointer from devicePtr() held across a basis-state fused run (relayout
    forced, so an unpinned state would be relabeled) sees the canonical state without calling
    devicePtr() again (reference include/StateVector.cuh:66-124: devicePtr() is the state), and the
    raw kernel entry on it acts on the right qubit.  Pinned states run the identity layout in place
    (capi.hip qsim_run), so no second buffer and no copy-back either."""
    from qsim_amd import _lib
    from qsim_amd.plan import set_jit, set_relayout
    set_relayout(2, 20)  # forced relayout plan at 22 qubits (taken by an unpinned state)
    set_jit(0, -1)       # (the interpreter: no compile wait)
    n = 22
    c = qsim.createRandomHCCircuit(n, 100, 42)
    ref = oracle.run_cpu(n, oracle.gates_of(c))
    free = qsim.StateVector(n)  # control: the same run unpinned takes the relayout plan
    free.run(c, qsim.RunMode.Fused)
    assert free.layoutInfo()["relayout"] and free.layoutInfo()["relabeled"]
    assert float(np.max(np.abs(free.toHost() - ref))) < 1e-12
    free.close()
    sv = qsim.StateVector(n)
    ptr = sv.devicePtr()
    sv.initializeZero()  # (a basis state again, pointer still out)
    sv.run(c, qsim.RunMode.Fused)
    info = sv.layoutInfo()
    assert not info["relayout"] and not info["relabeled"], info
    assert sv.getDeviceMemoryBytes() < 2 * (16 << n)  # one 2^n buffer
    assert float(np.max(np.abs(_read_device(ptr, n) - ref))) < 1e-12  # no devicePtr() call before
    # the raw entry on the held pointer, on the state's stream
    _lib.check(_lib.hip.qsim_apply_hadamard_optimized(ctypes.c_void_p(ptr), n, 17,
                                                      ctypes.c_void_p(sv.stream())))
    sv.synchronize()
    h = qsim.Circuit(n)
    h.h(17)
    ref2 = oracle.run_cpu(n, oracle.gates_of(h), state=ref)
    assert float(np.max(np.abs(sv.toHost() - ref2))) < 1e-12
    # a run from that (non-basis) state, then back to |0..0> and the memoised decision: still in place
    sv.run(c, qsim.RunMode.Fused)
    ref3 = oracle.run_cpu(n, oracle.gates_of(c), state=ref2)
    assert float(np.max(np.abs(_read_device(ptr, n) - ref3))) < 1e-12
    sv.initializeZero()
    sv.run(c, qsim.RunMode.Fused)
    assert not sv.layoutInfo()["relabeled"]
    assert float(np.max(np.abs(_read_device(ptr, n) - ref))) < 1e-12
    assert sv.devicePtr() == ptr


def _hip():
    lib = ctypes.CDLL("libamdhip64.so.7")  # the runtime libqsim_hip.so already loaded
    lib.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    lib.hipFree.argtypes = [ctypes.c_void_p]
    lib.hipMemGetInfo.argtypes = [ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]
    lib.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    lib.hipDeviceSynchronize.argtypes = []
    return lib


def test_relayout_buffer_that_does_not_fit_falls_back(qsim, gpu_ready, jit2):
    """Fill device memory until a second 26-qubit buffer (1 GiB) cannot fit: the first run must
    keep the in-place fixed-layout plan (no relayout, no extra buffer) and equal per-gate.
    Relayout is forced (the calibrated choice at 26 qubits may be a fixed layout either way)."""
    from qsim_amd.plan import set_relayout
    set_relayout(2, -1)
    n = 26
    c = qsim.createRandomHCCircuit(n, 100, 42)
    free_run = qsim.Simulator(n)
    free_run.run(c)
    assert free_run.state.layoutInfo()["relayout"]  # with room, this circuit takes relayout
    state_b = 16 << n
    assert free_run.state.getDeviceMemoryBytes() >= 2 * state_b
    free_run.state.close()
    ref = qsim.Simulator(n, mode=qsim.RunMode.PerGate)
    ref.run(c)
    sim = qsim.Simulator(n)
    assert sim.state.getDeviceMemoryBytes() < 2 * state_b
    ref.synchronize()
    hip = _hip()
    held = []
    try:
        free_b, total_b = ctypes.c_size_t(), ctypes.c_size_t()
        for chunk in (8 << 30, 1 << 30, 64 << 20):
            while True:
                assert hip.hipMemGetInfo(ctypes.byref(free_b), ctypes.byref(total_b)) == 0
                if free_b.value < chunk + (512 << 20):
                    break
                p = ctypes.c_void_p()
                if hip.hipMalloc(ctypes.byref(p), chunk) != 0:
                    break
                held.append(p)
        assert hip.hipMemGetInfo(ctypes.byref(free_b), ctypes.byref(total_b)) == 0
        assert free_b.value < state_b, free_b.value  # a second buffer cannot fit now
        sim.run(c)  # memoised decision says relayout; there is no room: fixed layout in place
        sim.synchronize()
        info = sim.state.layoutInfo()
        assert not info["relayout"], info
        assert sim.state.getDeviceMemoryBytes() < 2 * state_b
        err = sim.state.maxAbsDiff(ref.state)  # (the restore: SWAP network, in place)
        assert err < 1e-12, err
        sim.run(c)  # re-run from the identity layout, still in place
        ref.run(c)
        assert sim.state.maxAbsDiff(ref.state) < 1e-12
    finally:
        for p in held:
            hip.hipFree(p)
