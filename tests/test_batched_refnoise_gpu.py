"""BatchedSimulator under the reference's noise process (QSIM_BATCH_REFERENCE_NOISE; VERDICT r1
"reference-semantics batched noise").

The reference applies, after every gate, one applyBatchedDepolarizingKernel pass per
Depolarizing channel entry: every amplitude PAIR of every trajectory draws its own uniform and,
below p, a second one picks X/Y/Z applied to that pair only (src/NoiseModel.cu:815-892, SURVEY
F5/F7).  The engine runs that process with a counter hash in place of the per-pair curandState;
the oracle restates it with the same hash (oracle/numpy_oracle.py: batched_reference_run), so
the GPU trajectories are compared exactly (1e-12).  cuRAND's own stream is parity-unpinned; the
statistics test checks the process against its closed form.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _circuit(q, n, depth, seed):
    rng = np.random.default_rng(seed)
    c = q.Circuit(n)
    for _ in range(depth):
        a, b, d = (int(x) for x in rng.choice(n, 3, replace=False))
        k = int(rng.integers(0, 9))
        if k < 4:
            (c.x, c.y, c.z, c.h)[k](a)
        elif k == 4:
            c.cnot(a, b)
        elif k == 5:
            c.rx(a, float(rng.uniform(-3, 3)))
        elif k == 6:
            c.cz(a, b)
        elif k == 7:
            c.toffoli(a, b, d)
        else:
            c.swap(a, b)
    return c


def _entries(n, p_dep, p_flip):
    # NoiseModel order: addDepolarizingAll(n, p_dep) then addBitFlip([0, n-1], p_flip)
    return [(0, q, p_dep) for q in range(n)] + [(3, 0, p_flip), (3, n - 1, p_flip)]


@pytest.mark.parametrize("n,B,seed,refgates", [(6, 8, 1, False), (9, 4, 2, True), (11, 3, 3, False)])
def test_reference_noise_matches_oracle(qsim, oracle, gpu_ready, n, B, seed, refgates):
    c = _circuit(qsim, n, 25, seed)
    nm = qsim.NoiseModel()
    nm.addDepolarizingAll(n, 0.15)
    nm.addBitFlip([0, n - 1], 0.3)  # not a Depolarizing channel: the reference ignores it
    s = qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Reference,
                              gate_set=qsim.BatchedGateSet.Reference if refgates
                              else qsim.BatchedGateSet.Full)
    s.setSeed(seed)
    ref, counter = None, 0
    for _ in range(2):  # the second run continues the pass counter
        s.run(c)
        ref, counter = oracle.batched_reference_run(n, B, oracle.gates_of(c), _entries(n, 0.15, 0.3),
                                                    seed, refgates, states=ref, counter=counter)
    for t in range(B):
        np.testing.assert_allclose(s.getStateVector(t), ref[t], atol=1e-12, rtol=0)
    # per-pair flips act on a random subset of pairs: trajectories differ and stay normalised
    # (X/Y/Z on a pair preserve the norm)
    assert abs(np.sum(np.abs(s.getStateVector(0)) ** 2) - 1.0) < 1e-10


def test_reference_noise_statistics(qsim, gpu_ready):
    """n = 1: one pair per trajectory, so the per-pair process equals the channel: after X,
    P(|0>) = 2p/3 (X or Y flips back, Z keeps |1>)."""
    n, B, p = 1, 20000, 0.3
    nm = qsim.NoiseModel()
    nm.addDepolarizing([0], p)
    b = qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Reference)
    b.setSeed(42)
    c = qsim.Circuit(1)
    c.x(0)
    b.run(c)
    avg = b.getAverageProbabilities()
    assert abs(avg[0] - 2 * p / 3) < 0.015


def test_reference_noise_per_pair_subset(qsim, gpu_ready):
    """F7: the reference flips a random SUBSET of pairs — with p = 0.5 on qubit 0 of |+>^n the
    trajectory is no longer a product state, unlike any Pauli-channel realisation."""
    n, B = 8, 4
    nm = qsim.NoiseModel()
    nm.addDepolarizing([0], 0.5)
    c = qsim.Circuit(n)
    for q in range(n):
        c.z(q) if q == 0 else c.h(q)
    b = qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Reference)
    b.setSeed(1)
    b.run(c)
    psi = b.getStateVector(0).reshape(-1, 2)  # row k: the qubit-0 pair (a0, a1) of pair k
    mag = 1 / np.sqrt(psi.shape[0])
    one = np.abs(psi[:, 1]) > 0.5 * mag
    # every pair holds its amplitude on exactly one side, with its magnitude unchanged ...
    np.testing.assert_allclose(np.abs(psi).max(axis=1), mag, atol=1e-12)
    np.testing.assert_allclose(np.abs(psi).min(axis=1), 0, atol=1e-12)
    # ... and which side differs from pair to pair (8 passes at p = 0.5 over 128 pairs)
    assert 0 < np.count_nonzero(one) < psi.shape[0]


def test_reference_compatible_profile_cpp_names(qsim, gpu_ready):
    b = qsim.BatchedSimulator(3, 2)
    b.setReferenceCompatible()
    c = qsim.Circuit(3)
    c.h(0).s(1).cnot(0, 1)  # S ignored by the reference gate set
    b.run(c)
    p = b.getAverageProbabilities()
    np.testing.assert_allclose(p, [0.5, 0, 0, 0.5, 0, 0, 0, 0], atol=1e-12)


@pytest.mark.parametrize("n,B,seed,traj0", [(6, 8, 4, 0), (6, 5, 5, 3), (9, 6, 5, 2), (12, 4, 6, 0), (3, 50, 7, 3)])
def test_reference_noise_one_launch_per_gate(qsim, oracle, gpu_ready, monkeypatch, n, B, seed, traj0):
    """All Depolarizing passes after a gate in ONE launch (k_noise_units: a work-group per unit
    of whole trajectories, channels in order between work-group barriers), forced here at oracle
    sizes (QSIM_NOISE_UNIT_MIN=1), also on a trajectory shard whose pairs start mid-block.
    (The push kernels: the batched default below 12 qubits, the suffix kernel above.)"""
    monkeypatch.setenv("QSIM_NOISE_UNIT_MIN", "1")
    monkeypatch.setenv("QSIM_NOISE_PULL", "0")
    monkeypatch.setenv("QSIM_NOISE_TILE", "0")  # (the push kernels alone, also at 12 qubits)
    c = _circuit(qsim, n, 12, seed)
    nm = qsim.NoiseModel()
    nm.addDepolarizingAll(n, 0.2)
    s = qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Reference)
    s.setSeed(seed)
    s.setTrajectoryOffset(traj0)
    s.run(c)
    entries = [(0, q, 0.2) for q in range(n)]
    whole, _ = oracle.batched_reference_run(n, traj0 + B, oracle.gates_of(c), entries, seed)
    for t in range(B):
        np.testing.assert_allclose(s.getStateVector(t), whole[traj0 + t], atol=1e-12, rtol=0)


def test_reference_noise_one_launch_equals_per_channel_16q(qsim, gpu_ready, monkeypatch):
    """BASELINE config-4 shape (16 qubits, 256 trajectories, depolarizing on every qubit): the
    one-launch path (default at this size) and one launch per channel give identical states."""
    n, B = 16, 256
    c = qsim.createRandomHCCircuit(n, 20, 42)
    nm = qsim.NoiseModel()
    nm.addDepolarizingAll(n, 0.01)
    out = []
    monkeypatch.setenv("QSIM_NOISE_PULL", "0")
    monkeypatch.setenv("QSIM_NOISE_TILE", "0")
    for unit_min in ("128", str(1 << 40)):
        monkeypatch.setenv("QSIM_NOISE_UNIT_MIN", unit_min)
        s = qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Reference)
        s.setSeed(9)
        s.run(c)
        out.append(np.stack([s.getStateVector(t) for t in (0, 77, 255)]))
    assert np.array_equal(out[0], out[1])
    assert abs(np.sum(np.abs(out[0][1]) ** 2) - 1.0) < 1e-10


# ---- pulled noise (noise.hip: k_noise_words + k_pull_gate; opt-in for the batched ensemble,
# QSIM_NOISE_PULL=1 — measured no faster there; NoisySimulator's default) -----------
# The flips after gate i are applied by gate i+1's pass, reading its inputs through the noise
# permutation out of place; the flips after the last gate by one identity pass.  Same draws as
# the push kernels, so the states are the push path's and the oracle's.

@pytest.mark.parametrize("n,B,seed,traj0,refgates", [(9, 6, 5, 2, False), (10, 4, 8, 0, True),
                                                     (12, 3, 6, 5, False), (14, 2, 11, 1, False)])
def test_pulled_noise_matches_oracle(qsim, oracle, gpu_ready, monkeypatch, n, B, seed, traj0, refgates):
    monkeypatch.setenv("QSIM_NOISE_PULL", "1")  # (the batched default is the push kernels)
    c = _circuit(qsim, n, 14, seed)
    nm = qsim.NoiseModel()
    nm.addDepolarizingAll(n, 0.2)
    s = qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Reference,
                              gate_set=qsim.BatchedGateSet.Reference if refgates else qsim.BatchedGateSet.Full)
    s.setSeed(seed)
    s.setTrajectoryOffset(traj0)
    entries = [(0, q, 0.2) for q in range(n)]
    whole, counter = None, 0
    for _ in range(2):  # the second run continues the pass counter from the first's end
        s.run(c)
        whole, counter = oracle.batched_reference_run(n, traj0 + B, oracle.gates_of(c), entries, seed,
                                                      refgates, states=whole, counter=counter)
    for t in range(B):
        np.testing.assert_allclose(s.getStateVector(t), whole[traj0 + t], atol=1e-12, rtol=0)


def test_pulled_noise_equals_push_16q(qsim, gpu_ready, monkeypatch):
    """BASELINE config-4 shape (16 qubits, depolarizing 0.01 on every qubit, W-HC): pulled noise
    (its maps overlapped on a second stream or not) and pushed noise give bit-identical
    trajectories; also through a pinned device pointer."""
    n, B = 16, 128
    c = qsim.createRandomHCCircuit(n, 30, 42)
    nm = qsim.NoiseModel()
    nm.addDepolarizingAll(n, 0.01)
    out = []
    # pulled with the next step's map built on a second stream (the default), pulled on one
    # stream, pushed
    for pull, overlap in (("1", "1"), ("1", "0"), ("0", "1")):
        monkeypatch.setenv("QSIM_NOISE_PULL", pull)
        monkeypatch.setenv("QSIM_NOISE_MAP_OVERLAP", overlap)
        s = qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Reference)
        s.setSeed(9)
        s.run(c)
        s.run(c)
        out.append(np.stack([s.getStateVector(t) for t in (0, 63, 127)]))
        s.close()
    assert np.array_equal(out[0], out[1]) and np.array_equal(out[0], out[2])
    assert abs(np.sum(np.abs(out[0][1]) ** 2) - 1.0) < 1e-10
    # a raw pointer handed out: the pulled run copies its result back where it points
    monkeypatch.setenv("QSIM_NOISE_PULL", "1")
    s = qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Reference)
    s.setSeed(9)
    from qsim_amd import _lib
    import ctypes
    ptr = ctypes.c_void_p()
    _lib.check(_lib.hip.qsim_batch_device_ptr(s._h, ctypes.byref(ptr)))
    s.run(c)
    s.run(c)
    ptr2 = ctypes.c_void_p()
    _lib.check(_lib.hip.qsim_batch_device_ptr(s._h, ctypes.byref(ptr2)))
    assert ptr.value == ptr2.value
    assert np.array_equal(np.stack([s.getStateVector(t) for t in (0, 63, 127)]), out[0])


@pytest.mark.parametrize("n,B,seed,traj0", [(6, 5, 5, 3), (3, 50, 7, 3), (7, 9, 8, 1), (9, 6, 5, 2)])
def test_one_launch_noise_accesses_stay_in_unit(qsim, oracle, gpu_ready, monkeypatch, n, B, seed, traj0):
    """the one-launch kernel (k_noise_units) run range-checked on the device
    (QSIM_NOISE_CHECK=1: every load / store outside the work-group's pairs is counted and fails
    the run) on units whose pairs start and end mid-block (trajectory offsets at n <= 8): no
    violation, flips applied, and the states equal the oracle."""
    import ctypes
    from qsim_amd import _lib
    monkeypatch.setenv("QSIM_NOISE_UNIT_MIN", "1")
    monkeypatch.setenv("QSIM_NOISE_PULL", "0")
    monkeypatch.setenv("QSIM_NOISE_CHECK", "1")
    before = ctypes.c_uint64(0)
    _lib.check(_lib.hip.qsim_noise_check_flips(ctypes.byref(before)))
    c = _circuit(qsim, n, 12, seed)
    nm = qsim.NoiseModel()
    nm.addDepolarizingAll(n, 0.3)
    s = qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Reference)
    s.setSeed(seed)
    s.setTrajectoryOffset(traj0)
    s.run(c)  # raises if any access left its unit
    after = ctypes.c_uint64(0)
    _lib.check(_lib.hip.qsim_noise_check_flips(ctypes.byref(after)))
    assert after.value > before.value
    entries = [(0, q, 0.3) for q in range(n)]
    whole, _ = oracle.batched_reference_run(n, traj0 + B, oracle.gates_of(c), entries, seed)
    for t in range(B):
        np.testing.assert_allclose(s.getStateVector(t), whole[traj0 + t], atol=1e-12, rtol=0)


# ---- gate + in-tile noise (noise.hip: k_gate_noise_tile, the reference process's default from 12
# qubits, round 5) -------------------------------------------------------------------------------
# The gate and the channels whose qubits lie in its 4096-amplitude tile (qubits 0..10 and one
# more) in one LDS pass — the flips composed into per-amplitude code words and every output
# amplitude pulled through them — the remaining channels by the one-launch push kernel: the
# same result as applying the channels in order, so the same states as gate kernel + push.

@pytest.mark.parametrize("n,B,seed,traj0,refgates", [(12, 3, 21, 0, False), (13, 2, 22, 3, True),
                                                     (14, 2, 23, 1, False)])
def test_gate_noise_tile_matches_oracle(qsim, oracle, gpu_ready, monkeypatch, n, B, seed, traj0, refgates):
    monkeypatch.setenv("QSIM_NOISE_TILE", "1")
    c = _circuit(qsim, n, 14, seed)
    nm = qsim.NoiseModel()
    nm.addDepolarizingAll(n, 0.2)
    nm.addDepolarizing([0, 11], 0.3)  # (repeated qubits: a longer prefix than the tile's qubits)
    s = qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Reference,
                              gate_set=qsim.BatchedGateSet.Reference if refgates else qsim.BatchedGateSet.Full)
    s.setSeed(seed)
    s.setTrajectoryOffset(traj0)
    entries = [(0, q, 0.2) for q in range(n)] + [(0, 0, 0.3), (0, 11, 0.3)]
    whole, counter = None, 0
    for _ in range(2):
        s.run(c)
        whole, counter = oracle.batched_reference_run(n, traj0 + B, oracle.gates_of(c), entries, seed,
                                                      refgates, states=whole, counter=counter)
    for t in range(B):
        np.testing.assert_allclose(s.getStateVector(t), whole[traj0 + t], atol=1e-12, rtol=0)


@pytest.mark.parametrize("p", [0.5, 0.05])
def test_gate_noise_tile_dense_flips_match_oracle(qsim, oracle, gpu_ready, monkeypatch, p):
    """Flip densities where most code words hold several fields (p = 0.5: a pair flips on most
    channels, so the pulled walk moves through up to 12 partners), X / Y / Z channels mixed with
    depolarizing ones on repeated qubits, controlled gates with controls in and out of the tile."""
    monkeypatch.setenv("QSIM_NOISE_TILE", "1")
    n, B, seed = 13, 2, 31
    c = _circuit(qsim, n, 16, seed)
    c.cnot(12, 3).toffoli(12, 1, 5).cz(2, 12).swap(4, 12)
    nm = qsim.NoiseModel()
    nm.addDepolarizingAll(n, p)
    s = qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Reference)
    s.setSeed(seed)
    entries = [(0, q, p) for q in range(n)]
    whole, _ = oracle.batched_reference_run(n, B, oracle.gates_of(c), entries, seed)
    s.run(c)
    for t in range(B):
        np.testing.assert_allclose(s.getStateVector(t), whole[t], atol=1e-12, rtol=0)


@pytest.mark.parametrize("lists,cap", [("1", "0"), ("1", "8"), ("0", "0")])
def test_gate_noise_tile_lists_match_oracle(qsim, oracle, gpu_ready, monkeypatch, lists, cap):
    """The flip lists built on the second stream one step ahead (k_gn_lists), at their natural
    capacity, with a capacity of 8 (most lists overflow: the tile kernel walks the rest of those
    blocks itself), and without lists; two runs (the list sets alternate across the run boundary),
    a trajectory offset, a non-depolarizing flip channel in the prefix."""
    monkeypatch.setenv("QSIM_NOISE_TILE", "1")
    monkeypatch.setenv("QSIM_NOISE_TILE_LISTS", lists)
    if cap != "0":
        monkeypatch.setenv("QSIM_NOISE_LIST_CAP", cap)
    n, B, seed, traj0, p = 13, 3, 41, 2, 0.03
    c = _circuit(qsim, n, 15, seed)
    nm = qsim.NoiseModel()
    nm.addDepolarizingAll(n, p)
    s = qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Reference)
    s.setSeed(seed)
    s.setTrajectoryOffset(traj0)
    entries = [(0, q, p) for q in range(n)]
    whole, counter = None, 0
    for _ in range(2):
        s.run(c)
        whole, counter = oracle.batched_reference_run(n, traj0 + B, oracle.gates_of(c), entries, seed,
                                                      False, states=whole, counter=counter)
    for t in range(B):
        np.testing.assert_allclose(s.getStateVector(t), whole[traj0 + t], atol=1e-12, rtol=0)


def test_gate_noise_tile_equals_push_16q(qsim, gpu_ready, monkeypatch):
    """Config-4 shape (16 qubits, depolarizing 0.01 on every qubit, W-HC and the mixed gate
    set): the tile kernel and gate kernel + push give bit-identical trajectories."""
    n, B = 16, 64
    nm = qsim.NoiseModel()
    nm.addDepolarizingAll(n, 0.01)
    for c in (qsim.createRandomHCCircuit(n, 30, 42), _circuit(qsim, n, 30, 5)):
        out = []
        for tile in ("1", "0"):
            monkeypatch.setenv("QSIM_NOISE_TILE", tile)
            s = qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Reference)
            s.setSeed(9)
            s.run(c)
            s.run(c)
            out.append(np.stack([s.getStateVector(t) for t in (0, 31, 63)]))
            s.close()
        assert np.array_equal(out[0], out[1])


@pytest.mark.parametrize("k", ["2", "3"])
def test_gate_noise_tile_split_parts_equal_one_part(qsim, oracle, gpu_ready, monkeypatch, k):
    """QSIM_NOISE_SPLIT=k (default 2): the in-tile run as k trajectory parts on k streams gives the
    one-part run's trajectories bit for bit (draws keyed by the global pair index), over two runs."""
    n, B = 13, 7
    nm = qsim.NoiseModel()
    nm.addDepolarizingAll(n, 0.03)
    c = _circuit(qsim, n, 20, 17)
    out = []
    for split in ("1", k):
        monkeypatch.setenv("QSIM_NOISE_SPLIT", split)
        s = qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Reference)
        s.setSeed(17)
        s.run(c)
        s.run(c)
        out.append(np.stack([s.getStateVector(t) for t in range(B)]))
        s.close()
    assert np.array_equal(out[0], out[1])
    entries = [(0, q, 0.03) for q in range(n)]
    whole, counter = None, 0
    for _ in range(2):
        whole, counter = oracle.batched_reference_run(n, B, oracle.gates_of(c), entries, 17, False,
                                                      states=whole, counter=counter)
    np.testing.assert_allclose(out[1], whole, atol=1e-12, rtol=0)


@pytest.mark.parametrize("p", [0.01, 0.3, 1e-4, 0.9])
def test_single_precision_gap_draws_equal_double(qsim, gpu_ready, monkeypatch, p):
    """noise.hip next_flip takes each geometric gap from the hardware single-precision log2 unless
    the value lies within its error bound of an integer (then the double log): the trajectories
    equal the all-double walks bit for bit (QSIM_NOISE_FAST_LOG=0) — millions of draws at config-4
    shape, the in-tile lists, the pushed suffix and the pulled NoisySimulator words alike."""
    n, B = 16, 64
    nm = qsim.NoiseModel()
    nm.addDepolarizingAll(n, p)
    c = qsim.createRandomHCCircuit(n, 30, 7)
    out = []
    for fast in ("1", "0"):
        monkeypatch.setenv("QSIM_NOISE_FAST_LOG", fast)
        s = qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Reference)
        s.setSeed(11)
        s.run(c)
        out.append(np.stack([s.getStateVector(t) for t in (0, 17, 40, 63)]))
        s.close()
    assert np.array_equal(out[0], out[1])
    m = 20
    nm2 = qsim.NoiseModel()
    nm2.addDepolarizingAll(m, p)
    c2 = qsim.createRandomHCCircuit(m, 20, 8)
    got = []
    for fast in ("1", "0"):
        monkeypatch.setenv("QSIM_NOISE_FAST_LOG", fast)
        sim = qsim.NoisySimulator(m, nm2)
        sim.setSeed(5)
        sim.run(c2)
        got.append(sim.getStateVector())
        del sim
    assert np.array_equal(got[0], got[1])


@pytest.mark.gpu
@pytest.mark.parametrize("p", [0.01, 0.001, 1e-5, 0.05, 0.3, 0.75, 0.99])
def test_single_precision_gaps_never_differ(qsim, gpu_ready, p):
    """noise.hip flip_gap over 2^26 draws per probability: the single-precision-first gap equals
    floor(ln u / ln(1 - P)) in double every time (its error bound holds), and the double fallback
    stays rare (< 1 % of draws)."""
    import ctypes
    from qsim_amd import _lib
    mm, fb = ctypes.c_uint64(), ctypes.c_uint64()
    draws = 1 << 26
    _lib.check(_lib.hip.qsim_noise_gap_check(p, draws, 0x5eed + int(p * 1e6), ctypes.byref(mm), ctypes.byref(fb)))
    assert mm.value == 0
    assert fb.value < draws // 100


@pytest.mark.gpu
@pytest.mark.parametrize("p", [0.01, 0.001, 1e-5, 0.05, 0.3, 0.75, 0.99])
def test_single_precision_gaps_at_every_boundary(qsim, gpu_ready, p):
    """the targeted form of the check above — 2 x 4096 consecutive u values around every
    integer boundary of the gap up to the block (u_m = exp(m ln(1 - P)), m = 0..256) and around both
    ends of the float-rounding interval of u_m, where the single-precision try sees one input while
    the double answer changes: no draw may differ from the double formula."""
    import ctypes
    from qsim_amd import _lib
    mm, fb, dr = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    _lib.check(_lib.hip.qsim_noise_gap_check_edges(p, 4096, ctypes.byref(mm), ctypes.byref(fb), ctypes.byref(dr)))
    assert dr.value >= 3 * 8192  # (at least the m = 0 boundary; small p has all 257)
    assert mm.value == 0, (mm.value, fb.value, dr.value)
    assert fb.value > 0  # (the sweep reaches the undecidable draws: it is where the bound matters)
