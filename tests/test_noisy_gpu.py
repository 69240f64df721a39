"""NoisySimulator (reference include/NoiseModel.cuh:139-214, src/NoiseModel.cu:115-651) on the HIP
noise passes (csrc/hip/noise.hip).

* Exact: the engine's per-pair noise passes equal the oracle's restatement of the reference
  kernels (oracle/numpy_oracle.py noise_pass: per-pair draws, per-pair damping renormalisation)
  driven by the same counter hash, for every channel type, at 1e-12.
* The reference's own tests (tests/test_noise.cu:62-231, 345-447): zero-probability noise,
  bit flip p=1 undoing X, phase flip keeping probabilities, amplitude-damping statistics, high
  noise varying outcomes, same seed = same result.  cuRAND realisations are parity-unpinned.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _model(q, channels):
    nm = q.NoiseModel()
    adders = [nm.addDepolarizing, nm.addAmplitudeDamping, nm.addPhaseDamping, nm.addBitFlip,
              nm.addPhaseFlip, nm.addBitPhaseFlip]
    for t, qb, p in channels:
        adders[t]([qb], p)
    return nm


@pytest.mark.parametrize("n,seed", [(3, 1), (8, 2), (13, 3)])
def test_noise_passes_match_oracle(qsim, oracle, gpu_ready, n, seed):
    rng = np.random.default_rng(seed)
    c = qsim.createRandomCircuit(n, 12, seed)
    channels = [(int(t), int(rng.integers(0, n)), float(p))
                for t, p in zip(range(6), (0.3, 0.4, 0.35, 0.25, 0.5, 0.45))]
    sim = qsim.NoisySimulator(n, _model(qsim, channels))
    sim.setSeed(1000 + seed)
    sim.run(c)
    want, ctr = oracle.noisy_run(n, oracle.gates_of(c), channels, 1000 + seed)
    np.testing.assert_allclose(sim.getStateVector(), want, atol=1e-12, rtol=0)
    # a second run continues the noise stream (counter), like the reference's curand states
    sim.run(c)
    want2, _ = oracle.noisy_run(n, oracle.gates_of(c), channels, 1000 + seed, ctr, want)
    np.testing.assert_allclose(sim.getStateVector(), want2, atol=1e-12, rtol=0)


def test_apply_noise_to_qubit_matches_oracle(qsim, oracle, gpu_ready):
    n = 6
    sim = qsim.NoisySimulator(n)
    sim.setSeed(77)
    sim.run(qsim.createGHZCircuit(n))
    s = sim.getStateVector()
    for k, (t, qb, p) in enumerate([(0, 2, 0.6), (3, 5, 0.5), (1, 0, 0.7), (2, 4, 0.9)]):
        sim.applyNoiseToQubit(qsim.NoiseType(t), qb, p)
        s = oracle.noise_pass(s, n, t, qb, p, 77, k)
    np.testing.assert_allclose(sim.getStateVector(), s, atol=1e-12, rtol=0)


def test_reference_noise_suite(qsim, gpu_ready):
    NT = qsim.NoiseType
    # ZeroProbabilityNoEffect (:106-122)
    nm = qsim.NoiseModel()
    nm.addDepolarizing([0], 0.0)
    sim = qsim.NoisySimulator(2, nm)
    sim.setSeed(42)
    sim.run(qsim.createBellCircuit())
    p = sim.getProbabilities()
    assert abs(p[0] - 0.5) < 1e-10 and abs(p[3] - 0.5) < 1e-10
    # BitFlipAffectsState (:157-179): X then certain bit flip = |0>
    nm = qsim.NoiseModel()
    nm.addBitFlip([0], 1.0)
    sim = qsim.NoisySimulator(1, nm)
    c = qsim.Circuit(1)
    c.x(0)
    sim.run(c)
    assert abs(sim.getProbabilities()[0] - 1.0) < 1e-10
    # PhaseFlipDoesNotChangeComputationalBasis (:185-200)
    nm = qsim.NoiseModel()
    nm.addPhaseFlip([0], 1.0)
    sim = qsim.NoisySimulator(1, nm)
    sim.run(c)
    assert abs(sim.getProbabilities()[1] - 1.0) < 1e-10
    assert abs(sim.getStateVector()[1] + 1.0) < 1e-12  # Z|1> = -|1>
    # AmplitudeDampingDecayTowardGround (:206-231)
    nm = qsim.NoiseModel()
    nm.addAmplitudeDamping([0], 0.5)
    ground = 0
    for i in range(100):
        sim = qsim.NoisySimulator(1, nm)
        sim.setSeed(i)
        sim.run(c)
        ground += int(sim.sample(1)[0] == 0)
    assert 0 < ground < 100
    assert 30 < ground < 70  # P(decay) = |a1|^2 * gamma = 0.5
    # HighNoiseDestroysSuperposition (:124-151)
    nm = qsim.NoiseModel()
    nm.addDepolarizingAll(2, 0.5)
    counts = set()
    sim = qsim.NoisySimulator(2, nm)
    h = qsim.Circuit(2)
    h.h(0)
    for i in range(100):
        sim.reset()
        sim.setSeed(i)
        sim.run(h)
        counts.add(int(sim.sample(1)[0]))
    assert len(counts) > 1
    # SameSeedSameResults (:345-377)
    nm = qsim.NoiseModel()
    nm.addDepolarizing([0, 1], 0.1)
    runs = []
    for _ in range(2):
        sim = qsim.NoisySimulator(2, nm)
        sim.setSeed(12345)
        sim.run(qsim.createBellCircuit())
        runs.append(sim.getProbabilities())
    assert np.array_equal(runs[0], runs[1])
    # global channels act on no qubit (F6): same as ideal
    nm = qsim.NoiseModel()
    nm.addDepolarizing(0.9)
    sim = qsim.NoisySimulator(2, nm)
    sim.run(qsim.createBellCircuit())
    assert abs(sim.getProbabilities()[3] - 0.5) < 1e-12


def test_depolarizing_statistics(qsim, gpu_ready):
    """P(|1>) after depolarizing p on |0>: X or Y fire with probability 2p/3 (per pair draw)."""
    nm = qsim.NoiseModel()
    nm.addDepolarizing([0], 0.3)
    ones = 0
    trials = 600
    sim = qsim.NoisySimulator(1, nm)
    c = qsim.Circuit(1)
    c.z(0)
    for i in range(trials):
        sim.reset()
        sim.setSeed(i)
        sim.run(c)
        ones += int(sim.getProbabilities()[1] > 0.5)
    assert abs(ones / trials - 0.2) < 0.05


def test_noise_free_run_is_fused_and_exact(qsim, oracle, gpu_ready):
    n = 12
    c = qsim.createRandomCircuit(n, 200, 5)
    sim = qsim.NoisySimulator(n)
    sim.run(c)
    np.testing.assert_allclose(sim.getStateVector(), oracle.run_cpu(n, oracle.gates_of(c)),
                               atol=1e-12, rtol=0)
    with pytest.raises(IndexError):
        sim.applyNoiseToQubit(qsim.NoiseType.BitFlip, n, 0.5)


@pytest.mark.parametrize("mode", ["fused", "overlap", "serial"])
@pytest.mark.parametrize("n,seed,types", [(10, 4, (0, 3, 4, 5)), (12, 5, (0, 0, 5, 3)), (11, 6, (0, 1, 3)),
                                          (9, 7, (0,) * 20), (13, 8, (0,) * 18)])
def test_pulled_flip_noise_matches_oracle(qsim, oracle, gpu_ready, monkeypatch, n, seed, types, mode):
    """From 9 qubits, flip-only noise models run pulled (the noise after gate i applied by gate
    i+1's pass, out of place; noise.hip) — exactly the oracle's per-pair passes, with the next
    step's code words built on a second stream (the default), before the pass, or by the pass
    itself (fused, opt-in), and with > 16 channel entries (64-bit words, fourth and fifth cases).  A damping
    channel in the model keeps the per-channel passes (third)."""
    monkeypatch.setenv("QSIM_NOISE_MAP_FUSED", "1" if mode == "fused" else "0")
    monkeypatch.setenv("QSIM_NOISE_MAP_OVERLAP", "1" if mode == "overlap" else "0")
    monkeypatch.setenv("QSIM_NOISY_TILE", "0")  # (the default; the in-tile path is opt-in)
    rng = np.random.default_rng(seed)
    c = qsim.createRandomCircuit(n, 16, seed)
    channels = [(int(t), int(rng.integers(0, n)), float(rng.uniform(0.1, 0.5))) for t in types]
    sim = qsim.NoisySimulator(n, _model(qsim, channels))
    sim.setSeed(2000 + seed)
    sim.run(c)
    want, ctr = oracle.noisy_run(n, oracle.gates_of(c), channels, 2000 + seed)
    np.testing.assert_allclose(sim.getStateVector(), want, atol=1e-12, rtol=0)
    sim.run(c)
    want2, _ = oracle.noisy_run(n, oracle.gates_of(c), channels, 2000 + seed, ctr, want)
    np.testing.assert_allclose(sim.getStateVector(), want2, atol=1e-12, rtol=0)


def _read_device(ptr, n):
    """The 2^n complex amplitudes at a raw device pointer (hipMemcpy D2H via the loaded runtime)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    hip.hipDeviceSynchronize.argtypes = []
    out = np.empty(1 << n, dtype=np.complex128)
    assert hip.hipDeviceSynchronize() == 0
    assert hip.hipMemcpy(out.ctypes.data, ctypes.c_void_p(ptr), out.nbytes, 2) == 0  # D2H
    return out


@pytest.mark.parametrize("tile", ["0", "1"])
@pytest.mark.parametrize("keep", ["1", "0"])
def test_pulled_noise_on_a_pinned_pointer(qsim, oracle, gpu_ready, monkeypatch, keep, tile):
    """an unpinned pulled run with an odd gate count leaves the amplitudes in
    the second buffer; devicePtr() then hands that buffer out.  The next pulled runs must leave
    their result where that pointer points (odd and even gate counts), never free it, and the
    pointer must equal getStateVector and the oracle.  keep=0 frees the noise buffers after every
    run (the low-memory branch), keep=1 keeps them."""
    monkeypatch.setenv("QSIM_NOISE_KEEP_BUFFERS", keep)
    monkeypatch.setenv("QSIM_NOISY_TILE", tile)  # (tile = 1: the in-tile path, in place)
    n, seed = 12, 9
    channels = [(0, q, 0.2) for q in range(n)]
    c_odd = qsim.createRandomCircuit(n, 15, seed)
    c_even = qsim.createRandomCircuit(n, 16, seed + 1)
    assert len(c_odd.getGates()) % 2 == 1 and len(c_even.getGates()) % 2 == 0
    sim = qsim.NoisySimulator(n, _model(qsim, channels))
    sim.setSeed(77)
    sim.run(c_odd)
    want, ctr = oracle.noisy_run(n, oracle.gates_of(c_odd), channels, 77)
    ptr = sim.state.devicePtr()
    np.testing.assert_allclose(_read_device(ptr, n), want, atol=1e-12, rtol=0)
    for c in (c_odd, c_even, c_odd):
        sim.run(c)
        want, ctr = oracle.noisy_run(n, oracle.gates_of(c), channels, 77, ctr, want)
        np.testing.assert_allclose(_read_device(ptr, n), want, atol=1e-12, rtol=0)
        np.testing.assert_allclose(sim.getStateVector(), want, atol=1e-12, rtol=0)
    assert sim.state.devicePtr() == ptr
    # a basis-state fused run (the path that used to release the second buffer) keeps the pointer
    sim.state.initializeZero()
    c = qsim.createRandomHCCircuit(n, 40, 3)
    sim.state.run(c, qsim.RunMode.Fused)
    np.testing.assert_allclose(_read_device(ptr, n), oracle.run_cpu(n, oracle.gates_of(c)), atol=1e-12, rtol=0)


@pytest.mark.parametrize("lists", ["1", "0"])
@pytest.mark.parametrize("n,seed,types,p", [(12, 11, (0,) * 12, 0.05), (13, 12, (0, 3, 4, 5, 0, 3), 0.3),
                                            (14, 13, (0,) * 14, 0.01)])
def test_tile_noise_matches_oracle(qsim, oracle, gpu_ready, monkeypatch, lists, n, seed, types, p):
    """QSIM_NOISY_TILE=1: from 12 qubits flip-only models run through the in-tile path (noise.hip
    launch_gate_noise_run: the gate and the channel prefix inside its 4096-amplitude tile in one LDS
    pass, flips from per-step lists built on the noise stream, the rest pushed per channel) —
    exactly the oracle's per-pair passes, two runs (the counter continues), lists on and off."""
    monkeypatch.setenv("QSIM_NOISE_TILE_LISTS", lists)
    monkeypatch.setenv("QSIM_NOISY_TILE", "1")
    rng = np.random.default_rng(seed)
    c = qsim.createRandomCircuit(n, 24, seed)
    c.cnot(n - 1, 2).swap(3, n - 2).cz(0, n - 1)
    channels = [(int(t), int(q), p) for t, q in zip(types, rng.permutation(n))]
    sim = qsim.NoisySimulator(n, _model(qsim, channels))
    sim.setSeed(3000 + seed)
    sim.run(c)
    want, ctr = oracle.noisy_run(n, oracle.gates_of(c), channels, 3000 + seed)
    np.testing.assert_allclose(sim.getStateVector(), want, atol=1e-12, rtol=0)
    sim.run(c)
    want2, _ = oracle.noisy_run(n, oracle.gates_of(c), channels, 3000 + seed, ctr, want)
    np.testing.assert_allclose(sim.getStateVector(), want2, atol=1e-12, rtol=0)


@pytest.mark.parametrize("n,seed,p", [(12, 21, 0.3), (14, 22, 0.05), (16, 23, 0.01)])
def test_pull_chains_match_oracle(qsim, oracle, gpu_ready, monkeypatch, n, seed, p):
    """The pulled pass (k_pull_gate, sparse words) against the oracle with channels on every qubit
    (X / Y / Z / depolarizing; p = 0.3: long chains through partners, overflow words), a repeated
    channel, gates on qubit 11 and above, controls above the low qubits, SWAPs of two high qubits,
    two runs.  (Round 6 also ran a tile form of this pass — in-tile partners from LDS, the gate in
    LDS — through this test, 0.71 against 0.61 ms at 26 qubits: not kept)"""
    monkeypatch.setenv("QSIM_NOISY_TILE", "0")
    c = qsim.createRandomCircuit(n, 20, seed)
    c.cnot(n - 1, 2).swap(3, n - 2).swap(n - 1, n - 2).cz(0, n - 1).toffoli(n - 1, n - 2, 4)
    c.rx(n - 3, 0.4).h(11).cnot(5, 11)
    if n > 12:
        c.cnot(11, n - 1).swap(11, n - 1)
    types = (0, 3, 4, 5)
    channels = [(types[q % 4], q, p) for q in range(n)] + [(0, n - 1, p), (3, 0, p)]
    sim = qsim.NoisySimulator(n, _model(qsim, channels))
    sim.setSeed(4000 + seed)
    sim.run(c)
    want, ctr = oracle.noisy_run(n, oracle.gates_of(c), channels, 4000 + seed)
    np.testing.assert_allclose(sim.getStateVector(), want, atol=1e-12, rtol=0)
    sim.run(c)
    want2, _ = oracle.noisy_run(n, oracle.gates_of(c), channels, 4000 + seed, ctr, want)
    np.testing.assert_allclose(sim.getStateVector(), want2, atol=1e-12, rtol=0)
