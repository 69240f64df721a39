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


@pytest.mark.parametrize("overlap", ["1", "0"])
@pytest.mark.parametrize("n,seed,types", [(10, 4, (0, 3, 4, 5)), (12, 5, (0, 0, 5, 3)), (11, 6, (0, 1, 3)),
                                          (9, 7, (0,) * 20)])
def test_pulled_flip_noise_matches_oracle(qsim, oracle, gpu_ready, monkeypatch, n, seed, types, overlap):
    """From 9 qubits, flip-only noise models run pulled (the noise after gate i applied by gate
    i+1's pass, out of place; noise.hip) — exactly the oracle's per-pair passes, with the next
    step's code words built on a second stream or not, and with > 16 channel entries (64-bit
    words, fourth case).  A damping channel in the model keeps the per-channel passes (third)."""
    monkeypatch.setenv("QSIM_NOISE_MAP_OVERLAP", overlap)
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
