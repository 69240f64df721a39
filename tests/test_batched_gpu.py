"""Batched trajectories on fused tile passes (batched.hip + fused.hip): the Pauli-frame execution
must give exactly the trajectories of the per-gate execution (one kernel per gate and one Pauli
pass per noisy step — the reference's structure, src/NoiseModel.cu:815-892) for the same seed,
and noise-free trajectories must equal the oracle state."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _mixed(q, n, depth, seed, gateset="full"):
    rng = np.random.default_rng(seed)
    c = q.Circuit(n)
    for _ in range(depth):
        a, b, d = (int(x) for x in rng.choice(n, 3, replace=False))
        th = float(rng.uniform(-3.0, 3.0))
        k = int(rng.integers(0, 6 if gateset == "reference" else 17))
        if gateset == "reference":
            (c.x, c.y, c.z, c.h)[k](a) if k < 4 else c.cnot(a, b)
            continue
        if k < 8:
            getattr(c, ("x", "y", "z", "h", "s", "t", "sdag", "tdag")[k])(a)
        elif k < 11:
            getattr(c, ("rx", "ry", "rz")[k - 8])(a, th)
        elif k == 11:
            c.cnot(a, b)
        elif k == 12:
            c.cz(a, b)
        elif k == 13:
            c.cry(a, b, th)
        elif k == 14:
            c.crz(a, b, th)
        elif k == 15:
            c.swap(a, b)
        else:
            c.toffoli(a, b, d)
    return c


def _noise(q, n):
    nm = q.NoiseModel()
    nm.addDepolarizingAll(n, 0.12)
    nm.addBitFlip([0, n - 1], 0.2)
    nm.addPhaseFlip([1, n // 2], 0.2)
    nm.addBitPhaseFlip([2, n - 2], 0.1)
    return nm


@pytest.mark.parametrize("n,B,seed", [(10, 8, 1), (12, 16, 2), (13, 4, 3)])
def test_frames_equal_per_gate(qsim, gpu_ready, n, B, seed):
    c = _mixed(qsim, n, 60, seed)
    nm = _noise(qsim, n)
    fused, ref = qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Physical), qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Physical)
    fused.setSeed(seed)
    ref.setSeed(seed)
    for _ in range(2):  # the second run continues the noise stream (step counter)
        fused.run(c)
        ref.run(c, per_gate=True)
    for t in range(B):
        np.testing.assert_allclose(fused.getStateVector(t), ref.getStateVector(t), atol=1e-12, rtol=0)
    avg = fused.getAverageProbabilities()
    assert abs(avg.sum() - 1.0) < 1e-10


def test_carried_frames_through_mixed_runs(qsim, gpu_ready):
    """A fused noisy run leaves its Pauli frames unmaterialised: the next fused run composes them
    (also a noise-free one, whose non-Clifford gates are then conjugated by the carried frame),
    a per-gate run and every reader materialise them first, and sync() does too.  Against the
    per-gate execution (one Pauli pass per step) with the same seed."""
    n, B = 11, 6
    c1, c2 = _mixed(qsim, n, 40, 11), _mixed(qsim, n, 30, 12)
    nm, quiet = _noise(qsim, n), qsim.NoiseModel()
    fused, ref = qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Physical), qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Physical)
    for s in (fused, ref):
        s.setSeed(5)
    fused.run(c1)
    ref.run(c1, per_gate=True)
    for s in (fused, ref):
        s.setNoiseModel(quiet)
    fused.run(c2)  # noise-free, carried frame
    ref.run(c2, per_gate=True)
    for s in (fused, ref):
        s.setNoiseModel(nm)
    fused.run(c1, per_gate=True)  # per-gate run: materialises first
    ref.run(c1, per_gate=True)
    fused.run(c2)
    ref.run(c2, per_gate=True)
    fused.synchronize()
    fused.run(c1)
    ref.run(c1, per_gate=True)
    for t in range(B):
        np.testing.assert_allclose(fused.getStateVector(t), ref.getStateVector(t), atol=1e-12, rtol=0)
    np.testing.assert_allclose(fused.getAverageProbabilities(), ref.getAverageProbabilities(),
                               atol=1e-12, rtol=0)


def test_frames_reference_gateset(qsim, gpu_ready):
    n, B = 11, 8
    c = _mixed(qsim, n, 80, 7)
    c.rz(3, 0.4)  # ignored by the reference gate set, still followed by noise
    nm = _noise(qsim, n)
    out = []
    for per_gate in (False, True):
        s = qsim.BatchedSimulator(n, B, nm, gate_set=qsim.BatchedGateSet.Reference, noise=qsim.BatchedNoise.Physical)
        s.setSeed(5)
        s.run(c, per_gate=per_gate)
        out.append([s.getStateVector(t) for t in range(B)])
    for a, b in zip(*out):
        np.testing.assert_allclose(a, b, atol=1e-12, rtol=0)


def test_noise_free_fused_batch_matches_oracle(qsim, oracle, gpu_ready):
    n, B = 12, 6
    c = _mixed(qsim, n, 150, 11)
    s = qsim.BatchedSimulator(n, B)
    s.run(c)
    ref = oracle.run_cpu(n, oracle.gates_of(c))
    for t in range(B):
        np.testing.assert_allclose(s.getStateVector(t), ref, atol=1e-12, rtol=0)


def test_frames_noise_actually_applied(qsim, gpu_ready):
    """With p = 1 bit flips on qubit 0 after every gate the trajectories are deterministic."""
    n, B = 10, 4
    c = qsim.Circuit(n)
    c.h(3).cnot(3, 5).x(7)  # 3 gates -> 3 flips of qubit 0 -> net X on qubit 0
    nm = qsim.NoiseModel()
    nm.addBitFlip([0], 1.0)
    s = qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Physical)
    s.run(c)
    ideal = qsim.Simulator(n)
    ideal.run(c)
    ideal.applyGate(qsim.GateOp(qsim.GateType.X, [0]))
    for t in range(B):
        np.testing.assert_allclose(s.getStateVector(t), ideal.getStateVector(), atol=1e-12, rtol=0)


# ---- BASELINE config 4: 16 qubits x 1024 trajectories ("config 4 has no GPU test")
def test_config4_noise_free_matches_oracle(qsim, oracle, gpu_ready):
    """16q x 1024 trajectories (1 GiB of states), W-HC depth 100: a fixed sample of 64
    trajectories (first, last and 62 spread between) equals the oracle state at 1e-12."""
    n, B = 16, 1024
    c = qsim.createRandomHCCircuit(n, 100, 42)
    s = qsim.BatchedSimulator(n, B)
    s.run(c)
    ref = oracle.run_cpu(n, oracle.gates_of(c))
    for t in sorted({0, B - 1, *np.linspace(0, B - 1, 62).astype(int).tolist()}):
        np.testing.assert_allclose(s.getStateVector(t), ref, atol=1e-12, rtol=0)
    np.testing.assert_allclose(s.getAverageProbabilities(), np.abs(ref) ** 2, atol=1e-12)


def test_config4_noisy_frames_equal_per_gate(qsim, gpu_ready):
    """16q, depolarizing 0.01 on every qubit after every gate (W-BATCH's noise), 64 trajectories:
    the fused Pauli-frame execution == one kernel per gate + one Pauli pass per step."""
    n, B = 16, 64
    c = qsim.createRandomHCCircuit(n, 100, 42)
    nm = qsim.NoiseModel()
    nm.addDepolarizingAll(n, 0.01)
    fused, ref = qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Physical), qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Physical)
    fused.setSeed(42)
    ref.setSeed(42)
    fused.run(c)
    ref.run(c, per_gate=True)
    differ = 0
    ideal = qsim.BatchedSimulator(n, 1)
    ideal.run(c)
    psi = ideal.getStateVector(0)
    for t in range(B):
        a = fused.getStateVector(t)
        np.testing.assert_allclose(a, ref.getStateVector(t), atol=1e-12, rtol=0)
        differ += np.max(np.abs(a - psi)) > 1e-9
    # 16 x 100 channels at p = 0.01: a trajectory stays error-free with prob ~1e-7
    assert differ >= B - 2


def test_config4_full_size_noisy_run(qsim, gpu_ready):
    """The W-BATCH configuration itself (16q x 1024, depolarizing 0.01 everywhere): every
    trajectory stays normalised and the average distribution is a distribution."""
    n, B = 16, 1024
    c = qsim.createRandomHCCircuit(n, 100, 42)
    nm = qsim.NoiseModel()
    nm.addDepolarizingAll(n, 0.01)
    s = qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Physical)
    s.setSeed(42)
    s.run(c)
    avg = s.getAverageProbabilities()
    assert abs(avg.sum() - 1.0) < 1e-10 and avg.min() >= 0
    for t in (0, 511, 1023):
        assert abs(np.sum(np.abs(s.getStateVector(t)) ** 2) - 1.0) < 1e-10
    h = s.getHistogram(4)
    assert h.sum() == 4 * B


@pytest.mark.parametrize("noise", ["physical", "reference"])
@pytest.mark.parametrize("per_gate", [False, True])
def test_trajectory_shards_reproduce_the_ensemble(qsim, gpu_ready, noise, per_gate):
    """BatchedSimulator shards by trajectory.  G objects of B/G trajectories with
    offsets 0, B/G, ... and the same seed hold exactly the trajectories of one B-trajectory
    object (noise draws keyed by the global trajectory index), over two runs."""
    n, B, G = 12, 8, 4
    c = _mixed(qsim, n, 50, 9)
    nm = _noise(qsim, n)
    sem = qsim.BatchedNoise.Reference if noise == "reference" else qsim.BatchedNoise.Physical
    full = qsim.BatchedSimulator(n, B, nm, noise=sem)
    full.setSeed(21)
    shards = []
    for r in range(G):
        s = qsim.BatchedSimulator(n, B // G, nm, noise=sem)
        s.setSeed(21)
        s.setTrajectoryOffset(r * (B // G))
        shards.append(s)
    for _ in range(2):
        full.run(c, per_gate=per_gate)
        for s in shards:
            s.run(c, per_gate=per_gate)
    avg = np.zeros(1 << n)
    for r, s in enumerate(shards):
        for t in range(B // G):
            np.testing.assert_array_equal(s.getStateVector(t), full.getStateVector(r * (B // G) + t))
        avg += s.getAverageProbabilities() * (B // G) / B
    np.testing.assert_allclose(avg, full.getAverageProbabilities(), atol=1e-14, rtol=0)
    # the draws really differ between trajectories (the offset is not a no-op)
    assert any(np.max(np.abs(full.getStateVector(0) - full.getStateVector(t))) > 1e-6 for t in range(1, B))


@pytest.mark.parametrize("n,B", [(12, 16), (14, 8)])
def test_relabeled_batch_equals_per_gate(qsim, gpu_ready, n, B):
    """Layout-aware relabeling of the trajectories' qubits (first fused run of |0..0>, threshold
    lowered here): noise draws are keyed by channel index, so the relabeled fused run holds the
    same trajectories as the per-gate run (which never relabels), through two runs, every
    trajectory readout and the ensemble average."""
    from qsim_amd.plan import set_relabel
    c = _mixed(qsim, n, 60, 4)
    nm = _noise(qsim, n)
    set_relabel(1, 14)
    try:
        fused, ref = qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Physical), qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Physical)
        fused.setSeed(8)
        ref.setSeed(8)
        for _ in range(2):
            fused.run(c)
            ref.run(c, per_gate=True)
        np.testing.assert_allclose(fused.getAverageProbabilities(), ref.getAverageProbabilities(),
                                   atol=1e-12, rtol=0)
        for t in range(B):
            np.testing.assert_allclose(fused.getStateVector(t), ref.getStateVector(t), atol=1e-12, rtol=0)
        fused.reset()
        ref.reset()
        fused.run(c)  # relabels again from |0..0>
        ref.run(c, per_gate=True)
        u = np.random.default_rng(1).random((B, 64))
        np.testing.assert_array_equal(fused.sampleWith(u), ref.sampleWith(u))
    finally:
        set_relabel(1, 26)


def test_config4_physical_batch_plans_three_passes(qsim, gpu_ready):
    """BASELINE config 4 (16q x 1024, W-HC seed 42) under the physical process: the relabeled
    fused plan is 3 passes.  The labels are chosen under the frame path's tile-control rule
    (every control a tile qubit) in every planning thread (round-4 regression: the relabel
    workers planned with tile-constant controls, the frame path without, and ran 4 passes)."""
    n, B = 16, 1024
    c = qsim.createRandomHCCircuit(n, 100, 42)
    nm = qsim.NoiseModel()
    nm.addDepolarizingAll(n, 0.01)
    s = qsim.BatchedSimulator(n, B, nm, noise=qsim.BatchedNoise.Physical)
    s.setSeed(42)
    s.run(c)
    s.run(c)
    assert s.lastRunInfo()[0] == 3
    s.close()
