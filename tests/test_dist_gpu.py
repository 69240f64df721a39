"""GPU: the sharded engine (qsim_dist_*) with virtual ranks on one GPU vs the oracle.

Virtual mode runs W shards in one process on one device with the production planner, per-rank
lowering, fused local passes and pack/unpack exchange kernels; only the RCCL transport is replaced
by device copies (RCCL rejects two ranks on one GPU).  A 1-rank RCCL communicator is also created
to exercise the real create/run/gather path.
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def mixed_circuit(qsim, n, seed, depth=120):
    rng = np.random.default_rng(seed)
    c = qsim.Circuit(n)
    for _ in range(depth):
        t = int(rng.integers(0, 17))
        ar = 1 if t <= 10 else (2 if t <= 15 else 3)
        qs = [int(x) for x in rng.choice(n, size=ar, replace=False)]
        c.append(qsim.GateOp(t, qs, float(rng.uniform(0, 2 * math.pi))))
    return c


@pytest.mark.parametrize("world,n", [(2, 8), (4, 10), (8, 12), (8, 16), (2, 20)])
@pytest.mark.parametrize("fused", [True, False])
def test_virtual_ranks_match_oracle(qsim, oracle, gpu_ready, world, n, fused):
    from qsim_amd.dist import DistributedSimulator
    circs = [qsim.createRandomHCCircuit(n, 100, 42), qsim.createRandomCircuit(n, 100, 5)]
    if n <= 16:
        circs.append(mixed_circuit(qsim, n, n))
    for c in circs:
        d = DistributedSimulator.virtual(n, world)
        d.run(c, fused=fused)
        got = d.getStateVector()
        ref = oracle.run_cpu(n, oracle.gates_of(c))
        assert np.max(np.abs(got - ref)) < 1e-12
        assert abs(d.getTotalProbability() - 1.0) < 1e-12
        p = np.abs(ref) ** 2
        for q in (0, n // 2, n - 1):
            mask = ((np.arange(1 << n) >> q) & 1) == 0
            assert abs(d.probBitZero(q) - p[mask].sum()) < 1e-12


def test_virtual_ranks_run_twice_and_reset(qsim, oracle, gpu_ready):
    from qsim_amd.dist import DistributedSimulator
    n = 12
    c = qsim.createRandomHCCircuit(n, 100, 42)
    d = DistributedSimulator.virtual(n, 8)
    d.run(c)
    d.run(c)  # second run starts from the permuted layout left by the first
    g = oracle.gates_of(c)
    ref = oracle.run_cpu(n, g + g)
    assert np.max(np.abs(d.getStateVector() - ref)) < 1e-12
    d.reset()
    s = d.getStateVector()
    assert abs(s[0] - 1) < 1e-15 and np.all(np.abs(s[1:]) == 0)


@pytest.mark.parametrize("world,n", [(8, 16), (4, 20)])
def test_virtual_ranks_run_sequence(qsim, oracle, gpu_ready, world, n):
    """DistributedSimulator.runSequence: three circuits as one sharded run (remaps and passes planned
    over all of them) equal the oracle of the circuits in turn, twice."""
    from qsim_amd.dist import DistributedSimulator
    cs = [qsim.createRandomHCCircuit(n, 100, sd) for sd in (42, 43)] + [qsim.createRandomCircuit(n, 60, 9)]
    g = [x for c in cs for x in oracle.gates_of(c)]
    d = DistributedSimulator.virtual(n, world)
    d.runSequence(cs)
    ref = oracle.run_cpu(n, g)
    assert np.max(np.abs(d.getStateVector() - ref)) < 1e-12
    d.runSequence(cs)
    assert np.max(np.abs(d.getStateVector() - oracle.run_cpu(n, g, ref))) < 1e-12


@pytest.mark.parametrize("world,n", [(4, 22), (8, 23), (2, 21)])
def test_virtual_pipelined_remaps_match_single_gpu(qsim, gpu_ready, world, n):
    """Shards large enough that every remap is split into pipeline parts (transfers on the comm
    stream, packs/unpacks on the compute stream, event-ordered); three runs so the qubit map
    moves through several layouts.  Beyond the oracle's size the reference is the single-GPU
    engine."""
    from qsim_amd.dist import DistributedSimulator
    c = qsim.createRandomHCCircuit(n, 100, 7)
    d = DistributedSimulator.virtual(n, world)
    s = qsim.Simulator(n)
    for _ in range(3):
        d.run(c)
        s.run(c)
    np.testing.assert_allclose(d.getStateVector(), s.getStateVector(), atol=1e-12, rtol=0)


def test_single_rank_rccl_path(qsim, oracle, gpu_ready):
    from qsim_amd.dist import DistributedSimulator
    n = 14
    c = qsim.createRandomCircuit(n, 150, 9)
    d = DistributedSimulator(n, 0, 1)
    d.run(c)
    ref = oracle.run_cpu(n, oracle.gates_of(c))
    assert np.max(np.abs(d.getStateVector() - ref)) < 1e-12
    assert abs(d.getTotalProbability() - 1.0) < 1e-12


@pytest.mark.parametrize("world,n,fused", [(8, 16, True), (4, 18, True), (2, 20, True),
                                           (8, 24, True), (8, 16, False)])
def test_overlapped_remaps_match(qsim, oracle, gpu_ready, world, n, fused):
    """Remaps split in halves around a pivot qubit (half-exchanges on the copy / comm streams,
    the neighbouring local steps run per half on the compute stream, event-ordered): the state
    after several runs equals the single-GPU engine (and the oracle where it fits), and the
    planner did overlap remaps (per-gate mode falls back to whole-shard steps, same result)."""
    from qsim_amd.dist import DistributedSimulator, plan
    c = qsim.createRandomHCCircuit(n, 100, 42)
    steps, _ = plan(c, world, 0)
    assert any(s["kind"] == "exchange" and s["pivot"] >= 0 for s in steps)
    d = DistributedSimulator.virtual(n, world)
    s = qsim.Simulator(n)
    for _ in range(3):
        d.run(c, fused=fused)
        s.run(c)
        assert d.overlappedRemaps() >= 1
    got = d.getStateVector()
    np.testing.assert_allclose(got, s.getStateVector(), atol=1e-12, rtol=0)
    if n <= 18:
        g = oracle.gates_of(c)
        np.testing.assert_allclose(got, oracle.run_cpu(n, g + g + g), atol=1e-12, rtol=0)


@pytest.mark.parametrize("world,n", [(4, 20), (8, 21)])
def test_relabeled_local_positions_match(qsim, oracle, gpu_ready, world, n):
    """Layout-aware relabeling of the shards' local positions on the first fused run of |0..0>
    (threshold lowered to exercise it here): gathered states equal the oracle after three runs,
    and the map differs from the unrelabeled engine's."""
    from qsim_amd.dist import DistributedSimulator
    from qsim_amd.plan import set_relabel
    c = qsim.createRandomHCCircuit(n, 100, 42)
    g = oracle.gates_of(c)
    maps = {}
    try:
        for mode in (0, 1):
            set_relabel(mode, 14)
            d = DistributedSimulator.virtual(n, world)
            for _ in range(3):
                d.run(c)
            maps[mode] = d.perm()
            np.testing.assert_allclose(d.getStateVector(), oracle.run_cpu(n, g + g + g), atol=1e-12, rtol=0)
            d.close()
    finally:
        set_relabel(1, 26)
    assert maps[0] != maps[1]


@pytest.mark.parametrize("world,n,fused", [(8, 16, True), (4, 18, True), (2, 14, True),
                                           (8, 10, True), (8, 16, False)])
def test_virtual_shards_over_rccl(qsim, oracle, gpu_ready, world, n, fused):
    """Virtual shards whose slabs move as ncclSend / ncclRecv pairs to rank 0 of a world-1 RCCL
    communicator (non-blocking init, grouped calls, settle, watchdog, all-reduce): the RCCL call
    sequence of the multi-rank path, run on one GPU, for part-exchanges (n >= 14 here) and plain
    pipelined remaps (n = 10: 7 local qubits, no overlap)."""
    from qsim_amd.dist import DistributedSimulator
    c = qsim.createRandomHCCircuit(n, 100, 3)
    d = DistributedSimulator.virtual(n, world, rccl=True)
    s = qsim.Simulator(n)
    for _ in range(2):
        d.run(c, fused=fused)
        s.run(c)
    got = d.getStateVector()
    np.testing.assert_allclose(got, s.getStateVector(), atol=1e-12, rtol=0)
    assert abs(d.getTotalProbability() - 1.0) < 1e-10
    g = oracle.gates_of(c)
    np.testing.assert_allclose(got, oracle.run_cpu(n, g + g), atol=1e-12, rtol=0)


def test_virtual_30q_8_shards_over_rccl_matches_single_gpu(qsim, gpu_ready):
    """BASELINE config 5 at its own size on one GPU: 30 qubits in 8 virtual shards of 2 GiB
    (16 GiB of shards + 32 GiB of send / receive slabs), every slab moved by ncclSend / ncclRecv
    through a world-1 RCCL communicator, overlapped part-exchanges as planned for 8 ranks; W-HC run
    twice.  Reference: the single-GPU engine on the same circuit (16 GiB).  Compared: the full
    logical state vectors (1e-12 per component), getTotalProbability and probBitZero of every
    qubit (collectives of the sharded object)."""
    from qsim_amd.dist import DistributedSimulator, plan
    n, world = 30, 8
    c = qsim.createRandomHCCircuit(n, 100, 42)
    steps, _ = plan(c, world, 0)
    assert any(s["kind"] == "exchange" and s["pivots"] for s in steps)
    d = DistributedSimulator.virtual(n, world, rccl=True)
    for _ in range(2):
        d.run(c)
    d.synchronize()
    assert d.overlappedRemaps() >= 1
    assert abs(d.getTotalProbability() - 1.0) < 1e-10
    p0 = [d.probBitZero(q) for q in range(n)]
    got = d.getStateVector()
    d.close()
    del d
    s = qsim.Simulator(n)
    for _ in range(2):
        s.run(c)
    for q in range(n):
        assert abs(p0[q] - s.state.probBitZero(q)) < 1e-12, q
    ref = s.getStateVector()
    del s
    err = float(np.max(np.abs(got - ref)))
    assert err < 1e-12, err


@pytest.mark.parametrize("n,world", [(20, 8), (24, 8), (22, 4)])
def test_fused_remap_equals_pack_unpack(qsim, oracle, gpu_ready, monkeypatch, n, world):
    """The fused remap (qsim_dist_fused_remaps): the last pass before the exchange stores into the
    send buffer's slab layout, the step after loads from the receive buffer in that layout and
    stores back (sub-space relayout passes per pivot part) — the same state as the pack / unpack
    kernels, over two runs (the second from the first's map) and against the oracle."""
    from qsim_amd.dist import DistributedSimulator
    c = qsim.createRandomHCCircuit(n, 100, 42)
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("QSIM_DIST_FUSED_PACK", mode)
        d = DistributedSimulator.virtual(n, world)
        d.run(c)
        fused1 = d.fusedRemaps()
        d.run(c)
        fused2 = d.fusedRemaps()
        out[mode] = d.getStateVector()
        if mode == "1":
            assert fused1 + fused2 > 0
        else:
            assert fused1 == fused2 == 0
        d.close()
    g = oracle.gates_of(c)
    ref = oracle.run_cpu(n, g + g)
    assert np.max(np.abs(out["1"] - ref)) < 1e-12
    assert np.max(np.abs(out["0"] - ref)) < 1e-12


@pytest.mark.parametrize("fused_pack", ["1", "0"])
@pytest.mark.parametrize("world,n", [(4, 22), (8, 20)])
def test_cross_run_carry_matches_oracle(qsim, oracle, gpu_ready, monkeypatch, world, n, fused_pack):
    """the experimental cross-run carry (QSIM_DIST_CARRY=1: a run's last step is
    left pending and merged into the next run's first step).  Three runs of one circuit, with
    readers (probability, gather) and a reset in between — every state-touching entry must flush
    the pending step first — against the oracle at 1e-12, and the merge must have happened.
    World 8 / 20 qubits (dropped in round 5 after "the carry never merged"): some shards' last
    steps are lowered without the gates a global control drops, so not every shard's step lay
    wholly in the per-part head, and round 5 carried only when all did; the carry is now decided on
    the step skeleton alone and such a shard runs its step's other passes whole (flush_carry)."""
    from qsim_amd.dist import DistributedSimulator
    monkeypatch.setenv("QSIM_DIST_CARRY", "1")
    monkeypatch.setenv("QSIM_DIST_FUSED_PACK", fused_pack)
    c = qsim.createRandomHCCircuit(n, 100, 42)
    g = oracle.gates_of(c)
    d = DistributedSimulator.virtual(n, world)
    merged = 0
    for _ in range(3):
        d.run(c)
        merged += d.carriedRuns() > 0
    np.testing.assert_allclose(d.getStateVector(), oracle.run_cpu(n, g * 3), atol=1e-12, rtol=0)
    d.run(c)  # (carry pending again) then a reader
    assert abs(d.getTotalProbability() - 1.0) < 1e-12
    d.run(c)
    ref5 = oracle.run_cpu(n, g * 5)
    p = np.abs(ref5) ** 2
    mask = ((np.arange(1 << n) >> (n - 1)) & 1) == 0
    assert abs(d.probBitZero(n - 1) - p[mask].sum()) < 1e-12
    np.testing.assert_allclose(d.getStateVector(), ref5, atol=1e-12, rtol=0)
    d.run(c)
    d.reset()  # flushes, then |0..0>
    s = d.getStateVector()
    assert abs(s[0] - 1) < 1e-15 and np.all(np.abs(s[1:]) == 0)
    d.run(c)
    np.testing.assert_allclose(d.getStateVector(), oracle.run_cpu(n, g), atol=1e-12, rtol=0)
    print(f"carry merges: world {world} n {n} fused_pack {fused_pack}: {merged} of the first 3 runs, "
          f"{d.carriedRuns()} in all")
    assert d.carriedRuns() >= 1, "the carry never merged"
