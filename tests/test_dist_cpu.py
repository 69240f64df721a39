"""CPU, multi-process (gloo): the sharded path's planner + exchange logic against the oracle.

world_size 2, 4 and 8 ranks run as separate processes (torch.multiprocessing, gloo over
127.0.0.1); each plans its own rank in its own process (qsim_amd.dist.plan, the exact step list
qsim_dist_run launches — pivots included, decided independently per process) and executes it on a
numpy shard, performing every qubit remap (part by part when it has pivots) as real isend/irecv
exchanges over the engine's own slab maps (qsim_dist_slab_map).  Rank 0 gathers the shards,
undoes the logical->physical map and compares with the CPUSimulator restatement at 1e-12.
"""
import math
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def circuits(qsim, n):
    out = [qsim.createRandomHCCircuit(n, 300 if n == 16 else (100 if n >= 12 else 60), 3 if n == 16 else 42),
           qsim.createRandomCircuit(n, 80, 3)]
    rng = np.random.default_rng(n)
    c = qsim.Circuit(n)
    for _ in range(90):
        t = int(rng.integers(0, 17))
        ar = 1 if t <= 10 else (2 if t <= 15 else 3)
        qs = [int(x) for x in rng.choice(n, size=ar, replace=False)]
        c.append(qsim.GateOp(t, qs, float(rng.uniform(0, 2 * math.pi))))
    out.append(c)
    return out


def worker(rank, world, port, n, result_q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "cuda-quantum-simulator_amd"), os.path.join(root, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    import qsim_amd
    import dist_exec
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import datetime
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=120))
    try:
        for ci, c in enumerate(circuits(qsim_amd, n)):
            shard, perm = dist_exec.run_rank(n, world, rank, c, dist)
            if ci == 0:  # the planner must have overlapped a remap where the shard allows it
                steps, _ = qsim_amd.dist.plan(c, world, rank)
                result_q.put(("pivots", rank, [tuple(s["pivots"]) for s in steps if s["kind"] == "exchange"]))
            gathered = [torch.empty(2 * shard.size, dtype=torch.float64) for _ in range(world)] \
                if rank == 0 else None
            dist.gather(torch.from_numpy(shard.view(np.float64).copy()), gathered, dst=0)
            if rank == 0:
                full = dist_exec.assemble([g.numpy().view(np.complex128) for g in gathered], perm, n)
                result_q.put((ci, full))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 7), (4, 8), (2, 10), (2, 12), (4, 13), (8, 14), (8, 16)])
def test_sharded_plan_matches_oracle_gloo(qsim, oracle, world, n):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, pivots = {}, {}
    try:
        while len(got) < 3 or len(pivots) < world:
            item = q.get(timeout=240)
            if item[0] == "pivots":
                pivots[item[1]] = item[2]
            else:
                got[item[0]] = item[1]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    for ci, c in enumerate(circuits(qsim, n)):
        ref = oracle.run_cpu(n, oracle.gates_of(c))
        assert np.max(np.abs(got[ci] - ref)) < 1e-12, ci
    # every rank process chose the same pivots on its own; shards of >= 8 local qubits overlap
    assert all(pivots[r] == pivots[0] for r in range(world))
    if n - (world.bit_length() - 1) >= 11:
        assert any(pivots[0]), pivots[0]


def test_plan_structure(qsim):
    """SWAPs never move data; exchanges only when a target sits on a rank bit; all ranks share
    the exchange skeleton."""
    import qsim_amd.dist as qd
    n, world = 10, 8
    c = qsim.Circuit(n)
    c.swap(0, 9).swap(1, 8).h(9).cnot(9, 2).cz(8, 7).crz(7, 9, 0.4).h(7).toffoli(9, 8, 1)
    skel = None
    for r in range(world):
        steps, perm = qd.plan(c, world, r)
        kinds = [s["kind"] for s in steps]
        ex = [(s["k"], s["gpos"], s["lpos"]) for s in steps if s["kind"] == "exchange"]
        skel = skel or (kinds.count("exchange"), ex)
        assert (kinds.count("exchange"), ex) == skel
        assert sorted(perm) == list(range(n))
        for s in steps:
            if s["kind"] == "ops":
                for op in s["ops"]:
                    assert op["t0"] < n - 3 and (op["kind"] != 2 or op["t1"] < n - 3)
                    assert op["cmask"] < (1 << (n - 3))


@pytest.mark.parametrize("seed", [42, 1, 2, 3])
def test_plan_w_hc_30q_one_remap_per_run(qsim, seed):
    """Dependency-aware scheduling (gates move only past gates on disjoint qubits): the W-HC
    circuit at 30 qubits on 8 ranks needs at most one all-to-all remap per run, from the first
    run on and for every repetition (each run starts from the map the previous one left)."""
    import qsim_amd.dist as qd
    c = qsim.createRandomHCCircuit(30, 100, seed)
    perm = list(range(30))
    for _ in range(4):
        steps, perm = qd.plan(c, 8, 0, perm)
        assert sum(s["kind"] == "exchange" for s in steps) <= 1
        assert all(s["k"] == 3 for s in steps if s["kind"] == "exchange")


@pytest.mark.parametrize("n,seed", [(16, 3), (18, 8), (22, 7)])
def test_plan_pivots_rank_independent_fresh(qsim, n, seed):
    """Pivots are planned from rank-independent data only: each rank planned as if in its own
    fresh process (the pivot memo cleared before every rank) gets rank 0's pivots and roles, on a
    circuit with two or more pivoted remaps in a row (the ops step between them is the trailing
    step of one and the leading step of the other)."""
    import qsim_amd.dist as qd
    world = 8
    # (these circuits made ranks != 0 pick other pivots when the planner read the roles of
    # rank 0's reference plan instead of its own marks — ADVICE r2, dist.hip mark_overlap)
    c = qsim.createRandomHCCircuit(n, 300, seed)
    ref = None
    for r in range(world):
        qd.plan_memo_clear()
        steps, _ = qd.plan(c, world, r)
        sk = [(s["kind"], tuple(s.get("pivots", ())), s.get("role", 0)) for s in steps]
        ref = ref or sk
        assert sk == ref, r
    pivoted = [i for i, s in enumerate(ref) if s[0] == "exchange" and s[1]]
    assert len(pivoted) >= 2
    assert any(ref[i][2] == 3 for i in range(len(ref)) if ref[i][0] == "ops"), \
        "no ops step both follows and precedes a pivoted remap"


def test_slab_map_is_a_partition(qsim):
    """qsim_dist_slab_map (the pack / unpack index map): for every rank, every remap of a plan and
    every part, the slabs cover the shard exactly once; the parts of an overlapped remap cover it
    exactly once together; peers are an involution (my slab c goes to the rank whose slab my_c
    comes back) and differ from the rank only in the exchanged global bits."""
    import qsim_amd.dist as qd
    n, world = 14, 8
    g, L = 3, 11
    c = qsim.createRandomHCCircuit(n, 100, 42)
    for r in range(world):
        steps, _ = qd.plan(c, world, r)
        for st in (s for s in steps if s["kind"] == "exchange"):
            my_c, peer_of, idx = qd.slab_map(n, world, r, st, -1)
            assert np.array_equal(np.sort(idx), np.arange(1 << L))
            assert peer_of[my_c] == r
            gmask = sum(1 << (p - L) for p in st["gpos"])
            for cc, q in enumerate(peer_of):
                assert (q & ~gmask) == (r & ~gmask)
                qc, qpeer, _ = qd.slab_map(n, world, q, st, -1)
                assert qpeer[my_c] == r and qc == cc
            if st["pivots"]:
                allp = np.concatenate([qd.slab_map(n, world, r, st, h)[2]
                                       for h in range(1 << len(st["pivots"]))])
                assert np.array_equal(np.sort(allp), np.arange(1 << L))


def test_plan_pivots_rank_independent(qsim):
    """Overlapped remaps run in 2^m parts around m <= 4 pivot positions chosen by planning the
    neighbouring steps on rank 0's ops: every rank gets the same pivots (the part exchanges pair
    up across ranks); pivots are local positions >= 6 outside the exchanged ones, and the steps on
    both sides are marked to run their avoiding passes per part."""
    import qsim_amd.dist as qd
    n, world = 22, 8
    c = qsim.createRandomHCCircuit(n, 100, 7)
    perm0 = list(range(n))
    ref = None
    for r in range(world):
        steps, perm = qd.plan(c, world, r, list(perm0))
        piv = [(i, tuple(s["pivots"])) for i, s in enumerate(steps) if s["kind"] == "exchange"]
        ref = ref or piv
        assert piv == ref
        for i, pv in piv:
            s = steps[i]
            if not pv:
                continue
            assert 1 <= len(pv) <= 4 and s["pivot"] == pv[0]
            assert all(6 <= p < n - 3 and p not in s["lpos"] for p in pv)
            assert steps[i - 1]["role"] & 1 and steps[i + 1]["role"] & 2
    assert any(pv for _, pv in ref)


def test_plan_reorder_is_exact(qsim, oracle):
    """The executed op sequence of every rank, mapped back through the planner's qubit maps,
    is a reordering of the circuit that only swaps gates on disjoint qubits."""
    import qsim_amd.dist as qd
    n, world = 12, 8
    c = qsim.createRandomCircuit(n, 300, 11)
    gates = c.getGates()
    steps, _ = qd.plan(c, world, 0)
    order = [op["src"] for s in steps if s["kind"] == "ops" for op in s["ops"]]
    assert len(set(order)) == len(order)
    pos = {g: i for i, g in enumerate(order)}
    qs = [set(g.qubits) for g in gates]
    for a in range(len(gates)):
        for b in range(a + 1, len(gates)):
            if a in pos and b in pos and qs[a] & qs[b]:
                assert pos[a] < pos[b], (a, b)


def test_plan_sizes_output_for_the_given_map(qsim):
    """plan() from a non-identity start map returns every step (its output was once sized by a
    plan from the identity map, which can have fewer steps)."""
    import qsim_amd.dist as qd
    n, world = 14, 2
    c = qsim.createRandomHCCircuit(n, 300, 3)
    perm = list(range(n))
    for _ in range(3):
        steps, nxt = qd.plan(c, world, 0, perm)
        ex = [s for s in steps if s["kind"] == "exchange"]
        # the framed step list starts and ends with an ops step and alternates around remaps
        assert steps[0]["kind"] == "ops" and steps[-1]["kind"] == "ops"
        assert len(steps) == 2 * len(ex) + 1
        passes = qd_passes(qd, c, world, perm)
        assert len(passes) == len(steps)
        perm = nxt


def qd_passes(qd, c, world, perm):
    import ctypes
    from qsim_amd import _lib
    n = c.getNumQubits()
    arr, cnt = c.to_abi()
    p = (ctypes.c_int32 * n)(*perm)
    ns = ctypes.c_size_t(0)
    _lib.check(_lib.hip.qsim_dist_plan_passes(n, world, 0, arr, cnt, p, None, 0, ctypes.byref(ns)))
    return [0] * ns.value
