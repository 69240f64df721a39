"""Test helper: execute the distributed planner's step list (qsim_amd.dist.plan) for one rank on
a numpy shard, with every qubit-remap exchange carried out over torch.distributed (gloo, CPU).

This checks the multi-GPU logic — per-rank lowering of global controls/phases, the lookahead
remap choice, the pivots of overlapped remaps (planned independently in every rank process), the
engine's own pack/peer/unpack index maps (qsim_dist_slab_map, the C++ the kernels use) and the
final logical<->physical un-permutation — with real inter-process transfers and no GPU.  Op semantics follow engine.hpp (M1 / DIAG / SWAP).
"""
from __future__ import annotations

import numpy as np


def apply_op(s: np.ndarray, op: dict) -> None:
    idx = np.arange(s.size, dtype=np.int64)
    cm = np.int64(op["cmask"])
    ctrl = (idx & cm) == cm
    m = op["m"]
    if op["kind"] == 0:
        b = 1 << op["t0"]
        sel = idx[ctrl & ((idx & b) == 0)]
        a0, a1 = s[sel].copy(), s[sel | b].copy()
        s[sel] = m[0] * a0 + m[1] * a1
        s[sel | b] = m[2] * a0 + m[3] * a1
    elif op["kind"] == 1:
        b = 1 << op["t0"]
        bit = (idx & b) != 0
        f = np.where(bit, m[1], m[0])
        s[ctrl] = s[ctrl] * f[ctrl]
    else:
        b0, b1 = 1 << op["t0"], 1 << op["t1"]
        sel = idx[ctrl & ((idx & b0) != 0) & ((idx & b1) == 0)]
        j = sel ^ b0 ^ b1
        tmp = s[sel].copy()
        s[sel] = s[j]
        s[j] = tmp


def exchange(s: np.ndarray, n: int, world: int, rank: int, step: dict, dist) -> None:
    """One remap with the engine's own slab layout (qsim_dist_slab_map: the peer of every slab
    and the local index of every slab element, as the pack / unpack kernels compute them); an
    overlapped remap (pivots) is carried out part by part, as qsim_dist_run does."""
    import torch
    import qsim_amd.dist as qd
    k = step["k"]
    if k == 0:
        return
    parts = range(1 << len(step["pivots"])) if step["pivots"] else [-1]
    for part in parts:
        my_c, peer_of, idx = qd.slab_map(n, world, rank, step, part)
        chunk = idx.size >> k
        ops, recv = [], {}
        for c in range(1 << k):
            if c == my_c:
                continue
            sl = idx[c * chunk:(c + 1) * chunk]
            send = torch.from_numpy(np.ascontiguousarray(s[sl]).view(np.float64))
            recv[c] = (sl, torch.empty_like(send))
            ops.append(dist.P2POp(dist.isend, send, peer_of[c]))
            ops.append(dist.P2POp(dist.irecv, recv[c][1], peer_of[c]))
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        for sl, buf in recv.values():
            s[sl] = buf.numpy().view(np.complex128)


def run_rank(n: int, world: int, rank: int, circuit, dist) -> tuple:
    import qsim_amd.dist as qd
    g = world.bit_length() - 1
    L = n - g
    steps, perm = qd.plan(circuit, world, rank)
    s = np.zeros(1 << L, dtype=np.complex128)
    if rank == 0:
        s[0] = 1.0
    for st in steps:
        if st["kind"] == "ops":
            for op in st["ops"]:
                apply_op(s, op)
        else:
            exchange(s, n, world, rank, st, dist)
    return s, perm


def assemble(shards, perm, n: int) -> np.ndarray:
    phys = np.concatenate(shards)
    i = np.arange(1 << n, dtype=np.int64)
    p = np.zeros_like(i)
    for q in range(n):
        p |= ((i >> q) & 1) << perm[q]
    return phys[p]
