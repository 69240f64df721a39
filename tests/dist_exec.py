"""Test helper: execute the distributed planner's step list (qsim_amd.dist.plan) for one rank on
a numpy shard, with every qubit-remap exchange carried out over torch.distributed (gloo, CPU).

This checks the multi-GPU logic — per-rank lowering of global controls/phases, the lookahead
remap choice, the pack/peer/unpack index mapping and the final logical<->physical un-permutation —
with real inter-process collectives and no GPU.  Op semantics follow engine.hpp (M1 / DIAG / SWAP).
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


def chunk_index(L: int, lpos, c: int) -> np.ndarray:
    """Local indices whose bits at lpos[j] equal bit j of c, in ascending order."""
    k = len(lpos)
    rest = np.arange(1 << (L - k), dtype=np.int64)
    for p in sorted(lpos):
        lo = rest & ((1 << p) - 1)
        rest = ((rest ^ lo) << 1) | lo
    for j, p in enumerate(lpos):
        rest |= ((c >> j) & 1) << p
    return rest


def exchange(s: np.ndarray, L: int, rank: int, step: dict, dist) -> None:
    import torch
    k, gpos, lpos = step["k"], step["gpos"], step["lpos"]
    if k == 0:
        return
    my_c = sum(((rank >> (gpos[j] - L)) & 1) << j for j in range(k))
    ops, recv = [], {}
    for c in range(1 << k):
        if c == my_c:
            continue
        peer = rank
        for j in range(k):
            b = gpos[j] - L
            peer = (peer & ~(1 << b)) | (((c >> j) & 1) << b)
        send = torch.from_numpy(np.ascontiguousarray(s[chunk_index(L, lpos, c)]).view(np.float64))
        recv[c] = torch.empty_like(send)
        ops.append(dist.P2POp(dist.isend, send, peer))
        ops.append(dist.P2POp(dist.irecv, recv[c], peer))
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    for c, buf in recv.items():
        s[chunk_index(L, lpos, c)] = buf.numpy().view(np.complex128)


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
            exchange(s, L, rank, st, dist)
    return s, perm


def assemble(shards, perm, n: int) -> np.ndarray:
    phys = np.concatenate(shards)
    i = np.arange(1 << n, dtype=np.int64)
    p = np.zeros_like(i)
    for q in range(n):
        p |= ((i >> q) & 1) << perm[q]
    return phys[p]
