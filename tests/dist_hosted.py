"""Test helper: one rank process of a multi-process sharded run WITHOUT RCCL.

Each rank process creates `DistributedSimulator.hosted(n, rank, world, transport)` (one shard per
process, exactly the multi-rank path of qsim_dist_run: per-process planning with its own pivot
memo, rank-dependent lowering and slab maps, collectives), and the transfers go through the
`SocketMesh` below (TCP over 127.0.0.1, one connection per rank pair).  Several rank processes
can therefore share the single GPU of a test box, which RCCL refuses.

Run as a script: python dist_hosted.py RANK WORLD PORTS N OUT_DIR
(PORTS comma-separated, one per rank).  Rank 0 saves the gathered states; every rank writes its
collective readouts (total probability, probBitZero of every qubit) to OUT_DIR/rank<R>.json.
"""
from __future__ import annotations

import json
import os
import socket
import struct
import sys
import threading
import time
from collections import defaultdict


def _recv_exact(s: socket.socket, view: memoryview) -> None:
    got = 0
    while got < len(view):
        k = s.recv_into(view[got:])
        if k == 0:
            raise ConnectionError("peer closed the connection")
        got += k


class SocketMesh:
    """Full mesh of TCP connections; a post's payload is framed by its length so that posts
    which do not pair up (a planning mismatch between ranks) fail instead of corrupting data."""

    def __init__(self, rank: int, world: int, ports, timeout: float = 60.0):
        self.rank, self.socks = rank, {}
        srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        srv.bind(("127.0.0.1", ports[rank]))
        srv.listen(world)
        srv.settimeout(timeout)
        for r in range(rank):  # connect to the lower ranks (they listen first)
            t0 = time.time()
            while True:
                try:
                    s = socket.create_connection(("127.0.0.1", ports[r]), timeout=timeout)
                    break
                except OSError:
                    if time.time() - t0 > timeout:
                        raise
                    time.sleep(0.05)
            s.sendall(struct.pack("<i", rank))
            self.socks[r] = s
        for _ in range(world - 1 - rank):
            c, _ = srv.accept()
            hdr = bytearray(4)
            _recv_exact(c, memoryview(hdr))
            self.socks[struct.unpack("<i", hdr)[0]] = c
        srv.close()
        for s in self.socks.values():
            s.settimeout(timeout)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)

    def __call__(self, posts) -> None:
        by_peer = defaultdict(list)
        for peer, snd, rcv in posts:
            if peer == self.rank or peer not in self.socks:
                raise ValueError(f"bad peer {peer}")
            by_peer[peer].append((snd, rcv))
        errs = []

        def send_all(peer, items):
            try:
                for snd, _ in items:
                    if snd is not None:
                        self.socks[peer].sendall(struct.pack("<Q", len(snd)))
                        self.socks[peer].sendall(snd)
            except BaseException as e:  # noqa: BLE001
                errs.append(e)

        th = [threading.Thread(target=send_all, args=(p, it)) for p, it in by_peer.items()]
        for t in th:
            t.start()
        try:
            for peer, items in by_peer.items():
                for _, rcv in items:
                    if rcv is None:
                        continue
                    hdr = bytearray(8)
                    _recv_exact(self.socks[peer], memoryview(hdr))
                    size = struct.unpack("<Q", hdr)[0]
                    if size != len(rcv):
                        raise RuntimeError(f"rank {self.rank}: post from {peer} carries {size} "
                                           f"bytes, expected {len(rcv)} (ranks disagree)")
                    _recv_exact(self.socks[peer], rcv)
        finally:
            for t in th:
                t.join()
        if errs:
            raise errs[0]

    def close(self) -> None:
        for s in self.socks.values():
            s.close()


def circuits(q, n):
    """The circuits every hosted run executes (the parent test recomputes them)."""
    return [("hc300s3", q.createRandomHCCircuit(n, 300, 3)),
            ("rand150s5", q.createRandomCircuit(n, 150, 5)),
            ("hc100s42", q.createRandomHCCircuit(n, 100, 42))]


def main(argv) -> int:
    rank, world = int(argv[1]), int(argv[2])
    ports = [int(p) for p in argv[3].split(",")]
    n, out = int(argv[4]), argv[5]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "cuda-quantum-simulator_amd"))
    import numpy as np
    import qsim_amd as q
    from qsim_amd.dist import DistributedSimulator
    mesh = SocketMesh(rank, world, ports)
    rec = {"rank": rank, "runs": {}}
    for name, c in circuits(q, n):
        for fused in (True, False):
            if not fused and name != "rand150s5":
                continue
            d = DistributedSimulator.hosted(n, rank, world, mesh)
            perms, overlapped, sent = [], [], []
            for _ in range(3):  # the qubit map moves through several layouts
                perms.append(d.perm())
                d.run(c, fused=fused)
                overlapped.append(d.overlappedRemaps())
                sent.append(d.remapBytes())
            d.synchronize()
            key = f"{name}_{'fused' if fused else 'pergate'}"
            rec["runs"][key] = {
                "total": d.getTotalProbability(),
                "p0": [d.probBitZero(b) for b in range(n)],
                "perm": d.perm(), "perms_in": perms, "overlapped": overlapped,
                "remap_bytes": sent, "carried": d.carriedRuns()}
            st = d.getStateVector()
            if rank == 0:
                np.save(os.path.join(out, f"{key}.npy"), st)
            d.close()
    mesh.close()
    with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
        json.dump(rec, f)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
