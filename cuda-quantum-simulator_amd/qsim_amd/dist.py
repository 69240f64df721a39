"""Sharded multi-GPU state (qsim_dist_* of include/qsim_hip.h).

One process per GPU: `DistributedSimulator(n, rank, world, unique_id, device)`; rank 0 creates the
RCCL unique id with `unique_id()` and the launcher (torch.distributed over gloo, see
dist_bench.py) broadcasts it.  `DistributedSimulator.virtual(n, world)` keeps all `world` shards in
one process on one GPU (exchanges by device copies) — the same planner and kernels, used to test
the sharded path on a single GPU.  `plan()` exposes the host planner (no GPU needed).
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Tuple

import numpy as np

from . import _lib
from .circuit import Circuit

_c = ctypes
UNIQUE_ID_BYTES = 128


def unique_id() -> bytes:
    buf = _c.create_string_buffer(UNIQUE_ID_BYTES)
    _lib.check(_lib.hip.qsim_dist_unique_id(buf))
    return buf.raw


class DistributedSimulator:
    def __init__(self, num_qubits: int, rank: int = 0, world: int = 1,
                 uid: Optional[bytes] = None, device: int = 0, _virtual: bool = False):
        self._h = _c.c_void_p()
        self._n, self._world, self._rank = num_qubits, world, rank
        self._virtual = _virtual
        if _virtual:
            _lib.check(_lib.hip.qsim_dist_create_virtual(num_qubits, world, device,
                                                         _c.byref(self._h)))
        else:
            if uid is None:
                if world != 1:
                    raise ValueError("a unique id from rank 0 is required for world > 1")
                uid = unique_id()
            buf = _c.create_string_buffer(uid, UNIQUE_ID_BYTES)
            _lib.check(_lib.hip.qsim_dist_create(num_qubits, rank, world, buf, device,
                                                 _c.byref(self._h)))

    @classmethod
    def virtual(cls, num_qubits: int, world: int, device: int = 0,
                rccl: bool = False) -> "DistributedSimulator":
        """`world` shards in this process on one GPU.  rccl: move the slabs with ncclSend /
        ncclRecv pairs to rank 0 of a world-1 communicator (qsim_dist_virtual_rccl) instead of
        device copies — the multi-rank RCCL call sequence, on one GPU."""
        sim = cls(num_qubits, 0, world, None, device, _virtual=True)
        if rccl:
            buf = _c.create_string_buffer(unique_id(), UNIQUE_ID_BYTES)
            _lib.check(_lib.hip.qsim_dist_virtual_rccl(sim._h, buf))
        return sim

    @classmethod
    def hosted(cls, num_qubits: int, rank: int, world: int, transport, device: int = 0
               ) -> "DistributedSimulator":
        """One shard per process, as the RCCL path, but every transfer goes through the Python
        callable `transport(posts)` (qsim_dist_create_hosted): `posts` is a list of
        (peer, send, recv) with `send` / `recv` memoryviews of host staging (either may be None
        for a one-sided post); the k-th post naming q must meet q's k-th post naming this rank.
        An exception in `transport` fails the engine call.  Lets several rank processes share
        one GPU (tests: the per-rank planning and exchange of the multi-rank path without RCCL)."""
        sim = cls.__new__(cls)
        sim._h = _c.c_void_p()
        sim._n, sim._world, sim._rank, sim._virtual = num_qubits, world, rank, False
        sim._transport_error = None

        def cb(_ctx, posts, count):
            try:
                items = []
                for i in range(count):
                    p = posts[i]
                    snd = (memoryview((_c.c_char * p.bytes).from_address(p.send)).cast("B")
                           if p.send else None)
                    rcv = (memoryview((_c.c_char * p.bytes).from_address(p.recv)).cast("B")
                           if p.recv else None)
                    items.append((p.peer, snd, rcv))
                transport(items)
                return 0
            except BaseException as e:  # noqa: BLE001 — reported through the engine's error
                sim._transport_error = e
                return 1
        sim._cb = _lib.qsim_dist_transport_fn(cb)  # kept alive with the object
        _lib.check(_lib.hip.qsim_dist_create_hosted(num_qubits, rank, world, device, sim._cb, None,
                                                    _c.byref(sim._h)))
        return sim

    def __del__(self):
        self.close()

    def close(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            _lib.hip.qsim_dist_destroy(h)
            self._h = _c.c_void_p()

    def getNumQubits(self) -> int: return self._n
    def getWorldSize(self) -> int: return self._world

    def run(self, circuit: Circuit, fused: bool = True) -> None:
        if circuit.getNumQubits() != self._n:
            raise ValueError("Circuit qubit count doesn't match simulator")
        arr, cnt = circuit.to_abi()
        _lib.check(_lib.hip.qsim_dist_run(self._h, arr, cnt,
                                          _lib.QSIM_RUN_FUSED if fused else _lib.QSIM_RUN_PER_GATE))

    def runSequence(self, circuits, fused: bool = True) -> None:
        """run() of each circuit in turn as ONE sharded run (Simulator.runSequence): passes and
        global<->local remaps are planned over all of their gates."""
        from .simulator import sequence_circuit
        self.run(sequence_circuit(circuits, self._n), fused)

    def synchronize(self) -> None: _lib.check(_lib.hip.qsim_dist_sync(self._h))

    def barrier(self) -> None:
        """Collective: this rank's engine idle, then a one-value all-reduce over the communicator
        (the ranks leave within its latency of one another: bench.py's per-step timing barrier)."""
        _lib.check(_lib.hip.qsim_dist_barrier(self._h))

    def overlappedRemaps(self) -> int:
        """Remaps of the last run that were split in halves overlapping local work."""
        v = _c.c_int(0)
        _lib.check(_lib.hip.qsim_dist_overlapped(self._h, _c.byref(v)))
        return v.value
    def carriedRuns(self) -> int:
        """Runs whose first step merged the previous run's carried last step (QSIM_DIST_CARRY=1,
        experimental)."""
        v = _c.c_int(0)
        _lib.check(_lib.hip.qsim_dist_carried_runs(self._h, _c.byref(v)))
        return v.value
    def fusedRemaps(self) -> int:
        """Exchanges of the last run whose pack / unpack ran inside the local passes (the pass
        before stored into the slab layout, the step after loaded from it), summed over shards."""
        v = _c.c_int(0)
        _lib.check(_lib.hip.qsim_dist_fused_remaps(self._h, _c.byref(v)))
        return v.value

    def remapBytes(self) -> float:
        """Bytes this rank sent in the last run's remaps (it received as many)."""
        v = _c.c_double(0)
        _lib.check(_lib.hip.qsim_dist_remap_bytes(self._h, _c.byref(v)))
        return v.value

    def reset(self) -> None: _lib.check(_lib.hip.qsim_dist_reset(self._h))

    def perm(self) -> List[int]:
        p = (_c.c_int32 * self._n)()
        _lib.check(_lib.hip.qsim_dist_perm(self._h, p))
        return list(p)

    def getStateVector(self) -> Optional[np.ndarray]:
        """Full logical-order state on rank 0 (collective); None on other ranks."""
        out = np.empty(1 << self._n, dtype=np.complex128)
        root = self._virtual or self._rank == 0
        _lib.check(_lib.hip.qsim_dist_gather_state(self._h, out.ctypes.data_as(_c.c_void_p)
                                                   if root else None))
        return out if root else None

    def localState(self) -> np.ndarray:
        shards = self._world if self._virtual else 1
        out = np.empty(shards << (self._n - (self._world.bit_length() - 1)), dtype=np.complex128)
        _lib.check(_lib.hip.qsim_dist_local_state(self._h, out.ctypes.data_as(_c.c_void_p)))
        return out

    def getTotalProbability(self) -> float:
        t = _c.c_double()
        _lib.check(_lib.hip.qsim_dist_total_probability(self._h, _c.byref(t)))
        return t.value

    def probBitZero(self, q: int) -> float:
        t = _c.c_double()
        _lib.check(_lib.hip.qsim_dist_prob_bit_zero(self._h, q, _c.byref(t)))
        return t.value

    def profile(self, enable: bool = True) -> None:
        _lib.check(_lib.hip.qsim_dist_profile(self._h, 1 if enable else 0))

    def profileStats(self):
        n = _c.c_int(0)
        _lib.check(_lib.hip.qsim_dist_profile_count(self._h, _c.byref(n)))
        out = []
        for i in range(n.value):
            name = _c.create_string_buffer(64)
            ms, cnt, by = _c.c_double(), _c.c_int64(), _c.c_double()
            _lib.check(_lib.hip.qsim_dist_profile_get(self._h, i, name, 64, _c.byref(ms),
                                                      _c.byref(cnt), _c.byref(by)))
            out.append({"name": name.value.decode(), "ms": ms.value, "launches": cnt.value,
                        "alg_bytes": by.value})
        return out


def plan(circuit: Circuit, world: int, rank: int, perm: Optional[List[int]] = None):
    """Host planner output for `rank`: (steps, ops, perm_after).  steps are dicts
    {kind: 'ops'|'exchange', ...}; ops are dicts with the lowered op fields."""
    n = circuit.getNumQubits()
    arr, cnt = circuit.to_abi()
    p = (_c.c_int32 * n)(*(perm if perm is not None else range(n)))
    ns, no = _c.c_size_t(0), _c.c_size_t(0)
    p_size = (_c.c_int32 * n)(*p)  # size the output for the SAME start map (the call updates it)
    _lib.check(_lib.hip.qsim_dist_plan(n, world, rank, arr, cnt, p_size, None, 0, _c.byref(ns),
                                       None, 0, _c.byref(no)))
    steps = (_lib.qsim_dist_step * max(1, ns.value))()
    ops = (_lib.qsim_op * max(1, no.value))()
    _lib.check(_lib.hip.qsim_dist_plan(n, world, rank, arr, cnt, p, steps, ns.value, _c.byref(ns),
                                       ops, no.value, _c.byref(no)))
    out_ops = [{"kind": o.kind, "sub": o.sub, "t0": o.t0, "t1": o.t1, "cmask": o.cmask,
                "d0_one": o.d0_one, "src": o.src,
                "m": [complex(o.m[2 * i], o.m[2 * i + 1]) for i in range(4)]}
               for o in ops[:no.value]]
    out_steps = []
    for s in steps[:ns.value]:
        if s.kind == 1:
            out_steps.append({"kind": "exchange", "k": s.k, "gpos": list(s.gpos[:s.k]),
                              "lpos": list(s.lpos[:s.k]), "pivot": s.pivot, "pmask": s.pmask, "coarse": s.coarse,
                              "pivots": [b for b in range(64) if (s.pmask >> b) & 1]})
        else:
            out_steps.append({"kind": "ops", "ops": out_ops[s.op_begin:s.op_end],
                              "role": s.role, "pivot": s.pivot})
    return out_steps, list(p)


def plan_memo_clear() -> None:
    """Forget the process-wide pivot memo: the next plan() decides as a fresh rank process."""
    _lib.check(_lib.hip.qsim_dist_plan_memo_clear())


def slab_map(n: int, world: int, rank: int, step: dict, part: int = -1):
    """The pack / unpack layout of exchange `step` (a plan() dict) on `rank`, as the engine's
    kernels use it (qsim_dist_slab_map): (my_c, peer_of, index) where slab c goes to and comes
    from rank peer_of[c] and index[c * chunk + e] is the local amplitude index of its element e.
    part >= 0: part `part` of an overlapped remap (the pivot bits hold `part`)."""
    st = _lib.qsim_dist_step()
    st.kind, st.k = 1, step["k"]
    for j in range(step["k"]):
        st.gpos[j], st.lpos[j] = step["gpos"][j], step["lpos"][j]
    st.pmask = step.get("pmask", 0)
    g = world.bit_length() - 1
    m = bin(st.pmask).count("1") if part >= 0 else 0
    count = 1 << (n - g - m)
    my_c = _c.c_int32(0)
    peer_of = (_c.c_int32 * (1 << st.k))()
    index = np.empty(count, dtype=np.uint64)
    _lib.check(_lib.hip.qsim_dist_slab_map(n, world, rank, _c.byref(st), part, _c.byref(my_c), peer_of,
                                           index.ctypes.data_as(_c.POINTER(_c.c_uint64)), count))
    return my_c.value, list(peer_of), index.astype(np.int64)
