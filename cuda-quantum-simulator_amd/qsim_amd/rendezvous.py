"""Single-node rank rendezvous without torch: unique-id broadcast, barriers, max-reduce.

Why not torch.distributed here: importing torch after the engine library loads a second HIP
runtime into the process (torch-ROCm ships its own libamdhip64 / hiprtc / comgr and its
libc10_hip asks for the unversioned soname, so the loader cannot reuse /opt/rocm's copy); the
process then aborts in the duplicated runtimes' static destructors at exit.  The sharded bench
only needs three host-side operations between ranks of ONE node — broadcast the 128-byte RCCL
unique id, barrier, max over ranks of a wall time — so they go through small files in a
directory private to the job (key: the launcher's pid, MASTER_PORT, TORCHELASTIC_RUN_ID and
TORCHELASTIC_RESTART_COUNT; every rank of one torchrun / bench launcher has the same parent, and a
restarted attempt gets a fresh directory instead of reading the crashed attempt's files, e.g. an
old RCCL unique id).  All state traffic is RCCL.

Every wait is bounded (QSIM_DIST_INIT_TIMEOUT, default 300 s): a rank that never arrives makes
the others raise instead of hanging.
"""
from __future__ import annotations

import os
import shutil
import tempfile
import time
from typing import List, Optional


class FileGroup:
    def __init__(self, rank: int, world: int, key: Optional[str] = None,
                 timeout_s: Optional[float] = None, root: Optional[str] = None):
        self.rank, self.world = rank, world
        if key is None:
            key = os.environ.get("QSIM_RDZV_KEY")  # set by qsim_amd/launch.py
        if key is None:
            key = "{}_{}_{}_r{}".format(os.getppid(), os.environ.get("MASTER_PORT", "0"),
                                        os.environ.get("TORCHELASTIC_RUN_ID", "none"),
                                        os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
        self.dir = os.path.join(root or tempfile.gettempdir(), "qsim_rdzv_" + key)
        self.timeout = float(timeout_s if timeout_s is not None
                             else os.environ.get("QSIM_DIST_INIT_TIMEOUT", "300"))
        self._seq = 0
        os.makedirs(self.dir, exist_ok=True)

    # -- primitives ------------------------------------------------------------------------
    def _put(self, name: str, data: bytes) -> None:
        tmp = os.path.join(self.dir, f".{name}.{self.rank}.tmp")
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, os.path.join(self.dir, name))  # atomic: readers see all or nothing

    def _get(self, name: str) -> bytes:
        path = os.path.join(self.dir, name)
        t0 = time.monotonic()
        delay = 1e-4
        while True:
            try:
                with open(path, "rb") as f:
                    return f.read()
            except FileNotFoundError:
                pass
            if time.monotonic() - t0 > self.timeout:
                raise TimeoutError(f"rank {self.rank}: no '{name}' from a peer within "
                                   f"{self.timeout:.0f} s ({self.dir})")
            time.sleep(delay)
            delay = min(delay * 2, 5e-3)

    # -- collectives -----------------------------------------------------------------------
    def broadcast(self, data: Optional[bytes], src: int = 0) -> bytes:
        self._seq += 1
        name = f"bc{self._seq}"
        if self.rank == src:
            self._put(name, data)
            return data
        return self._get(name)

    def all_gather(self, data: bytes) -> List[bytes]:
        self._seq += 1
        self._put(f"ag{self._seq}_{self.rank}", data)
        return [self._get(f"ag{self._seq}_{r}") for r in range(self.world)]

    def barrier(self) -> None:
        self.all_gather(b"")

    def all_reduce_max(self, value: float) -> float:
        return max(float(v.decode()) for v in self.all_gather(repr(float(value)).encode()))

    def all_reduce_min(self, value: float) -> float:
        return min(float(v.decode()) for v in self.all_gather(repr(float(value)).encode()))

    def close(self) -> None:
        """Collective: the last barrier, then rank 0 removes the job directory."""
        self.barrier()
        # every peer says it has finished reading; only then does rank 0 delete the files
        if self.rank != 0:
            self._put(f"done_{self.rank}", b"")
            return
        for r in range(1, self.world):
            self._get(f"done_{r}")
        shutil.rmtree(self.dir, ignore_errors=True)
