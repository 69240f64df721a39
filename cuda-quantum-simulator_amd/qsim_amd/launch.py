"""Self-launch of the one-process-per-GPU bench (bench.py --gpus N with no external launcher).

The driver may start `bench.py --gpus N` directly instead of through `torch.distributed.run`.
Then this parent (which never touches the GPU) starts N copies of the same command as rank
processes with RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT set
(device = LOCAL_RANK), forwards rank 0's stdout (the one JSON line) and every rank's stderr, and
exits with the first non-zero rank status.  When one rank fails or the time limit passes, the
others are terminated (SIGTERM to their process group, SIGKILL after a grace period), so a dead
rank never leaves its peers blocked in a collective.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import threading
import time
from typing import List, Optional


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _pump(src, dst, keep: Optional[list]):
    for line in iter(src.readline, b""):
        if keep is not None:
            keep.append(line)
        dst.write(line)
        dst.flush()
    src.close()


def _stop(procs, grace: float = 10.0):
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
    t0 = time.time()
    while time.time() - t0 < grace and any(p.poll() is None for p in procs):
        time.sleep(0.1)
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()


def launch_ranks(script: str, argv: List[str], world: int, timeout_s: float = 1500.0,
                 port: Optional[int] = None, python: Optional[str] = None) -> int:
    """Run `python script argv` as `world` ranks; return the exit status for the parent."""
    port = port or free_port()
    key = f"{os.getpid()}_{port}_{time.time_ns()}"  # private rendezvous directory of this job
    procs, pumps = [], []
    out_bin = sys.stdout.buffer
    err_bin = sys.stderr.buffer
    for r in range(world):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(world),
                    "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0",
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                    "QSIM_RDZV_KEY": key})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        p = subprocess.Popen([python or sys.executable, "-u", script] + list(argv), env=env,
                             stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL,
                             stderr=subprocess.PIPE, start_new_session=True)
        procs.append(p)
        if r == 0:
            t = threading.Thread(target=_pump, args=(p.stdout, out_bin, None), daemon=True)
            t.start()
            pumps.append(t)
        t = threading.Thread(target=_pump, args=(p.stderr, err_bin, None), daemon=True)
        t.start()
        pumps.append(t)
    rc = 0
    t0 = time.time()
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0] if bad[0] > 0 else 128 - bad[0]
                failed = [r for r, c in enumerate(codes) if c not in (None, 0)]
                sys.stderr.write(f"[launch] rank(s) {failed} failed (status {bad[0]}); stopping "
                                 f"the others\n")
                break
            if all(c == 0 for c in codes):
                break
            if time.time() - t0 > timeout_s:
                sys.stderr.write(f"[launch] time limit {timeout_s:.0f} s reached; stopping ranks\n")
                rc = 124
                break
            time.sleep(0.05)
    except KeyboardInterrupt:
        rc = 130
    finally:
        _stop(procs)
        for t in pumps:
            t.join(timeout=5)
    return rc
