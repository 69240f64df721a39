"""GPU: the multi-rank sharded path with one process per rank, on the box's single GPU.

RCCL refuses two ranks on one device, so these ranks use the engine's host-staged transport
(qsim_dist_create_hosted, TCP between the processes, tests/dist_hosted.py).  Everything else is the
production multi-rank path of qsim_dist_run: every process plans only its own rank (its own pivot
memo, as on an 8-GPU node), lowers global controls / phases for its rank, packs and unpacks with
its rank's slab maps, and the readouts are collectives.  The gathered states must equal the oracle
(three runs of each circuit, so the qubit map moves through several layouts) at 1e-12, and every
rank must report the same collective values.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _ports(k):
    socks, ports = [], []
    for _ in range(k):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        socks.append(s)
        ports.append(s.getsockname()[1])
    for s in socks:
        s.close()
    return ports


def _launch(world, n, tmp_path, carry=False):
    sys.path.insert(0, HERE)
    ports = _ports(world)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if carry:
        env["QSIM_DIST_CARRY"] = "1"
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "dist_hosted.py"), str(r), str(world),
                               ",".join(map(str, ports)), str(n), str(tmp_path)], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(world)]
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=100)
            outs.append(out.decode(errors="replace")[-3000:])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} failed:\n{outs[r]}"
    return [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]


@pytest.mark.subprocess  # started before this process initialises the GPU (pool rule)
@pytest.mark.parametrize("world,n", [(8, 16), (4, 16)])
def test_rank_processes_with_cross_run_carry(qsim, oracle, tmp_path, world, n):
    """The cross-run carry (QSIM_DIST_CARRY=1) with one process per rank: each rank decides to
    carry its run's last step from the step skeleton alone (roles and pivots, the same on every
    rank) — not from its own passes, whose lowering differs per rank — so every rank carries the
    same runs and plans the next run's pivots with the same carried ones.  States equal the oracle
    at 1e-12, every rank reports the same carried-run count and collective values, and the carry
    merged at least once."""
    sys.path.insert(0, HERE)
    import dist_hosted
    recs = _launch(world, n, tmp_path, carry=True)
    merged = 0
    for name, c in dist_hosted.circuits(qsim, n):
        g = oracle.gates_of(c)
        ref = oracle.run_cpu(n, g + g + g)
        for mode in ("fused", "pergate"):
            key = f"{name}_{mode}"
            if key not in recs[0]["runs"]:
                continue
            np.testing.assert_allclose(np.load(tmp_path / f"{key}.npy"), ref, atol=1e-12, rtol=0, err_msg=key)
            for rec in recs:
                run = rec["runs"][key]
                assert run["carried"] == recs[0]["runs"][key]["carried"], key
                assert run["perm"] == recs[0]["runs"][key]["perm"]
                assert abs(run["total"] - 1.0) < 1e-12
            merged += recs[0]["runs"][key]["carried"]
    assert merged >= 1


@pytest.mark.subprocess  # started before this process initialises the GPU (pool rule)
@pytest.mark.parametrize("world,n", [(2, 14), (4, 16), (8, 16), (8, 10)])
def test_rank_processes_match_oracle(qsim, oracle, tmp_path, world, n):
    sys.path.insert(0, HERE)
    import dist_hosted
    ports = _ports(world)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "dist_hosted.py"), str(r), str(world),
                               ",".join(map(str, ports)), str(n), str(tmp_path)], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(world)]
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=100)
            outs.append(out.decode(errors="replace")[-3000:])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} failed:\n{outs[r]}"
    recs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]
    for name, c in dist_hosted.circuits(qsim, n):
        g = oracle.gates_of(c)
        ref = oracle.run_cpu(n, g + g + g)
        p = np.abs(ref) ** 2
        for mode in ("fused", "pergate"):
            key = f"{name}_{mode}"
            if key not in recs[0]["runs"]:
                continue
            got = np.load(tmp_path / f"{key}.npy")
            np.testing.assert_allclose(got, ref, atol=1e-12, rtol=0, err_msg=key)
            for rec in recs:
                run = rec["runs"][key]
                assert run["perm"] == recs[0]["runs"][key]["perm"]
                assert abs(run["total"] - 1.0) < 1e-12
                for b in range(n):
                    want = p[((np.arange(1 << n) >> b) & 1) == 0].sum()
                    assert abs(run["p0"][b] - want) < 1e-12, (key, b)
            from qsim_amd.dist import plan
            run0 = recs[0]["runs"][key]
            for i, perm_in in enumerate(run0["perms_in"]):
                steps, perm_out = plan(c, world, 0, list(perm_in))
                if i + 1 < len(run0["perms_in"]):
                    assert perm_out == run0["perms_in"][i + 1], (key, i)
                ex = [s for s in steps if s["kind"] == "exchange"]
                piv = sum(1 for s in ex if s["pivots"])
                # every run overlapped exactly its planned pivoted remaps (fused mode)
                assert run0["overlapped"][i] == piv, (key, i, run0["overlapped"], piv)
                if name == "hc300s3" and n - (world.bit_length() - 1) >= 11:
                    assert piv >= 1
                # every rank sent the same share, (1 - 2^-k) of its shard per remap
                L = n - (world.bit_length() - 1)
                want = sum(16.0 * (1 << L) * (1 - 2.0 ** -s["k"]) for s in ex)
                for rec in recs:
                    assert rec["runs"][key]["remap_bytes"][i] == want, (key, i)
