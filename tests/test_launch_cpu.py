"""CPU: bench.py's N-rank launch contract (no GPU).

* `bench.py --gpus N --dry-run` with no WORLD_SIZE self-launches N rank processes
  (qsim_amd/launch.py), runs the sharded bench skeleton (rendezvous, per-rank host remap planner,
  barriers, max-over-ranks timing) and prints exactly ONE JSON line from rank 0.
* A failing rank makes the launcher stop its peers and exit non-zero; a rank that never arrives
  makes the rendezvous raise instead of hanging.
"""
import json
import os
import subprocess
import sys
import tempfile
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "QSIM_RDZV_KEY"):
        env.pop(k, None)
    return env


@pytest.mark.parametrize("world", [2, 4])
def test_dry_run_launch_prints_one_json_line(world):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(world), "--dry-run", "--steps", "2",
                        "--warmup", "1", "--qubits", "24", "--cpu-budget", "1"], capture_output=True,
                       text=True, timeout=300, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == world and out["dry_run"] is True
    assert out["steps"] == 2 and out["value"] > 0 and out["scaling"] == "strong"
    assert out["config"]["remaps_per_step"] >= 1  # W-HC at 24q needs at least one remap per run
    # the N > 1 line's complete shape — roofline, comm and cpu_baseline (rank 0,
    # after the timed region)
    L = 24 - (world.bit_length() - 1)
    roof = out["roofline"]
    assert roof["bound"] == "hbm" and roof["peak"] == 8000.0 and roof["alg_bytes_per_launch"] == 32.0 * 2 ** L
    for k in ("achieved", "frac", "traffic", "avg_launch_ms"):
        assert k in roof
    assert out["comm"]["bytes_sent_per_step"] >= 16 * 2 ** L * 0.5  # at least one remap of k >= 1
    cb = out["cpu_baseline"]
    assert cb["kind"] == "port" and cb["cores"] == 1 and cb["value"] > 0 and "prefix" in cb["sample"]
    assert cb["w_hc_20q"]["value"] > 0
    # the N = 1 line's statistic (gates / median synchronised step) at every N,
    # and the PMC traffic field with its source
    assert "median" in out["value_is"] and out["value_mean"] > 0
    assert abs(out["value"] - out["config"]["gates"] / (out["ms_per_step"] / 1e3)) <= 0.01 * out["value"]
    assert "traffic_source" in roof


def test_launcher_parent_does_not_load_the_engine():
    """The self-launching parent of `bench.py --gpus N` never touches the GPU: after its ranks
    have run, its own /proc/self/maps holds no libqsim_hip / RCCL / hipRTC / HIP runtime."""
    code = ("import importlib.util, sys\n"
            f"sys.argv = [{BENCH!r}, '--gpus', '2', '--dry-run', '--steps', '1', '--warmup', '1', "
            "'--qubits', '20']\n"
            f"spec = importlib.util.spec_from_file_location('bench', {BENCH!r})\n"
            "m = importlib.util.module_from_spec(spec); spec.loader.exec_module(m)\n"
            "try:\n    m.main()\n    rc = 0\nexcept SystemExit as e:\n    rc = e.code\n"
            "maps = open('/proc/self/maps').read()\n"
            "bad = [k for k in ('libqsim_hip', 'librccl', 'libhiprtc', 'libamdhip64') if k in maps]\n"
            "print('PARENT_MAPS', bad, file=sys.stderr)\n"
            "sys.exit(rc if not bad else 9)\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       env=_env())
    assert "PARENT_MAPS []" in r.stderr, r.stderr[-2000:]
    assert r.returncode == 0, r.stderr[-2000:]
    assert len([ln for ln in r.stdout.splitlines() if ln.strip()]) == 1


def test_failing_rank_stops_launch():
    sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))
    from qsim_amd.launch import launch_ranks
    with tempfile.TemporaryDirectory() as d:
        script = os.path.join(d, "rank.py")
        with open(script, "w") as f:
            f.write("import os, sys, time\n"
                    "r = int(os.environ['RANK'])\n"
                    "if r == 1: sys.exit(3)\n"
                    "time.sleep(120)\n")
        t0 = time.time()
        rc = launch_ranks(script, [], 3, timeout_s=100)
        assert rc == 3
        assert time.time() - t0 < 60  # the sleeping ranks were stopped, not waited for


def test_rendezvous_times_out_on_missing_rank():
    sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))
    from qsim_amd.rendezvous import FileGroup
    with tempfile.TemporaryDirectory() as d:
        g = FileGroup(0, 2, key="t", timeout_s=0.5, root=d)
        with pytest.raises(TimeoutError):
            g.barrier()


def test_rendezvous_collectives_in_process():
    sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))
    from qsim_amd.rendezvous import FileGroup
    import threading
    with tempfile.TemporaryDirectory() as d:
        res = {}

        def rank(r):
            g = FileGroup(r, 3, key="c", timeout_s=30, root=d)
            uid = g.broadcast(b"id-bytes" if r == 0 else None)
            m = g.all_reduce_max(float(r) * 1.5)
            lo = g.all_reduce_min(float(r) + 2)
            g.close()
            res[r] = (uid, m, lo)

        ts = [threading.Thread(target=rank, args=(r,)) for r in range(3)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(60)
        assert res == {r: (b"id-bytes", 3.0, 2.0) for r in range(3)}
        assert not os.path.exists(os.path.join(d, "qsim_rdzv_c"))


@pytest.mark.parametrize("world,total", [(2, 1024), (4, 1023)])
def test_batch_dry_run_shards_trajectories(world, total):
    """`bench.py --workload batch --gpus N --dry-run`: N ranks take contiguous trajectory shares
    (sizes differ by at most one, covering the ensemble), the trajectory-weighted reduction of the
    ranks' averages is a probability vector, one JSON line."""
    r = subprocess.run([sys.executable, BENCH, "--workload", "batch", "--gpus", str(world), "--dry-run",
                        "--steps", "2", "--warmup", "1", "--qubits", "10", "--trajectories", str(total),
                        "--cpu-budget", "1"],
                       capture_output=True, text=True, timeout=300, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    per = out["config"]["trajectories_per_rank"]
    assert out["n_gpus"] == world and out["dry_run"] is True and out["unit"] == "trajectory-gates/s"
    assert sum(per) == total and max(per) - min(per) <= 1
    assert abs(out["config"]["ensemble_probability_sum"] - 1.0) < 1e-12
    # median statistic and the CPU baseline on rank 0 (the oracle's batched
    # reference-process restatement on a bounded sample)
    assert "median" in out["value_is"]
    cb = out["cpu_baseline"]
    assert cb["kind"] == "port" and cb["unit"] == "trajectory-gates/s" and cb["value"] > 0


def test_split_trajectories_covers_the_ensemble():
    sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))
    from qsim_amd.dist_bench import split_trajectories
    for total in (1, 7, 1024, 1023):
        for world in (1, 2, 3, 8):
            spans = [split_trajectories(total, world, r) for r in range(world)]
            assert spans[0][0] == 0
            for (f0, c0), (f1, _) in zip(spans, spans[1:]):
                assert f0 + c0 == f1
            assert spans[-1][0] + spans[-1][1] == total
