"""bench.py's N > 1 leg: the sharded state over N GPUs of one node (strong scaling: the n-qubit
circuit is fixed, each of the N ranks holds 2^n / N amplitudes).

One process per GPU (device = LOCAL_RANK), started by `torch.distributed.run` or by bench.py's
own launcher (`qsim_amd/launch.py`, when no WORLD_SIZE is set).  The host-side rendezvous —
broadcast of the RCCL unique id, the timing barriers, the max-over-ranks wall time — goes through
`qsim_amd.rendezvous.FileGroup` (single node; torch is deliberately not imported next to the
engine, see that module), every wait bounded by QSIM_DIST_INIT_TIMEOUT.  All state traffic goes
through the engine's RCCL communicator over xGMI (non-blocking communicator, aborted on error or
timeout, csrc/hip/dist.hip).

`--dry-run` runs the same skeleton without the GPU: rendezvous, the host remap planner of this
rank once per step (its qubit map carried from step to step as in a real run), barriers and the
max-over-ranks timing; the JSON line says "dry_run": true and its value is planner speed, not a
measurement of the engine.
"""
from __future__ import annotations

import json
import os
import time

from .rendezvous import FileGroup


def _rank_world(args):
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(args.gpus)))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def _circuit(args):
    from . import circuit as qc
    n = args.qubits
    if args.workload == "hc":
        return (qc.createRandomHCCircuit(n, args.depth, args.seed),
                f"W-HC random H+CNOT depth-{args.depth} seed {args.seed}")
    return qc.createScalingBenchmarkCircuit(n), "W-REF benchmark_scaling.cu:69-76 (100 H + 20 CNOT)"


def _median(xs):
    xs = sorted(xs)
    m = len(xs) // 2
    return xs[m] if len(xs) % 2 else 0.5 * (xs[m - 1] + xs[m])


def _step_max(grp, step_s):
    """Per-step max over ranks of each rank's synchronised step times (one all-gather after the
    timed region): the statistic of the N = 1 line (bench.py: gates / median step) at every N."""
    import struct
    parts = grp.all_gather(struct.pack(f"{len(step_s)}d", *step_s))
    per_rank = [struct.unpack(f"{len(step_s)}d", p) for p in parts]
    return [max(col) for col in zip(*per_rank)]


def _pmc_traffic(name: str, kernel: str):
    """HBM bytes per launch of `kernel` from profiles/<name> (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE,
    corrected as profiles/ README says), or (None, None) when no such measurement is committed."""
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    path = os.path.join(root, "profiles", name)
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        ent = json.load(f).get("kernels", {}).get(kernel, {})
    t = ent.get("hbm_bytes_per_launch")
    return t, (os.path.relpath(path, root) if t is not None else None)


def _cpu_baseline(cpu_fn, circuit, n):
    """Rank 0, after the timed region and its max-over-ranks reduction (so it cannot disturb the
    measurement): bench.py's cpu_baseline leg (the oracle's single-thread restatement of the
    reference CPUSimulator on a bounded prefix of the same circuit, plus its 20q / 28q entries)."""
    if cpu_fn is None:
        return None
    from . import circuit as qc
    return cpu_fn(circuit, n, qc)


def run_dry(args, metric: str, peak_gbps: float = 8000.0, cpu_fn=None) -> None:
    from .dist import plan
    rank, world, _ = _rank_world(args)
    grp = FileGroup(rank, world)
    circuit, wl = _circuit(args)
    n = args.qubits
    L = n - (world.bit_length() - 1)
    perm = list(range(n))
    remaps, sent = 0, 0.0
    for _ in range(args.warmup):
        steps, perm = plan(circuit, world, rank, perm)
    grp.barrier()
    step_s = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        grp.barrier()  # (the GPU run's per-step device barrier)
        ts = time.perf_counter()
        steps, perm = plan(circuit, world, rank, perm)
        xs = [s for s in steps if s["kind"] == "exchange"]
        remaps += len(xs)
        # each exchange of k global qubits sends (1 - 2^-k) of this rank's 16 B x 2^L shard
        sent += sum(16.0 * (1 << L) * (1.0 - 2.0 ** -s["k"]) for s in xs)
        step_s.append(time.perf_counter() - ts)
    t1 = time.perf_counter()
    grp.barrier()
    wall = max(grp.all_reduce_max(t1 - t0), 1e-9)
    step_max = [max(x, 1e-9) for x in _step_max(grp, step_s)]
    med = _median(step_max)
    # every rank must plan the same exchange skeleton (the lockstep contract of qsim_dist_run)
    if grp.all_reduce_min(remaps) != grp.all_reduce_max(remaps):
        raise RuntimeError("ranks planned different numbers of remaps")
    if rank == 0:
        gates = circuit.getGateCount()
        # the line's full shape; what only the GPU run measures is null (dry_run: true)
        roof = {"bound": "hbm", "kernel": "fused_tile", "achieved": None, "peak": peak_gbps, "unit": "GB/s",
                "frac": None, "traffic": None, "traffic_source": None, "alg_bytes_per_launch": 32.0 * (1 << L),
                "avg_launch_ms": None, "launches": None}
        comm = {"bytes_sent_per_step": sent / max(1, args.steps), "bytes_sent_last_run": None,
                "transfer_ms_per_step": None, "transfer_parts_per_step": None, "sent_GBps": None,
                "local_kernel_ms_per_step": None, "exposed_ms_per_step": None,
                "overlapped_ms_per_step": None, "source": "host planner (bytes); times need the GPU run"}
        print(json.dumps({
            "metric": metric, "value": round(gates / med, 2), "unit": "gates/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(med * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "c128 (complex<double>)",
            "data": "synthetic", "dry_run": True,
            "value_is": "gates / median over steps of the max-over-ranks step time",
            "value_mean": round(gates * args.steps / sum(step_max), 2), "wall_s": round(wall, 4),
            "config": {"workload": wl, "qubits": n, "gates": gates,
                       "remaps_per_step": remaps / max(1, args.steps),
                       "parallelism": f"dry run: host planner on {world} ranks, no GPU"},
            "roofline": roof, "comm": comm,
            "cpu_baseline": _cpu_baseline(cpu_fn, circuit, n)}), flush=True)
    grp.close()


def run(args, metric: str, peak_gbps: float, cpu_fn=None) -> None:
    """cpu_fn(circuit, n, circuit_module) -> the cpu_baseline object (bench.py), timed on rank 0
    after the timed region; None leaves it null."""
    if getattr(args, "dry_run", False):
        run_dry(args, metric, peak_gbps, cpu_fn)
        return
    from .dist import DistributedSimulator, unique_id
    rank, world, local = _rank_world(args)
    grp = FileGroup(rank, world)
    n = args.qubits
    circuit, wl = _circuit(args)
    uid = grp.broadcast(unique_id() if rank == 0 else None, src=0)
    sim = DistributedSimulator(n, rank, world, uid, device=local)
    fused = args.mode == "fused"
    jit = getattr(args, "jit", 2)
    from .plan import set_jit
    set_jit(jit, -1)
    # Each run starts from the qubit map the previous one ended with; the maps soon cycle (the
    # remap planner is deterministic).  Warm up until the start map repeats, so every plan (and,
    # with the JIT on, every compiled pass kernel) the timed runs use has been seen.
    seen = {tuple(sim.perm())}
    for i in range(max(12, args.warmup)):
        sim.run(circuit, fused=fused)
        p = tuple(sim.perm())
        if i + 1 >= args.warmup and p in seen:
            break
        seen.add(p)
    sim.synchronize()
    sim.profile(True)
    grp.barrier()
    # Every step synchronised and timed on its own between device barriers (an all-reduce on the
    # communicator: the ranks leave it within its latency), value = gates / the median over steps
    # of the max-over-ranks step time — the N = 1 line's statistic (bench.py run_single).
    step_s = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sim.barrier()
        ts = time.perf_counter()
        sim.run(circuit, fused=fused)
        sim.synchronize()
        step_s.append(time.perf_counter() - ts)
    t1 = time.perf_counter()
    grp.barrier()
    wall = grp.all_reduce_max(t1 - t0)
    step_max = _step_max(grp, step_s)
    med = _median(step_max)
    stats = sim.profileStats()
    gates = circuit.getGateCount()
    comm = comm_summary(stats, args.steps, sum(step_max), sim.remapBytes())
    comm["fused_remaps_last_run"] = sim.fusedRemaps()
    comm["remap_path"] = ("fused: the last pass before the remap stores into the send buffer's slab "
                          "layout, the step after loads from the receive buffer (no pack / unpack "
                          "kernels)" if comm["fused_remaps_last_run"] else "pack / unpack kernels")
    comms = [json.loads(b.decode()) for b in grp.all_gather(json.dumps(comm).encode())]
    if rank == 0:
        dom = max((s for s in stats if s["name"] != "alltoall_remap"), key=lambda s: s["ms"],
                  default=None)
        roof = None
        if dom and dom["launches"]:
            per = dom["alg_bytes"] / dom["launches"]
            avg_s = dom["ms"] / dom["launches"] / 1e3
            # per-launch HBM bytes of this kernel at the shard's size (rocprofv3 --pmc of the
            # same sharded run on virtual shards, profiles/pmc_dist_<wl>_<n>q_<G>.json)
            traffic, tsrc = _pmc_traffic(f"pmc_dist_{args.workload}_{n}q_{world}.json", dom["name"])
            roof = {"bound": "hbm", "kernel": dom["name"], "achieved": round(per / avg_s / 1e9, 1),
                    "peak": peak_gbps, "unit": "GB/s",
                    "frac": round(per / avg_s / 1e9 / peak_gbps, 4), "traffic": traffic,
                    "traffic_source": tsrc,
                    "alg_bytes_per_launch": per, "avg_launch_ms": round(dom["ms"] / dom["launches"], 4),
                    "launches": dom["launches"]}
        out = {
            "metric": metric, "value": round(gates / med, 2), "unit": "gates/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(med * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "c128 (complex<double>)",
            "data": "synthetic",
            "value_is": "gates / median over steps of the max-over-ranks synchronised step time "
                        "(device barrier before each step); value_mean = gates x steps / sum of them",
            "value_mean": round(gates * args.steps / sum(step_max), 2),
            "ms_per_step_min_max": [round(min(step_max) * 1e3, 3), round(max(step_max) * 1e3, 3)],
            "wall_s": round(wall, 4),
            "config": {"workload": wl, "qubits": n, "gates": gates,
                       "mode": "Fused" if fused else "PerGate", "state_bytes": 16 << n,
                       "pass_kernels": "jit" if jit else "interpreter",
                       "parallelism": f"state sharded by high qubits over {world} GPUs (RCCL all-to-all remaps)"},
            "roofline": roof, "kernels_rank0": stats, "cpu_baseline": None,
            "comm": dict(comms[0], per_rank_transfer_ms=[c["transfer_ms_per_step"] for c in comms],
                         max_exposed_ms=max(c["exposed_ms_per_step"] for c in comms)),
        }
    sim.close()
    if rank == 0:
        out["cpu_baseline"] = _cpu_baseline(cpu_fn, circuit, n)
        print(json.dumps(out), flush=True)
    grp.close()


REMAP_STATS = ("alltoall_remap", "xgmi_transfer")


def comm_summary(stats, steps: int, wall_s: float, sent_last_run: float) -> dict:
    """This rank's remap traffic and where its time went, per step (events on the engine's
    streams, csrc/hip/dist.hip): `xgmi_transfer` spans the grouped ncclSend / ncclRecv of every
    remap part on the comm stream (its bytes: sent + received); the local pass kernels run on the
    compute stream.  exposed = step time - local kernel time (what the remaps add to the step);
    overlapped = transfer time hidden behind local work."""
    by = {s["name"]: s for s in stats}
    xfer = by.get("xgmi_transfer", {"ms": 0.0, "alg_bytes": 0.0, "launches": 0})
    local_ms = sum(s["ms"] for s in stats if s["name"] not in REMAP_STATS) / max(1, steps)
    step_ms = wall_s / max(1, steps) * 1e3
    t_ms = xfer["ms"] / max(1, steps)
    sent = xfer["alg_bytes"] / 2 / max(1, steps)
    exposed = max(0.0, step_ms - local_ms)
    return {"bytes_sent_per_step": sent, "bytes_sent_last_run": sent_last_run,
            "transfer_ms_per_step": round(t_ms, 4),
            "transfer_parts_per_step": xfer["launches"] / max(1, steps),
            "sent_GBps": round(sent / (t_ms / 1e3) / 1e9, 2) if t_ms > 0 else None,
            "local_kernel_ms_per_step": round(local_ms, 4),
            "exposed_ms_per_step": round(exposed, 4),
            "overlapped_ms_per_step": round(max(0.0, t_ms - exposed), 4)}


def split_trajectories(total: int, world: int, rank: int):
    """(first, count) of rank's share of `total` trajectories: contiguous, sizes differing by at
    most one.  The shards' noise draws are keyed by the global index (setTrajectoryOffset)."""
    base, extra = divmod(total, world)
    return rank * base + min(rank, extra), base + (1 if rank < extra else 0)


def run_batch(args, metric: str, peak_gbps: float, cpu_fn=None) -> None:
    """W-BATCH over N GPUs (SURVEY §8(e) "BatchedSimulator shards trivially by trajectory"): each
    rank runs its contiguous share of the --trajectories total (replicas, no data-path exchange;
    strong scaling: the ensemble is fixed), and the ensemble's average probabilities are the
    trajectory-weighted sum of the ranks' averages, reduced once after the timed region.  The
    noise realisations are those of a single-GPU run of the whole ensemble (global trajectory
    keys), so the reduced average is the single-GPU one up to summation order."""
    import numpy as np
    rank, world, local = _rank_world(args)
    grp = FileGroup(rank, world)
    first, count = split_trajectories(args.trajectories, world, rank)
    n = args.qubits
    dry = getattr(args, "dry_run", False)
    from . import circuit as qc
    circuit = qc.createRandomHCCircuit(n, args.depth, args.seed)
    gates = circuit.getGateCount()
    step_s = []
    if dry:  # skeleton only: split, barriers, max-over-ranks timing, the weighted reduction
        grp.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            grp.barrier()
            ts = time.perf_counter()
            step_s.append(time.perf_counter() - ts)
        t1 = time.perf_counter()
        avg = np.full(1 << n, 1.0 / (1 << n))
        stats, roof = [], None
    else:
        from . import simulator as qs
        from .plan import set_jit
        ndev = qs.device_count()
        if local >= ndev:  # replicas may share a GPU (e.g. a 2-rank rehearsal on a 1-GPU box)
            import sys
            print(f"rank {rank}: LOCAL_RANK {local} >= {ndev} visible GPUs, using GPU {local % ndev}",
                  file=sys.stderr)
        qs.set_device(local % ndev)
        set_jit(getattr(args, "jit", 2), -1)
        nm = qs.NoiseModel()
        nm.addDepolarizingAll(n, args.noise)
        sem = qs.BatchedNoise.Reference if args.batch_noise == "reference" else qs.BatchedNoise.Physical
        sim = qs.BatchedSimulator(n, count, nm, noise=sem)
        sim.setSeed(args.seed)
        sim.setTrajectoryOffset(first)
        for _ in range(max(1, args.warmup)):
            sim.run(circuit)
        sim.synchronize()
        sim.profile(True)
        grp.barrier()
        # replicas exchange nothing, so a host barrier's release skew cannot enter a rank's own
        # step time: each step synchronised and timed per rank, max over ranks per step, median
        t0 = time.perf_counter()
        for _ in range(args.steps):
            grp.barrier()
            ts = time.perf_counter()
            sim.run(circuit)
            sim.synchronize()
            step_s.append(time.perf_counter() - ts)
        t1 = time.perf_counter()
        stats = sim.profileStats()
        gate_stats = [s for s in stats if s["alg_bytes"] > 0]
        dom = max(gate_stats, key=lambda s: s["ms"]) if gate_stats else None
        roof = None
        if dom and dom["launches"]:
            per = dom["alg_bytes"] / dom["launches"]
            avg_s = dom["ms"] / dom["launches"] / 1e3
            # per-launch HBM bytes: the same kernels at the same per-rank shape would need a PMC
            # pass per shard size; the committed one is the 1-GPU ensemble's (16q x 1024), used
            # only when this rank runs that shape
            pmc = "pmc_batch_ref_16q.json" if args.batch_noise == "reference" else "pmc_batch_16q.json"
            traffic, tsrc = _pmc_traffic(pmc, dom["name"]) if (n, count) == (16, 1024) else (None, None)
            roof = {"bound": "hbm", "kernel": dom["name"], "achieved": round(per / avg_s / 1e9, 1),
                    "peak": peak_gbps, "unit": "GB/s", "frac": round(per / avg_s / 1e9 / peak_gbps, 4),
                    "traffic": traffic, "traffic_source": tsrc, "alg_bytes_per_launch": per,
                    "avg_launch_ms": round(avg_s * 1e3, 4), "launches": dom["launches"]}
        avg = sim.getAverageProbabilities()
    grp.barrier()
    wall = max(grp.all_reduce_max(t1 - t0), 1e-9)
    step_max = [max(x, 1e-9) for x in _step_max(grp, step_s)]
    med = _median(step_max)
    # ensemble average: sum over ranks of (count_r / total) * average_r (after the timed region)
    parts = grp.all_gather((avg * (count / args.trajectories)).astype(np.float64).tobytes())
    ens = np.sum([np.frombuffer(p, dtype=np.float64) for p in parts], axis=0)
    if rank == 0:
        total = args.trajectories
        print(json.dumps({
            "metric": metric, "value": round(gates * total / med, 1),
            "unit": "trajectory-gates/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(med * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "c128 (complex<double>)",
            "data": "synthetic", "dry_run": bool(dry),
            "value_is": "trajectory-gates / median over steps of the max-over-ranks synchronised step time",
            "value_mean": round(gates * total * args.steps / sum(step_max), 1), "wall_s": round(wall, 4),
            "config": {"workload": f"W-BATCH {n}q x {total} trajectories, depolarizing {args.noise} "
                                   f"on all qubits after every gate, W-HC depth {args.depth} seed {args.seed}",
                       "qubits": n, "trajectories": total, "gates": gates,
                       "trajectories_per_rank": [split_trajectories(total, world, r)[1] for r in range(world)],
                       "ensemble_probability_sum": float(ens.sum()),
                       "parallelism": f"trajectories sharded over {world} GPUs (replicas, no exchange)"},
            "roofline": roof, "kernels_rank0": stats,
            # rank 0, after the timed region and the reductions
            "cpu_baseline": cpu_fn(args) if cpu_fn is not None else None}), flush=True)
    grp.close()
