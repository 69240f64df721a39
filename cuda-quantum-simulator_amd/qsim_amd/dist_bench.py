"""bench.py's N > 1 leg: the sharded state over N GPUs of one node (strong scaling: the n-qubit
circuit is fixed, each of the N ranks holds 2^n / N amplitudes).

Launched one process per GPU by `torch.distributed.run`; torch.distributed (gloo, CPU only) is
used for the bootstrap (broadcast of the RCCL unique id), the timing barriers and the max-over-
ranks reduction.  All state traffic goes through the engine's RCCL communicator over xGMI.
"""
from __future__ import annotations

import json
import os
import time


def run(args, metric: str, peak_gbps: float) -> None:
    from . import circuit as qc
    from .dist import DistributedSimulator, unique_id
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(args.gpus)))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29517")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = args.qubits
    if args.workload == "hc":
        circuit = qc.createRandomHCCircuit(n, args.depth, args.seed)
        wl = f"W-HC random H+CNOT depth-{args.depth} seed {args.seed}"
    else:
        circuit = qc.createScalingBenchmarkCircuit(n)
        wl = "W-REF benchmark_scaling.cu:69-76 (100 H + 20 CNOT)"
    obj = [unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    sim = DistributedSimulator(n, rank, world, obj[0], device=local)
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
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sim.run(circuit, fused=fused)
    sim.synchronize()
    t1 = time.perf_counter()
    dist.barrier()
    wall = torch.tensor([t1 - t0], dtype=torch.float64)
    dist.all_reduce(wall, op=dist.ReduceOp.MAX)
    wall = float(wall.item())
    stats = sim.profileStats()
    gates = circuit.getGateCount()
    if rank == 0:
        dom = max((s for s in stats if s["name"] != "alltoall_remap"), key=lambda s: s["ms"],
                  default=None)
        roof = None
        if dom and dom["launches"]:
            per = dom["alg_bytes"] / dom["launches"]
            avg_s = dom["ms"] / dom["launches"] / 1e3
            roof = {"bound": "hbm", "kernel": dom["name"], "achieved": round(per / avg_s / 1e9, 1),
                    "peak": peak_gbps, "unit": "GB/s",
                    "frac": round(per / avg_s / 1e9 / peak_gbps, 4), "traffic": None,
                    "alg_bytes_per_launch": per, "avg_launch_ms": round(dom["ms"] / dom["launches"], 4),
                    "launches": dom["launches"]}
        out = {
            "metric": metric, "value": round(gates * args.steps / wall, 2), "unit": "gates/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "c128 (complex<double>)",
            "data": "synthetic",
            "config": {"workload": wl, "qubits": n, "gates": gates,
                       "mode": "Fused" if fused else "PerGate", "state_bytes": 16 << n,
                       "pass_kernels": "jit" if jit else "interpreter",
                       "parallelism": f"state sharded by high qubits over {world} GPUs (RCCL all-to-all remaps)"},
            "roofline": roof, "kernels_rank0": stats, "cpu_baseline": None,
        }
        print(json.dumps(out))
    sim.close()
    dist.barrier()
    dist.destroy_process_group()
