#!/usr/bin/env python3
"""bench.py — gates/s and achieved HBM bandwidth of the MI355X state-vector engine.

Workload (BASELINE.json metric "gates/s + achieved HBM GB/s (% peak), 100-gate H+CNOT circuit @ n
qubits"): W-HC, the seeded random {H, CNOT} depth-100 circuit (factory
createRandomHCCircuit, mt19937 seed 42) on a complex<double> state of n qubits starting at |0..0>.
Default n = 30: the one configuration that is both HBM-bound on one GPU (16 GiB state >> 256 MiB
Infinity Cache) and the north_star's 1/2/4/8-GPU scaling case (BASELINE.json configs[4]); --qubits
20 / 28 give configs[1] / configs[2].  A step = one run of the circuit (inputs resident in HBM).

One process per GPU (torch.distributed launcher for N > 1): the state is sharded by its high
qubits across ranks (strong scaling: the total work is fixed).  Rank 0 prints ONE JSON line.

roofline: the dominant kernel's algorithmic bytes per launch (a fused pass reads and
writes every amplitude once = 32 B x 2^n; per-gate kernels use the per-gate byte table) divided
by its HIP-event-timed average duration inside the timed region (events on the last tenth of the
timed steps, at least one: at 20 qubits events on every launch would add ~35 % to the step), against
8 TB/s.
roofline_1q28 / roofline_batch16: north_star's single-qubit target (W-1Q, 28 qubits) and BASELINE
config 4 (W-BATCH 16q x 1024 under the reference noise process, the BatchedSimulator default, and
under the physical process) measured in the same run.
cpu_baseline: the oracle's single-threaded C++ restatement of the reference CPUSimulator
(kind "port"), timed on this host on a bounded prefix of the same circuit.
"""
from __future__ import annotations

import argparse
import json
import os
import resource
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cuda-quantum-simulator_amd"))
resource.setrlimit(resource.RLIMIT_CORE, (0, 0))  # an abort fails fast, no core dump
# Every measurement below is a cold one: no kernels or layout decisions from an on-disk cache of
# earlier processes (csrc/hip/cache.hip).  The `first_run_cache` object measures that cache on its
# own, in child processes with a private cache directory.
os.environ.setdefault("QSIM_CACHE", "0")

METRIC = "gates/s + achieved HBM GB/s (% peak), 100-gate H+CNOT circuit @ n qubits"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


PROFILE_REGION = ["none"]


class region:
    """A roctx range named "timed_<name>" (rocprofv3 --marker-trace: scripts/roofline_check.py
    keeps the kernels that start inside it) and roctxProfilerResume(0) / roctxProfilerPause(0)
    (rocprofv3 --selected-regions) around a timed region when --profile-region names it; a no-op
    otherwise (the roctx library is loaded only then)."""
    _lib = None

    def __init__(self, name):
        self.name = name
        self.on = PROFILE_REGION[0] == name

    def __enter__(self):
        if self.on:
            if region._lib is None:
                import ctypes
                region._lib = ctypes.CDLL("librocprofiler-sdk-roctx.so.1")
                region._lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            region._lib.roctxProfilerResume(0)
            region._lib.roctxRangePushA(f"timed_{self.name}".encode())
        return self

    def __exit__(self, *exc):
        if self.on:
            region._lib.roctxRangePop()
            region._lib.roctxProfilerPause(0)
        return False


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--qubits", type=int, default=None,
                   help="default 30 (W-HC / ref / 1q), 16 for --workload batch (W-BATCH)")
    p.add_argument("--depth", type=int, default=100)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--mode", choices=["fused", "per-gate"], default="fused")
    p.add_argument("--jit", type=int, choices=[0, 1, 2], default=2,
                   help="circuit-specialised pass kernels: 0 interpreter only, 1 background "
                        "compile, 2 compile during the first warmup run (default)")
    p.add_argument("--workload", choices=["hc", "ref", "1q", "batch", "dm", "noisy"], default="hc",
                   help="hc: W-HC random H+CNOT; ref: reference benchmark_scaling circuit; "
                        "1q: 100 unfused H gates on targets i %% n; batch: W-BATCH, the W-HC "
                        "circuit on --trajectories noisy trajectories (depolarizing on every "
                        "qubit after every gate, SURVEY §8(d)); dm: DensityMatrixSimulator (default 14 "
                        "qubits); noisy: NoisySimulator (default 26 qubits), both W-HC with "
                        "depolarizing --noise on all qubits")
    p.add_argument("--trajectories", type=int, default=1024)
    p.add_argument("--batch-noise", choices=["physical", "reference"], default="reference",
                   help="W-BATCH noise process: reference (the BatchedSimulator default: per-pair "
                        "draws after every gate, src/NoiseModel.cu:834-892) or physical (one draw "
                        "per trajectory, channel and gate; Pauli frames)")
    p.add_argument("--no-1q28", action="store_true",
                   help="skip the W-1Q 28q single-qubit roofline object of the default line")
    p.add_argument("--no-batch16", action="store_true",
                   help="skip the W-BATCH 16q x 1024 object (BASELINE config 4) of the default line")
    p.add_argument("--no-extras", action="store_true",
                   help="skip the default line's extra objects (seeds, default_mode, w_ref, "
                        "gate_table_20q, dm_14q, noisy_26q)")
    p.add_argument("--extras", default="seeds,default_mode,w_ref,w_hc_28q,w_hc_seq,first_run_cache,h_single,gate_table,dm,noisy",
                   help="which extra objects of the default W-HC line to measure (comma list; "
                        "--no-extras: none)")
    p.add_argument("--noise", type=float, default=0.01)
    p.add_argument("--cpu-budget", type=float, default=12.0,
                   help="seconds of single-thread CPU oracle work for cpu_baseline (0 = skip)")
    p.add_argument("--launch-timeout", type=float, default=1500.0,
                   help="N > 1 without an external launcher: seconds before the rank processes "
                        "are stopped")
    p.add_argument("--dry-run", action="store_true",
                   help="N-rank skeleton without the GPU: gloo bootstrap, the host remap planner "
                        "per rank and step, barriers and max-over-ranks timing (CPU tests)")
    p.add_argument("--pmc-json", default=None,
                   help="per-launch HBM traffic measured by rocprofv3 --pmc (see profiles/)")
    p.add_argument("--profile-region", default="none",
                   choices=["none", "hc", "hc28", "1q28", "batch16ref", "noisy26", "dm14"],
                   help="bracket that timed region (only) with roctxProfilerResume / Pause, for "
                        "rocprofv3 --selected-regions: the profile then holds exactly the launches "
                        "the line's roofline averages (scripts/roofline_check.py recomputes it)")
    a = p.parse_args()
    PROFILE_REGION[0] = a.profile_region
    if a.qubits is None:
        a.qubits = {"batch": 16, "dm": 14, "noisy": 26}.get(a.workload, 30)
    return a


def make_circuit(q, args):
    n = args.qubits
    if args.workload == "hc":
        return q.createRandomHCCircuit(n, args.depth, args.seed), \
            f"W-HC random H+CNOT depth-{args.depth} seed {args.seed}"
    if args.workload == "ref":
        return q.createScalingBenchmarkCircuit(n), "W-REF benchmark_scaling.cu:69-76 (100 H + 20 CNOT)"
    c = q.Circuit(n)
    for i in range(args.depth):
        c.h(i % n)
    return c, f"W-1Q {args.depth} H gates on targets i % n"


def alg_bytes_of_circuit(circuit, n):
    """Sum of per-gate algorithmic bytes — the 'effective' traffic of the circuit."""
    N = float(1 << n)
    total = 0.0
    for g in circuit.getGates():
        t = int(g.type)
        if t in (0, 1, 3, 8, 9, 10):
            total += 32 * N
        elif t in (2, 4, 5, 6, 7, 11, 13, 14, 15):
            total += 16 * N
        else:  # CZ, Toffoli
            total += 8 * N
    return total


def cpu_baseline(circuit, n, budget, q=None, args=None):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy_oracle as orc  # test infrastructure: the CPU baseline leg only
    gates = orc.gates_of(circuit)
    # median of >= 3 runs — three prefix runs of budget / 3 each, median rate
    runs_n = [orc.time_prefix(n, gates, budget / 3.0) for _ in range(3)]
    rates_n = sorted(d / s for d, s in runs_n if s > 0)
    done, secs = runs_n[0]
    full20 = None
    if q is not None and args is not None and args.workload == "hc":
        # BASELINE.md §3 plan: the same W-HC circuit at 20 qubits, whole runs, median of 3
        c20 = q.createRandomHCCircuit(20, args.depth, args.seed)
        g20 = orc.gates_of(c20)
        runs = []
        for _ in range(3):
            d20, s20 = orc.time_prefix(20, g20, 120.0)
            if d20 == len(g20):
                runs.append(s20)
        if runs:
            m = sorted(runs)[len(runs) // 2]
            full20 = {"value": round(len(g20) / m, 2), "unit": "gates/s", "cores": 1, "kind": "port",
                      "sample": f"W-HC depth {args.depth} seed {args.seed} at 20 qubits, median of "
                                f"{len(runs)} whole runs ({', '.join(f'{r:.3f}' for r in runs)} s)"}
    pre28 = None
    if q is not None and args is not None and args.workload == "hc" and budget > 0:
        # BASELINE.md §3 plan: the same circuit family at 28 qubits (config 3), a prefix of it
        c28 = q.createRandomHCCircuit(28, args.depth, args.seed)
        g28 = orc.gates_of(c28)
        r28 = [orc.time_prefix(28, g28, min(budget, 9.0) / 3.0) for _ in range(3)]
        v28 = sorted(d / s for d, s in r28 if d and s > 0)
        if v28:
            pre28 = {"value": round(v28[len(v28) // 2], 3), "unit": "gates/s", "cores": 1, "kind": "port",
                     "sample": f"prefix-extrapolated: W-HC depth {args.depth} seed {args.seed} at 28 qubits, "
                               f"median of 3 prefix runs ({', '.join(str(d) for d, _ in r28)} gates in "
                               f"{', '.join(f'{s:.1f}' for _, s in r28)} s), single thread"}
    cpu_model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": rates_n[len(rates_n) // 2] if rates_n else None, "unit": "gates/s", "cores": 1,
            "kind": "port", "w_hc_20q": full20, "w_hc_28q": pre28,
            "sample": f"prefix-extrapolated: median of 3 prefix runs of the same circuit at n={n} "
                      f"({', '.join(str(d) for d, _ in runs_n)} gates in "
                      f"{', '.join(f'{s:.1f}' for _, s in runs_n)} s), single thread ({cpu_model}; host "
                      f"has {os.cpu_count()} logical CPUs); value = median of prefix gates / prefix time"}


def batch_cpu_baseline(args, trajectories=4):
    """W-BATCH CPU baseline (kind "port"): the oracle's restatement of the reference batched noise
    process (oracle/numpy_oracle.py batched_reference_run: per gate the C++ CPUSimulator
    restatement on every trajectory, then one per-pair depolarizing pass per channel entry,
    src/NoiseModel.cu:815-892) on `trajectories` trajectories of the same circuit and noise, gate by
    gate until --cpu-budget seconds; value = trajectories x gates done / seconds."""
    if args.cpu_budget <= 0:
        return None
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy_oracle as orc  # test infrastructure: the CPU baseline leg only
    from qsim_amd import circuit as qc
    n = args.qubits
    gates = orc.gates_of(qc.createRandomHCCircuit(n, args.depth, args.seed))
    chans = [(0, qq, args.noise) for qq in range(n)]
    st, counter, done = None, 0, 0
    t0 = time.perf_counter()
    while done < len(gates) and time.perf_counter() - t0 < args.cpu_budget:
        st, counter = orc.batched_reference_run(n, trajectories, [gates[done]], chans, args.seed,
                                                states=st, counter=counter)
        done += 1
    secs = time.perf_counter() - t0
    return {"value": round(trajectories * done / secs, 2), "unit": "trajectory-gates/s", "cores": 1,
            "kind": "port",
            "sample": f"{trajectories} trajectories x the first {done} of {len(gates)} gates at {n} qubits "
                      f"with depolarizing {args.noise} on all qubits after every gate, {secs:.1f} s, single "
                      f"thread (numpy + the C++ oracle; same process and draws as the engine's reference "
                      f"noise path)"}


H_SINGLE_REF_MS = {20: 0.035, 24: 2.7, 26: 9.9}  # README.md:373-377 (benchmark_custatevec.cu)


def h_single_synced(q, sizes=(12, 16, 18, 20, 22, 24, 26), warmup=3, iterations=10):
    """The reference's Hadamard scaling benchmark (benchmarks/benchmark_custatevec.cu:60-78 timing
    helper, :233-290 loop): one H on target 0 of an n-qubit |0..0> state, `warmup` synchronised
    launches, then `iterations` launches back to back between two device synchronisations, the
    mean per launch; here through the per-gate kernel entry (StateVector.applyGate, the
    applyH<<<>>> analogue), beside the published times (README.md:373-377, RTX 4070 laptop)."""
    rows = []
    for n in sizes:
        sv = q.StateVector(n)
        op = q.GateOp(q.GateType.H, [0])
        for _ in range(warmup):
            sv.applyGate(op)
            sv.synchronize()
        sv.synchronize()
        t0 = time.perf_counter()
        for _ in range(iterations):
            sv.applyGate(op)
        sv.synchronize()
        ms = (time.perf_counter() - t0) / iterations * 1e3
        sv.close()
        rows.append({"qubits": n, "ms": round(ms, 4), "GBps": round(32.0 * (1 << n) / (ms / 1e3) / 1e9, 1),
                     "reference_readme_ms": H_SINGLE_REF_MS.get(n),
                     "speedup_vs_reference": round(H_SINGLE_REF_MS[n] / ms, 1) if n in H_SINGLE_REF_MS else None})
    return {"workload": "one H on target 0, mean of 10 back-to-back launches between synchronisations "
                        "(benchmark_custatevec.cu benchmarkScaling)", "rows": rows}


def w_hc_28q(q, args, steps=10):
    """BASELINE config 3 in the default line: createRandomHCCircuit(28, depth, seed) in the line's
    mode (calibrated first run, specialised pass kernels), gates / median synchronised step, and
    the pass kernels' roofline from per-launch HIP events on every timed step (the launches a
    --profile-region hc28 rocprof profile records), PMC traffic from profiles/pmc_hc_28q.json."""
    from qsim_amd.plan import set_jit
    set_jit(args.jit, -1)
    n = 28
    c = q.createRandomHCCircuit(n, args.depth, args.seed)
    sim = q.Simulator(n)
    tf = time.perf_counter()
    sim.run(c)
    sim.synchronize()
    first = time.perf_counter() - tf
    sim.run(c)
    sim.synchronize()
    sim.state.profileReset()
    sim.state.profile(True)
    ts_ = []
    with region("hc28"):
        for _ in range(steps):
            t0 = time.perf_counter()
            sim.run(c)
            sim.synchronize()
            ts_.append(time.perf_counter() - t0)
    stats = sim.state.profileStats()
    sim.state.profile(False)
    info = sim.state.layoutInfo()
    passes = sim.state.lastRunInfo()[0]
    del sim
    med = _median(ts_)
    # the pass kernels together (every launch moves 32 B x 2^28 whatever its name)
    pk = [s_ for s_ in stats if s_["alg_bytes"] > 0 and s_["launches"]]
    launches = sum(s_["launches"] for s_ in pk)
    ms = sum(s_["ms"] for s_ in pk)
    by = sum(s_["alg_bytes"] for s_ in pk)
    roof = None
    if launches:
        ach = by / (ms / 1e3) / 1e9
        traffic, tsrc = None, None
        pmc_path = os.path.join(ROOT, "profiles", "pmc_hc_28q.json")
        if os.path.exists(pmc_path):
            with open(pmc_path) as f:
                kern = json.load(f).get("kernels", {})
            ents = [kern[s_["name"]] for s_ in pk if s_["name"] in kern]
            tl = sum(e["launches"] for e in ents)
            if ents and tl:
                traffic = sum(e["hbm_bytes_per_launch"] * e["launches"] for e in ents) / tl
                tsrc = os.path.relpath(pmc_path, ROOT)
        roof = {"bound": "hbm", "kernels": sorted(s_["name"] for s_ in pk), "achieved": round(ach, 1),
                "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBPS, 4),
                "traffic": traffic, "traffic_source": tsrc, "alg_bytes_per_launch": by / launches,
                "avg_launch_ms": round(ms / launches, 4), "launches": launches}
    return {"workload": f"W-HC createRandomHCCircuit(28, {args.depth}, {args.seed}) (BASELINE config 3)",
            "value": round(c.getGateCount() / med, 1), "unit": "gates/s", "ms_per_step": round(med * 1e3, 3),
            "steps": steps, "passes": passes, "tile_qubits": info["tile_qubits"], "relayout": info["relayout"],
            "calibrated": info["calibrated"], "first_run_ms": round(first * 1e3, 1), "roofline": roof,
            "kernels": stats}


def w_hc_seq(q, args, reps=4, steps=5):
    """Consecutive W-HC circuits as ONE engine run (Simulator.runSequence; not the headline, whose
    step is one run() of one circuit): `reps` copies of the line's circuit, and `reps` circuits of
    consecutive seeds, each planned as a whole — a pass may hold the end of one circuit and the
    start of the next.  Per sequence: calibrated first run on |0..0>, one warm-up, the median of
    `steps` synchronised sequences; value = gates of the sequence / that median."""
    from qsim_amd.plan import set_jit
    set_jit(args.jit, -1)
    n = args.qubits
    out = {"workload": f"{reps} consecutive createRandomHCCircuit({n}, {args.depth}, .) per "
                       f"Simulator.runSequence call (same mode as the line)", "runs": []}
    for label, seeds in (("same", [args.seed] * reps), ("seeds", [args.seed + i for i in range(reps)])):
        circs = [q.createRandomHCCircuit(n, args.depth, sd) for sd in seeds]
        gates = sum(c.getGateCount() for c in circs)
        sim = q.Simulator(n)
        t0 = time.perf_counter()
        sim.runSequence(circs)
        sim.synchronize()
        first = time.perf_counter() - t0
        sim.runSequence(circs)
        sim.synchronize()
        ts_ = []
        for _ in range(steps):
            t0 = time.perf_counter()
            sim.runSequence(circs)
            sim.synchronize()
            ts_.append(time.perf_counter() - t0)
        med = _median(ts_)
        info = sim.state.layoutInfo()
        passes = sim.state.lastRunInfo()[0]
        del sim
        out["runs"].append({"circuits": label, "seeds": seeds, "gates": gates, "value": round(gates / med, 1),
                            "unit": "gates/s", "ms_per_sequence": round(med * 1e3, 3),
                            "passes": passes, "passes_per_circuit": round(passes / reps, 3),
                            "relayout": info["relayout"], "tile_qubits": info["tile_qubits"],
                            "first_run_ms": round(first * 1e3, 1)})
    return out


def first_run_cache(n, seed):
    """The first run of the same circuit in a NEW process, without and with the on-disk cache of
    an earlier process (csrc/hip/cache.hip: pass-kernel code objects and the layout decision):
    scripts/first_run.py in three child processes sharing one private cache directory — cold
    (empty cache), warm (the first one's entries), and the library with the cache off."""
    import subprocess
    import tempfile
    out = {"workload": f"first sim.run of W-HC seed {seed} at {n} qubits in a new process (jit = 2, "
                       f"calibrated first run), private cache directory"}
    with tempfile.TemporaryDirectory() as d:
        env = dict(os.environ, QSIM_CACHE="1", QSIM_CACHE_DIR=d)
        for tag in ("cold", "warm"):
            r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "first_run.py"), str(n), str(seed)],
                               capture_output=True, text=True, timeout=600, env=env)
            if r.returncode != 0:
                out[tag] = {"error": r.stderr[-500:]}
                return out
            rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
            rec.pop("p0", None)
            out[tag] = rec
    return out


def run_single(args):
    import qsim_amd as q
    n = args.qubits
    circuit, wl = make_circuit(q, args)
    mode = q.RunMode.Fused if args.mode == "fused" else q.RunMode.PerGate
    if args.workload == "1q":
        mode = q.RunMode.PerGate
    from qsim_amd.plan import set_jit
    set_jit(args.jit, -1)
    sim = q.Simulator(n, mode=mode)
    # the first run() on |0..0> alone: what a one-shot sim.run(c) user pays (layout choice,
    # calibration candidates timed on the device, pass-kernel compiles, the run itself)
    first_run_ms = None
    for i in range(max(1, args.warmup) if args.jit else args.warmup):
        tf = time.perf_counter()
        sim.run(circuit)
        if i == 0:
            sim.synchronize()
            first_run_ms = round((time.perf_counter() - tf) * 1e3, 1)
    sim.synchronize()
    sim.state.profileReset()
    sim.synchronize()
    # Per-launch HIP events cost ~5 us per launch: negligible against a pass of >= 24 qubits
    # (0.08 ms and up), so there every timed step carries them and the roofline averages exactly
    # the launches a --profile-region hc profile records; below 24 qubits (a 20-qubit pass is
    # ~15 us) only the last tenth of the timed steps (at least one) does.
    # Every step is synchronised and timed on its own (the median of >= 10 steps);
    # at 30 qubits a step is ~25 ms, the per-step synchronisation ~20 us.
    prof_from = 0 if n >= 24 else args.steps - max(1, args.steps // 10)
    step_s = []
    t0 = time.perf_counter()
    with region("hc"):
        for i in range(args.steps):
            if i == prof_from:
                sim.state.profile(True)
            ts = time.perf_counter()
            sim.run(circuit)
            sim.synchronize()
            step_s.append(time.perf_counter() - ts)
    t1 = time.perf_counter()
    stats = sim.state.profileStats()
    sim.state.profile(False)
    wall = t1 - t0
    med = sorted(step_s)[len(step_s) // 2] if len(step_s) % 2 else \
        0.5 * sum(sorted(step_s)[len(step_s) // 2 - 1:len(step_s) // 2 + 1])
    gates = circuit.getGateCount()
    layout = sim.state.layoutInfo()
    run_passes = sim.state.lastRunInfo()[0]
    # what the timed loop never pays: the first index-based readback after a relabeled run
    # restores the identity layout with a fused SWAP network
    restore_ms = None
    if layout["relabeled"]:
        tr = time.perf_counter()
        sim.state.restoreLayout()
        sim.synchronize()
        restore_ms = round((time.perf_counter() - tr) * 1e3, 3)
        restore_passes = 1 if os.environ.get("QSIM_RESTORE_ONE_PASS", "1") != "0" and n >= 16 else None
    dom = max(stats, key=lambda s: s["ms"]) if stats else None
    roof = None
    if dom and dom["launches"]:
        per_launch_bytes = dom["alg_bytes"] / dom["launches"]
        avg_s = dom["ms"] / dom["launches"] / 1e3
        achieved = per_launch_bytes / avg_s / 1e9
        traffic, traffic_src = None, None
        pmc_path = args.pmc_json or os.path.join(ROOT, "profiles", f"pmc_{args.workload}_{n}q.json")
        if os.path.exists(pmc_path):
            with open(pmc_path) as f:
                pmc = json.load(f)
            ent = pmc.get("kernels", pmc).get(dom["name"], {})
            traffic = ent.get("hbm_bytes_per_launch")
            traffic_src = os.path.relpath(pmc_path, ROOT) if traffic is not None else None
        roof = {"bound": "hbm", "kernel": dom["name"], "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic, "traffic_source": traffic_src,
                "alg_bytes_per_launch": per_launch_bytes,
                "avg_launch_ms": round(dom["ms"] / dom["launches"], 4),
                "launches": dom["launches"]}
    eff = alg_bytes_of_circuit(circuit, n) * args.steps / wall / 1e9
    out = {
        "metric": METRIC, "value": round(gates / med, 2), "unit": "gates/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(med * 1e3, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "c128 (complex<double>)",
        "data": "synthetic",
        "value_mean": round(gates * args.steps / wall, 2),
        "ms_per_step_mean": round(wall / args.steps * 1e3, 3),
        "ms_per_step_min_max": [round(min(step_s) * 1e3, 3), round(max(step_s) * 1e3, 3)],
        "config": {"workload": wl, "qubits": n, "gates": gates, "mode": mode.name,
                   "pass_kernels": "jit" if args.jit else "interpreter",
                   "jit_mode": args.jit, "tile_qubits": layout["tile_qubits"],
                   "calibrated": layout["calibrated"], "relabel": layout["relabeled"],
                   "relayout": layout["relayout"], "passes": run_passes,
                   "state_bytes": 16 << n, "parallelism": "single GPU"},
        "value_is": "gates / median step time (every step synchronised); value_mean = gates x steps / wall",
        "first_run_ms": first_run_ms,
        "restore_ms": restore_ms,
        "restore_passes": restore_passes if restore_ms is not None else None,
        "roofline": roof,
        "effective_GBps": round(eff, 1),
        "kernels": stats,
    }
    del sim
    ex = set() if args.no_extras else set(args.extras.split(","))
    if args.workload == "hc":
        if "seeds" in ex:
            out["seeds"] = hc_seeds(q, args)
        if "default_mode" in ex:
            out["default_mode"] = default_mode(q, args, circuit)
        if "w_ref" in ex:
            out["w_ref"] = w_ref(q, args)
        if "w_hc_28q" in ex:
            out["w_hc_28q"] = w_hc_28q(q, args)
        if "w_hc_seq" in ex:
            out["w_hc_seq"] = w_hc_seq(q, args)
        if "first_run_cache" in ex:
            out["first_run_cache"] = first_run_cache(n, args.seed)
        if "h_single" in ex:
            out["h_single_synced"] = h_single_synced(q)
        if "gate_table" in ex:
            out["gate_table_20q"] = gate_table_20q(q)
        if "dm" in ex:
            out["dm_14q"] = measure_dm(q, 14, 3, 1, args.jit, args.seed, args.depth, 0.01)
        if "noisy" in ex:
            out["noisy_26q"] = measure_noisy(q, 26, 3, 1, args.seed, args.depth, 0.01)
    if args.workload == "hc" and not args.no_1q28:
        out["roofline_1q28"] = roofline_1q28(q)
    if args.workload == "hc" and not args.no_batch16:
        out["roofline_batch16"] = roofline_batch16(q, args)
    if args.cpu_budget > 0:
        out["cpu_baseline"] = cpu_baseline(circuit, n, args.cpu_budget, q, args)
    else:
        out["cpu_baseline"] = None
    print(json.dumps(out))


def _median(xs):
    xs = sorted(xs)
    m = len(xs) // 2
    return xs[m] if len(xs) % 2 else 0.5 * (xs[m - 1] + xs[m])


def _timed_runs(sim, circuit, steps):
    """Median wall time of `steps` synchronised runs (seconds)."""
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        sim.run(circuit)
        sim.synchronize()
        ts.append(time.perf_counter() - t0)
    return _median(ts)


def hc_seeds(q, args, seeds=(1, 2, 3, 4), steps=5):
    """W-HC at the line's size for seeds 1-4 beside the headline seed: each seed's
    calibrated first run on |0..0> (its first_run_ms), one warm-up run, then the median of
    `steps` synchronised runs; passes / relayout / tile height of the plan it keeps."""
    n = args.qubits
    from qsim_amd.plan import set_jit
    set_jit(args.jit, -1)
    sim = q.Simulator(n)
    out = {"workload": f"W-HC depth {args.depth} at {n} qubits, seeds {list(seeds)}, same mode as the line",
           "runs": []}
    for sd in seeds:
        sim.reset()
        c = q.createRandomHCCircuit(n, args.depth, sd)
        t0 = time.perf_counter()
        sim.run(c)
        sim.synchronize()
        first = time.perf_counter() - t0
        sim.run(c)
        med = _timed_runs(sim, c, steps)
        info = sim.state.layoutInfo()
        out["runs"].append({"seed": sd, "value": round(c.getGateCount() / med, 1), "unit": "gates/s",
                            "ms_per_step": round(med * 1e3, 3), "passes": sim.state.lastRunInfo()[0],
                            "relayout": info["relayout"], "tile_qubits": info["tile_qubits"],
                            "first_run_ms": round(first * 1e3, 1)})
    del sim
    vals = [r["value"] for r in out["runs"]]
    out["min"], out["max"] = min(vals), max(vals)
    return out


def default_mode(q, args, circuit, steps=10, compile_wait_s=60.0):
    """The same circuit at the library defaults (jit = 1: pass kernels compiled in the background
    while the interpreter runs; no device calibration: the layout model's untimed choice).  The
    first run is timed alone (what a one-shot user pays); then runs continue until every pass
    runs its compiled kernel, and `steps` synchronised runs are timed."""
    from qsim_amd.plan import DEFAULTS, set_jit
    set_jit(*DEFAULTS["jit"])
    try:
        n = circuit.getNumQubits()
        sim = q.Simulator(n)
        t0 = time.perf_counter()
        sim.run(circuit)
        sim.synchronize()
        first = time.perf_counter() - t0
        runs_before_compiled = 1
        tw = time.perf_counter()
        while True:
            passes, jit_passes = sim.state.lastRunInfo()
            if jit_passes >= passes or time.perf_counter() - tw > compile_wait_s:
                break
            sim.run(circuit)
            sim.synchronize()
            runs_before_compiled += 1
        med = _timed_runs(sim, circuit, steps)
        info = sim.state.layoutInfo()
        passes, jit_passes = sim.state.lastRunInfo()
        out = {"value": round(circuit.getGateCount() / med, 1), "unit": "gates/s",
               "ms_per_step": round(med * 1e3, 3), "first_run_ms": round(first * 1e3, 1),
               "runs_before_compiled": runs_before_compiled, "passes": passes,
               "jit_passes": jit_passes, "relayout": info["relayout"], "relabel": info["relabeled"],
               "tile_qubits": info["tile_qubits"], "calibrated": info["calibrated"],
               "mode": "library default: jit 1 (background compile), no calibration"}
        del sim
        return out
    finally:
        set_jit(args.jit, -1)


# README.md:30-38 (RTX 4070 laptop, GPU times taken without a device synchronisation) and :58-63
REF_W_REF_MS = {20: {"gpu_ms": 0.28, "cpu_ms": 143.50}, 22: {"gpu_ms": 0.28, "cpu_ms": 720.39}}
REF_GATE_TABLE_20Q = {"CNOT": 53200, "X": 34300, "H": 24600, "Rz": 5940}


def w_ref(q, args, sizes=(20, 22), steps=20):
    """The reference's own GPU-vs-CPU workload (benchmarks/benchmark_scaling.cu:69-76: 100 H on
    i % n plus a CNOT(i % n, (i+1) % n) every 5th, 120 gates) at 20 and 22 qubits: the engine in
    the line's mode (median of `steps` synchronised runs after warm-up) beside the oracle's
    single-thread CPUSimulator restatement on this host (one whole run) and the README numbers."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy_oracle as orc  # test infrastructure: the CPU column only
    from qsim_amd.plan import set_jit
    set_jit(args.jit, -1)
    rows = []
    for n in sizes:
        c = q.createScalingBenchmarkCircuit(n)
        sim = q.Simulator(n)
        for _ in range(3):
            sim.run(c)
        sim.synchronize()
        med = _timed_runs(sim, c, steps)
        del sim
        g = orc.gates_of(c)
        done, secs = orc.time_prefix(n, g, 60.0)
        rows.append({"qubits": n, "gates": c.getGateCount(), "gpu_ms": round(med * 1e3, 4),
                     "gates_per_s": round(c.getGateCount() / med, 1),
                     "cpu_ms": round(secs * 1e3, 2) if done == len(g) else None, "cpu_cores": 1,
                     "speedup_vs_cpu": round(secs / med, 1) if done == len(g) else None,
                     "reference_readme": REF_W_REF_MS.get(n)})
    return {"workload": "W-REF benchmark_scaling.cu:69-76 (100 H + 20 CNOT)", "rows": rows,
            "note": "reference README GPU times are taken without a device synchronisation (launch "
                    "time); ours are synchronised"}


def gate_table_20q(q, n=20, count=1000, reps=3):
    """The reference's gate-throughput table (benchmarks/benchmark_gates.cu:36-88, README.md:58-63):
    1000 gates of one type on targets i % n (CNOT: control i % (n-1), target control + 1) at 20
    qubits, one run after a warm-up run and reset; here synchronised, median of `reps`, in the
    reference's one-kernel-per-gate mode and in the default fused mode."""
    def circ(kind):
        c = q.Circuit(n)
        for i in range(count):
            if kind == "H":
                c.h(i % n)
            elif kind == "X":
                c.x(i % n)
            elif kind == "Rz":
                c.rz(i % n, 0.5)
            else:
                c.cnot(i % (n - 1), i % (n - 1) + 1)
        return c
    rows = {}
    for kind in ("H", "X", "Rz", "CNOT"):
        c = circ(kind)
        row = {"reference_readme_gates_per_s": REF_GATE_TABLE_20Q[kind]}
        for mode in (q.RunMode.PerGate, q.RunMode.Fused):
            sim = q.Simulator(n, mode=mode)
            sim.run(c)
            sim.synchronize()
            ts = []
            for _ in range(reps):
                sim.reset()
                t0 = time.perf_counter()
                sim.run(c)
                sim.synchronize()
                ts.append(time.perf_counter() - t0)
            del sim
            row["per_gate" if mode == q.RunMode.PerGate else "fused"] = round(count / _median(ts), 1)
        rows[kind] = row
    return {"workload": f"{count} gates per type at {n} qubits (benchmark_gates.cu)", "unit": "gates/s",
            "rows": rows}


def _dominant_roofline(stats):
    byte_stats = [s for s in stats if s["alg_bytes"] > 0 and s["launches"]]
    if not byte_stats:
        return None
    dom = max(byte_stats, key=lambda s: s["ms"])
    per = dom["alg_bytes"] / dom["launches"]
    avg_s = dom["ms"] / dom["launches"] / 1e3
    ach = per / avg_s / 1e9
    return {"bound": "hbm", "kernel": dom["name"], "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS,
            "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBPS, 4), "alg_bytes_per_launch": per,
            "avg_launch_ms": round(avg_s * 1e3, 4), "launches": dom["launches"]}


def measure_dm(q, n, steps, warmup, jit, seed, depth, p_noise):
    """DensityMatrixSimulator (src/DensityMatrix.cu:978-1122): rho of n qubits as a 2n-index-bit
    engine state (4^n x 16 B), the W-HC circuit with depolarizing p on all qubits (the reference
    applies each channel after a gate that touches its qubit).  gates/s = circuit gates / median
    synchronised run; roofline of the dominant kernel from per-launch HIP events."""
    from qsim_amd.density import DensityMatrixSimulator
    from qsim_amd.plan import set_jit
    set_jit(jit, -1)
    c = q.createRandomHCCircuit(n, depth, seed)
    nm = q.NoiseModel()
    nm.addDepolarizingAll(n, p_noise)
    sim = DensityMatrixSimulator(n, nm)
    sv = sim.density.state
    for _ in range(max(1, warmup)):
        sim.run(c)
        sv.synchronize()
    sv.profile(True)
    sv.profileReset()
    ts = []
    for _ in range(steps):
        sim.reset()
        sv.synchronize()
        t0 = time.perf_counter()
        with region("dm14" if n == 14 else "-"):
            sim.run(c)
            sv.synchronize()
        ts.append(time.perf_counter() - t0)
    stats = sv.profileStats()
    sv.profile(False)
    passes, jit_passes = sv.lastRunInfo()
    tr = sim.getTrace()
    del sim
    med = _median(ts)
    return {"workload": f"DensityMatrixSimulator {n} qubits (rho: {2 * n} index bits, {16 << (2 * n)} B), "
                        f"W-HC depth {depth} seed {seed}, depolarizing {p_noise} on all qubits",
            "value": round(c.getGateCount() / med, 1), "unit": "gates/s", "ms_per_step": round(med * 1e3, 3),
            "passes": passes, "jit_passes": jit_passes, "trace": tr, "roofline": _dominant_roofline(stats),
            "kernels": stats}


def measure_noisy(q, n, steps, warmup, seed, depth, p_noise):
    """NoisySimulator (src/NoiseModel.cu:117-314): the W-HC circuit with depolarizing p on all n
    qubits, every channel entry a per-pair Monte-Carlo pass after every gate (the reference's
    structure; flips walked geometrically, noise.hip).  gates/s = circuit gates / median run."""
    c = q.createRandomHCCircuit(n, depth, seed)
    nm = q.NoiseModel()
    nm.addDepolarizingAll(n, p_noise)
    sim = q.NoisySimulator(n, nm)
    sim.setSeed(seed)
    for _ in range(max(1, warmup)):
        sim.run(c)
    sim.synchronize()
    sv = sim.state
    sv.profile(True)
    sv.profileReset()
    ts = []
    for _ in range(steps):
        sim.reset()
        sim.synchronize()
        t0 = time.perf_counter()
        sim.run(c)
        sim.synchronize()
        ts.append(time.perf_counter() - t0)
    stats = sv.profileStats()
    # The pulled path builds the next step's code words (noise_map) on a second stream beside the
    # pull pass, so their HIP-event spans overlap and each includes time shared with the other
    # kernel.  One more run with the map on the main stream (QSIM_NOISE_MAP_OVERLAP=0, same states)
    # gives each kernel's own duration: the kernel table and the rooflines come from that run.
    prev = os.environ.get("QSIM_NOISE_MAP_OVERLAP")
    os.environ["QSIM_NOISE_MAP_OVERLAP"] = "0"
    try:
        sim.reset()
        sim.synchronize()
        sv.profileReset()
        with region("noisy26" if n == 26 else "-"):  # (the run the kernel table and rooflines come from)
            sim.run(c)
            sim.synchronize()
        serial = sv.profileStats()
    finally:
        if prev is None:
            os.environ.pop("QSIM_NOISE_MAP_OVERLAP", None)
        else:
            os.environ["QSIM_NOISE_MAP_OVERLAP"] = prev
    sv.profile(False)
    del sim
    med = _median(ts)
    # the noise kernels: the per-channel passes (push) or the pull pass, which applies the flips
    # of the step before while it applies the gate (its bytes: one read + one write of the state
    # plus the code words), with its PMC traffic (profiles/pmc_noisy_26q.json)
    noise = [s for s in serial if s["name"] in ("noise", "pull_gate", "pull_gate_map")]
    noise_roof = _dominant_roofline(noise) if noise else None
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_noisy_{n}q.json")
    if noise_roof and os.path.exists(pmc_path):
        with open(pmc_path) as f:
            ent = json.load(f).get("kernels", {}).get(noise_roof["kernel"], {})
        noise_roof["traffic"] = ent.get("hbm_bytes_per_launch")
        noise_roof["traffic_source"] = os.path.relpath(pmc_path, ROOT) if noise_roof["traffic"] else None
    return {"workload": f"NoisySimulator {n} qubits, W-HC depth {depth} seed {seed}, depolarizing "
                        f"{p_noise} on all qubits after every gate ({n} channel passes per gate)",
            "value": round(c.getGateCount() / med, 1), "unit": "gates/s", "ms_per_step": round(med * 1e3, 3),
            "roofline": _dominant_roofline(serial), "noise_roofline": noise_roof,
            "kernels": serial, "kernels_note": "per-kernel durations from one run with the code-word map "
                                               "on the main stream (no overlap); the timed runs overlap it",
            "kernels_overlapped": stats}


def roofline_1q28(q, steps=3):
    """north_star's single-qubit target, measured in the same run: W-1Q at 28 qubits (BASELINE
    configs[2], 4 GiB state) — 100 H gates on targets i % 28, one kernel per gate, unfused —
    per-launch HIP events on the state's stream; algorithmic bytes 32 B x 2^28 per gate."""
    n = 28
    c = q.Circuit(n)
    for i in range(100):
        c.h(i % n)
    sim = q.Simulator(n, mode=q.RunMode.PerGate)
    sim.run(c)
    sim.synchronize()
    sim.state.profile(True)
    sim.state.profileReset()
    t0 = time.perf_counter()
    with region("1q28"):
        for _ in range(steps):
            sim.run(c)
        sim.synchronize()
    wall = time.perf_counter() - t0
    stats = sim.state.profileStats()
    sim.state.profile(False)
    launches = sum(s["launches"] for s in stats)
    ms = sum(s["ms"] for s in stats)
    by = sum(s["alg_bytes"] for s in stats)
    achieved = by / (ms / 1e3) / 1e9
    # PMC traffic per launch (profiles/pmc_1q_28q.json, the same W-1Q command under rocprofv3
    # --pmc), launch-weighted over the kernels this workload ran
    traffic, traffic_src = None, None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_1q_28q.json")
    if os.path.exists(pmc_path):
        with open(pmc_path) as f:
            kern = json.load(f).get("kernels", {})
        ents = [kern[s["name"]] for s in stats if s["name"] in kern]
        tl = sum(e["launches"] for e in ents)
        if ents and tl:
            traffic = sum(e["hbm_bytes_per_launch"] * e["launches"] for e in ents) / tl
            traffic_src = os.path.relpath(pmc_path, ROOT)
    return {"workload": "W-1Q 100 unfused H gates on targets i % 28, 28 qubits",
            "traffic": traffic, "traffic_source": traffic_src,
            "kernels": sorted({s["name"] for s in stats}), "launches": launches,
            "avg_launch_ms": round(ms / launches, 4), "alg_bytes_per_launch": by / launches,
            "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "gates_per_s": round(100 * steps / wall, 1), "target_frac": 0.70}


def measure_batch(q, n, B, steps, warmup, jit, seed, depth, p_noise, process, pmc_path=None):
    """W-BATCH (BASELINE config 4): BatchedSimulator, n qubits x B trajectories, depolarizing p on
    every qubit after every gate (NoiseModel.addDepolarizingAll), the W-HC circuit, under one noise
    process.  Returns value (trajectory-gates/s), ms per step, the kernel table and the dominant
    kernel's roofline (its per-launch algorithmic bytes: a pass / gate its streaming bytes, a
    reference noise step 32 B x the expected flipped pairs)."""
    circuit = q.createRandomHCCircuit(n, depth, seed)
    nm = q.NoiseModel()
    nm.addDepolarizingAll(n, p_noise)
    from qsim_amd.plan import set_jit
    set_jit(jit, -1)  # specialised pass kernels, compiled during the first warmup run
    sem = q.BatchedNoise.Reference if process == "reference" else q.BatchedNoise.Physical
    sim = q.BatchedSimulator(n, B, nm, noise=sem)
    sim.setSeed(seed)
    for _ in range(max(1, warmup) if jit else warmup):
        sim.run(circuit)
    sim.synchronize()
    sim.profile(True)
    split = process == "reference"  # (the in-tile path runs two trajectory halves on two streams)
    t0 = time.perf_counter()
    with region("batch16ref" if process == "reference" and n == 16 and B == 1024 and not split else "-"):
        for _ in range(steps):
            sim.run(circuit)
        sim.synchronize()
    wall = time.perf_counter() - t0
    stats = sim.profileStats()
    overlapped = None
    if split:
        # The timed steps overlap the two halves' kernels (each launch's HIP-event span includes
        # time shared with the other half), so the kernel table and the roofline come from as
        # many steps more with one part on one stream (QSIM_NOISE_SPLIT=1, the same states): each
        # kernel's own duration over the whole ensemble.
        prev = os.environ.get("QSIM_NOISE_SPLIT")
        os.environ["QSIM_NOISE_SPLIT"] = "1"
        try:
            with region("batch16ref" if n == 16 and B == 1024 else "-"):
                for _ in range(steps):
                    sim.run(circuit)
                sim.synchronize()
            after = sim.profileStats()
        finally:
            if prev is None:
                os.environ.pop("QSIM_NOISE_SPLIT", None)
            else:
                os.environ["QSIM_NOISE_SPLIT"] = prev
        before = {s_["name"]: s_ for s_ in stats}
        serial = []
        for s_ in after:
            b_ = before.get(s_["name"], {"ms": 0.0, "launches": 0, "alg_bytes": 0.0})
            d = {"name": s_["name"], "ms": s_["ms"] - b_["ms"], "launches": s_["launches"] - b_["launches"],
                 "alg_bytes": s_["alg_bytes"] - b_["alg_bytes"]}
            if d["launches"] > 0:
                serial.append(d)
        overlapped, stats = stats, serial
    sim.profile(False)
    passes, jit_passes = sim.lastRunInfo()
    gates = circuit.getGateCount()
    byte_stats = [s for s in stats if s["alg_bytes"] > 0]  # (frame builds carry no byte count)
    dom = max(byte_stats, key=lambda s: s["ms"]) if byte_stats else None
    roof = None
    if dom and dom["launches"]:
        per = dom["alg_bytes"] / dom["launches"]
        avg_s = dom["ms"] / dom["launches"] / 1e3
        ach = per / avg_s / 1e9
        traffic, traffic_src = None, None
        if pmc_path and os.path.exists(pmc_path):
            with open(pmc_path) as f:
                ent = json.load(f).get("kernels", {}).get(dom["name"], {})
            traffic = ent.get("hbm_bytes_per_launch")
            traffic_src = os.path.relpath(pmc_path, ROOT) if traffic is not None else None
        roof = {"bound": "hbm", "kernel": dom["name"], "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": traffic,
                "traffic_source": traffic_src,
                "alg_bytes_per_launch": per, "avg_launch_ms": round(avg_s * 1e3, 4),
                "launches": dom["launches"],
                "source": ("as many steps more with one part on one stream after the timed ones "
                           "(QSIM_NOISE_SPLIT=1, same states): each kernel's own duration; the timed "
                           "steps run two parts on two streams") if split else "the timed steps"}
    del sim
    return {"value": round(gates * B * steps / wall, 1), "ms_per_step": round(wall / steps * 1e3, 3),
            "gates": gates, "tile_passes": passes, "jit_passes": jit_passes, "roofline": roof,
            "kernels": stats,
            **({"kernels_note": "per-kernel durations (and the roofline) from as many steps more with the "
                                "ensemble as one part on one stream (QSIM_NOISE_SPLIT=1, same states); the "
                                "timed steps run two halves on two streams",
                "kernels_overlapped": overlapped} if overlapped is not None else {}),
            "noise_process": ("reference: per-pair draws, one pass per channel entry after every "
                              "gate (src/NoiseModel.cu:834-892); the BatchedSimulator default"
                              if process == "reference" else
                              "physical: one draw per trajectory, channel and gate (Pauli frames)")}


def batch_pmc_path(n, process):
    return os.path.join(ROOT, "profiles", f"pmc_batch_{n}q.json" if process == "physical"
                        else f"pmc_batch_ref_{n}q.json")


def roofline_batch16(q, args):
    """BASELINE config 4 in the default line: W-BATCH 16q x 1024 under both noise processes
    (reference first: the drop-in default), 5 timed steps each."""
    out = {}
    for proc in ("reference", "physical"):
        m = measure_batch(q, 16, 1024, 5, 1, args.jit, args.seed, args.depth, 0.01, proc,
                          batch_pmc_path(16, proc))
        out[proc] = {"value": m["value"], "unit": "trajectory-gates/s", "ms_per_step": m["ms_per_step"],
                     "roofline": m["roofline"], "noise_process": m["noise_process"],
                     **({"roofline_note": m["kernels_note"]} if "kernels_note" in m else {})}
    out["workload"] = (f"W-BATCH 16q x 1024 trajectories, depolarizing 0.01 on all qubits after every "
                       f"gate, W-HC depth {args.depth} seed {args.seed}")
    return out


def run_batch(args):
    """W-BATCH line (--workload batch): value = trajectory-gates/s."""
    import qsim_amd as q
    n, B = args.qubits, args.trajectories
    m = measure_batch(q, n, B, args.steps, args.warmup, args.jit, args.seed, args.depth, args.noise,
                      args.batch_noise, args.pmc_json or batch_pmc_path(n, args.batch_noise))
    out = {
        "metric": "trajectory-gates/s, W-HC circuit on noisy trajectories (BatchedSimulator)",
        "value": m["value"], "unit": "trajectory-gates/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": m["ms_per_step"], "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "c128 (complex<double>)", "data": "synthetic",
        "config": {"workload": f"W-BATCH {n}q x {B} trajectories, depolarizing {args.noise} on all "
                               f"qubits after every gate, W-HC depth {args.depth} seed {args.seed}",
                   "noise_process": m["noise_process"],
                   "qubits": n, "trajectories": B, "gates": m["gates"], "state_bytes": (16 << n) * B,
                   "tile_passes": m["tile_passes"], "jit_passes": m["jit_passes"]},
        "roofline": m["roofline"], "kernels": m["kernels"], "cpu_baseline": batch_cpu_baseline(args),
        **{k: m[k] for k in ("kernels_note", "kernels_overlapped") if k in m},
    }
    print(json.dumps(out))


def run_model_line(args):
    """--workload dm / noisy: one line for the §8(f) simulators (value = circuit gates/s)."""
    import qsim_amd as q
    if args.workload == "dm":
        m = measure_dm(q, args.qubits, args.steps, args.warmup, args.jit, args.seed, args.depth, args.noise)
        metric = "gates/s, W-HC circuit with depolarizing noise (DensityMatrixSimulator)"
    else:
        m = measure_noisy(q, args.qubits, args.steps, args.warmup, args.seed, args.depth, args.noise)
        metric = "gates/s, W-HC circuit with depolarizing noise (NoisySimulator)"
    out = {"metric": metric, "value": m["value"], "unit": "gates/s", "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": m["ms_per_step"], "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "c128 (complex<double>)", "data": "synthetic",
           "config": {"workload": m["workload"], "qubits": args.qubits},
           "roofline": m["roofline"], "cpu_baseline": None}
    out.update({k: v for k, v in m.items() if k not in out and k not in ("value", "workload")})
    print(json.dumps(out))


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # No launcher around us: start the N rank processes ourselves and relay rank 0's JSON
        # line (qsim_amd/launch.py).  launch.py is loaded by file path, not through the package:
        # importing qsim_amd would load libqsim_hip.so (and RCCL / hipRTC) into this parent,
        # which never uses the GPU.
        import importlib.util
        spec = importlib.util.spec_from_file_location(
            "qsim_launch", os.path.join(ROOT, "cuda-quantum-simulator_amd", "qsim_amd", "launch.py"))
        launch = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(launch)
        sys.exit(launch.launch_ranks(os.path.abspath(__file__), sys.argv[1:], args.gpus,
                                     timeout_s=args.launch_timeout))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.workload in ("dm", "noisy"):
        if world > 1 or args.gpus > 1:
            sys.exit("--workload dm / noisy run on one GPU")
        run_model_line(args)
        return
    if args.workload == "batch":
        if world > 1 or args.dry_run:
            from qsim_amd import dist_bench  # trajectory-sharded replicas
            dist_bench.run_batch(args, "trajectory-gates/s, W-HC circuit on noisy trajectories "
                                       "(BatchedSimulator)", HBM_PEAK_GBPS, batch_cpu_baseline)
        else:
            run_batch(args)
        return
    if world > 1 or args.gpus > 1 or args.dry_run:
        from qsim_amd import dist_bench  # sharded strong-scaling path (RCCL over xGMI)
        cpu_fn = None
        if args.cpu_budget > 0:  # rank 0, after the timed region (dist_bench._cpu_baseline)
            def cpu_fn(circuit, n, qmod):
                return cpu_baseline(circuit, n, args.cpu_budget, qmod, args)
        dist_bench.run(args, METRIC, HBM_PEAK_GBPS, cpu_fn)
    else:
        run_single(args)


if __name__ == "__main__":
    main()
