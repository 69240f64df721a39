#!/usr/bin/env python3
"""Recompute a bench line's roofline fraction from a rocprofv3 kernel trace of its timed region.

    python scripts/roofline_check.py <region> <bench.json> <kernel_trace.csv> [out.json]
        [--markers=<marker_api_trace.csv>]

<region> is one of bench.py's --profile-region names.  The trace comes from
    rocprofv3 --selected-regions --kernel-trace --stats --output-format csv -- \
        python3 bench.py --profile-region <region> ...
so it holds only the launches of that timed region (roctxProfilerResume / Pause around it).  The
line's roofline for the region (achieved = algorithmic bytes per launch / average launch time from
HIP events on the engine's stream) is recomputed from the rocprof durations of the same kernels:
average and median per launch, frac = bytes / average / 8 TB/s, and the relative gap to the line.
"""
import csv
import json
import re
import statistics
import sys

PEAK = 8000.0  # GB/s, MI355X HBM3E (MI355X_MICROARCH.md)

# region -> (how to find the line's roofline object, rocprof kernel-name pattern)
REGIONS = {
    "hc": (lambda o: o["roofline"], r"^(qk\d+|.*k_fused_(staged|tile).*)"),
    "hc28": (lambda o: o["w_hc_28q"]["roofline"], r"^(qk\d+|.*k_fused_(staged|tile).*)"),
    "1q28": (lambda o: o["roofline_1q28"], r".*k_m1_(slice|lane).*"),
    "batch16ref": (lambda o: o["roofline_batch16"]["reference"]["roofline"], None),
    # (the default line's nested objects, or the --workload noisy / dm line itself)
    "noisy26": (lambda o: o.get("noisy_26q", o)["noise_roofline"], None),
    "dm14": (lambda o: o.get("dm_14q", o)["roofline"], r"^(qk\d+|.*k_fused_(staged|tile).*)"),
}
# the engine's kernel-table names -> rocprof symbol patterns (bench.py / engine Timer names)
ENGINE_NAMES = {
    "noise_units": r".*k_noise_units.*",
    "noise": r".*k_noise_(units|flips).*",
    "gate_noise": r".*k_gate_noise_tile.*",
    # k_pull_gate<W, PAIR, U, NT, MAP[, SPARSE]>: the fifth argument says whether the map is fused in
    "pull_gate": r".*k_pull_gate<[^,]+, *[a-z]+, *\d+, *[a-z]+(, *false(, *[a-z]+)?)?>\(.*",
    "pull_gate_map": r".*k_pull_gate<[^,]+, *[a-z]+, *\d+, *[a-z]+, *true(, *[a-z]+)?>\(.*",
    "noise_map": r".*k_noise_words.*",
    "fused_tile": r"^(qk\d+|.*k_fused_(staged|tile).*)",
}


def load_line(path):
    with open(path) as f:
        for line in f:
            line = line.strip()
            if line.startswith("{"):
                return json.loads(line)
    raise SystemExit(f"no JSON line in {path}")


def marker_window(marker_csv, region):
    """[(start, end), ...] of every roctx range "timed_<region>" (rocprofv3 --marker-trace csv; a
    region entered once per timed step gives one range per step)."""
    out = []
    with open(marker_csv, newline="") as f:
        for row in csv.DictReader(f):
            msg = row.get("Function") or row.get("Message") or row.get("Name") or ""
            if msg == f"timed_{region}" or row.get("Message", "") == f"timed_{region}":
                out.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
    if not out:
        raise SystemExit(f"no range timed_{region} in {marker_csv}")
    return out


def durations(trace_csv, pattern, window=None):
    rx = re.compile(pattern)
    out = {}
    with open(trace_csv, newline="") as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name") or row.get("KernelName") or row.get("Name")
            if name is None or not rx.match(name):
                continue
            t0, t1 = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
            if window and not any(a <= t0 <= b for a, b in window):
                continue
            out.setdefault(name, []).append(t1 - t0)
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--markers=")]
    markers = [a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--markers=")]
    sys.argv = [sys.argv[0]] + args
    region, bench_json, trace = args[:3]
    window = marker_window(markers[0], region) if markers else None
    line = load_line(bench_json)
    get_roof, pattern = REGIONS[region]
    roof = get_roof(line)
    if pattern is None:
        pattern = ENGINE_NAMES[roof["kernel"]]
    per_name = durations(trace, pattern, window)
    allv = [d for v in per_name.values() for d in v]
    if not allv:
        raise SystemExit(f"no launches matching {pattern} in {trace}")
    avg_ns, med_ns = statistics.fmean(allv), statistics.median(allv)
    per = roof["alg_bytes_per_launch"]
    frac_avg = per / (avg_ns * 1e-9) / 1e9 / PEAK
    frac_med = per / (med_ns * 1e-9) / 1e9 / PEAK
    res = {
        "region": region, "kernel_pattern": pattern, "launches": len(allv),
        "selection": (f"kernels starting inside the roctx range timed_{region} (--marker-trace)" if window
                      else "every launch in the trace (--selected-regions)"),
        "line_launches": roof.get("launches"),
        "rocprof_avg_ms": round(avg_ns / 1e6, 4), "rocprof_median_ms": round(med_ns / 1e6, 4),
        "line_avg_launch_ms": roof.get("avg_launch_ms"),
        "alg_bytes_per_launch": per,
        "frac_from_rocprof_avg": round(frac_avg, 4), "frac_from_rocprof_median": round(frac_med, 4),
        "line_frac": roof["frac"], "rel_gap_avg": round(frac_avg / roof["frac"] - 1.0, 4),
        "per_kernel": {k: {"launches": len(v), "avg_ms": round(statistics.fmean(v) / 1e6, 4),
                           "median_ms": round(statistics.median(v) / 1e6, 4)}
                       for k, v in sorted(per_name.items())},
    }
    js = json.dumps(res, indent=1)
    print(js)
    if len(sys.argv) > 4:
        with open(sys.argv[4], "w") as f:
            f.write(js + "\n")
        # the rocprof kernel summary of the timed region alone (every kernel in the window)
        allk = durations(trace, r".*", window)
        rows = sorted(allk.items(), key=lambda kv: -sum(kv[1]))
        with open(sys.argv[4].replace(".json", "_timed_kernel_stats.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MedianNs", "MinNs", "MaxNs"])
            for name, v in rows:
                w.writerow([name, len(v), sum(v), round(statistics.fmean(v), 1), statistics.median(v), min(v), max(v)])


if __name__ == "__main__":
    main()
