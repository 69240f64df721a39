#!/usr/bin/env python3
"""Reduce rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes to per-launch HBM bytes per kernel.

Usage: pmc_summary.py <pmc_dir> <out.json> [--min-bytes B]
  <pmc_dir>/p1/*counter_collection.csv holds FETCH_SIZE, <pmc_dir>/p2/... WRITE_SIZE (gpu_pmc.sh).

Corrections (MI355X_MICROARCH.md, HBM section): both counters are in KiB; on gfx950 FETCH_SIZE
reports half the bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled;
WRITE_SIZE is exact for 16 B/lane streaming stores.  Only launches moving >= --min-bytes are kept
(drops the setup/copy kernels), and rows are keyed by the engine's timer label (bench.py's
`roofline.kernel`) as well as by the demangled kernel name.
"""
import csv
import glob
import json
import os
import sys

LABELS = [("k_fused_staged", "fused_tile"), ("k_fused_tile", "fused_tile"),
          ("k_m1_slice", "m1_slice"), ("k_m1_lane", "m1_lane"), ("k_diag", "diag"),
          ("k_swap_hh", "swap_hh"), ("k_swap_lh", "swap_lh"), ("k_swap_ll", "swap_ll"),
          ("k_pauli_apply", "pauli_apply"), ("k_exchange_copy", "alltoall_remap"),
          ("k_noise_units", "noise"), ("k_noise_flips", "noise"),
          ("k_gate_noise_tile", "gate_noise"), ("k_gn_lists", "noise_lists"),
          ("k_pull_gate", "pull_gate"), ("k_noise_map", "noise_map"), ("k_noise_words", "noise_map"),
          ("qk", "fused_tile")]  # circuit-specialised pass kernels (jit.hip) are named qk<pass>


def label_of(name):
    if "k_pull_gate<" in name:
        # k_pull_gate<W, PAIR, U, NT, MAP[, SPARSE]>: MAP = true is the word map fused in
        args = name.split("(")[0].split("<", 1)[1].rstrip(">").replace(" ", "").split(",")
        return "pull_gate_map" if len(args) >= 5 and args[4] == "true" else "pull_gate"
    for key, lab in LABELS:
        if key in name:
            return lab
    return None


def read(pdir, counter):
    rows = {}
    for path in glob.glob(os.path.join(pdir, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] != counter:
                    continue
                key = int(r["Dispatch_Id"])
                rows[key] = (r["Kernel_Name"], rows.get(key, ("", 0.0))[1] + float(r["Counter_Value"]))
    return rows


def main():
    src, out = sys.argv[1], sys.argv[2]
    min_bytes = float(sys.argv[sys.argv.index("--min-bytes") + 1]) if "--min-bytes" in sys.argv else 1 << 26
    fetch = read(os.path.join(src, "p1"), "FETCH_SIZE")
    write = read(os.path.join(src, "p2"), "WRITE_SIZE")
    per = {}
    # the two passes are separate runs of the same deterministic command: match launches by
    # their order within each kernel name
    def by_name(rows):
        d = {}
        for k in sorted(rows):
            d.setdefault(rows[k][0], []).append(rows[k][1] * 1024.0)
        return d
    fb, wb = by_name(fetch), by_name(write)
    for name in sorted(set(fb) | set(wb)):
        f, w = fb.get(name, []), wb.get(name, [])
        m = min(len(f), len(w))
        if m == 0:
            continue
        tot = [2.0 * f[i] + w[i] for i in range(m)]
        keep = [i for i in range(m) if tot[i] >= min_bytes]
        if not keep:
            continue
        ent = {"launches": len(keep),
               "fetch_bytes_per_launch": sum(2.0 * f[i] for i in keep) / len(keep),
               "write_bytes_per_launch": sum(w[i] for i in keep) / len(keep)}
        ent["hbm_bytes_per_launch"] = ent["fetch_bytes_per_launch"] + ent["write_bytes_per_launch"]
        per[name] = ent
        lab = label_of(name)
        if lab:
            agg = per.setdefault(lab, {"launches": 0, "fetch_bytes_per_launch": 0.0,
                                       "write_bytes_per_launch": 0.0, "hbm_bytes_per_launch": 0.0})
            n0, n1 = agg["launches"], ent["launches"]
            for k in ("fetch_bytes_per_launch", "write_bytes_per_launch", "hbm_bytes_per_launch"):
                agg[k] = (agg[k] * n0 + ent[k] * n1) / (n0 + n1)
            agg["launches"] = n0 + n1
    # further passes (p3, p4, ...): every other counter, averaged per launch of each kernel
    other = {}
    for pdir in sorted(glob.glob(os.path.join(src, "p[0-9]*"))):
        if os.path.basename(pdir) in ("p1", "p2"):
            continue
        for path in glob.glob(os.path.join(pdir, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                acc = {}
                for r in csv.DictReader(f):
                    key = (r["Kernel_Name"], r["Counter_Name"], int(r["Dispatch_Id"]))
                    acc[key] = acc.get(key, 0.0) + float(r["Counter_Value"])
            for (kname, cname, _), v in acc.items():
                lab = label_of(kname)
                for k in ([kname] + ([lab] if lab else [])):
                    d = other.setdefault(k, {}).setdefault(cname, [0.0, 0])
                    d[0] += v
                    d[1] += 1
    for k, cs in other.items():
        tgt = per.setdefault(k, {})
        tgt["counters_per_launch"] = {c: v[0] / v[1] for c, v in sorted(cs.items())}
    with open(out, "w") as f:
        json.dump({"source": src, "fetch_correction": 2.0, "unit": "bytes", "kernels": per}, f, indent=1)
    for k, v in per.items():
        if "hbm_bytes_per_launch" in v:
            print(f"{k[:60]:60s} {v['launches']:5d} {v['hbm_bytes_per_launch'] / 2**30:8.3f} GiB/launch")
        for c, x in v.get("counters_per_launch", {}).items():
            print(f"    {c:28s} {x:16.1f}")


if __name__ == "__main__":
    main()
