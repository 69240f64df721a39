"""Kernel statistics (rocprofv3 --stats layout: Name, Calls, TotalDurationNs, AverageNs,
Percentage, MinNs, MaxNs) from a rocprofv3 SQLite database (`*_results.db`).
Usage: python scripts/rocpd_stats.py <results.db> [out.csv]"""
import csv
import sqlite3
import sys


def stats(db_path):
    db = sqlite3.connect(db_path)
    rows = db.execute(
        "select s.display_name, count(*), sum(d.end - d.start), min(d.end - d.start), max(d.end - d.start) "
        "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id "
        "group by s.display_name order by sum(d.end - d.start) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    return [{"Name": r[0], "Calls": r[1], "TotalDurationNs": r[2], "AverageNs": r[2] / r[1],
             "Percentage": 100.0 * r[2] / total, "MinNs": r[3], "MaxNs": r[4]} for r in rows]


if __name__ == "__main__":
    out = stats(sys.argv[1])
    f = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.DictWriter(f, fieldnames=list(out[0].keys()))
    w.writeheader()
    w.writerows(out)
