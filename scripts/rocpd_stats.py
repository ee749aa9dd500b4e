"""Kernel statistics (name, calls, total/avg/min/max ns, share) from a
rocprofv3 SQLite output (run_results.db), as rocprofv3's kernel_stats.csv.
Usage: python scripts/rocpd_stats.py DB [OUT.csv]"""
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else cols[0])
    rows = c.execute(f"select {name}, start, end from kernels").fetchall()
    agg = {}
    for n, s, e in rows:
        d = e - s
        a = agg.setdefault(n, [0, 0, None, 0])
        a[0] += 1
        a[1] += d
        a[2] = d if a[2] is None else min(a[2], d)
        a[3] = max(a[3], d)
    tot = sum(v[1] for v in agg.values()) or 1
    out = [(n, v[0], v[1], v[1] / v[0], v[2], v[3], 100.0 * v[1] / tot) for n, v in agg.items()]
    return sorted(out, key=lambda r: -r[2])


if __name__ == "__main__":
    rows = stats(sys.argv[1])
    w = csv.writer(open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
    for r in rows:
        w.writerow([r[0], r[1], r[2], round(r[3], 1), r[4], r[5], round(r[6], 2)])
