#!/usr/bin/env python3
"""rocprofv3's default rocpd output (SQLite) -> the --stats kernel summary
as CSV (Name, Calls, TotalDurationNs, AverageNs, Percentage), the columns
of rocprofv3 --stats --output-format csv (the rocpd view reports us).  Usage:
  rocpd_stats.py run_results.db > kernel_stats.csv"""
import csv
import sqlite3
import sys


def main():
    con = sqlite3.connect(sys.argv[1])
    rows = con.execute("select name, total_calls, total_duration, average, percentage "
                       "from top_kernels order by total_duration desc").fetchall()
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
    for name, calls, tot, avg, pct in rows:
        w.writerow([name, calls, f"{tot * 1e3:.0f}", f"{avg * 1e3:.0f}", f"{pct:.2f}"])


if __name__ == "__main__":
    main()
