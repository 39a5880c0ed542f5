#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run (SQLite .db or CSV dir)
into profiles/<name>.csv (per-kernel calls / total / average duration, us)."""
import csv
import glob
import os
import sqlite3
import sys


def main(src_dir, dst):
    rows = []
    dbs = glob.glob(os.path.join(src_dir, "**", "*.db"), recursive=True)
    if dbs:
        con = sqlite3.connect(dbs[0])
        for name, calls, total, avg, pct in con.execute(
                "select name, total_calls, total_duration, average, percentage "
                "from top_kernels"):
            # rocpd top_kernels durations are in microseconds
            rows.append([name.split("(")[0], calls, total, avg, pct])
    else:
        stats = glob.glob(os.path.join(src_dir, "**", "*kernel_stats.csv"), recursive=True)
        for r in csv.DictReader(open(stats[0])):
            rows.append([r["Name"].split("(")[0], int(r["Calls"]),
                         float(r["TotalDurationNs"]) / 1e3,
                         float(r["AverageNs"]) / 1e3, float(r["Percentage"])])
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "average_us", "percent"])
        for r in rows:
            w.writerow([r[0], r[1], "%.3f" % r[2], "%.3f" % r[3], "%.2f" % r[4]])
    for r in rows[:12]:
        print("%-28s %6d %12.1f %10.2f %6.2f" % tuple(r))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
