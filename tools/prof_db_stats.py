"""Kernel statistics from a rocprofv3 results database (rocpd SQLite, what
`rocprofv3 --kernel-trace --stats` writes when no --output-format is given): one row per
kernel name with calls, total / average / min / max duration in ns and the share of the
total -- the columns of rocprofv3's kernel_stats.csv.

    python tools/prof_db_stats.py <run_results.db> <out.csv>
"""
import collections
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    acc = collections.defaultdict(list)
    for name, dur in c.execute("select name, duration from kernels"):
        acc[name].append(int(dur))
    total = sum(sum(v) for v in acc.values()) or 1
    rows = sorted(acc.items(), key=lambda kv: -sum(kv[1]))
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, v in rows:
            w.writerow([name, len(v), sum(v), round(sum(v) / len(v), 1), round(100.0 * sum(v) / total, 3),
                        min(v), max(v)])
    for name, v in rows[:12]:
        print(f"{len(v):6d} x {sum(v) / len(v) / 1e3:10.2f} us  {name[:110]}")


if __name__ == "__main__":
    main(*sys.argv[1:3])
