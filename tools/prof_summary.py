"""Summarise a rocprofv3 --kernel-trace results database (rocpd SQLite) into CSV:
kernel name, calls, total/avg/min/max duration (us), VGPR/SGPR/scratch per dispatch."""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = c.execute(
        "select name, count(*), sum(duration)/1e3, avg(duration)/1e3, min(duration)/1e3, max(duration)/1e3, "
        "max(vgpr_count), max(accum_vgpr_count), max(sgpr_count), max(scratch_size), max(grid_x), max(workgroup_x) "
        "from kernels group by name order by sum(duration) desc").fetchall()
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "min_us", "max_us", "vgpr", "agpr", "sgpr",
                    "scratch_bytes", "grid_x", "workgroup_x"])
        for r in rows:
            w.writerow([r[0]] + [round(x, 3) if isinstance(x, float) else x for x in r[1:]])
    for r in rows:
        print(f"{r[3]:10.1f} us avg  x{r[1]:4d}  {r[0][:90]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
