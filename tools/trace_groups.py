"""Group a rocprofv3 kernel trace by (kernel, grid size): dispatches, mean / total duration and the
busy span of each group, so that a bench run's full frames and its frame parts (smaller grids)
can be told apart.  Usage: python tools/trace_groups.py <run_kernel_trace.csv> [out.txt]"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    m = re.match(r"(?:void )?(?:rtg::)?([A-Za-z_0-9]+)(<[^()]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main(path, out=None):
    g = defaultdict(list)
    for row in csv.DictReader(open(path)):
        if "rocclr" in row["Kernel_Name"]:
            continue
        grid = int(row["Grid_Size_X"]) * int(row["Grid_Size_Y"]) * int(row["Grid_Size_Z"])
        wg = int(row["Workgroup_Size_X"]) * int(row["Workgroup_Size_Y"]) * int(row["Workgroup_Size_Z"])
        s, e = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
        g[(short(row["Kernel_Name"]), grid // max(1, wg), row["VGPR_Count"], row["Scratch_Size"])].append((s, e))
    lines = [f"{'kernel':60s} {'blocks':>8s} {'vgpr':>5s} {'scr':>5s} {'n':>6s} {'mean_us':>9s} {'total_ms':>9s}"]
    for k in sorted(g, key=lambda k: -sum(e - s for s, e in g[k])):
        d = g[k]
        tot = sum(e - s for s, e in d)
        lines.append(f"{k[0][:60]:60s} {k[1]:8d} {k[2]:>5s} {k[3]:>5s} {len(d):6d} {tot / len(d) / 1e3:9.2f} {tot / 1e6:9.3f}")
    text = "\n".join(lines)
    print(text)
    if out:
        open(out, "w").write(text + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
