"""A rocprofv3 --kernel-trace of tools/diag_parts8.py (frames in flight on several streams):
per kernel, launch count and mean duration; for the kernels of the run's last window of
`--tail` dispatches, how the GPU's time splits -- wall span, time with at least one kernel
running (union of intervals), mean number of kernels in flight, and per queue the gaps between a
kernel's end and the next kernel's start on that queue.

    python tools/trace_parts.py <dir with *kernel_trace.csv> [--tail N]"""
import argparse
import collections
import csv
import glob
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("d")
    ap.add_argument("--tail", type=int, default=2000)
    a = ap.parse_args()
    path = glob.glob(f"{a.d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = []
    for r in csv.DictReader(open(path)):
        m = re.search(r"rtg::(k_\w+)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:30]
        if r["Kernel_Name"].startswith("void rtg::k_shade<") and ", 2, " in r["Kernel_Name"]:
            name = "k_shade_shadow"
        q = r.get("Queue_Id") or r.get("Stream_Id") or "0"
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, q,
                     int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)))
    rows.sort()
    per = collections.defaultdict(list)
    for s, e, n, q, g in rows:
        per[(n, g)].append(e - s)
    print("kernel, grid: launches, mean us")
    for (n, g), v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {n:18s} grid {g:9d}: {len(v):6d}  {sum(v) / len(v) / 1e3:8.2f}")
    w = rows[-a.tail:]
    t0, t1 = w[0][0], max(e for _, e, _, _, _ in w)
    busy, cur_s, cur_e = 0, None, None
    for s, e, *_ in w:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    inflight = sum(e - s for s, e, *_ in w) / (t1 - t0)
    print(f"last {len(w)} dispatches: span {(t1 - t0) / 1e3:.1f} us, busy {busy / (t1 - t0):.4f}, "
          f"mean kernels in flight {inflight:.2f}")
    byq = collections.defaultdict(list)
    for s, e, n, q, g in w:
        byq[q].append((s, e, n))
    gaps = []
    for q, v in byq.items():
        v.sort()
        gaps += [v[i + 1][0] - v[i][1] for i in range(len(v) - 1)]
    gaps.sort()
    if gaps:
        print(f"queues {len(byq)}; gaps between consecutive kernels of a queue: median {gaps[len(gaps) // 2] / 1e3:.2f} us, "
              f"p90 {gaps[int(len(gaps) * 0.9)] / 1e3:.2f} us, mean {sum(gaps) / len(gaps) / 1e3:.2f} us")


if __name__ == "__main__":
    main()
