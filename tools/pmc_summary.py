"""Summarise two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; -f csv) into per-kernel
HBM bytes per launch, with the gfx950 correction of /opt/skills/guides/MI355X_MICROARCH.md
(HBM section): FETCH_SIZE reports half the bytes of a wide read -> doubled; WRITE_SIZE
is taken as is.  Both counters are in KiB.

    python tools/pmc_summary.py <fetch_dir> <write_dir> <out.json>
"""
import collections
import csv
import glob
import json
import re
import sys


def per_kernel(d, counter):
    path = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        m = re.search(r"rtg::(k_\w+)(<(\w+)[^>]*>)?", r["Kernel_Name"])
        name = m.group(1) + ("" if not m.group(3) else f"<{m.group(3)}>")
        acc[name].append(float(r["Counter_Value"]) * 1024.0)
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main(fetch_dir, write_dir, out):
    f = per_kernel(fetch_dir, "FETCH_SIZE")
    w = per_kernel(write_dir, "WRITE_SIZE")
    res = {"note": "bytes per launch; read = 2 x FETCH_SIZE (gfx950 correction), write = WRITE_SIZE",
           "kernels": {}}
    for k in sorted(set(f) | set(w)):
        rd = 2.0 * f.get(k, (0.0, 0))[0]
        wr = w.get(k, (0.0, 0))[0]
        res["kernels"][k] = {"read_bytes": round(rd), "write_bytes": round(wr), "traffic_bytes": round(rd + wr),
                             "launches": max(f.get(k, (0, 0))[1], w.get(k, (0, 0))[1])}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res["kernels"].items():
        print(f"{k:22s} read {v['read_bytes'] / 1e6:9.2f} MB  write {v['write_bytes'] / 1e6:9.2f} MB  x{v['launches']}")


if __name__ == "__main__":
    main(*sys.argv[1:4])
