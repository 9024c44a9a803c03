"""Summarise rocprofv3 --pmc passes (-f csv) of bench.py into per-kernel bytes per launch,
with the gfx950 correction of /opt/skills/guides/MI355X_MICROARCH.md (HBM section):
FETCH_SIZE reports half the bytes of a wide read -> doubled; WRITE_SIZE is taken as is
(both in KiB).  An optional third pass with TCC_HIT_sum / TCC_MISS_sum / TCC_REQ_sum gives
the L2 hit rate and request count per launch.

    python tools/pmc_summary.py <fetch_dir> <write_dir> <out.json> [--tcc DIR] [--K K] [--gpus N]
"""
import argparse
import collections
import csv
import glob
import json
import re


def per_kernel(d, counter):
    path = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        m = re.search(r"rtg::(k_\w+)(<([^>]*)>)?", r["Kernel_Name"])
        if not m:
            continue
        base, targs = m.group(1), [t.strip() for t in (m.group(3) or "").split(",") if t.strip()]
        if base == "k_shade" and len(targs) >= 3 and targs[2] == "2":
            base = "k_shade_shadow"                      # SH_FUSED: shading + the shadow ray
        name = base + (f"<{targs[0]}>" if targs else "")
        acc[name].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("out")
    ap.add_argument("--tcc")
    ap.add_argument("--K", type=int, default=100352)
    ap.add_argument("--gpus", type=int, default=1)
    a = ap.parse_args()
    f = per_kernel(a.fetch_dir, "FETCH_SIZE")
    w = per_kernel(a.write_dir, "WRITE_SIZE")
    hit = per_kernel(a.tcc, "TCC_HIT_sum") if a.tcc else {}
    miss = per_kernel(a.tcc, "TCC_MISS_sum") if a.tcc else {}
    req = per_kernel(a.tcc, "TCC_REQ_sum") if a.tcc else {}
    res = {"note": "bytes per launch; read = 2 x FETCH_SIZE (gfx950 correction), write = WRITE_SIZE; "
                   "l2_hit_rate = TCC_HIT / (TCC_HIT + TCC_MISS)",
           "config": {"workload": "headline", "K": a.K, "n_gpus": a.gpus}, "kernels": {}}
    for k in sorted(set(f) | set(w)):
        rd = 2.0 * f.get(k, (0.0, 0))[0] * 1024.0
        wr = w.get(k, (0.0, 0))[0] * 1024.0
        e = {"read_bytes": round(rd), "write_bytes": round(wr), "traffic_bytes": round(rd + wr),
             "launches": max(f.get(k, (0, 0))[1], w.get(k, (0, 0))[1])}
        if k in hit and k in miss and hit[k][0] + miss[k][0] > 0:
            e["l2_hit_rate"] = round(hit[k][0] / (hit[k][0] + miss[k][0]), 4)
            e["l2_requests"] = round(req.get(k, (0.0, 0))[0])
        res["kernels"][k] = e
    json.dump(res, open(a.out, "w"), indent=1)
    for k, v in res["kernels"].items():
        print(f"{k:22s} read {v['read_bytes'] / 1e6:9.2f} MB  write {v['write_bytes'] / 1e6:9.2f} MB  "
              f"L2 hit {v.get('l2_hit_rate', '-')}  x{v['launches']}")


if __name__ == "__main__":
    main()
