"""Summarise a tools/gpu_ab_env.sh run: value and per-kernel ms per (setting, config)."""
import glob
import json
import os
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "bench_*.log"))):
    lines = [l for l in open(f) if l.startswith("{")]
    if not lines:
        print(os.path.basename(f), "no result")
        continue
    r = json.loads(lines[-1])
    k = r.get("roofline", {}).get("kernels_ms", {})
    print(f"{os.path.basename(f)[6:-4]:40s} {r['value']:9.1f} {r['ms_per_step']:8.4f}  " +
          " ".join(f"{n}={v:.4f}" for n, v in k.items()))
