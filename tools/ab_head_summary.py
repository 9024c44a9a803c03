"""Summarise tools/gpu_ab_head.sh output (bench_<lib>_<config>_<rep>.log): per library and
configuration, each repetition's Mrays/s (frames in flight), ms per step, the serial ms per
frame and the per-kernel HIP-event times.

    python tools/ab_head_summary.py gpurun_out/<tag>/ab"""
import glob
import json
import os
import re
import sys


def main():
    d = sys.argv[1]
    rows = []
    for f in sorted(glob.glob(os.path.join(d, "bench_*.log"))):
        m = re.match(r"bench_(.+)_([a-z0-9]+)_(\d+)\.log$", os.path.basename(f))
        if not m:
            continue
        lines = [l for l in open(f) if l.startswith("{")]
        if not lines:
            rows.append((m.group(1), m.group(2), m.group(3), "no result"))
            continue
        j = json.loads(lines[-1])
        rows.append((m.group(1), m.group(2), m.group(3),
                     f"{j['value']:10.1f} Mrays/s  {j['ms_per_step']:.4f} ms/step  serial "
                     f"{j['config']['serial']['ms_per_step']:.4f} ms  kernels {j['roofline'].get('kernels_ms')}"))
    for lib, cfg, rep, txt in sorted(rows, key=lambda r: (r[1], r[0], r[2])):
        print(f"{cfg:8s} {lib:24s} rep {rep}: {txt}")
    st = os.path.join(d, "status.txt")
    if os.path.exists(st):
        print(open(st).read())


if __name__ == "__main__":
    main()
