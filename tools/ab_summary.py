"""Summarise tools/gpu_ab.sh output: python tools/ab_summary.py <tag>"""
import json
import sys

d = f"gpurun_out/{sys.argv[1]}"
for k in ("base", "exp"):
    try:
        line = [l for l in open(f"{d}/bench_{k}.log") if l.startswith("{")][-1]
        j = json.loads(line)
        print(k, j["value"], j["unit"], j["ms_per_step"], j["roofline"].get("kernels_ms"))
    except Exception as e:  # noqa: BLE001
        print(k, "n/a", e)
print(open(f"{d}/status.txt").read())
