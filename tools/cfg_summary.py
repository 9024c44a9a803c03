"""One line per configuration bench (bench.py --config): throughput in flight and serial, the
kernels of the timed pass, the N-GPU prediction from the part timings, the CPU baseline.

    python tools/cfg_summary.py gpurun_out/<tag>/cfg_*.log"""
import json
import sys

for path in sys.argv[1:]:
    rec = None
    for line in open(path):
        if line.startswith("{"):
            rec = json.loads(line)
    if rec is None:
        print(path, "no result line")
        continue
    c = rec["config"]
    parts = rec.get("parts", {})
    cpu = rec.get("cpu_baseline") or {}
    print(f"{c['workload'][:34]:34s} value {rec['value']:9.1f}  serial {c.get('serial', {}).get('mrays_s', 0):9.1f} "
          f"({c.get('serial', {}).get('ms_per_step')} ms)  ms/step {rec['ms_per_step']}  "
          f"eff2/4/8 {[parts.get(n, {}).get('predicted_efficiency') for n in ('2', '4', '8')]}  "
          f"kernels {rec['roofline'].get('kernels_ms')}  cpu {cpu.get('value')} {cpu.get('kind', '')}")
