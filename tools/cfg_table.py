"""DESIGN.md §5 rows from a configs run: serial rate first, then 16 frames in flight, the N = 8
prediction and the CPU baseline.   python tools/cfg_table.py <cfg_*.log ...>"""
import json
import sys

NAMES = {"C2": "C2", "C3 70k": "C3", "C3 on": "C3-ton", "C4": "C4", "C5": "C5"}


def name(workload):
    for k, v in NAMES.items():
        if workload.startswith(k):
            return v
    return workload[:12]


def main(paths):
    for p in paths:
        lines = [l for l in open(p) if l.startswith("{")]
        # a bench log ends with its line; a .jsonl holds one line per configuration
        for d in ([json.loads(lines[-1])] if lines and not p.endswith((".jsonl", ".txt")) else
                  [json.loads(l) for l in lines]):
            row(d)


def row(d):
    c = d["config"]
    ser = c.get("serial", {})
    parts = d.get("parts", {}).get("8", {})
    cpu = d.get("cpu_baseline") or {}
    cpu_s = f"{cpu.get('value')} ({cpu.get('kind')}, {cpu.get('cores')} threads)" if cpu else "--"
    print(f"| {name(c['workload'])} | **{ser.get('mrays_s', 0):,.0f}** ({ser.get('ms_per_step', 0):.4g} ms) | "
          f"{d['value']:,.0f} ({d['ms_per_step']:.4g} ms) | {parts.get('predicted_efficiency', '--')} | {cpu_s} |")

if __name__ == "__main__":
    main(sys.argv[1:])
