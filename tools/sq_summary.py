"""Per-kernel averages of a rocprofv3 --pmc SQ counter pass (-f csv)."""
import collections
import csv
import glob
import re
import sys

path = glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(path)):
    m = re.search(r"rtg::(k_\w+)(<(\w+)>)?", r["Kernel_Name"])
    agg[m.group(1) + (m.group(2) or "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    a = {c: sum(v) / len(v) for c, v in d.items()}
    w = a.get("SQ_WAVES", 1)
    print(f"{k:20s} waves {w:8.0f}  valu/wave {a.get('SQ_INSTS_VALU', 0) / w:7.0f}  salu/wave {a.get('SQ_INSTS_SALU', 0) / w:7.0f}"
          f"  vmem/wave {a.get('SQ_INSTS_VMEM_RD', 0) / w:6.1f}  wait {a.get('SQ_WAIT_ANY', 0) / max(a.get('SQ_WAVE_CYCLES', 1), 1):.2f}"
          f"  active {a.get('SQ_ACTIVE_INST_ANY', 0) / max(a.get('SQ_WAVE_CYCLES', 1), 1):.2f}")
