"""Per-kernel averages of every counter in rocprofv3 --pmc csv passes under a directory."""
import collections
import csv
import glob
import re
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for path in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        m = re.search(r"rtg::(k_\w+)(<([\w, ]+)>)?", r["Kernel_Name"])
        agg[m.group(1) + (m.group(2) or "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(agg):
    print(k, {c: f"{sum(v) / len(v):.4g}" for c, v in sorted(agg[k].items())})
