"""Summarise rocprofv3 --pmc CSVs per kernel (average per dispatch)."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for path in glob.glob(root + "/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, cs in acc.items():
    if "tile" not in name and len(sys.argv) < 3:
        continue
    print(name[:100])
    for c, v in sorted(cs.items()):
        print("   %-24s %16.1f  (n=%d)" % (c, sum(v) / len(v), len(v)))
