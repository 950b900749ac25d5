"""Per-dispatch PMC values of one kernel (in dispatch order), grouped in runs of N."""
import csv
import glob
import sys
from collections import defaultdict

root, kname, group = sys.argv[1], sys.argv[2], int(sys.argv[3])
rows = defaultdict(dict)
for path in glob.glob(root + "/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        if kname not in r["Kernel_Name"]:
            continue
        rows[(path.split("/pmc")[1].split("/")[0], int(r["Dispatch_Id"]))][r["Counter_Name"]] = float(r["Counter_Value"])
by_pass = defaultdict(list)
for (p, d), cs in sorted(rows.items()):
    by_pass[p].append(cs)
for p, lst in sorted(by_pass.items()):
    print("pass", p, "dispatches", len(lst))
    for g in range(0, len(lst), group):
        chunk = lst[g:g + group][1:]   # drop the warm-up of each group
        keys = sorted(chunk[0]) if chunk else []
        waves = None
        out = []
        for k in keys:
            v = sum(c[k] for c in chunk) / len(chunk)
            out.append("%s=%.4g" % (k, v))
        print("  group %d: %s" % (g // group, " ".join(out)))
