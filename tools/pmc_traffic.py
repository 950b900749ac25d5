"""Summarise tools/pmc_traffic.sh output into profiles/pmc_traffic.json.

FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KiB per dispatch.
MI355X_MICROARCH.md (HBM section): on gfx950 FETCH_SIZE reports exactly half
of the bytes of a wide coalesced streaming read (16 B/lane loads), so the
read figure is doubled; WRITE_SIZE is exact for 16 B/lane streaming stores.
The scan kernel's loads are 16 B/lane coalesced streams, so the correction
applies to it; other kernels are reported raw as well.
usage: python tools/pmc_traffic.py gpurun_out/TAG KEY [out.json]
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

root, key = sys.argv[1], sys.argv[2]
out_path = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                                "pmc_traffic.json")
vals = defaultdict(lambda: defaultdict(list))
for path in glob.glob(root + "/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        m = re.findall(r"kmerhip::(\w+)", name)
        short = m[0] if m else name[:40]
        vals[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
summary = {}
for k, cs in vals.items():
    d = {c: sum(v) / len(v) for c, v in cs.items()}
    d["dispatches"] = max(len(v) for v in cs.values())
    summary[k] = d
kname = "scan_planes_kernel" if "scan_planes_kernel" in summary else "scan_tile_kernel"
scan = summary.get(kname, {})
entry = {
    "kernel": kname,
    "fetch_size_kib_raw": scan.get("FETCH_SIZE"),
    "write_size_kib": scan.get("WRITE_SIZE"),
}
if scan.get("FETCH_SIZE") is not None and scan.get("WRITE_SIZE") is not None:
    entry["hbm_read_bytes_per_launch"] = 2 * scan["FETCH_SIZE"] * 1024
    entry["hbm_write_bytes_per_launch"] = scan["WRITE_SIZE"] * 1024
    entry["hbm_bytes_per_launch"] = entry["hbm_read_bytes_per_launch"] + entry["hbm_write_bytes_per_launch"]
entry["correction"] = "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); KiB -> bytes x1024"
entry["all_kernels"] = summary
data = {}
if os.path.exists(out_path):
    with open(out_path) as f:
        data = json.load(f)
data[key] = entry
with open(out_path, "w") as f:
    json.dump(data, f, indent=1, sort_keys=True)
print(json.dumps({k: v for k, v in entry.items() if k != "all_kernels"}, indent=1))
