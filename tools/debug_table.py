"""Run table-mode golden cases one at a time with progress (debugging aid)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kmerjs_amd import _native  # noqa: E402

G = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")
g = json.load(open(os.path.join(G, "golden.json")))
for c in g["cases"]:
    p = c["prefix"]
    if not (c["step"] == 1 and c["k"] <= 32 and len(p) <= c["k"] and all(ch in "ACGT" for ch in p)):
        continue
    data = open(os.path.join(G, "inputs", c["input"]), "rb").read()
    print("case", c["input"], repr(p), c["k"], len(data), end=" ", flush=True)
    t0 = time.time()
    ctr = _native.Counter(k=c["k"], prefix=p.encode(), flags=_native.FLAG_UNORDERED)
    r = ctr.count_buffer(data)
    print("size", len(r), c["size"], "%.3fs" % (time.time() - t0), ctr.phase_times(), flush=True)
    ctr.close()
