"""Inspect the device table of one small table-mode count (debugging aid)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from kmerjs_amd import _native  # noqa: E402
from kmerjs_amd.multi import device_u64  # noqa: E402

G = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "inputs")
data = open(os.path.join(G, "test_short.fastq"), "rb").read()
ctr = _native.Counter(k=int(sys.argv[1]), prefix=sys.argv[2].encode(), flags=_native.FLAG_UNORDERED)
r = ctr.count_buffer(data)
print("size", len(r), "stats", ctr.table_stats(), flush=True)
e, st, ln, bg, nb = ctr.table_device()
start = device_u64(st, (1 << 20) + 1, torch.device("cuda")).cpu().numpy()
nd = device_u64(ln, 1 << 19, torch.device("cuda")).cpu().numpy().view(np.uint32)
print("start[-1]", start[-1], "nonempty buckets", int((np.diff(start) > 0).sum()), "sum nd", int(nd.sum()),
      "max nd", int(nd.max()), flush=True)
nz = np.nonzero(np.diff(start))[0][:5]
for q in nz:
    print("q", q, "start", start[q], "n", start[q + 1] - start[q], "nd", nd[q])
print("nd>0 where empty:", int(((np.diff(start) == 0) & (nd > 0)).sum()))
ctr.close()
