"""GPU experiment: tile kernel time by mode vs a plain HBM read of the batch."""
import json
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402
from kmerjs_amd import Counter, synth_fastq_device  # noqa: E402
from kmerjs_amd import _native  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
buf = torch.empty(n * 317, dtype=torch.uint8, device="cuda")
synth_fastq_device(buf.data_ptr(), 1, 0, n)
torch.cuda.synchronize()
out = {"bytes": n * 317}
# plain read bandwidth reference (torch reduction over the same bytes)
v = buf[: (n * 317 // 8) * 8].view(torch.int64)
for _ in range(3):
    v.sum()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    v.sum()
torch.cuda.synchronize()
out["torch_sum_GBs"] = n * 317 * 10 / (time.perf_counter() - t0) / 1e9
modes = (("full", 0), ("byte_scan", 4), ("no_hits", 1 << 8), ("no_emit", 1 << 10))
for name, flags in modes:
    ctr = Counter(k=16, prefix=b"ATGAC", flags=flags)
    ts, fs, fin = [], [], []
    for i in range(6):
        ctr.reset()
        ctr.feed_device(buf.data_ptr(), n * 317)
        t = ctr.last_timing()
        r = ctr.finish(want_result=(i == 5))
        ts.append(t[0])
        fs.append(t[1])
        fin.append(ctr.last_timing()[2])
    out[name] = {"scan_ms": ts[1:], "feed_ms": fs[1:], "finish_ms": fin[1:], "distinct": len(r),
                 "scan_GBs": n * 317 / (min(ts[1:]) * 1e-3) / 1e9}
    ctr.close()
print(json.dumps(out))
