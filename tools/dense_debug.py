"""Dense-path (kmer_dense.hip) diagnostics on the GPU: synthetic reads of
several sizes and prefixes through feed_device and count_buffer, each result
compared with the CPU oracle (test infrastructure); one JSON line per case."""
import json
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from kmerjs_amd import _native, synth_fastq_device  # noqa: E402
from oracle import oracle  # noqa: E402

for n, k, p in ((1000, 12, b"ACG"), (131072, 12, b"ACG"), (131073, 12, b"ACG"), (200000, 12, b"ACG"),
                (200000, 16, b"AT"), (50000, 40, b"AT"), (20000, 64, b"A")):
    buf = torch.empty(n * 317, dtype=torch.uint8, device="cuda")
    synth_fastq_device(buf.data_ptr(), 1, 0, n)
    torch.cuda.synchronize()
    host = buf.cpu().numpy().tobytes()
    want = oracle.count_buffer(host, p, k, 1)
    row = {"reads": n, "k": k, "prefix": p.decode()}
    for how in ("device", "buffer"):
        ctr = _native.Counter(k=k, prefix=p)
        try:
            if how == "device":
                ctr.reset()
                ctr.feed_device(buf.data_ptr(), len(host))
                got = ctr.finish().entries()
            else:
                got = ctr.count_buffer(host).entries()
            row[how] = "ok" if got == want else "MISMATCH %d vs %d" % (len(got), len(want))
        except Exception as e:  # noqa: BLE001
            row[how] = "ERR " + str(e)[:300]
        finally:
            ctr.close()
    print(json.dumps(row), flush=True)
