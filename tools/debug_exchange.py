"""Two ranks' worth on one device: hit exchange + per-owner finish vs one pass
(distinct keys, sum of counts) at growing sizes (debugging aid)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from kmerjs_amd import _native, synth_fastq_device  # noqa: E402
from kmerjs_amd.multi import device_u64  # noqa: E402

dev = torch.device("cuda")
for n in [int(x) for x in sys.argv[1:]]:
    buf = torch.empty(n * 317, dtype=torch.uint8, device=dev)
    synth_fastq_device(buf.data_ptr(), 4, 0, n)
    torch.cuda.synchronize()
    one = _native.Counter(k=16, prefix=b"ATGAC")
    one.reset()
    one.feed_device(buf.data_ptr(), buf.numel())
    one.finish(want_result=False)
    _, dc, _, m = one.result_device()
    s1 = int(device_u64(dc, m, dev).sum())
    half = n // 2
    ctrs = [_native.Counter(k=16, prefix=b"ATGAC") for _ in range(2)]
    runs, tot_send = [], []
    for r, c in enumerate(ctrs):
        c.reset()
        c.set_position(4 * half * r, 317 * half * r)
        c.feed_device(buf.data_ptr() + 317 * half * r, 317 * half)
        d_x, counts = c.exchange_prepare(2)
        x = device_u64(d_x, 2 * sum(counts), dev).clone()
        runs.append((x[:2 * counts[0]], x[2 * counts[0]:]))
        tot_send.append(counts)
    tot = 0
    ms, ss = [], []
    for o, c in enumerate(ctrs):
        recv = torch.cat([runs[0][o], runs[1][o]])
        if os.environ.get("DBG_WAIT_STREAM") == "1":
            c.finish_exchanged(recv.data_ptr(), recv.numel() // 2, 4 * n,
                               stream=torch.cuda.current_stream().cuda_stream)
        else:
            torch.cuda.synchronize()
            c.finish_exchanged(recv.data_ptr(), recv.numel() // 2, 4 * n)
        _, oc, _, om = c.result_device()
        ms.append(om)
        ss.append(int(device_u64(oc, om, dev).sum()))
    print("reads", n, "one-pass distinct", m, "sum", s1, "| exchange sent", tot_send, "distinct", ms, sum(ms),
          "sum", ss, sum(ss), flush=True)
    for c in ctrs + [one]:
        c.close()
    del buf
