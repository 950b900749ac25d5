"""Experiment: cost of the N > 1 finish on one GPU (world size 1, RCCL).

Times the single-GPU step next to the distributed step (partial -> key-range
all-to-all -> merged finish) with the all-to-all degenerate (self copy), and
a per-phase breakdown with a device sync after each phase.
  python tools/exp_dist.py [--reads N] [--steps S]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=10_000_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--prefix", default="ATGAC")
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    from kmerjs_amd import Counter, synth_fastq_device
    from kmerjs_amd import multi
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    n = args.reads * 317
    buf = torch.empty(n, dtype=torch.uint8, device=dev)
    synth_fastq_device(buf.data_ptr(), 1, 0, args.reads)
    torch.cuda.synchronize()
    P = args.prefix.encode()
    ctr = Counter(k=args.k, prefix=P, device=0)
    tl = args.reads * 4

    def feed():
        ctr.reset()
        ctr.set_position(0, 0)
        ctr.feed_device(buf.data_ptr(), n)

    def one():
        feed()
        ctr.finish(want_result=False)

    def distd():
        feed()
        multi.finish_distributed(ctr, args.k, len(P), tl)

    def timeit(fn, label):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps * 1e3
        print("%-34s %8.3f ms" % (label, dt), flush=True)
        return dt

    def exch():
        feed()
        multi.finish_exchange(ctr, args.k, len(P), tl)

    timeit(one, "N=1 step")
    timeit(distd, "partials all-to-all step (world 1)")
    timeit(exch, "hit exchange step (world 1)")
    # parity of the exchange finish with the single-GPU finish
    feed()
    want = ctr.finish(want_result=True).entries()
    feed()
    got = multi.finish_exchange(ctr, args.k, len(P), tl, want_result=True).entries()
    print("exchange == single finish:", got == want, len(got), flush=True)

    # phase breakdown
    ph = {"feed": 0.0, "partial": 0.0, "shuffle": 0.0, "records": 0.0, "merged": 0.0}
    for it in range(args.steps + 2):
        rec = it >= 2
        torch.cuda.synchronize()
        t = time.perf_counter()
        feed()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        d_k, d_v, m = ctr.partial_device()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        keys = multi.device_u64(d_k, m, dev)
        vals = multi.device_u64(d_v, 2 * m, dev).view(m, 2)
        rk, rv = multi.shuffle_partials(keys, vals, 2 * (args.k - len(P)))
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        multi.gather_records(ctr)
        t4 = time.perf_counter()
        ctr._keepalive = (rk, rv)
        ctr.finish_merged(rk.data_ptr(), rv.data_ptr(), rk.numel(), tl, want_result=False)
        torch.cuda.synchronize()
        t5 = time.perf_counter()
        if rec:
            for key, a, b in (("feed", t, t1), ("partial", t1, t2), ("shuffle", t2, t3), ("records", t3, t4),
                              ("merged", t4, t5)):
                ph[key] += (b - a) * 1e3 / args.steps
    for key, v in ph.items():
        print("  phase %-10s %8.3f ms" % (key, v), flush=True)
    ctr.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
