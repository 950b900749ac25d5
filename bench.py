"""Benchmark: kmerjs FASTQ k-mer counting on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): per GPU, 10 M synthetic
150 bp reads (317 B FASTQ records, 3.17 GB, generated on the device), k=16,
prefix 'ATGAC'.  A step = one pass of the hot path over the resident batch:
the single-pass scan kernel (line framing + both strands + prefix filter ->
packed hit per accepted window), hit resolution, the per-rank reduce of
packed keys (radix sort + reduce-by-key), the RCCL gather of the partials to
rank 0 when N > 1, and the finish on rank 0 (merged reduce, radix sort by
first occurrence, key decode): the ordered Map-equivalent result, in HBM.

value = windows examined on both strands (k-mers) per second,
whole job.  Also reported: distinct k-mers/s, the tile kernel's roofline
(algorithmic bytes / kernel time vs 8 TB/s HBM), and the CPU baseline (the
oracle restatement, 1 core, bounded sample).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

RECORD = 317
READ_LEN = 150
HBM_PEAK_GBS = 8000.0


def windows_per_read(k):
    return 2 * max(0, READ_LEN - k + 1)


def cpu_baseline(k, prefix, seconds_target=10.0):
    """Oracle (C restatement, 1 thread) on a bounded sample of the same workload."""
    from oracle import oracle
    n = 20000
    data = oracle.synth_fastq(1, 0, n)
    t0 = time.perf_counter()
    oracle.count_buffer(data, prefix, k, 1)
    dt = time.perf_counter() - t0
    n = int(max(20000, min(5_000_000, n * seconds_target / max(dt, 1e-6))))
    data = oracle.synth_fastq(1, 0, n)
    t0 = time.perf_counter()
    oracle.count_buffer(data, prefix, k, 1)
    dt = time.perf_counter() - t0
    return {"value": n * windows_per_read(k) / dt, "unit": "k-mers/s", "cores": 1, "kind": "port",
            "sample": "%d synthetic reads (seed 1), k=%d, prefix %r, oracle/kmer_oracle.c single-threaded, %.1f s"
                      % (n, k, prefix.decode(), dt)}


def load_traffic(args):
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        key = "k%d_%s_r%d" % (args.k, args.prefix, args.reads)
        return d.get(key, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--reads", type=int, default=10_000_000, help="reads per GPU")
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--prefix", default="ATGAC")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pcie", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from kmerjs_amd import Counter, synth_fastq_device
    from kmerjs_amd.multi import merge_to, shard_plan

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    prefix = args.prefix.encode()
    plan = shard_plan(args.reads, rank)
    nbytes = args.reads * RECORD
    buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    synth_fastq_device(buf.data_ptr(), args.seed, plan["first_read"], args.reads)
    torch.cuda.synchronize()

    ctr = Counter(k=args.k, prefix=prefix, device=local, flags=args.flags)
    total_lines = world * args.reads * 4
    tile_ms, feed_ms_l = [], []

    def step(record):
        ctr.reset()
        ctr.set_position(plan["lines_before"], plan["byte_offset"])
        ctr.feed_device(buf.data_ptr(), nbytes)
        scan_ms, feed_ms, _ = ctr.last_timing()
        if record:
            tile_ms.append(scan_ms)
            feed_ms_l.append(feed_ms)
        if world > 1:
            merge_to(ctr, args.k, len(prefix), total_lines, dst=0, want_result=False)
        else:
            ctr.finish(want_result=False)

    for _ in range(args.warmup):
        step(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # one more pass to read the result size / accepted windows (outside the timed region)
    ctr.reset()
    ctr.set_position(plan["lines_before"], plan["byte_offset"])
    ctr.feed_device(buf.data_ptr(), nbytes)
    distinct, accepted = 0, 0
    res = merge_to(ctr, args.k, len(prefix), total_lines, dst=0) if world > 1 else ctr.finish(want_result=True)
    if rank == 0:
        distinct = len(res)
        accepted = int(res.counts.sum())
        assert res.lines == total_lines, (res.lines, total_lines)

    if rank == 0:
        windows_step = world * args.reads * windows_per_read(args.k)
        ms_per_step = elapsed / args.steps * 1e3
        value = windows_step * args.steps / elapsed
        kern_ms = sum(tile_ms) / len(tile_ms)
        # algorithmic bytes per scan launch: the whole FASTQ batch is read
        # once (B_in) + one 24-B hit record written per accepted window
        algo_bytes = nbytes + 24 * (accepted / world)
        achieved = algo_bytes / (kern_ms * 1e-3) / 1e9
        traffic = load_traffic(args)
        out = {
            "metric": "k-mers/sec + distinct-kmers/sec, k=%d 150bp synthetic FASTQ, 1/2/4/8 GPU" % args.k,
            "value": value,
            "unit": "k-mers/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (on-device splitmix64 FASTQ, 317 B records, seed %d)" % args.seed,
            "config": {"workload": "C2: %d synthetic 150bp reads per GPU, k=%d, prefix '%s'"
                                   % (args.reads, args.k, args.prefix),
                       "reads_per_gpu": args.reads, "k": args.k, "prefix": args.prefix,
                       "bytes_per_gpu": nbytes, "parallelism": "dp%d (reads sharded, RCCL gather of partials)" % world},
            "distinct_kmers_per_s": distinct * args.steps / elapsed,
            "distinct_kmers": distinct,
            "accepted_windows": accepted,
            "scan_kernel_ms": kern_ms,
            "feed_device_ms": sum(feed_ms_l) / len(feed_ms_l),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic},
        }
        if not args.no_pcie and world == 1:
            # PCIe-inclusive rate (host bytes -> H2D -> count -> ordered host result); never `value`
            host = buf.cpu().numpy().tobytes()
            c2 = Counter(k=args.k, prefix=prefix, device=local)
            t0 = time.perf_counter()
            r = c2.count_buffer(host)
            dt = time.perf_counter() - t0
            c2.close()
            out["pcie_inclusive_kmers_per_s"] = args.reads * windows_per_read(args.k) / dt
            out["pcie_inclusive_ms"] = dt * 1e3
            assert len(r) == distinct
            del host
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(args.k, prefix)
        print(json.dumps(out), flush=True)
    ctr.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
