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


def cpu_baseline(k, prefix, seconds_target=8.0):
    """Oracle (C restatement) on a bounded sample of the same workload: one
    thread, and one thread per host core on record-aligned shards whose
    per-shard Maps are then merged (whole-job time, merge included)."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle
    n = 20000
    data = oracle.synth_fastq(1, 0, n)
    t0 = time.perf_counter()
    r0 = oracle.count_buffer(data, prefix, k, 1)
    dt = time.perf_counter() - t0
    n_cap = int(20_000_000 / max(1e-9, len(r0) / n))       # (host result lists of <= ~20 M entries)
    n = int(max(20000, min(5_000_000, n_cap, n * seconds_target / max(dt, 1e-6))))
    data = oracle.synth_fastq(1, 0, n)
    t0 = time.perf_counter()
    r1 = oracle.count_buffer(data, prefix, k, 1)
    dt1 = time.perf_counter() - t0
    # one thread per core (the box's CPU share is 16; ctypes calls release the GIL);
    # the Python merge of the shards' Maps is bounded to ~20 M entries (dense
    # prefixes: nearly every hit a distinct key)
    cores = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()))
    per_read = max(1e-9, len(r1) / n)
    nt = max(cores, min(n * cores, int(20_000_000 / per_read)))
    data = oracle.synth_fastq(1, 0, nt)
    per = (nt + cores - 1) // cores
    shards = [data[i * per * RECORD:min(nt, (i + 1) * per) * RECORD] for i in range(cores)]
    t0 = time.perf_counter()
    with ThreadPoolExecutor(cores) as ex:
        parts = list(ex.map(lambda b: oracle.count_buffer(b, prefix, k, 1), shards))
    merged = {}
    for part in parts:                       # shard order = read order: first occurrence kept
        for key, v in part:
            merged[key] = merged.get(key, 0) + v
    dtn = time.perf_counter() - t0
    return {"value": n * windows_per_read(k) / dt1, "unit": "k-mers/s", "cores": 1, "kind": "port",
            "sample": "%d synthetic reads (seed 1), k=%d, prefix %r, oracle/kmer_oracle.c single-threaded, %.1f s"
                      % (n, k, prefix.decode(), dt1),
            "threads": {"value": nt * windows_per_read(k) / dtn, "unit": "k-mers/s", "cores": cores, "kind": "port",
                        "sample": "%d reads in %d record-aligned shards, one thread each, + merge of the per-shard "
                                  "Maps; %.1f s" % (nt, cores, dtn)}}


def reference_js_c2(args):
    """The reference's own Node.js path (lib/kmers.js readFile(), unmodified) on
    this exact C2 workload, timed ONCE in the build container by
    tools/time_ref_c2.py (the reference never travels to the GPU box, SURVEY
    §8c): profiles/ref_js_c2.json.  Reported beside the C port's timing."""
    if args.reads != 10_000_000 or args.k != 16 or args.prefix != "ATGAC" or args.seed != 1:
        return None
    path = os.path.join(REPO, "profiles", "ref_js_c2.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    runs = {r["progress"]: r for r in d["runs"]}
    r0 = runs[False]
    return {"value": r0["kmers_per_s"], "unit": "k-mers/s", "cores": 1, "kind": "reference",
            "seconds": r0["seconds"], "progress_true": {"value": runs[True]["kmers_per_s"],
                                                       "seconds": runs[True]["seconds"]},
            "digest_equals_oracle": r0["digest_equals_oracle"],
            "sample": "the whole C2 workload (10 M reads, 3.17 GB), node %s, progress=false (default progress=true "
                      "beside it)" % d["host"]["node"],
            "where": d["where"] + " (%s, %d vCPU)" % (d["host"]["cpu"], d["host"]["vcpus"])}


def end_to_end(buf, args):
    """readFile() -> Map through the Node drop-in on the same input written to
    a file: a child `node` process, timed inside it."""
    import shutil
    import subprocess
    import tempfile
    node = shutil.which("node")
    if node is None:
        return {"skipped": "node not installed"}
    fd, path = tempfile.mkstemp(suffix=".fastq", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        with os.fdopen(fd, "wb") as f:
            step = 1 << 30
            for lo in range(0, buf.numel(), step):
                f.write(buf[lo:lo + step].cpu().numpy().tobytes())
        p = subprocess.run([node, os.path.join(REPO, "tools", "e2e_readfile.js"), path, args.prefix, str(args.k)],
                           capture_output=True, text=True, timeout=600)
        if p.returncode != 0:
            return {"error": p.stderr[-500:]}
        r = json.loads(p.stdout.strip().splitlines()[-1])
        r["what"] = ("Node KmerJS.readFile() on a %.2f GB FASTQ file: host read + H2D + GPU count + ordered result "
                     "+ N-API + lazy KmerMap; iterate = one full for..of; first_get = index build on the first "
                     "keyed access; eager_map = new Map(map) for comparison" % (buf.numel() / 1e9))
        return r
    finally:
        os.unlink(path)


def count_windows(lines_bytes_lengths, first_line, k):
    """Windows on both strands of the sequence lines (index % 4 == 1, length > 1)."""
    tot = 0
    for i, L in enumerate(lines_bytes_lengths):
        if (first_line + i) % 4 == 1 and L > 1 and L >= k:
            tot += 2 * (L - k + 1)
    return tot


def make_contigs(seed, target_bytes, k, width=0):
    """C5: FASTA '>c%08d\n' + contig of 10 kb - 1 Mb, seed 5;
    single-line (width 0: the reference reads it as FASTQ, line index % 4 == 1
    counts) or wrapped at `width` columns (KMER_FLAG_FASTA input, .fsa style).
    Returns (bytes, line lengths) -- for width > 0 the contig lengths instead."""
    import numpy as np
    rng = np.random.default_rng(seed)
    parts, lens, n, i = [], [], 0, 0
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    while n < target_bytes:
        L = int(rng.integers(10_000, 1_000_001))
        head = b">c%08d\n" % i
        seq = acgt[rng.integers(0, 4, L)]
        if width:
            full = L // width
            body = np.full(full * (width + 1), ord("\n"), np.uint8).reshape(full, width + 1)
            body[:, :width] = seq[:full * width].reshape(full, width)
            tail = seq[full * width:].tobytes()
            parts += [head, body.tobytes(), tail + (b"\n" if tail else b"")]
            lens.append(L)
            n += len(head) + body.size + len(tail) + (1 if tail else 0)
        else:
            parts += [head, seq.tobytes(), b"\n"]
            lens += [len(head) - 1, L]
            n += len(head) + L + 1
        i += 1
    return b"".join(parts), lens


def make_workload(args, rank, world, dev):
    """Input of this rank, resident in HBM, and its line / byte position in the whole job."""
    import torch
    import torch.distributed as dist
    from kmerjs_amd import synth_fastq_device
    from kmerjs_amd.multi import shard_plan
    if args.config in ("c2", "c3", "c4"):
        plan = shard_plan(args.reads, rank)
        nbytes = args.reads * RECORD
        buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        synth_fastq_device(buf.data_ptr(), args.seed, plan["first_read"], args.reads)
        torch.cuda.synchronize()
        per = args.reads * windows_per_read(args.k)
        return {"buf": buf, "nbytes": nbytes, "lines_before": plan["lines_before"], "byte_offset": plan["byte_offset"],
                "total_lines": world * args.reads * 4, "windows": per, "windows_total": world * per,
                "desc": "%s: %d synthetic 150bp reads per GPU, k=%d, prefix '%s'"
                        % (args.config.upper(), args.reads, args.k, args.prefix)}
    if args.config == "c5" and args.fasta:
        # .fsa-style multi-line contigs (60 columns), every record counted
        # (KMER_FLAG_FASTA; parity unpinned by the reference, which has no FASTA
        # parser: test/kmerFinderServer.js:158)
        data, lens = make_contigs(5 + rank, args.contig_bytes, args.k, width=60)
        n_lines = data.count(b"\n")
        info = torch.tensor([len(data), n_lines], dtype=torch.int64, device=dev)
        if world > 1:
            allv = [torch.zeros_like(info) for _ in range(world)]
            dist.all_gather(allv, info)
            sizes = [(int(x[0]), int(x[1])) for x in allv]
        else:
            sizes = [(len(data), n_lines)]
        per = sum(2 * (L - args.k + 1) for L in lens if L >= args.k and L > 1)
        tot = torch.tensor([per], dtype=torch.int64, device=dev)
        if world > 1:
            dist.all_reduce(tot)
        buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
        return {"buf": buf, "nbytes": len(data), "lines_before": sum(n for _, n in sizes[:rank]),
                "byte_offset": sum(b for b, _ in sizes[:rank]), "total_lines": sum(n for _, n in sizes),
                "windows": per, "windows_total": int(tot.item()), "records": len(lens),
                "desc": "C5 FASTA: contigs 10 kb-1 Mb in 60-column lines (seed 5+rank), %.2f GB per GPU, "
                        "every record counted (KMER_FLAG_FASTA), k=%d, prefix '%s'" % (len(data) / 1e9, args.k,
                                                                                    args.prefix)}
    if args.config == "c5":
        data, lens = make_contigs(5 + rank, args.contig_bytes, args.k)
        info = torch.tensor([len(data), len(lens)], dtype=torch.int64, device=dev)
        if world > 1:
            allv = [torch.zeros_like(info) for _ in range(world)]
            dist.all_gather(allv, info)
            sizes = [(int(x[0]), int(x[1])) for x in allv]
        else:
            sizes = [(len(data), len(lens))]
        byte_offset = sum(b for b, _ in sizes[:rank])
        lines_before = sum(n for _, n in sizes[:rank])
        per = count_windows(lens, lines_before, args.k)
        tot = torch.tensor([per], dtype=torch.int64, device=dev)
        if world > 1:
            dist.all_reduce(tot)
        buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
        return {"buf": buf, "nbytes": len(data), "lines_before": lines_before, "byte_offset": byte_offset,
                "total_lines": sum(n for _, n in sizes), "windows": per, "windows_total": int(tot.item()),
                "desc": "C5: single-line FASTA contigs 10 kb-1 Mb (seed 5+rank), %.2f GB per GPU, k=%d, prefix '%s'"
                        % (len(data) / 1e9, args.k, args.prefix)}
    if args.config == "c1":
        path = os.path.join(REPO, "tests", "golden", "inputs", "test_short.fastq")
        with open(path, "rb") as f:
            data = f.read()
        lens = [len(x) for x in data.split(b"\n")]
        if data.endswith(b"\n"):
            lens = lens[:-1]
        per = count_windows(lens, 0, args.k)
        buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
        return {"buf": buf, "nbytes": len(data), "lines_before": 0, "byte_offset": 0, "total_lines": len(lens),
                "windows": per, "windows_total": per,
                "desc": "C1: test_data/test_short.fastq, k=%d, prefix '%s' (plumbing)" % (args.k, args.prefix)}
    raise SystemExit("unknown config " + args.config)


def load_traffic(args, kern_name):
    """HBM bytes per launch of the kernel(s) `kern_name` names ("a + b (note)":
    the sum over a and b) in this config, from the committed PMC passes
    (profiles/pmc_traffic.json, keyed by config name and kernel)."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get(args.config + ("fa" if getattr(args, "fasta", False) else ""), {})
        reads = args.reads if args.config in ("c2", "c3", "c4") else 0   # (c1/c5 inputs are not read-based)
        if e.get("reads") not in (None, reads) or e.get("k") not in (None, args.k) or \
                e.get("prefix") not in (None, args.prefix):
            return None
        total = 0.0
        for kernel in kern_name.split(" (")[0].split(" + "):
            v = e.get("kernels", {}).get(kernel.strip(), {}).get("hbm_bytes_per_launch")
            if v is None:
                return None
            total += v
        return total
    except Exception:
        return None


# table mode (C3): algorithmic bytes of each phase per launch, from the
# pass-1 key count n (8-B keys) -- DESIGN.md §5.  final: every key read once
# (a bucket is held in registers across its LDS ranges) + one 8-B entry written
# per distinct canonical k-mer.
def table_phase_bytes(nbytes, n_keys, canonical, key_bytes=8):
    """Algorithmic bytes of the table phases: pass-1 keys of `key_bytes` (4:
    narrow keys, k <= 21 -- kmer_internal.hpp TAB_NSH), entries of 8 B."""
    kb = key_bytes
    return {"lines": nbytes, "hist1": nbytes, "scatter1": nbytes + kb * n_keys, "hist2": kb * n_keys,
            "scatter2": 2 * kb * n_keys, "final": kb * n_keys + 8 * canonical}


def print_shard_plan(args, world, strong):
    """--dry-run: the record-aligned shard each rank would count (reads-based
    configs: multi.shard_plan; c5: the rank's own contig file), one JSON line
    per rank -- no GPU is touched."""
    from kmerjs_amd.multi import shard_plan
    for r in range(world):
        row = {"rank": r, "world": world, "config": args.config, "k": args.k, "prefix": args.prefix,
               "merge": args.merge if world > 1 else None, "scaling": "strong" if strong else "weak"}
        if args.config in ("c2", "c3", "c4"):
            row.update(shard_plan(args.reads, r))
            row["windows"] = args.reads * windows_per_read(args.k)
        elif args.config == "c5":
            row.update({"contig_seed": 5 + r, "contig_bytes": args.contig_bytes, "fasta": bool(args.fasta)})
        print(json.dumps(row), flush=True)


def rank_envs(n, port, base=None):
    """Environment of each of the n worker processes `--gpus n` starts when no
    launcher set WORLD_SIZE: one process per GPU, rank r on device r."""
    base = dict(os.environ if base is None else base)
    envs = []
    for r in range(n):
        e = dict(base)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                  "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")     # (RCCL across processes: dmabuf IPC only)
        envs.append(e)
    return envs


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, dry_run=False, script=None):
    """`python bench.py --gpus N` without a launcher: start N child processes
    of this script, one per GPU (ranks 0..N-1, rendezvous on 127.0.0.1), and
    return the exit status of the job (the first failing rank's, else 0).
    Runs before anything touches the GPU, and never execs: the children are
    fresh processes whose stdout is this process's (rank 0 prints the line)."""
    import subprocess
    envs = rank_envs(n, free_port())
    cmd = [sys.executable, script or os.path.abspath(__file__)] + [a for a in argv if a != "--dry-run-launch"]
    if dry_run:
        keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
        for e in envs:
            print(json.dumps({"cmd": cmd, "env": {k: e[k] for k in keys}}))
        return 0
    procs = [subprocess.Popen(cmd, env=e) for e in envs]
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                r = p.poll()
                if r is None:
                    continue
                live.remove(p)
                if r != 0 and rc == 0:
                    rc = r
                    for q in live:            # one rank failed: the others would wait forever in a collective
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc if rc >= 0 else 128 - rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs (ranks).  Under torch.distributed.run WORLD_SIZE must equal it; without a launcher "
                         "bench.py starts the N rank processes itself")
    ap.add_argument("--dry-run-launch", action="store_true",
                    help="print the rank environments --gpus N would start and exit (no GPU)")
    ap.add_argument("--dry-run", action="store_true",
                    help="print the shard plan of each of the --gpus N ranks (one JSON line per rank) and exit "
                         "(no GPU, no launch)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--reads", type=int, default=10_000_000, help="reads per GPU")
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--prefix", default="ATGAC")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pcie", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the Node readFile() -> Map end-to-end run")
    ap.add_argument("--no-pipelined", action="store_true",
                    help="skip the extra two-session (double-buffered) throughput measurement")
    ap.add_argument("--no-match", action="store_true",
                    help="skip the template-matching record (C2's result joined against a synthetic kmerFinder DB)")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="sessions in rotation (>= 2: a step's finish overlaps the next steps' scans)")
    ap.add_argument("--config", default="c2", choices=("c1", "c2", "c3", "c4", "c5"),
                    help="BASELINE.json config: c2 (default, the headline); c3 100 M reads, k=31, no prefix "
                         "(table mode); c4 125 M reads per GPU (1 B on 8), k=16; c5 long contigs k=21")
    ap.add_argument("--contig-bytes", type=int, default=1_000_000_000, help="c5: bytes of contigs per GPU")
    ap.add_argument("--ordered", action="store_true", help="c5: the reference's ordered Map instead of canonical")
    ap.add_argument("--fasta", action="store_true",
                    help="c5: .fsa-style contigs in 60-column lines, counted by record (KMER_FLAG_FASTA, an "
                         "extension: parity unpinned by the reference, which has no FASTA parser)")
    ap.add_argument("--collect", action="store_true",
                    help="N > 1: the timed step also gathers every rank's ordered key range to rank 0 and merges "
                         "them on the device into ONE result in Map order (kmer_merge_ordered)")
    ap.add_argument("--merge", default=None, choices=("hits", "alltoall", "gather", "dense"),
                    help="N > 1: hits: key-range all-to-all of the hits + per-rank finish (result distributed by "
                         "key range); alltoall: the same with per-rank partials; dense: per-rank partials as dense "
                         "count / first-occurrence arrays, one reduce-scatter each (SURVEY §8e; short keys); "
                         "gather: all partials to rank 0.  Default: dense for c4 (bytes independent of the input "
                         "size), hits otherwise")
    args = ap.parse_args()
    if "WORLD_SIZE" not in os.environ and (args.gpus > 1 or args.dry_run_launch) and not args.dry_run:
        sys.exit(launch_ranks(max(1, args.gpus), sys.argv[1:], dry_run=args.dry_run_launch))
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        sys.exit("bench.py: WORLD_SIZE=%s but --gpus %d" % (os.environ["WORLD_SIZE"], args.gpus))
    # per-config defaults (explicit flags still win)
    argv = " ".join(sys.argv)
    from kmerjs_amd._native import FLAG_UNORDERED
    if args.config == "c3":
        # hash-table pressure: 24 G windows, ~12 G distinct canonical 31-mers -- far
        # beyond an ordered Map (the reference stops at 2^24 keys), so table mode
        if "--k" not in argv:
            args.k = 31
        if "--prefix" not in argv:
            args.prefix = ""
        if "--reads" not in argv:
            args.reads = 100_000_000
        if "--seed" not in argv:
            args.seed = 3
        args.flags |= FLAG_UNORDERED
    if args.config == "c4":
        # 1 B reads over 8 GPUs: 125 M per GPU (39.6 GB shard), seed 4
        if "--reads" not in argv:
            args.reads = 125_000_000
        if "--seed" not in argv:
            args.seed = 4
    if args.config == "c5":
        # long contigs, k = 21, canonical k-mers (BASELINE configs[4]): table
        # mode with KMER_FLAG_CANONICAL, no prefix (an extension: the reference
        # Map has no canonical form; parity of the underlying counts is tested)
        from kmerjs_amd._native import FLAG_CANONICAL
        if "--k" not in argv:
            args.k = 21
        if "--prefix" not in argv:
            args.prefix = ""
        if "--ordered" not in argv:
            args.flags |= FLAG_CANONICAL
        if args.fasta:
            from kmerjs_amd._native import FLAG_FASTA
            args.flags |= FLAG_FASTA
    if args.config != "c2":
        args.no_pcie = True
    if args.merge is None:
        args.merge = "dense" if args.config == "c4" and 2 * (args.k - len(args.prefix)) <= 26 else "hits"
    from kmerjs_amd._native import FLAG_CANONICAL as _FC
    table = bool(args.flags & (FLAG_UNORDERED | _FC))
    world_env = args.gpus if args.dry_run else int(os.environ.get("WORLD_SIZE", "1"))
    strong = False
    if args.config == "c3" and world_env > 1 and "--reads" not in argv:
        # C3 names a job (100 M reads), not a per-GPU size; one rank's 100 M reads
        # plus the exchange's send and receive key buffers would not fit 288 GB:
        # N ranks split the 100 M reads (strong scaling)
        args.reads = 100_000_000 // world_env
        strong = True
    if args.dry_run:
        print_shard_plan(args, world_env, strong)
        return

    import torch
    import torch.distributed as dist
    from kmerjs_amd import Counter
    from kmerjs_amd.multi import (collect_ordered_device, device_u64, finish_dense, finish_distributed,
                                  finish_exchange, finish_table_exchange, merge_to)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (never used by the driver): all ranks on one device, gloo instead of RCCL
    if os.environ.get("KMERHIP_ONE_DEVICE") == "1":
        local = 0
    backend = os.environ.get("KMERHIP_DIST_BACKEND", "nccl")
    one_device = os.environ.get("KMERHIP_ONE_DEVICE") == "1"
    rccl_ranks = 0
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        world = dist.get_world_size()
        rank = dist.get_rank()
        if dist.get_backend() == "nccl":
            rccl_ranks = world
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    prefix = args.prefix.encode()
    wl = make_workload(args, rank, world, dev)
    buf, nbytes = wl["buf"], wl["nbytes"]
    plan = {"lines_before": wl["lines_before"], "byte_offset": wl["byte_offset"]}

    # --pipeline N (N >= 2): N sessions in rotation.  Step i's chunk is queued
    # (kmer_feed_device returns without waiting), then the oldest session in
    # flight is settled and its finish queued on its high-priority stream, so
    # finishes (chains of small latency-bound kernels) overlap the following
    # scans instead of idling the chip.  Every step still does all of its work
    # inside the timed region: the sessions in flight are drained before the
    # clock stops.  Default: one session, steps strictly in sequence.
    nctx = max(1, args.pipeline)
    ctrs = [Counter(k=args.k, prefix=prefix, device=local, flags=args.flags) for _ in range(nctx)]
    ctr = ctrs[0]
    total_lines = wl["total_lines"]
    tile_ms, feed_ms_l = [], []
    phase_ms = []                 # table mode: per-step phase times
    inflight = []                 # (session, recorded) fed, finish not yet queued

    def feed(c):
        c.reset()
        c.set_position(plan["lines_before"], plan["byte_offset"])
        c.feed_device(buf.data_ptr(), nbytes)

    def retire():
        c, rec = inflight.pop(0)
        # the finish first (it settles the chunk itself), so that its kernels
        # are queued as soon as the scan's counters are back; the scan's own
        # time is read afterwards (those events are complete by then)
        multi_finish(c, rec, collect=args.collect)
        if rec:
            scan_ms, feed_ms, _ = c.last_timing(finish=False)
            tile_ms.append(scan_ms)
            feed_ms_l.append(feed_ms)

    def step(i, record):
        feed(ctrs[i % nctx])      # (its previous finish is ahead of it on its stream)
        inflight.append((ctrs[i % nctx], record))
        while len(inflight) > nctx - 1:
            retire()

    def drain():
        while inflight:
            retire()

    def multi_finish(c, record=False, collect=False):
        if world == 1:
            c.finish(want_result=False)
        elif table:
            # pass-1 keys to the owners of their hash-space slices (one RCCL
            # all-to-all), pass 2 + final on each owner's buckets
            finish_table_exchange(c)
        if table:
            if record:
                phase_ms.append(c.phase_times())
            return
        if world == 1:
            return
        if args.merge == "hits":
            finish_exchange(c, args.k, len(prefix), total_lines)
        elif args.merge == "alltoall":
            finish_distributed(c, args.k, len(prefix), total_lines)
        elif args.merge == "dense":
            finish_dense(c, args.k, len(prefix), total_lines)
        else:
            merge_to(c, args.k, len(prefix), total_lines, dst=0, want_result=False)
        if collect and args.merge != "gather":
            collect_ordered_device(c, args.k, total_lines, dst=0)

    for i in range(args.warmup):
        step(i, False)
    drain()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i, True)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # Also measured (single GPU, ordered paths): the same K steps with two
    # sessions in rotation, each step's finish overlapping the next step's
    # scan -- the double-buffered throughput of a batch pipeline.  Reported
    # beside `value`, which (like the roofline) comes from the steps above, run
    # strictly in sequence.
    pipelined = None
    if world == 1 and nctx == 1 and not table and not args.no_pipelined:
        extra = Counter(k=args.k, prefix=prefix, device=local, flags=args.flags)
        saved = ctrs
        ctrs, nctx = [ctr, extra], 2
        for i in range(2):
            step(i, False)
        drain()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for i in range(args.steps):
            step(i, False)
        drain()
        torch.cuda.synchronize()
        pel = time.perf_counter() - t1
        ctrs, nctx = saved, 1
        extra.close()
        pipelined = {"sessions": 2, "ms_per_step": pel * 1e3 / args.steps,
                     "value": wl["windows_total"] * args.steps / pel, "unit": "k-mers/s"}

    # one more pass to read the result size / accepted windows (outside the timed region)
    feed(ctr)
    distinct, accepted = 0, 0
    multi_finish(ctr)
    # counted on the device (a C3-sized result has ~10^9 entries): ordered device
    # entries (every rank's key range after the all-to-all, or all on rank 0) +
    # the host-side records (non-ACGT windows, on rank 0)
    canonical = None
    if table:
        canonical, n_keys_map, map_sum = ctr.table_stats()
        n_dev, dev_sum, n_rec, rec_sum = n_keys_map, map_sum, 0, 0
        if world > 1:                     # the ranks' shares of the table add up
            tc = torch.tensor([canonical], dtype=torch.int64, device=dev)
            dist.all_reduce(tc)
            canonical = int(tc.item())
    else:
        d_keys, d_cnt, d_first, n_dev = ctr.result_device() if (rank == 0 or args.merge != "gather") else (0, 0, 0, 0)
        dev_sum = int(device_u64(d_cnt, n_dev, dev).sum().item()) if n_dev else 0
        if n_dev > 1 and not (args.flags >> 8):      # (ablation experiments: results are wrong by design)
            f = device_u64(d_first, n_dev, dev)
            assert bool((f[1:] > f[:-1]).all().item()), "first-occurrence order broken"
        n_rec, rec_sum = 0, 0
        if rank == 0:
            kb, off, cnts, firsts = ctr.records_export()
            n_rec, rec_sum = len(cnts), int(cnts.sum())
    tot = torch.tensor([n_dev + n_rec, dev_sum + rec_sum], dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(tot)
    distinct, accepted = int(tot[0].item()), int(tot[1].item())
    if os.environ.get("KMERHIP_BENCH_VERIFY") == "1" and args.config in ("c2", "c4") and world > 1:
        # rehearsal check (never set by the driver): the distributed result, merged
        # by first occurrence, equals the oracle on the whole job's input
        from kmerjs_amd.multi import collect_ordered
        assert args.merge != "gather"
        got = collect_ordered(ctr, args.k, total_lines)
        if rank == 0:
            from oracle import oracle
            want = oracle.count_buffer(oracle.synth_fastq(args.seed, 0, world * args.reads), prefix, args.k, 1)
            assert got == want, "distributed result differs from the oracle"
            print("verify: %d entries equal the oracle" % len(want), file=sys.stderr)
    verified_table = None
    if os.environ.get("KMERHIP_BENCH_VERIFY") == "1" and table and world > 1 and args.config in ("c3", "c4", "c2"):
        # rehearsal check of the table exchange: the ranks' table digests (linear in
        # the counts, kmer_table_digest) add up to the digest of ONE context's table
        # over the whole job's input, and so do the table statistics
        d = ctr.table_digest()
        dig = torch.tensor([d - (1 << 64) if d >= (1 << 63) else d], dtype=torch.int64)   # (sum wraps mod 2^64)
        st = torch.tensor(list(ctr.table_stats()), dtype=torch.int64)
        cdev = "cpu" if dist.get_backend() == "gloo" else dev
        dig, st = dig.to(cdev), st.to(cdev)
        dist.all_reduce(dig)
        dist.all_reduce(st)
        if rank == 0:
            whole = torch.empty(world * args.reads * RECORD, dtype=torch.uint8, device=dev)
            from kmerjs_amd import synth_fastq_device
            synth_fastq_device(whole.data_ptr(), args.seed, 0, world * args.reads)
            torch.cuda.synchronize()
            one = Counter(k=args.k, prefix=prefix, device=local, flags=args.flags)
            one.reset()
            one.feed_device(whole.data_ptr(), whole.numel())
            one.finish(want_result=False)
            want_d, want_s = one.table_digest(), one.table_stats()
            one.close()
            del whole
            got_d = int(dig.item()) & ((1 << 64) - 1)
            got_s = tuple(int(x) for x in st.tolist())
            # (record keys were moved to rank 0, so their share of stats counts once)
            assert got_d == want_d, "table digest of the ranks %x != one context's %x" % (got_d, want_d)
            assert got_s == tuple(want_s), "table stats of the ranks %s != one context's %s" % (got_s, want_s)
            verified_table = {"digest": "%016x" % want_d, "stats": list(want_s)}
            print("verify: table digest %016x and stats %s of the %d ranks equal one context's table"
                  % (want_d, list(want_s), world), file=sys.stderr)

    if rank == 0:
        windows_step = wl["windows_total"]
        ms_per_step = elapsed / args.steps * 1e3
        value = windows_step * args.steps / elapsed
        kern_ms = sum(tile_ms) / len(tile_ms)
        # step-level fraction: SURVEY.md §8d algorithmic bytes per window (input
        # B_in + table B_table) x windows of the step / step time
        b_in = RECORD / windows_per_read(args.k) if args.config in ("c2", "c3", "c4") else nbytes / max(1, wl["windows"])
        if table:
            b_table = 16.0      # SURVEY §8d hash path: 16-B slot read + write per forward position / 2 windows
        else:
            b_table = 24.0 * accepted / max(1, windows_step)  # one slot update per accepted window
        step_bytes = (b_in + b_table) * windows_step / world
        step_frac = step_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS
        phases = None
        if table:
            # the dominant phase of the table pipeline (HIP events on the library's stream)
            phases = {kname: sum(p[kname] for p in phase_ms) / len(phase_ms) for kname in phase_ms[0]}
            # pass-1 keys = forward windows counted (no prefix): the Map sum is
            # twice that, the canonical sum once
            n_keys = (accepted if args.flags & _FC else accepted // 2) if not args.prefix else None
            pbytes = table_phase_bytes(nbytes, n_keys or 0, canonical, 4 if args.k <= 21 else 8)
            pbytes["fasta"] = 2 * nbytes      # (the rewrite: the chunk read once, about its size written)
            kern_name = max(phases, key=lambda x: phases[x])
            kern_ms = phases[kern_name]
            algo_bytes = pbytes[kern_name]
            # pass 1 without the counting pass (fixed runs: "hist1" is then only
            # the window counts per workgroup, well under a tenth of scatter1)
            fixed = phases.get("hist1", 0.0) < 0.1 * phases.get("scatter1", 1.0)
            kern_name = {"lines": "nl_slots_kernel + seq_lines_slots_kernel",
                         "hist1": "tab_hist1_kernel (+ scan)",
                         "scatter1": "tab_scatter1f_kernel" if fixed else "tab_scatter1h_kernel",
                         "hist2": "tab_hist2_kernel (+ scan)", "scatter2": "tab_scatter2f_kernel (fixed regions; counted route: tab_scatter2c_kernel)",
                         "final": "tab_sort_final_kernel (+ tab_final_kernel on its leftover units)",
                         "fasta": "fa_tiles_kernel + fa_write_kernel (FASTA rewrite)"}[kern_name]
        elif args.k > 64 or (not args.prefix and args.k > 31):
            # general path (k > 64, unprefixed k > 31): line arrays, the windows
            # (A/C/G/T prefix: plane candidates; else one lane per window
            # position); the accepted windows are merged on the device
            # (general_merge: hash sort + byte-checked groups) -- the feed
            # kernels together (lines, windows, append)
            wk = ("gen_cand_kernel" if args.prefix and set(args.prefix) <= set("ACGT") and not args.flags & 4
                  else "gen_windows_kernel")
            kern_name = "nl_slots_kernel + seq_lines_slots_kernel + " + wk + " + gen_append_kernel " \
                        "(general path feed; device merge at finish)"
            kern_ms = sum(feed_ms_l) / len(feed_ms_l)
            algo_bytes = nbytes + (24 + args.k) * (accepted / world)
        elif args.flags & 2 or not set(args.prefix) <= set("ACGT"):
            # tile path with records (records forced, or a non-ACGT prefix): the
            # plane scan for A/C/G/T prefixes (else the byte-SWAR scan)
            kern_name = ("scan_planes_kernel" if set(args.prefix) <= set("ACGT") else
                         "scan_tile_kernel") + " (tile records path; host record merge dominates the step)"
            algo_bytes = nbytes + 24 * (accepted / world)
        elif args.prefix and len(args.prefix) <= 3:
            # dense-hit path with a 1-3 base prefix (k <= 64): the timed phase
            # is the line split -- one streaming pass over the input
            # (nl_slots_kernel) + the sequence-line descriptors -- and the count
            # pass over the sequence lines (dense_windows_kernel<count>: the
            # 150 sequence bytes of a 317-B record read once more)
            kern_name = "nl_slots_kernel + seq_lines_slots_kernel + dense_windows_kernel<count> (dense-hit path)"
            algo_bytes = nbytes * (1.0 + 150.0 / 317.0)
        elif not args.prefix:
            # dense-hit path without a prefix (every window ranked): the timed
            # phase is the line split alone
            kern_name = "nl_slots_kernel + seq_lines_slots_kernel (dense-hit path line split)"
            algo_bytes = nbytes
        elif args.k > 32:
            # packed path with 128-bit window codes (k in 33..64, ACGT prefix)
            kern_name = "scan_planes_kernel (k > 32: 128-bit window codes)"
            algo_bytes = nbytes + 32 * (accepted / world)
        else:
            # algorithmic bytes per scan launch: the whole FASTQ batch is
            # read once (B_in) + one 24-B hit record written per accepted window
            kern_name = "scan_planes_kernel"
            algo_bytes = nbytes + 24 * (accepted / world)
        achieved = algo_bytes / (kern_ms * 1e-3) / 1e9
        traffic = load_traffic(args, kern_name)
        coll = "RCCL" if rccl_ranks else (dist.get_backend().upper() if world > 1 else "")
        out = {
            "metric": "k-mers/sec + distinct-kmers/sec, k=%d 150bp synthetic FASTQ, 1/2/4/8 GPU" % args.k,
            "value": value,
            "unit": "k-mers/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": {"c1": "test_data/test_short.fastq (reference fixture)",
                     "c5": "synthetic contigs (numpy PCG64, seed 5 + rank)%s" % (
                         ", 60-column FASTA records" if args.fasta else "")}.get(
                         args.config, "synthetic (on-device splitmix64 FASTQ, 317 B records, seed %d)" % args.seed),
            "config": {"workload": wl["desc"], "name": args.config,
                       "reads_per_gpu": args.reads if args.config in ("c2", "c3", "c4") else None,
                       "mode": ("table, canonical k-mers (KMER_FLAG_CANONICAL)" if args.flags & _FC else
                                "table (unordered canonical counts, KMER_FLAG_UNORDERED)") if table
                               else "ordered (reference Map insertion order)",
                       "k": args.k, "prefix": args.prefix, "windows_per_step": windows_step,
                       "bytes_per_gpu": nbytes,
                       "pipeline": ("%d sessions in rotation: finishes overlap later scans" % nctx if nctx > 1
                                    else "off (steps in sequence)"),
                       "parallelism": "dp1 (one GPU; no collective)" if world == 1 else
                       "dp%d (reads sharded; %s%s%s)" % (
                           world, coll + " all-to-all of pass-1 keys by hash-space slice, per-rank table finish"
                           if table else {"hits": coll + " all-to-all of hits by key range, per-rank finish",
                        "alltoall": coll + " all-to-all of partials by key range, per-rank finish",
                        "dense": coll + " reduce-scatter of dense count / first-occurrence arrays, per-rank finish"}.get(
                            args.merge, coll + " gather of partials, finish on rank 0"),
                           "; + alltoallv gather of the ordered ranges to rank 0 and device merge into one "
                           "Map-order result" if args.collect else "",
                           "; REHEARSAL: every rank on device 0" if one_device else ""),
                       "backend": "none" if world == 1 else ("rccl" if rccl_ranks else dist.get_backend())},
            "rccl_ranks": rccl_ranks,
            "distinct_kmers_per_s": distinct * args.steps / elapsed,
            "distinct_kmers": distinct,
            "accepted_windows": accepted,
            "scan_kernel_ms": kern_ms,
            "feed_device_ms": sum(feed_ms_l) / len(feed_ms_l),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": kern_name,
                         "algorithmic_bytes_per_launch": algo_bytes, "kernel_ms": kern_ms,
                         "step_frac": step_frac, "step_bytes_per_window": b_in + b_table},
        }
        if verified_table is not None:
            out["verified_table"] = verified_table
        if phases is not None:
            out["table_phase_ms"] = phases
            out["canonical_kmers"] = canonical
        if pipelined is not None:
            out["pipelined"] = pipelined
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
        if not args.no_e2e and world == 1 and args.config == "c2":
            out["end_to_end"] = end_to_end(buf, args)
        if not args.no_cpu_baseline and world == 1 and args.config == "c2":
            out["cpu_baseline"] = cpu_baseline(args.k, prefix)
            ref = reference_js_c2(args)
            if ref is not None:
                out["cpu_baseline"]["reference_js"] = ref
        if (not args.no_match and world == 1 and args.config == "c2" and args.pipeline == 1 and args.k == 16
                and args.prefix == "ATGAC"):
            # §8(f3): the count just measured, still in HBM, joined against a
            # synthetic template DB (tools/bench_match.py)
            sys.path.insert(0, os.path.join(REPO, "tools"))
            import bench_match
            d_keys, d_cnt, _, nq = ctr.result_device()
            out["template_matching"] = bench_match.measure(d_keys, d_cnt, nq, args.k, args.reads,
                                                           cpu_baseline=not args.no_cpu_baseline)
        print(json.dumps(out), flush=True)
    for c in ctrs:
        c.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
