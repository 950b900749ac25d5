"""Multi-GPU sharding of the k-mer count (one process per GPU).

Reads are independent units (lib/kmers.js:151-155), so an input is split into
per-rank shards at record boundaries; each rank counts its shard with the
global line index / byte offset of its first line (kmer_set_position), which
makes first-occurrence order keys comparable across ranks.  Each rank reduces
its shard to a partial result (unique packed keys + {first, count}, in
first-occurrence order).  Two ways to finish:

* finish_exchange (the default): no per-rank reduce at all -- the session's
  counting hits are partitioned by owning rank on the device
  (kmer_exchange_prepare: equal slices of the packed-key space, stable), ONE
  all-to-all (RCCL over xGMI) moves each run to its owner, and the owner
  counts what it received with the single-GPU finish (kmer_finish_exchanged).
  The received runs, concatenated by source rank, are in first-occurrence
  order (shards are in line order), so each rank ends with its key range of
  the result, ordered by first occurrence.  The global Map order is the merge
  of the ranks' lists by first occurrence: collect_ordered_device gathers the
  lists to one rank (alltoallv over RCCL) and re-orders them on the device
  (kmer_merge_ordered).  Work per rank stays constant as ranks are added.
* finish_distributed: the same key-range all-to-all, but of per-rank partials
  (unique keys + {first, count}, kmer_partial_device) merged with
  kmer_finish_merged -- fewer bytes on the wire when keys repeat a lot within
  a shard (high coverage), one more reduce per rank.
* finish_dense (short keys, 2(k - |P|) <= 26 bits): SURVEY §8(e)'s dense
  merge -- per-rank partials scattered into dense count / first-occurrence
  arrays over the key space, one reduce-scatter each (sum, min): constant
  bytes on the wire whatever the input size (C4).
* merge_to: gather every partial to one rank and finish there (one ordered
  result on one GPU; the gather and the merge grow with the rank count).

Table mode (KMER_FLAG_UNORDERED / _CANONICAL, C3) shards the same way:
finish_table_exchange sends each rank's pass-1 keys to the rank owning their
slice of the hash space (kmer_table_exchange_prepare: 1024 partitions, rank o
owns a contiguous 1024/world of them), ONE all-to-all of the keys plus an
all-gather of the per-partition counts, and each owner runs pass 2 + the
final kernel over its buckets (kmer_table_finish_exchanged).  Partitions are
disjoint, so the ranks' table statistics add up (table_stats_all).

Record (non-ACGT) keys are merged on the host of one rank with a small object
gather.
"""
import torch
import torch.distributed as dist


class _CudaArray:
    """Expose a raw device pointer to torch via __cuda_array_interface__."""

    def __init__(self, ptr, n, typestr="<u8"):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False), "version": 2,
                                         "strides": None}


def device_u64(ptr, n, device):
    """int64 view (uint64 bits) of n words of device memory owned by the library."""
    t = torch.as_tensor(_CudaArray(ptr, n), device=device)
    assert t.data_ptr() == ptr
    return t.view(torch.int64)


def shard_plan(n_reads_per_rank, rank, record_bytes=317, lines_per_record=4):
    """Weak-scaling synthetic shards: rank r holds reads [r*n, (r+1)*n)."""
    first_read = rank * n_reads_per_rank
    return {"first_read": first_read, "lines_before": first_read * lines_per_record,
            "byte_offset": first_read * record_bytes, "n_reads": n_reads_per_rank}


def split_at_records(buf: bytes, world):
    """Split a FASTQ byte string into `world` shards that start at record
    starts (line index % 4 == 0); returns [(start, end, lines_before)]."""
    n = len(buf)
    # line starts
    starts = [0]
    pos = buf.find(b"\n")
    while pos != -1:
        if pos + 1 < n:
            starts.append(pos + 1)
        pos = buf.find(b"\n", pos + 1)
    rec_starts = starts[::4]
    out = []
    for r in range(world):
        lo = rec_starts[(len(rec_starts) * r) // world] if r else 0
        hi = rec_starts[(len(rec_starts) * (r + 1)) // world] if r + 1 < world else n
        if r + 1 < world and (len(rec_starts) * (r + 1)) // world >= len(rec_starts):
            hi = n
        lines_before = 4 * ((len(rec_starts) * r) // world)
        out.append((lo, hi, lines_before))
    return out


def invalid_key(k, plen):
    """Packed-key sentinel of the device reduce: 1 << 2(k-|P|) (kmer_finish.hip)."""
    return 1 << (2 * (k - plen))


def gather_partials(keys, vals, pad_key, dst=0, group=None):
    """Gather variable-length partials (keys int64[n], vals int64[n, 2]) to `dst`.

    Every rank pads to the largest n with (pad_key, {first=-1, count=0}); the
    padding sorts into the sentinel group that the merged reduce drops.
    Returns the concatenated (keys, vals) on dst, (None, None) elsewhere.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = keys.device
    host_coll = dist.get_backend(group) == "gloo"
    n = torch.tensor([keys.numel()], dtype=torch.int64, device="cpu" if host_coll else dev)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    maxn = max(int(x.item()) for x in sizes)
    if maxn == 0:
        return (keys[:0], vals[:0]) if rank == dst else (None, None)
    kp = torch.full((maxn,), pad_key, dtype=torch.int64, device=dev)
    vp = torch.empty((maxn, 2), dtype=torch.int64, device=dev)
    vp[:, 0] = -1
    vp[:, 1] = 0
    kp[:keys.numel()] = keys
    vp[:keys.numel()] = vals
    staged = host_coll and kp.is_cuda     # gloo: gather host tensors
    if staged:
        kp, vp = kp.cpu(), vp.cpu()
    if rank == dst:
        kl = [torch.empty_like(kp) for _ in range(world)]
        vl = [torch.empty_like(vp) for _ in range(world)]
        dist.gather(kp, kl, dst=dst, group=group)
        dist.gather(vp, vl, dst=dst, group=group)
        gk, gv = torch.cat(kl), torch.cat(vl)
        return (gk.to(dev), gv.to(dev)) if staged else (gk, gv)
    dist.gather(kp, None, dst=dst, group=group)
    dist.gather(vp, None, dst=dst, group=group)
    return None, None


def gather_records(ctr, dst=0, group=None, total=None, mine=None):
    """Move every rank's host record keys (non-ACGT windows) into rank dst's context.

    total: the number of records over all ranks when the caller already knows
    it (else one all-reduce finds it); mine: this rank's records_export()."""
    rank = dist.get_rank(group)
    if mine is None:
        mine = ctr.records_export()
    # skip the object gather when no rank has records (the common case)
    if total is None:
        dev = "cpu" if dist.get_backend(group) == "gloo" else torch.device("cuda", torch.cuda.current_device())
        tot = torch.tensor([len(mine[2])], dtype=torch.int64, device=dev)
        dist.all_reduce(tot, group=group)
        total = int(tot.item())
    if total == 0:
        return
    payload = (mine[0], mine[1].tolist(), mine[2].tolist(), mine[3].tolist())
    got = [None] * dist.get_world_size(group) if rank == dst else None
    dist.gather_object(payload, got, dst=dst, group=group)
    if rank != dst:
        ctr.records_clear()          # moved: a later host result of this rank must not repeat them
    if rank == dst:
        import numpy as np
        for r, (kb, off, cnt, fst) in enumerate(got):
            if r != dst and cnt:
                ctr.records_import(kb, np.array(off, dtype=np.uint64), np.array(cnt, dtype=np.uint64),
                                   np.array(fst, dtype=np.uint64))


def key_owner(keys, kbits, world):
    """Owning rank of each packed key: equal slices of the key space."""
    s = max(0, kbits - 40)
    return (((keys >> s) * world) >> (kbits - s)).clamp_(0, world - 1)


def shuffle_partials(keys, vals, kbits, group=None):
    """All-to-all of partial entries by key range.

    keys int64[n] (packed keys), vals int64[n, 2] ({first, count}), in
    first-occurrence order.  Returns this rank's key range from every rank,
    concatenated by source rank -- i.e. still in first-occurrence order."""
    world = dist.get_world_size(group)
    dev = keys.device
    host_coll = dist.get_backend(group) == "gloo"
    owner = key_owner(keys, kbits, world)
    order = torch.sort(owner, stable=True).indices       # stable: first order kept per destination
    ks, vs = keys[order], vals[order]
    send = torch.bincount(owner, minlength=world).to(torch.int64)
    recv = torch.empty_like(send)
    if host_coll:
        send, recv, ks, vs = send.cpu(), recv.cpu(), ks.cpu(), vs.cpu()
    dist.all_to_all_single(recv, send, group=group)
    send_l, recv_l = send.tolist(), recv.tolist()
    rk = torch.empty(sum(recv_l), dtype=torch.int64, device=ks.device)
    rv = torch.empty((sum(recv_l), 2), dtype=torch.int64, device=ks.device)
    dist.all_to_all_single(rk, ks, recv_l, send_l, group=group)
    dist.all_to_all_single(rv.view(-1), vs.reshape(-1), [2 * x for x in recv_l], [2 * x for x in send_l], group=group)
    if host_coll:
        rk, rv = rk.to(dev), rv.to(dev)
    return rk, rv


def exchange_counts(counts, n_records, device, group=None):
    """All-to-all of the per-destination run lengths, with this rank's host
    record count riding along.  Returns (received run lengths by source rank,
    record counts by rank) as host lists -- one device->host sync."""
    world = dist.get_world_size(group)
    assert len(counts) == world
    if dist.get_backend(group) == "gloo":
        device = "cpu"
    send = torch.tensor([[c, n_records] for c in counts], dtype=torch.int64).to(device, non_blocking=True)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    r = recv.cpu().tolist()
    return [x[0] for x in r], [x[1] for x in r]


def exchange_runs(send, counts, recv_counts, words=2, group=None):
    """All-to-all of owner-major runs of `words` int64 words per record:
    send = int64[words * sum(counts)] (run o goes to rank o); returns the
    received runs concatenated by source rank, int64[words * sum(recv_counts)]."""
    dev = send.device
    host_coll = dist.get_backend(group) == "gloo"
    out = torch.empty(words * sum(recv_counts), dtype=torch.int64, device="cpu" if host_coll else dev)
    src = send.cpu() if host_coll else send
    dist.all_to_all_single(out, src, [words * x for x in recv_counts], [words * x for x in counts], group=group)
    return out.to(dev) if host_coll else out


def finish_exchange(ctr, k, plen, total_lines, group=None, want_result=False, records=True, dst=0):
    """Finish a sharded count by exchanging hits (module docstring): afterwards
    every rank holds its key range of the result, ordered by first occurrence
    (device, kmer_result_device).  Record keys are merged on rank `dst`."""
    world = dist.get_world_size(group)
    dev = torch.device("cuda", torch.cuda.current_device())
    d_x, counts = ctr.exchange_prepare(world)
    mine = ctr.records_export() if records else None
    recv_counts, rec_counts = exchange_counts(counts, len(mine[2]) if mine else 0, dev, group=group)
    n_send = sum(counts)
    send = device_u64(d_x, 2 * n_send, dev) if n_send else torch.empty(0, dtype=torch.int64, device=dev)
    recv = exchange_runs(send, counts, recv_counts, group=group)
    if records:
        gather_records(ctr, dst=dst, group=group, total=sum(rec_counts), mine=mine)
    # the finish runs on the context's stream after the collective (stream wait,
    # no host sync) and may read `recv` after returning: keep it alive
    ctr._keepalive = (recv,)
    return ctr.finish_exchanged(recv.data_ptr(), recv.numel() // 2, total_lines,
                                stream=torch.cuda.current_stream(dev).cuda_stream, want_result=want_result)


def table_part_range(o, world, parts=1024):
    """Pass-1 partitions [lo, hi) owned by rank o (tab_part_lo, kmer_api.hip / kmer_tabhost.hip)."""
    return o * parts // world, (o + 1) * parts // world


def exchange_table_keys(send, counts, parts, group=None):
    """The collectives of the table exchange: per-destination run lengths
    (all-to-all), every rank's per-partition counts (all-gather), and the key
    runs (all-to-all).  send = int64[sum(counts)] (runs in owner order);
    returns (received runs by source rank, int64[world, len(parts)])."""
    world = dist.get_world_size(group)
    host_coll = dist.get_backend(group) == "gloo"
    cdev = "cpu" if host_coll else send.device
    send_n = torch.tensor(counts, dtype=torch.int64).to(cdev)
    recv_n = torch.empty_like(send_n)
    dist.all_to_all_single(recv_n, send_n, group=group)
    mine = torch.tensor(parts, dtype=torch.int64).to(cdev)
    allp = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allp, mine, group=group)
    recv_l = recv_n.cpu().tolist()
    recv = exchange_runs(send, counts, recv_l, words=1, group=group)
    return recv, torch.stack(allp).cpu()


def finish_table_exchange(ctr, group=None, records=True, dst=0):
    """Finish a sharded table-mode count (module docstring): afterwards every
    rank holds its buckets of the table (kmer_table_device).  Record keys are
    moved to rank `dst`, so table_stats_all counts each once."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = torch.device("cuda", torch.cuda.current_device())
    d_x, counts, parts = ctr.table_exchange_prepare(world)
    n_send = sum(counts)
    send = device_u64(d_x, n_send, dev) if n_send else torch.empty(0, dtype=torch.int64, device=dev)
    recv, parts_all = exchange_table_keys(send, counts, parts, group=group)
    if records:
        gather_records(ctr, dst=dst, group=group)
    # the table is written over `recv` (and read from it) on the context's
    # stream after the collective: keep it alive until the next reset
    ctr._keepalive = (recv,)
    ctr.table_finish_exchanged(recv.data_ptr() if recv.numel() else 0, recv.numel(), parts_all.numpy(),
                               world, rank, stream=torch.cuda.current_stream(dev).cuda_stream)


def table_stats_all(ctr, group=None):
    """(canonical, keys, total) of the whole sharded table: the ranks' shares summed."""
    dev = "cpu" if dist.get_backend(group) == "gloo" else torch.device("cuda", torch.cuda.current_device())
    t = torch.tensor(list(ctr.table_stats()), dtype=torch.int64, device=dev)
    dist.all_reduce(t, group=group)
    return tuple(int(x) for x in t.tolist())


def finish_distributed(ctr, k, plen, total_lines, group=None, want_result=False, records=True, dst=0):
    """Finish a sharded count with the key-range all-to-all: afterwards every
    rank holds its key range of the result, ordered by first occurrence
    (device, kmer_result_device).  Record keys are merged on rank `dst`."""
    d_k, d_v, n = ctr.partial_device()
    dev = torch.device("cuda", torch.cuda.current_device())
    keys = device_u64(d_k, n, dev) if n else torch.empty(0, dtype=torch.int64, device=dev)
    vals = device_u64(d_v, 2 * n, dev).view(n, 2) if n else torch.empty((0, 2), dtype=torch.int64, device=dev)
    rk, rv = shuffle_partials(keys, vals, 2 * (k - plen), group=group)
    if records:
        gather_records(ctr, dst=dst, group=group)
    torch.cuda.synchronize()
    # the merged finish runs on the context's own stream and may still read the
    # received buffers after returning: keep them alive until the next finish
    ctr._keepalive = (rk, rv)
    return ctr.finish_merged(rk.data_ptr(), rv.data_ptr(), rk.numel(), total_lines, want_result=want_result)


INT64_MAX = (1 << 63) - 1


def dense_reduce(keys, vals, kbits, group=None):
    """SURVEY.md §8(e)'s dense merge, for short packed keys (2(k - |P|) <= 26
    bits: C2 / C4 have 22): this rank's partial entries (unique packed keys,
    {first, count}) are scattered into dense arrays over the whole key space
    -- counts and first-occurrence keys -- and ONE reduce-scatter each (sum,
    min) leaves every rank its equal slice of the key space, summed over the
    ranks.  Bytes on the wire are 16 B x 2^kbits whatever the input size
    (C4: 67 MB per rank against 16 B per hit = 527 MB for the hit exchange).
    Returns this rank's entries (keys int64[m], vals int64[m, 2] {first,
    count}) in first-occurrence order."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = keys.device
    n_slots = 1 << kbits
    per = -(-n_slots // world)
    cnt = torch.zeros(per * world, dtype=torch.int64, device=dev)
    fst = torch.full((per * world,), INT64_MAX, dtype=torch.int64, device=dev)
    ok = keys < n_slots                                  # (the reduce's invalid-key sentinel)
    kk = keys[ok]
    cnt[kk] = vals[ok, 1]
    fst[kk] = vals[ok, 0]
    if dist.get_backend(group) == "gloo":                # (CPU tests: gloo has no reduce_scatter)
        cnt, fst = cnt.cpu(), fst.cpu()
        dist.all_reduce(cnt, op=dist.ReduceOp.SUM, group=group)
        dist.all_reduce(fst, op=dist.ReduceOp.MIN, group=group)
        out_c = cnt[rank * per:(rank + 1) * per].to(dev)
        out_f = fst[rank * per:(rank + 1) * per].to(dev)
    else:
        out_c = torch.empty(per, dtype=torch.int64, device=dev)
        out_f = torch.empty(per, dtype=torch.int64, device=dev)
        dist.reduce_scatter_tensor(out_c, cnt, op=dist.ReduceOp.SUM, group=group)
        dist.reduce_scatter_tensor(out_f, fst, op=dist.ReduceOp.MIN, group=group)
    idx = torch.nonzero(out_c > 0).flatten()
    f = out_f[idx]
    o = torch.argsort(f)
    return idx[o] + rank * per, torch.stack([f[o], out_c[idx][o]], dim=1).contiguous()


def finish_dense(ctr, k, plen, total_lines, group=None, want_result=False, records=True, dst=0):
    """Finish a sharded count with the dense reduce (dense_reduce): afterwards
    every rank holds its key range of the result, ordered by first occurrence
    (device, kmer_result_device), as after finish_exchange.  Record keys are
    merged on rank `dst`."""
    d_k, d_v, n = ctr.partial_device()
    dev = torch.device("cuda", torch.cuda.current_device())
    keys = device_u64(d_k, n, dev) if n else torch.empty(0, dtype=torch.int64, device=dev)
    vals = device_u64(d_v, 2 * n, dev).view(n, 2) if n else torch.empty((0, 2), dtype=torch.int64, device=dev)
    torch.cuda.synchronize()                     # (the partial is on the context's stream)
    rk, rv = dense_reduce(keys, vals, 2 * (k - plen), group=group)
    if records:
        gather_records(ctr, dst=dst, group=group)
    torch.cuda.synchronize()
    ctr._keepalive = (rk, rv)                    # (see finish_distributed)
    return ctr.finish_merged(rk.data_ptr(), rv.data_ptr(), rk.numel(), total_lines, want_result=want_result)


def gather_rows(tensors, n, dst=0, group=None):
    """Gather variable-length row blocks to `dst` with one all-to-all per
    tensor (alltoallv: only dst receives, no padding).  tensors: list of
    (tensor, elements per row); returns (received tensors concatenated by
    source rank, total rows) on dst, (None, 0) elsewhere."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    host_coll = dist.get_backend(group) == "gloo"
    dev = tensors[0][0].device
    cnt_dev = "cpu" if host_coll else dev
    send = torch.zeros(world, dtype=torch.int64, device=cnt_dev)
    send[dst] = n
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    recv_l = recv.cpu().tolist() if rank == dst else [0] * world
    total = sum(recv_l)
    out = []
    for t, per in tensors:
        src = t.cpu() if host_coll else t
        split_out = [per * x for x in recv_l]
        split_in = [per * n if r == dst else 0 for r in range(world)]
        o = torch.empty(per * total, dtype=t.dtype, device=src.device)
        dist.all_to_all_single(o, src, split_out, split_in, group=group)
        out.append(o.to(dev) if host_coll else o)
    return (out, total) if rank == dst else (None, 0)


def collect_ordered_device(ctr, k, total_lines, dst=0, group=None, want_result=False):
    """One result in Map order on rank `dst` after finish_exchange /
    finish_distributed (each rank holds its key range, ordered by first
    occurrence): every rank's (keys, counts, firsts) go to dst in one
    alltoallv each (RCCL over xGMI), and dst re-orders the union by first
    occurrence on the device (kmer_merge_ordered).  The record keys were
    already merged on dst.  Returns dst's Result when want_result (host
    entries, records merged in), else None; the ordered device result is
    dst's kmer_result_device."""
    d_keys, d_cnt, d_first, n = ctr.result_device()
    dev = torch.device("cuda", torch.cuda.current_device())
    if n:
        keys = torch.as_tensor(_CudaArray(d_keys, n * k, "|u1"), device=dev)
        cnt = device_u64(d_cnt, n, dev)
        fst = device_u64(d_first, n, dev)
    else:
        keys = torch.empty(0, dtype=torch.uint8, device=dev)
        cnt = torch.empty(0, dtype=torch.int64, device=dev)
        fst = torch.empty(0, dtype=torch.int64, device=dev)
    got, total = gather_rows([(keys, k), (cnt, 1), (fst, 1)], n, dst=dst, group=group)
    if got is None:
        return None
    torch.cuda.synchronize()                  # (the merge runs on the context's stream)
    rk, rc, rf = got
    ctr._keepalive = (rk, rc, rf)
    return ctr.merge_ordered(rk.data_ptr(), rc.data_ptr(), rf.data_ptr(), total, total_lines,
                             want_result=want_result)


def collect_ordered(ctr, k, total_lines, dst=0, group=None):
    """The whole Map in reference order on `dst` (device gather + device merge,
    collect_ordered_device): [(key bytes, count)] on dst, None elsewhere."""
    r = collect_ordered_device(ctr, k, total_lines, dst=dst, group=group, want_result=True)
    return r.entries() if r is not None else None


def merge_to(ctr, k, plen, total_lines, dst=0, group=None, want_result=True, records=True):
    """Finish a sharded count: gather every rank's partial to `dst` and finish there.

    ctr: kmerjs_amd.Counter that has fed this rank's shard.  Returns the merged
    ordered Result on dst (None elsewhere or when want_result is False).
    """
    d_k, d_v, n = ctr.partial_device()
    dev = torch.device("cuda", torch.cuda.current_device())
    keys = device_u64(d_k, n, dev) if n else torch.empty(0, dtype=torch.int64, device=dev)
    vals = device_u64(d_v, 2 * n, dev).view(n, 2) if n else torch.empty((0, 2), dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    gk, gv = gather_partials(keys, vals, invalid_key(k, plen), dst=dst, group=group)
    if records:
        gather_records(ctr, dst=dst, group=group)
    if dist.get_rank(group) != dst:
        return None
    torch.cuda.synchronize()
    ctr._keepalive = (gk, gv)                     # (see finish_distributed)
    return ctr.finish_merged(gk.data_ptr(), gv.data_ptr(), gk.numel(), total_lines, want_result=want_result)
