"""Multi-GPU sharding of the k-mer count (one process per GPU).

Reads are independent units (lib/kmers.js:151-155), so an input is split into
per-rank shards at record boundaries; each rank counts its shard with the
global line index / byte offset of its first line (kmer_set_position), which
makes first-occurrence order keys comparable across ranks.  The only exchange
is one gather of the per-rank partial results to rank 0 (RCCL over xGMI):
unique packed keys + {first, count} pairs, padded to the largest rank with the
invalid key (which the merged reduce drops), followed by one reduce/order/
decode on rank 0 (kmer_finish_merged).  Record (non-ACGT) keys
are merged on the host with a small object gather.
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
    """Packed-key sentinel of the device reduce: 1 << 2(k-|P|) (kmer_api.hip)."""
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


def gather_records(ctr, dst=0, group=None):
    """Move every rank's host record keys (non-ACGT windows) into rank dst's context."""
    rank = dist.get_rank(group)
    mine = ctr.records_export()
    payload = (mine[0], mine[1].tolist(), mine[2].tolist(), mine[3].tolist())
    got = [None] * dist.get_world_size(group) if rank == dst else None
    dist.gather_object(payload, got, dst=dst, group=group)
    if rank == dst:
        import numpy as np
        for r, (kb, off, cnt, fst) in enumerate(got):
            if r != dst and cnt:
                ctr.records_import(kb, np.array(off, dtype=np.uint64), np.array(cnt, dtype=np.uint64),
                                   np.array(fst, dtype=np.uint64))


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
    return ctr.finish_merged(gk.data_ptr(), gv.data_ptr(), gk.numel(), total_lines, want_result=want_result)
