"""Multi-GPU sharding of the k-mer count (one process per GPU).

Reads are independent units (lib/kmers.js:151-155), so an input is split into
per-rank shards at record boundaries; each rank counts its shard into its own
dense table with the global line index / byte offset of its first line
(kmer_set_position), and the only exchange is one merge of the tables: an
RCCL reduce over xGMI, SUM for counts and MIN for first-occurrence orders
(SURVEY.md §8e).  Record (non-ACGT) keys are merged on the host with a small
object gather.
"""
import torch
import torch.distributed as dist


class _CudaArray:
    """Expose a raw device pointer to torch via __cuda_array_interface__."""

    def __init__(self, ptr, n, typestr="<u8"):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False), "version": 2,
                                         "strides": None}


def device_u64(ptr, n, device):
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


def merge_dense_tables(counts: torch.Tensor, first: torch.Tensor, dst=0, group=None):
    """In-place reduce of per-rank dense tables to rank `dst`.

    counts: int64 (uint64 bits) counts, SUM.  first: first-occurrence orders
    as uint64 bits, MIN.  Orders are < 2^63 and the empty value is
    0xFFFF_FFFF_FFFF_FFFF (-1 as int64), so MIN on int64 would pick the empty
    marker; flip to order-preserving signed form (x ^ 2^63) around the reduce.
    """
    sign = torch.tensor(-(1 << 63), dtype=torch.int64, device=first.device)
    first.bitwise_xor_(sign)
    dist.reduce(counts, dst, op=dist.ReduceOp.SUM, group=group)
    dist.reduce(first, dst, op=dist.ReduceOp.MIN, group=group)
    first.bitwise_xor_(sign)
