"""The multi-GPU paths over RCCL itself (backend "nccl" = RCCL on ROCm), at
world size 1 on the one-GPU box: every collective of bench.py's N-GPU step
(hit exchange + alltoallv collect, table-mode key exchange + stats
all-reduce) runs on device tensors and the context streams, and the results
equal the single-context count.  (Several ranks need several GPUs: the gloo
tests in test_dist.py and the in-process exchanges in test_gpu_parity.py /
test_table_gpu.py cover the N > 1 data movement.)"""
import socket

import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_world1_exchange_collect_and_table():
    import torch
    import torch.distributed as dist
    from kmerjs_amd import _native, multi, synth_fastq_device
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _free_port(), rank=0, world_size=1,
                            device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        n = 200_000
        buf = torch.empty(n * 317, dtype=torch.uint8, device=dev)
        synth_fastq_device(buf.data_ptr(), 11, 0, n)
        torch.cuda.synchronize()
        host = buf.cpu().numpy().tobytes()
        # ordered: hit exchange + device collect (Map order)
        ref = _native.Counter(k=16, prefix=b"ATGAC")
        want = ref.count_buffer(host).entries()
        ref.close()
        ctr = _native.Counter(k=16, prefix=b"ATGAC")
        ctr.reset()
        ctr.set_position(0, 0)
        ctr.feed_device(buf.data_ptr(), buf.numel())
        multi.finish_exchange(ctr, 16, 5, 4 * n)
        got = multi.collect_ordered(ctr, 16, 4 * n)
        ctr.close()
        assert got == want
        # ordered: dense reduce-scatter merge + device collect
        ctr = _native.Counter(k=16, prefix=b"ATGAC")
        ctr.reset()
        ctr.set_position(0, 0)
        ctr.feed_device(buf.data_ptr(), buf.numel())
        multi.finish_dense(ctr, 16, 5, 4 * n)
        got = multi.collect_ordered(ctr, 16, 4 * n)
        ctr.close()
        assert got == want
        # table mode: key exchange by hash-space slice + stats all-reduce
        one = _native.Counter(k=31, prefix=b"", flags=_native.FLAG_UNORDERED)
        one.reset()
        one.feed_device(buf.data_ptr(), buf.numel())
        one.finish(want_result=False)
        want_stats = one.table_stats()
        want_digest = one.table_digest()
        one.close()
        tab = _native.Counter(k=31, prefix=b"", flags=_native.FLAG_UNORDERED)
        tab.reset()
        tab.feed_device(buf.data_ptr(), buf.numel())
        multi.finish_table_exchange(tab)
        assert multi.table_stats_all(tab) == want_stats
        assert tab.table_digest() == want_digest
        tab.close()
    finally:
        dist.destroy_process_group()
