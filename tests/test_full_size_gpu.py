"""Full-size tests of the BASELINE configurations (C2, C3, the C4 per-GPU
shard).  Pinned to answers computed ahead of time at the same sizes: C2's
ordered Map digest is the reference's own (lib/kmers.js run unmodified on the
same bytes, profiles/ref_js_c2.json) and the oracle's; the C4 shard's Map
digest and C3's table digest come from the oracle streamed over the same
synthetic reads (tests/golden/fullsize.json, tests/golden/gen_fullsize.py).
Plus properties that hold at any size -- Σ counts against windows counted
independently on the device, sortedness of first-occurrence keys, key
uniqueness, sharded == whole, and the linear table digest (the digest over
input A + B is the sum of the digests over A and B).  Marked `fullsize`:
tests/conftest.py runs them after every parity test."""
import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.fullsize]


@pytest.fixture(scope="module")
def native():
    from kmerjs_amd import _native
    return _native


def test_c2_full_size_properties(native):
    # BASELINE configs[1] at its size (10 M reads, 3.17 GB): properties that need no oracle
    import torch
    from kmerjs_amd import synth_fastq_device
    n = 10_000_000
    k, prefix = 16, b"ATGAC"
    buf = torch.empty(n * 317, dtype=torch.uint8, device="cuda")
    synth_fastq_device(buf.data_ptr(), 1, 0, n)
    torch.cuda.synchronize()
    ctr = native.Counter(k=k, prefix=prefix)
    ctr.reset()
    ctr.feed_device(buf.data_ptr(), buf.numel())
    res = ctr.finish()
    assert res.lines == 4 * n
    # accepted windows counted independently: forward windows start with P, reverse-strand
    # windows end (in forward coordinates) with rc(P) at q >= k - |P|
    seq = buf.view(n, 317)[:, 13:163]
    fwd = torch.ones((n, 150 - 5 + 1), dtype=torch.bool, device="cuda")
    rev = torch.ones_like(fwd)
    for i in range(5):
        fwd &= seq[:, i:146 + i] == prefix[i]
        rev &= seq[:, i:146 + i] == b"GTCAT"[i]
    accepted = int(fwd[:, :150 - k + 1].sum()) + int(rev[:, k - 5:].sum())
    del fwd, rev
    assert int(res.counts.sum()) == accepted
    # the reference's own output on this workload: lib/kmers.js readFile()
    # (:106-185) run unmodified on the same 3.17 GB in the build container
    # (profiles/ref_js_c2.json), and the oracle's streamed count
    # (tests/golden/fullsize.json, tests/golden/gen_fullsize.py)
    from tests.util import fullsize_golden, map_digest_arrays
    ref = {"size": 1_956_210, "sum": 2_635_074, "digest": "aadbad6b77b37001"}
    gold = fullsize_golden()["c2"]
    assert {x: gold[x] for x in ref} == ref
    assert len(res) == ref["size"] and int(res.counts.sum()) == ref["sum"]
    keys = np.frombuffer(res.keybuf, dtype=np.uint8).reshape(-1, k)
    assert map_digest_arrays(keys, res.counts) == ref["digest"]
    assert len(set(res.keys())) == len(res)
    assert all(key.startswith(prefix) for key in res.keys()[:100000])
    f = res.firsts.astype(np.uint64)
    assert bool(np.all(f[1:] > f[:-1]))
    # sharded (4 ranks' worth) + merged finish reproduces the whole result
    from kmerjs_amd.multi import device_u64, invalid_key
    per = n // 4
    keys, vals = [], []
    for r in range(4):
        ctr.reset()
        ctr.set_position(4 * per * r, 317 * per * r)
        ctr.feed_device(buf.data_ptr() + 317 * per * r, 317 * per)
        d_k, d_v, m = ctr.partial_device()
        keys.append(device_u64(d_k, m, torch.device("cuda")).clone())
        vals.append(device_u64(d_v, 2 * m, torch.device("cuda")).view(m, 2).clone())
    del buf
    gk, gv = torch.cat(keys), torch.cat(vals)
    merged = ctr.finish_merged(gk.data_ptr(), gv.data_ptr(), gk.numel(), 4 * n)
    ctr.close()
    assert merged.lines == res.lines
    assert np.array_equal(merged.counts, res.counts)
    assert np.array_equal(merged.firsts, res.firsts)
    assert merged.keybuf == res.keybuf


def test_c3_full_size_properties(native):
    """BASELINE configs[2] at its size: 100 M synthetic reads (31.7 GB, seed 3),
    k = 31, no prefix, table mode (lib/kmers.js:88-100 on both strands).
    Σ Map counts = 2 x 120 windows per read = 24,000,000,000 exactly; with odd
    k there are no palindromes and the uniform reads hold no non-ACGT byte, so
    the Map has exactly twice as many keys as the table has canonical classes;
    the table over all reads has the digest of the tables over the two halves
    added (linearity), the halves' Σ add up, and a repeat is identical."""
    import torch
    from kmerjs_amd import synth_fastq_device
    n, k = 100_000_000, 31
    buf = torch.empty(n * 317, dtype=torch.uint8, device="cuda")
    synth_fastq_device(buf.data_ptr(), 3, 0, n)
    torch.cuda.synchronize()
    ctr = native.Counter(k=k, prefix=b"", flags=native.FLAG_UNORDERED)
    try:
        parts = []
        half = n // 2
        for lo in (0, half):
            ctr.reset()
            ctr.set_position(4 * lo, 317 * lo)
            ctr.feed_device(buf.data_ptr() + 317 * lo, 317 * half)
            ctr.finish(want_result=False)
            parts.append((ctr.table_stats(), ctr.table_digest()))
        ctr.reset()
        ctr.feed_device(buf.data_ptr(), buf.numel())
        ctr.finish(want_result=False)
        assert ctr.lines() == 4 * n
        canon, keys, total = ctr.table_stats()
        d = ctr.table_digest()
        assert ctr.table_routes()["p2_fixed"] == 1          # (pass 2 without its histogram pass)
        assert total == 2 * 120 * n == 24_000_000_000
        assert keys == 2 * canon
        # the oracle's table digest of the same 100 M reads (a streamed sum
        # over forward windows, tests/golden/gen_fullsize.py)
        from tests.util import fullsize_golden
        gold = fullsize_golden()["c3"]
        assert gold["forward_windows"] == total // 2
        assert d == gold["table_digest"]
        assert 11_900_000_000 < canon <= 12_000_000_000
        assert total == parts[0][0][2] + parts[1][0][2]
        assert canon <= parts[0][0][0] + parts[1][0][0]
        assert d == (parts[0][1] + parts[1][1]) % (1 << 64)
        ctr.reset()
        ctr.feed_device(buf.data_ptr(), buf.numel())
        ctr.finish(want_result=False)
        assert ctr.table_stats() == (canon, keys, total) and ctr.table_digest() == d
    finally:
        ctr.close()
        del buf


def test_c3_exchange_digests_add_up(native):
    """Table mode across 2 ranks' worth of contexts at 20 M reads (k = 31): the
    owners' exchanged tables (kmer_table_exchange_prepare / _finish_exchanged)
    have digests and statistics that add up to the one-context table's."""
    import torch
    from kmerjs_amd import synth_fastq_device
    from kmerjs_amd.multi import device_u64
    n, k, world = 20_000_000, 31, 2
    buf = torch.empty(n * 317, dtype=torch.uint8, device="cuda")
    synth_fastq_device(buf.data_ptr(), 3, 0, n)
    torch.cuda.synchronize()
    one = native.Counter(k=k, prefix=b"", flags=native.FLAG_UNORDERED)
    one.reset()
    one.feed_device(buf.data_ptr(), buf.numel())
    one.finish(want_result=False)
    want = (one.table_stats(), one.table_digest())
    one.close()
    ctrs = [native.Counter(k=k, prefix=b"", flags=native.FLAG_UNORDERED) for _ in range(world)]
    sends = []
    for r, c in enumerate(ctrs):
        lo = n * r // world
        c.reset()
        c.set_position(4 * lo, 317 * lo)
        c.feed_device(buf.data_ptr() + 317 * lo, 317 * (n * (r + 1) // world - lo))
        d, counts, parts = c.table_exchange_prepare(world)
        sends.append((device_u64(d, sum(counts), buf.device).clone(), counts, parts))
    del buf
    parts_all = np.array([p for _, _, p in sends], dtype=np.uint64)
    recvs, stats, dig = [], np.zeros(3, dtype=np.int64), 0
    for o, c in enumerate(ctrs):
        recv = torch.cat([keys[sum(counts[:o]):sum(counts[:o]) + counts[o]] for keys, counts, _ in sends])
        recvs.append(recv)
        c.table_finish_exchanged(recv.data_ptr(), recv.numel(), parts_all, world, o,
                                 stream=torch.cuda.current_stream().cuda_stream)
        stats += np.array(c.table_stats(), dtype=np.int64)
        dig = (dig + c.table_digest()) % (1 << 64)
    for c in ctrs:
        c.close()
    assert tuple(stats.tolist()) == want[0] and dig == want[1]


def test_c4_shard_full_size_properties(native):
    # BASELINE configs[3] per-GPU shard: 125 M reads (39.6 GB, seed 4) -- the
    # 1 B-read job's share of one of 8 GPUs -- properties that need no oracle,
    # checked on the device; then the shard as 2 ranks' worth, hit exchange +
    # device-side ordered collect (kmer_merge_ordered) == the one-pass result
    import torch
    from kmerjs_amd import synth_fastq_device
    from kmerjs_amd.multi import _CudaArray, device_u64
    n, k, prefix = 125_000_000, 16, b"ATGAC"
    dev = torch.device("cuda")
    buf = torch.empty(n * 317, dtype=torch.uint8, device=dev)
    synth_fastq_device(buf.data_ptr(), 4, 0, n)
    torch.cuda.synchronize()
    ctr = native.Counter(k=k, prefix=prefix)
    ctr.reset()
    ctr.set_position(0, 0)
    ctr.feed_device(buf.data_ptr(), buf.numel())
    ctr.finish(want_result=False)
    assert ctr.lines() == 4 * n
    dk, dc, df, m = ctr.result_device()
    keys = torch.as_tensor(_CudaArray(dk, m * k, "|u1"), device=dev).view(m, k).clone()
    cnt = device_u64(dc, m, dev).clone()
    fst = device_u64(df, m, dev).clone()
    # accepted windows counted independently, 10 M reads at a time
    accepted = 0
    for lo in range(0, n, 10_000_000):
        seq = buf.view(n, 317)[lo:lo + 10_000_000, 13:163]
        fwd = torch.ones((seq.shape[0], 146), dtype=torch.bool, device=dev)
        rev = torch.ones_like(fwd)
        for i in range(5):
            fwd &= seq[:, i:146 + i] == prefix[i]
            rev &= seq[:, i:146 + i] == b"GTCAT"[i]
        accepted += int(fwd[:, :150 - k + 1].sum()) + int(rev[:, k - 5:].sum())
        del fwd, rev, seq
    assert int(cnt.sum()) == accepted
    assert m <= 4 ** 11 and bool((keys[:, :5] == torch.tensor(list(prefix), dtype=torch.uint8, device=dev)).all())
    assert bool((fst[1:] > fst[:-1]).all())
    # the oracle's Map of the same 125 M reads (streamed on 8 record-aligned
    # shards and merged by first occurrence, tests/golden/gen_fullsize.py)
    from tests.util import fullsize_golden, map_digest_arrays
    gold = fullsize_golden()["c4"]
    assert m == gold["size"] and int(cnt.sum()) == gold["sum"] and gold["lines"] == 4 * n
    assert map_digest_arrays(keys.cpu().numpy(), cnt.cpu().numpy().view(np.uint64)) == gold["digest"]
    # 2 ranks' worth on the same device: exchange by key range, per-owner finish,
    # then the owners' ordered lists merged by first occurrence on "rank 0"
    half = n // 2
    ctrs = [native.Counter(k=k, prefix=prefix) for _ in range(2)]
    runs = []
    for r, c in enumerate(ctrs):
        c.reset()
        c.set_position(4 * half * r, 317 * half * r)
        c.feed_device(buf.data_ptr() + 317 * half * r, 317 * half)
        d_x, counts = c.exchange_prepare(2)
        x = device_u64(d_x, 2 * sum(counts), dev).clone()
        runs.append((x[:2 * counts[0]], x[2 * counts[0]:]))
    del buf
    parts = []
    for o, c in enumerate(ctrs):
        recv = torch.cat([runs[0][o], runs[1][o]])
        c.finish_exchanged(recv.data_ptr(), recv.numel() // 2, 4 * n,
                           stream=torch.cuda.current_stream().cuda_stream)   # (after the cat)
        ok, oc, of, om = c.result_device()
        parts.append((torch.as_tensor(_CudaArray(ok, om * k, "|u1"), device=dev).clone(),
                      device_u64(oc, om, dev).clone(), device_u64(of, om, dev).clone()))
    del runs
    gk = torch.cat([p[0] for p in parts])
    gc = torch.cat([p[1] for p in parts])
    gf = torch.cat([p[2] for p in parts])
    torch.cuda.synchronize()
    ctrs[0].merge_ordered(gk.data_ptr(), gc.data_ptr(), gf.data_ptr(), gc.numel(), 4 * n)
    mk, mc, mf, mm = ctrs[0].result_device()
    assert mm == m
    assert torch.equal(device_u64(mc, mm, dev), cnt) and torch.equal(device_u64(mf, mm, dev), fst)
    assert torch.equal(torch.as_tensor(_CudaArray(mk, mm * k, "|u1"), device=dev).view(mm, k), keys)
    for c in ctrs + [ctr]:
        c.close()


@pytest.mark.parametrize("fasta", [False, True], ids=["single_line", "fasta60"])
def test_c5_full_size_pins(native, fasta):
    """BASELINE configs[4] at the size bench.py times: 1 GB of contigs (10 kb -
    1 Mb, bench.make_contigs seed 5 = rank 0's), k = 21, canonical table mode.
    Single-line: only lines with index % 4 == 1 count (lib/kmers.js:151);
    fasta60: 60-column records joined (KMER_FLAG_FASTA, an extension).  The
    table digest and Σ counts equal the oracle's streamed over the same bytes
    (tests/golden/fullsize.json "c5" / "c5fa"), on the route the bench takes
    (pass 1's workgroup shares merged: kmer_table_routes) and with that
    merging disabled (KMER_FLAG_TABLE_FIXED_TEST)."""
    import torch
    from bench import make_contigs
    from tests.util import fullsize_golden
    gold = fullsize_golden()["c5fa" if fasta else "c5"]
    data, _ = make_contigs(5, 1_000_000_000, 21, width=60 if fasta else 0)
    assert len(data) == gold["bytes"]
    buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    del data
    base = native.FLAG_CANONICAL | (native.FLAG_FASTA if fasta else 0)
    seen = []
    for flags in (base, base | native.FLAG_TABLE_FIXED_TEST):
        ctr = native.Counter(k=21, prefix=b"", flags=flags)
        try:
            for _ in range(2):                       # (a second finish on the reused buffers)
                ctr.reset()
                ctr.feed_device(buf.data_ptr(), buf.numel())
                ctr.finish(want_result=False)
                canon, keys, total = ctr.table_stats()
                assert total == gold["forward_windows"] and keys == canon
                assert ctr.table_digest() == gold["table_digest"]
                routes = ctr.table_routes()
                seen.append(routes)
                assert routes["fixed"] >= 1
                if flags & native.FLAG_TABLE_FIXED_TEST:
                    assert routes["merged"] == 0
                elif not fasta:
                    assert routes["merged"] == routes["fixed"] and routes["counted"] == 0, routes
                assert routes["p2_fixed"] == 1, routes   # (regions of 11 / 6 small buckets)
        finally:
            ctr.close()
    print("c5 routes", "fasta" if fasta else "single", seen)
