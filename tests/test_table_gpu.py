"""GPU parity of table mode (KMER_FLAG_UNORDERED, kmer_table.hip): the same
k-mer -> count Map as the reference (lib/kmers.js:88-100, :151-155), entries
sorted by key bytes instead of insertion order.  Checked against the goldens
(size, sum, lines; full entries where the golden holds them) and the oracle
(every entry, sorted)."""
import numpy as np
import pytest

from tests.util import first_diff

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    from kmerjs_amd import _native
    return _native


def _table_ok(c):
    p = c["prefix"]
    return c["step"] == 1 and c["k"] <= 32 and len(p) <= c["k"] and all(ch in "ACGT" for ch in p)


def _check_cases(native, golden, inputs, flags):
    from oracle import oracle
    bad = []
    by_cfg = {}
    for c in golden["cases"]:
        if _table_ok(c):
            by_cfg.setdefault((c["prefix"], c["k"]), []).append(c)
    for (p, k), cases in by_cfg.items():
        ctr = native.Counter(k=k, prefix=p.encode(), flags=native.FLAG_UNORDERED | flags)
        try:
            for c in cases:
                r = ctr.count_buffer(inputs[c["input"]])
                e = r.entries()
                ok = len(e) == c["size"] and sum(v for _, v in e) == c["sum"] and r.lines == c["lines"]
                if ok and "entries" in c:
                    ok = e == sorted((kk.encode("latin-1"), v) for kk, v in c["entries"])
                if ok and "entries" not in c:
                    ok = e == sorted(oracle.count_buffer(inputs[c["input"]], p.encode(), k, 1))
                if ok:
                    _, keys, total = ctr.table_stats()
                    ok = keys == c["size"] and total == c["sum"]
                if not ok:
                    bad.append((c["input"], p, k, len(e), c["size"], r.lines, c["lines"]))
        finally:
            ctr.close()
    return bad


def test_table_every_golden_case(native, golden, inputs):
    assert sum(_table_ok(c) for c in golden["cases"]) >= 455
    bad = _check_cases(native, golden, inputs, 0)
    assert not bad, bad[:5]


def test_table_range_splits(native, golden, inputs):
    # 64-key LDS ranges: every bucket with more keys is split (and redone)
    bad = _check_cases(native, golden, inputs, native.FLAG_TABLE_SPLIT_TEST)
    assert not bad, bad[:5]


def _device_input(n, seed=3):
    import torch
    from kmerjs_amd import synth_fastq_device
    buf = torch.empty(n * 317, dtype=torch.uint8, device="cuda")
    synth_fastq_device(buf.data_ptr(), seed, 0, n)
    torch.cuda.synchronize()
    return buf


@pytest.mark.parametrize("k,prefix", [(31, b""), (16, b""), (21, b"A"), (16, b"ATGAC"), (32, b"GT")])
def test_table_synthetic_vs_oracle(native, k, prefix):
    # every entry (keys compared as sorted 2-bit codes: byte order) vs the oracle
    from oracle import oracle
    from tests.util import packed_sorted, result_packed_sorted, same_packed
    buf = _device_input(30_000)
    host = buf.cpu().numpy().tobytes()
    keys_o, cnt_o = oracle.count_arrays(host, prefix, k)
    want = packed_sorted(keys_o, cnt_o)
    ctr = native.Counter(k=k, prefix=prefix, flags=native.FLAG_UNORDERED)
    ctr.reset()
    ctr.feed_device(buf.data_ptr(), len(host))
    res = ctr.finish()
    canon, keys, total = ctr.table_stats()
    with pytest.raises(native.KmerError):          # no ordered device result in table mode
        ctr.result_device()
    ctr.close()
    assert len(res) == len(cnt_o)
    assert same_packed(result_packed_sorted(res, k), want)
    assert keys == len(cnt_o) and total == int(cnt_o.sum())
    if len(res):                                   # the host result is in key byte order
        kb = np.frombuffer(res.keybuf, dtype=np.uint8).reshape(-1, k)
        assert bytes(kb[0]) <= bytes(kb[len(kb) // 2]) <= bytes(kb[-1])


@pytest.mark.parametrize("read_len", [3, 9, 30, 150])
def test_line_split_short_and_long_lines(native, read_len):
    # the one-pass line split keeps 1,024 newline positions per 16 KiB tile:
    # reads of 3 and 9 bases (lines of ~4-7 bytes) overflow it and take the
    # two-pass route, 30 and 150 do not; every route must give the oracle's
    # Map (ordered dense-hit path and table mode), mixed lengths included
    from oracle import oracle
    rng = np.random.default_rng(read_len)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    recs = []
    for i in range(12000):
        L = read_len if i % 5 else 150
        s = acgt[rng.integers(0, 4, L)].tobytes()
        recs.append(b"@r%d\n%s\n+\n%s\n" % (i, s, b"I" * L))
    data = b"".join(recs)
    for k, prefix in ((3, b""), (16, b""), (12, b"A")):
        want = oracle.count_buffer(data, prefix, k, 1)
        ctr = native.Counter(k=k, prefix=prefix)
        got = ctr.count_buffer(data).entries()
        ctr.close()
        assert got == want, (k, prefix)
        ctr = native.Counter(k=k, prefix=prefix, flags=native.FLAG_UNORDERED)
        e = ctr.count_buffer(data).entries()
        ctr.close()
        assert e == sorted(want), (k, prefix, "table")


def test_table_chunked_feeds_match_one_feed(native):
    import torch
    buf = _device_input(60_000, seed=9)
    n = buf.numel()
    ctr = native.Counter(k=31, prefix=b"", flags=native.FLAG_UNORDERED)
    ctr.reset()
    ctr.feed_device(buf.data_ptr(), n)
    ctr.finish(want_result=False)
    d1, s1 = ctr.table_digest(), ctr.table_stats()
    ctr.reset()
    cuts = [0, 317 * 7, 317 * 20_000, 317 * 20_001, 317 * 45_000, n]
    for lo, hi in zip(cuts, cuts[1:]):
        ctr.feed_device(buf.data_ptr() + lo, hi - lo)
    torch.cuda.synchronize()
    ctr.finish(want_result=False)
    assert ctr.table_digest() == d1 and ctr.table_stats() == s1
    # (entry by entry at a smaller size)
    small = buf[:317 * 8000].cpu().numpy().tobytes()
    one = ctr.count_buffer(small)
    ctr.reset()
    for lo, hi in ((0, 317 * 3), (317 * 3, 317 * 5000), (317 * 5000, len(small))):
        ctr.feed_device(buf.data_ptr() + lo, hi - lo)
    many = ctr.finish()
    ctr.close()
    assert many.keybuf == one.keybuf and np.array_equal(many.counts, one.counts)


def test_table_realistic_reads_with_n(native):
    from oracle import oracle
    rng = np.random.default_rng(12)
    arr = np.frombuffer(bytearray(oracle.synth_fastq(4, 0, 20000)), dtype=np.uint8).reshape(-1, 317).copy()
    seq = arr[:, 13:163]
    seq[rng.random(seq.shape) < 0.002] = ord("N")
    seq[rng.random(len(seq)) < 0.8, 0] = ord("N")
    arr[:, 13:163] = seq
    data = arr.tobytes()
    from tests.util import packed_sorted, result_packed_sorted, same_packed
    for k, p in ((16, b""), (31, b""), (21, b"GT")):
        want = packed_sorted(*oracle.count_arrays(data, p, k))
        assert len(want[2]) > 100                   # record keys (windows with N)
        ctr = native.Counter(k=k, prefix=p, flags=native.FLAG_UNORDERED)
        got = result_packed_sorted(ctr.count_buffer(data), k)
        ctr.close()
        assert same_packed(got, want), (k, p)


def test_table_big_counts(native):
    # one canonical k-mer seen > 2^20 times (count beyond the entry's 20-bit
    # field -> big list), plus palindromes (even k: AT-repeats)
    from oracle import oracle
    polya = b"".join(b"@r%010d\n%s\n+\n%s\n" % (i, b"A" * 150, b"I" * 150) for i in range(9000))
    at = b"".join(b"@s%010d\n%s\n+\n%s\n" % (i, b"AT" * 75, b"I" * 150) for i in range(300))
    data = polya + at
    for k, p in ((16, b""), (16, b"A"), (15, b"T"), (15, b"")):
        want = sorted(oracle.count_buffer(data, p, k, 1))
        ctr = native.Counter(k=k, prefix=p, flags=native.FLAG_UNORDERED)
        got = ctr.count_buffer(data).entries()
        ctr.close()
        assert got == want, (k, p, got[:4], want[:4])
    assert dict(want).get(b"A" * 15) == 9000 * 136


@pytest.mark.parametrize("k", [16, 31])
def test_table_fixed_runs_spill(native, k):
    # no prefix: pass 1 writes fixed per-workgroup runs (tab_scatter1f); keys
    # past a run go to their partition's spill area; a poly-A read every 8th
    # record crowds one partition far past its runs and its spill area, so the
    # chunk is redone with the counting pass, and a second feed of poly-A alone
    # does the same -- every route must give the oracle's Map
    from oracle import oracle
    from tests.util import packed_sorted, result_packed_sorted, same_packed
    arr = np.frombuffer(bytearray(oracle.synth_fastq(21, 0, 24000)), dtype=np.uint8).reshape(-1, 317).copy()
    arr[::8, 13:163] = ord("A")
    mixed = arr.tobytes()
    polya = b"".join(b"@p%010d\n%s\n+\n%s\n" % (i, b"A" * 150, b"I" * 150) for i in range(9000))
    data = mixed + polya
    want = packed_sorted(*oracle.count_arrays(data, b"", k))
    # (small shares: the fixed runs are forced, FLAG_TABLE_FIXED_TEST)
    ctr = native.Counter(k=k, prefix=b"", flags=native.FLAG_UNORDERED | native.FLAG_TABLE_FIXED_TEST)
    got = result_packed_sorted(ctr.count_buffer(mixed), k)
    assert same_packed(got, packed_sorted(*oracle.count_arrays(mixed, b"", k)))
    import torch
    dev = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    ctr.reset()
    ctr.feed_device(dev.data_ptr(), len(mixed))
    ctr.feed_device(dev.data_ptr() + len(mixed), len(polya))
    torch.cuda.synchronize()
    got = result_packed_sorted(ctr.finish(), k)
    canon, keys, total = ctr.table_stats()
    ctr.close()
    assert same_packed(got, want)
    assert total == int(want[1].sum()) + sum(want[2].values())


def test_table_matches_ordered_path_at_scale(native):
    # 2 M reads, k = 31, no prefix (C3's configuration): the table's Map keys
    # and counts equal the ordered dense path's result (960 windows per 2 reads)
    buf = _device_input(2_000_000, seed=3)
    ctr = native.Counter(k=31, prefix=b"", flags=native.FLAG_UNORDERED)
    ctr.reset()
    ctr.feed_device(buf.data_ptr(), buf.numel())
    ctr.finish(want_result=False)
    canon, keys, total = ctr.table_stats()
    ctr.close()
    assert total == 2_000_000 * 2 * 120
    assert keys == 2 * canon            # odd k: no palindromes
    ordered = native.Counter(k=31, prefix=b"")
    ordered.reset()
    ordered.feed_device(buf.data_ptr(), buf.numel())
    ordered.finish(want_result=False)
    _, d_counts, _, n = ordered.result_device()
    from kmerjs_amd.multi import device_u64
    ordered_sum = int(device_u64(d_counts, n, buf.device).sum().item())
    ordered.close()
    assert n == keys and ordered_sum == total


def _canonical_from_map(entries):
    """Canonical counts derived from the reference Map (App. A.6: Map(x) =
    fwd(x) + fwd(rc x)): class {x, rc x} under min(x, rc x) counts its forward
    windows = Map(c), or Map(c) / 2 for a self-complementary c."""
    from oracle import oracle
    m = dict(entries)
    out = []
    for key, v in m.items():
        rc = oracle.complement(key)
        if key <= rc:
            out.append((key, v // 2 if key == rc else v))
    return sorted(out)


@pytest.mark.parametrize("k,prefix,fixed", [(21, b"", False), (16, b"A", False), (31, b"", False), (12, b"GT", False),
                                            (21, b"", True), (31, b"", True)])
def test_canonical_mode_vs_oracle(native, golden, inputs, k, prefix, fixed):
    # KMER_FLAG_CANONICAL (BASELINE C5's "canonical k-mers"): one key per
    # {x, rc x} class, counted once per forward window; `fixed`: pass 1 with
    # fixed runs and filler slots forced (FLAG_TABLE_FIXED_TEST)
    from oracle import oracle
    rng = np.random.default_rng(k)
    arr = np.frombuffer(bytearray(oracle.synth_fastq(6, 0, 6000)), dtype=np.uint8).reshape(-1, 317).copy()
    seq = arr[:, 13:163]
    seq[rng.random(seq.shape) < 0.002] = ord("N")
    arr[:, 13:163] = seq
    datas = [arr.tobytes(), inputs["test_kmers.fastq"], inputs["test_long.kmer.fastq"], inputs["edge_contigs.fsa"]]
    ctr = native.Counter(k=k, prefix=prefix, flags=native.FLAG_CANONICAL | (native.FLAG_TABLE_FIXED_TEST if fixed else 0))
    for data in datas:
        want = _canonical_from_map(oracle.count_buffer(data, prefix, k, 1))
        got = ctr.count_buffer(data).entries()
        assert first_diff(got, want) is None, (k, prefix)
        _, keys, total = ctr.table_stats()
        assert keys == len(want) and total == sum(v for _, v in want)
    ctr.close()
    with pytest.raises(native.KmerError):          # canonical counts need a table-mode configuration
        native.Counter(k=16, prefix=b"N", flags=native.FLAG_CANONICAL)


@pytest.mark.parametrize("k,flags_name", [(31, "FLAG_UNORDERED"), (16, "FLAG_UNORDERED"), (21, "FLAG_CANONICAL")])
def test_table_digest_matches_oracle(native, k, flags_name):
    """kmer_table_digest (the linear checksum the full-size tests rely on)
    equals the digest of the oracle's Map at a size the oracle covers; reads
    with N (record keys are outside the digest) and even k (palindromes)."""
    from oracle import oracle
    from tests.util import canonical_summary
    rng = np.random.default_rng(k)
    arr = np.frombuffer(bytearray(oracle.synth_fastq(8, 0, 12000)), dtype=np.uint8).reshape(-1, 317).copy()
    seq = arr[:, 13:163]
    seq[rng.random(seq.shape) < 0.001] = ord("N")
    arr[:, 13:163] = seq
    data = arr.tobytes()
    keys, cnt = oracle.count_arrays(data, b"", k)
    acgt = ~(keys == ord("N")).any(axis=1)
    classes, fwd, dig = canonical_summary(keys[acgt], cnt[acgt], k)
    ctr = native.Counter(k=k, prefix=b"", flags=getattr(native, flags_name))
    ctr.count_buffer(data)
    assert ctr.table_digest() == dig
    assert ctr.table_stats()[0] == classes
    ctr.close()


def test_c5_contigs_canonical_vs_oracle(native):
    """BASELINE configs[4]'s shape at a size the oracle covers: single-line
    FASTA contigs of 10 kb - 1 Mb (bench.make_contigs, seed 5; only lines with
    index % 4 == 1 count, lib/kmers.js:151), k = 21, canonical k-mers on a
    device-resident feed: classes, Σ counts and the table digest equal those
    derived from the oracle's Map, and a sample of entries matches."""
    import torch
    from bench import make_contigs
    from oracle import oracle
    from tests.util import canonical_summary
    k = 21
    data, lens = make_contigs(5, 3_000_000, k)
    assert max(lens) > 100_000
    keys, cnt = oracle.count_arrays(data, b"", k)
    classes, fwd, dig = canonical_summary(keys, cnt, k)
    assert fwd == sum(L - k + 1 for i, L in enumerate(lens) if i % 4 == 1 and L >= k)
    buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    ctr = native.Counter(k=k, prefix=b"", flags=native.FLAG_CANONICAL)
    ctr.reset()
    ctr.feed_device(buf.data_ptr(), buf.numel())
    res = ctr.finish()
    assert ctr.table_stats() == (classes, classes, fwd)
    assert ctr.table_digest() == dig and len(res) == classes
    got = dict(res.entries())
    for i in range(0, len(cnt), 1009):
        kk = keys[i].tobytes()
        rc = oracle.complement(kk)
        c = min(kk, rc)
        assert got[c] == (int(cnt[i]) // 2 if kk == rc else int(cnt[i]))
    ctr.close()


@pytest.mark.parametrize("devs", [[0, 0], [0, 0, 0]])
def test_table_group_through_the_c_abi(native, inputs, devs, tmp_path):
    """kmer_params.ndev in table and canonical mode (BASELINE C3 / C5 on several
    GPUs through the reference's entry point, lib/kmers.js:106): the input
    streams in batches dealt round robin over the group (an ordinal repeated on
    a one-GPU box), pass-1 keys go to the child owning their hash-space slice,
    every child builds its slice -- the host result, the statistics and the
    table digest equal the one-context table's; through kmer_count_buffer and
    through kmer_count_file in small batches, plain and gzip."""
    import gzip
    from oracle import oracle
    rng = np.random.default_rng(len(devs))
    arr = np.frombuffer(bytearray(oracle.synth_fastq(12, 0, 6000)), dtype=np.uint8).reshape(-1, 317).copy()
    seq = arr[:, 13:163]
    seq[rng.random(seq.shape) < 0.001] = ord("N")
    arr[:, 13:163] = seq
    datas = [arr.tobytes(), inputs["test_long.kmer.fastq"], inputs["edge_contigs.fsa"], inputs["edge_blank.fastq"]]
    fx = native.FLAG_TABLE_FIXED_TEST           # (fixed runs with filler slots through the group's key exchange)
    for flags, k, p in ((native.FLAG_UNORDERED, 31, b""), (native.FLAG_CANONICAL, 21, b""),
                        (native.FLAG_UNORDERED, 16, b"AC"), (native.FLAG_UNORDERED | fx, 31, b""),
                        (native.FLAG_CANONICAL | fx, 21, b"")):
        one = native.Counter(k=k, prefix=p, flags=flags)
        grp = native.Counter(k=k, prefix=p, flags=flags, devices=devs)
        small = native.Counter(k=k, prefix=p, flags=flags, devices=devs, batch_bytes=1 << 16)
        for di, data in enumerate(datas):
            want = one.count_buffer(data)
            ws, wd = one.table_stats(), one.table_digest()
            got = grp.count_buffer(data)
            assert got.entries() == want.entries() and got.lines == want.lines, (flags, k, di)
            assert grp.table_stats() == ws and grp.table_digest() == wd
            f = tmp_path / ("in%d.fastq" % di)
            f.write_bytes(data)
            fz = tmp_path / ("in%d.fastq.gz" % di)
            fz.write_bytes(gzip.compress(data))
            for path in (f, fz):
                got = small.count_file(str(path))
                assert got.entries() == want.entries() and got.lines == want.lines, (flags, k, di, str(path))
                assert small.table_stats() == ws and small.table_digest() == wd
        for c in (one, grp, small):
            c.close()


def test_ordered_group_streams_small_batches(native, inputs, tmp_path):
    """An ordered group count of a file in 64 KiB batches dealt round robin
    over 3 children (positions from a running newline count) equals the
    oracle's Map, order included; a trailing line without '\n' too."""
    from oracle import oracle
    data = oracle.synth_fastq(13, 0, 8000) + inputs["test_kmers.fastq"] + b"@x\nACGTACGTACGTACGTACGTAAA"
    f = tmp_path / "s.fastq"
    f.write_bytes(data)
    for k, p in ((16, b"ATGAC"), (21, b"")):
        want = oracle.count_buffer(data, p, k, 1)
        ctr = native.Counter(k=k, prefix=p, devices=[0, 0, 0], batch_bytes=1 << 16)
        r = ctr.count_file(str(f))
        assert first_diff(r.entries(), want) is None and r.lines == data.count(b"\n") + 1
        r = ctr.count_buffer(data)
        assert first_diff(r.entries(), want) is None
        ctr.close()


def _table_dump(native, ctr):
    """The device table as sorted (h, count) arrays (kmer_table_device layout)."""
    import torch
    from kmerjs_amd.multi import _CudaArray, device_u64
    nq = 1 << 20
    e, st, ln, bg, nb = ctr.table_device()
    if not e:
        return np.zeros(0, np.uint64), np.zeros(0, np.uint64)
    dev = torch.device("cuda", torch.cuda.current_device())
    start = device_u64(st, nq + 1, dev).cpu().numpy().view(np.uint64)
    lens = torch.as_tensor(_CudaArray(ln, nq, "<i4"), device=dev).cpu().numpy().astype(np.int64)
    tot = int(lens.sum())
    ent = device_u64(e, int(start[-1]), dev).cpu().numpy().view(np.uint64)
    q = np.repeat(np.arange(nq, dtype=np.uint64), lens)
    first = np.cumsum(lens) - lens
    idx = np.repeat(start[:-1].astype(np.int64), lens) + (np.arange(tot) - np.repeat(first, lens))
    x = ent[idx]
    h = (q << np.uint64(44)) | (x >> np.uint64(20))
    cnt = x & np.uint64(0xFFFFF)
    if nb:
        big = device_u64(bg, 2 * nb, dev).cpu().numpy().view(np.uint64).reshape(-1, 2)
        bigmap = dict(zip(big[:, 0].tolist(), big[:, 1].tolist()))
        for i in np.nonzero(cnt == np.uint64(0xFFFFF))[0]:
            cnt[i] = bigmap[int(h[i])]
    o = np.argsort(h)
    return h[o], cnt[o]


@pytest.mark.parametrize("world,k,flags_name,with_n,fixed", [
    (2, 31, "FLAG_UNORDERED", False, False), (3, 21, "FLAG_CANONICAL", True, False),
    (1, 16, "FLAG_UNORDERED", True, False), (2, 31, "FLAG_UNORDERED", False, True),
    (3, 21, "FLAG_CANONICAL", True, True), (2, 31, "FLAG_UNORDERED", "polya", True)])
def test_table_exchange_matches_one_table(native, world, k, flags_name, with_n, fixed):
    """Multi-GPU table mode in one process: `world` contexts count record-aligned
    shards, their pass-1 keys are exchanged by owning partition range
    (kmer_table_exchange_prepare / _finish_exchanged, the all-to-all done with
    device copies), and the union of the owners' tables equals the one-context
    table entry for entry; the ranks' statistics add up to its statistics.
    `fixed`: the ranks' pass 1 writes fixed runs (FLAG_TABLE_FIXED_TEST), so
    filler slots, the chunks' alignment gaps and (poly-A reads crowding one
    partition) spill chunks travel through the segment-copy exchange."""
    import torch
    from kmerjs_amd import multi
    from oracle import oracle
    flags = getattr(native, flags_name)
    n_reads = 150_000
    if with_n:
        rng = np.random.default_rng(k)
        arr = np.frombuffer(bytearray(oracle.synth_fastq(5, 0, n_reads)), dtype=np.uint8).reshape(-1, 317).copy()
        seq = arr[:, 13:163]
        if with_n == "polya":
            seq[::16] = ord("A")          # (~560 K copies per rank: spill chunks, no list overflow)
        else:
            seq[rng.random(seq.shape) < 0.001] = ord("N")
        arr[:, 13:163] = seq
        buf = torch.from_numpy(arr.reshape(-1)).cuda()
    else:
        buf = _device_input(n_reads, seed=5)
    one = native.Counter(k=k, prefix=b"", flags=flags)
    one.reset()
    one.feed_device(buf.data_ptr(), buf.numel())
    one.finish(want_result=False)
    want_h, want_c = _table_dump(native, one)
    want_stats = one.table_stats()
    one.close()
    cuts = [317 * (n_reads * r // world) for r in range(world + 1)]
    ctrs = [native.Counter(k=k, prefix=b"", flags=flags | (native.FLAG_TABLE_FIXED_TEST if fixed else 0))
            for _ in range(world)]
    sends = []
    for r, c in enumerate(ctrs):
        c.reset()
        lo, hi = cuts[r], cuts[r + 1]
        if r == 0:                                    # two chunks: the segment-copy path
            mid = lo + 317 * ((hi - lo) // 634)
            c.feed_device(buf.data_ptr() + lo, mid - lo)
            c.feed_device(buf.data_ptr() + mid, hi - mid)
        else:
            c.feed_device(buf.data_ptr() + lo, hi - lo)
        d, counts, parts = c.table_exchange_prepare(world)
        assert sum(counts) == sum(parts)
        from kmerjs_amd.multi import device_u64
        keys = device_u64(d, sum(counts), buf.device).clone() if sum(counts) else torch.empty(0, dtype=torch.int64,
                                                                                           device=buf.device)
        sends.append((keys, counts, parts))
    parts_all = np.array([p for _, _, p in sends], dtype=np.uint64)
    # records (non-ACGT windows) move to rank 0, as multi.gather_records does
    for c in ctrs[1:]:
        kb, off, cnt, fst = c.records_export()
        ctrs[0].records_import(kb, off, cnt, fst)
        c.records_clear()
    recvs = []
    for o, c in enumerate(ctrs):
        runs = []
        for keys, counts, _ in sends:
            a = sum(counts[:o])
            runs.append(keys[a:a + counts[o]])
        recv = torch.cat(runs) if runs else torch.empty(0, dtype=torch.int64, device=buf.device)
        recvs.append(recv)
        c.table_finish_exchanged(recv.data_ptr() if recv.numel() else 0, recv.numel(), parts_all, world, o,
                                 stream=torch.cuda.current_stream().cuda_stream)
    hs, cs, stats = [], [], np.zeros(3, dtype=np.int64)
    for o, c in enumerate(ctrs):
        h, cnt = _table_dump(native, c)
        lo, hi = multi.table_part_range(o, world)
        assert ((h >> np.uint64(54)) >= lo).all() and ((h >> np.uint64(54)) < hi).all()
        hs.append(h)
        cs.append(cnt)
        stats += np.array(c.table_stats(), dtype=np.int64)
    h = np.concatenate(hs)
    cnt = np.concatenate(cs)
    o = np.argsort(h)
    assert np.array_equal(h[o], want_h) and np.array_equal(cnt[o], want_c)
    assert tuple(stats.tolist()) == want_stats
    for c in ctrs:
        c.close()
    del recvs


@pytest.mark.parametrize("n,k", [(20_000_000, 31), (3_000_000, 31), (3_000_000, 21)])
def test_table_fixed_pass2_vs_oracle(native, n, k):
    """Pass 2 without its histogram pass (tab_scatter2f, kmer_table_routes
    p2_fixed): at 20 M reads and k = 31 the buckets average 2,289 keys (>= 2,048),
    so each gets a fixed capacity region; at 3 M reads (343 keys) 16
    consecutive buckets share one (the sort final splits a region by bucket);
    k = 21: narrow keys (tab_mix_n, 32-bit keys in B2), 31 buckets per region
    (C5's case).  The table digest and Σ counts equal the oracle's streamed
    over the same reads (lib/kmers.js:88-100 on both strands).  Then 100
    copies of one read appended: its k-mers' bins hold > 64 keys, so their
    regions go to the general final (still p2_fixed); then 300 K copies: each
    of its k-mers' regions far past its capacity -> ERR_TAB_CAP -> the counted
    route redoes pass 2 (p2_fixed 0).  The digests are the sums of the parts
    (linearity)."""
    import torch
    from oracle import oracle
    buf = _device_input(n, seed=13)
    want_d, want_w = oracle.table_digest_synth(13, 0, n, k, 16)
    ctr = native.Counter(k=k, prefix=b"", flags=native.FLAG_UNORDERED)
    try:
        ctr.reset()
        ctr.feed_device(buf.data_ptr(), buf.numel())
        ctr.finish(want_result=False)
        assert ctr.table_routes()["p2_fixed"] == 1
        canon, keys, total = ctr.table_stats()
        assert total == 2 * want_w and ctr.table_digest() == want_d
        rec = buf[:317].clone()
        one_d, one_w = oracle.table_digest(bytes(rec.cpu().numpy()), k)
        for reps, fixed in ((100, 1), (300_000, 0)):
            buf2 = torch.cat([buf, rec.repeat(reps)])
            ctr.reset()
            ctr.feed_device(buf2.data_ptr(), buf2.numel())
            ctr.finish(want_result=False)
            del buf2
            assert ctr.table_routes()["p2_fixed"] == fixed, reps
            assert ctr.table_stats()[2] == 2 * (want_w + reps * one_w)
            assert ctr.table_digest() == (want_d + reps * one_d) % (1 << 64)
    finally:
        ctr.close()
