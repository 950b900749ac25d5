"""GPU parity: the HIP path (through the C-ABI) against the reference goldens
and the oracle, bit-exact (ordered keys + counts + line count)."""
import collections

import numpy as np
import pytest

from tests.util import digest, first_diff

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    from kmerjs_amd import _native
    return _native


def _run_cases(native, golden, inputs, flags=0, batch_bytes=0, select=None):
    by_cfg = collections.defaultdict(list)
    for c in golden["cases"]:
        if select is None or select(c):
            by_cfg[(c["prefix"], c["k"], c["step"])].append(c)
    bad = []
    for (p, k, step), cases in by_cfg.items():
        ctr = native.Counter(k=k, prefix=p.encode(), step=step, flags=flags, batch_bytes=batch_bytes)
        try:
            for c in cases:
                r = ctr.count_buffer(inputs[c["input"]])
                e = r.entries()
                if digest(e) != c["digest"] or r.lines != c["lines"]:
                    exp = [(kk.encode("latin-1"), v) for kk, v in c.get("entries", c.get("head", []))]
                    bad.append((c["input"], p, k, step, len(e), c["size"], r.lines, c["lines"],
                                first_diff(e[:len(exp)], exp)))
        finally:
            ctr.close()
    return bad


def test_c1_count_file_pins_reference_digest(native):
    """BASELINE configs[0] through the C-ABI (kmer_count_file): test_short.fastq,
    'ATGAC', k = 16 -> the reference's ordered Map (SURVEY.md App. C digest
    14056308710d569d; first-key KAT of test/kmers.js:12-19), 40 lines."""
    import os
    from tests.conftest import GOLDEN_DIR
    ctr = native.Counter(k=16, prefix=b"ATGAC")
    r = ctr.count_file(os.path.join(GOLDEN_DIR, "inputs", "test_short.fastq"))
    ctr.close()
    assert digest(r.entries()).startswith("14056308710d569d") and r.lines == 40
    assert r.entries() == [(b"ATGACGCAATACTCCT", 1), (b"ATGACCTGAGAGCCTT", 1)]


def test_every_golden_case(native, golden, inputs):
    bad = _run_cases(native, golden, inputs)
    assert not bad, bad[:5]


def test_two_pass_mode_matches(native, golden, inputs):
    bad = _run_cases(native, golden, inputs, flags=native.FLAG_TWO_PASS,
                     select=lambda c: c["step"] == 1 and c["k"] in (16, 31))
    assert not bad, bad[:5]


def test_long_line_mode_matches(native, golden, inputs):
    # long-line order keys (40-bit position field) must not change any result
    assert not _run_cases(native, golden, inputs, flags=native.FLAG_LONG_LINES)


def test_record_path_matches(native, golden, inputs):
    bad = _run_cases(native, golden, inputs, flags=native.FLAG_NO_DENSE,
                     select=lambda c: c["prefix"] == "ATGAC" and c["step"] == 1)
    assert not bad, bad[:5]


def test_byte_scan_kernel_matches(native, golden, inputs):
    # the byte-SWAR scan kernel (used for non-ACGT prefixes) on ACGT prefixes too
    bad = _run_cases(native, golden, inputs, flags=native.FLAG_BYTE_SCAN,
                     select=lambda c: c["step"] == 1 and c["prefix"] in ("ATGAC", "A", "GTCAT", "AT"))
    assert not bad, bad[:5]


def test_sort_finish_matches(native, golden, inputs):
    # the radix-sort finish (used for keys wider than 24 bits) on narrow keys too
    bad = _run_cases(native, golden, inputs, flags=native.FLAG_SORT_FINISH,
                     select=lambda c: c["step"] == 1 and c["k"] <= 16)
    assert not bad, bad[:5]


def test_chunks_must_end_at_line_ends(native):
    import torch
    data = b"@r\nACGTATGACGGGTTTACGATGACA\n+\nIIIIIIIIIIIIIIIIIIIIIIII\n"
    t = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    ctr = native.Counter(k=8, prefix=b"ATGAC")
    ctr.reset()
    ctr.feed_device(t.data_ptr(), 10)            # ends inside the sequence line
    torch.cuda.synchronize()
    with pytest.raises(native.KmerError):
        ctr.feed_device(t.data_ptr() + 10, len(data) - 10)
    ctr.reset()
    ctr.feed_device(t.data_ptr(), len(data))
    from oracle import oracle
    assert ctr.finish().entries() == oracle.count_buffer(data, b"ATGAC", 8, 1)
    ctr.close()


def test_small_batches_chain_lines(native, golden, inputs):
    # 4 KiB batches: many chunks per input, lines carried across chunk boundaries
    bad = _run_cases(native, golden, inputs, batch_bytes=4096,
                     select=lambda c: c["input"] in ("edge_longline.fastq", "edge_ragged.fastq",
                                                    "test_long.kmer.fastq", "edge_crlf.fastq")
                     and c["step"] == 1)
    assert not bad, bad[:5]


def test_count_file_and_missing_file(native, tmp_path, inputs):
    p = tmp_path / "s.fastq"
    p.write_bytes(inputs["test_short.fastq"])
    ctr = native.Counter()
    r = ctr.count_file(str(p))
    assert r.entries() == [(b"ATGACGCAATACTCCT", 1), (b"ATGACCTGAGAGCCTT", 1)] and r.lines == 40
    with pytest.raises(native.KmerError) as ei:
        ctr.count_file(str(tmp_path / "missing.fastq"))
    assert ei.value.status == 1
    ctr.close()


def test_count_file_reads_ahead_with_progress(native, tmp_path, inputs, golden):
    """kmer_count_file reads the file ahead in batches (FileBatches) and calls
    kmer_params.progress after each (lib/kmers.js:108-110's progress-stream):
    monotone byte counts ending at the file size; results equal the one-batch
    count, for plain and gzip files and a line longer than a batch."""
    import gzip
    from oracle import oracle
    data = inputs["test_long.kmer.fastq"] + b"@long\n" + b"ACGT" * 50_000 + b"\n+\n" + b"I" * 200_000 + b"\n"
    want = oracle.count_buffer(data, b"AC", 16, 1)
    f = tmp_path / "a.fastq"
    f.write_bytes(data)
    fz = tmp_path / "a.fastq.gz"
    fz.write_bytes(gzip.compress(data))
    for path, size in ((f, len(data)), (fz, fz.stat().st_size)):
        seen = []
        ctr = native.Counter(k=16, prefix=b"AC", batch_bytes=1 << 16, progress=lambda d, t: seen.append((d, t)))
        r = ctr.count_file(str(path))
        ctr.close()
        assert r.entries() == want
        assert len(seen) >= 3 and seen[-1] == (size, size), (str(path), seen[-3:])
        assert all(b[0] >= a[0] for a, b in zip(seen, seen[1:]))
    seen = []
    ctr = native.Counter(k=16, prefix=b"AC", batch_bytes=1 << 16, progress=lambda d, t: seen.append((d, t)))
    assert ctr.count_buffer(data).entries() == want
    ctr.close()
    assert len(seen) >= 3 and seen[-1] == (len(data), len(data))


def test_non_ascii_rejected(native):
    ctr = native.Counter()
    with pytest.raises(native.KmerError) as ei:
        ctr.count_buffer(b"@a\nATGAC\xc3\xa9GTCAT\n+\nII\n")
    assert ei.value.status == 6
    ctr.close()


def test_max_keys_mirrors_map_cap(native, inputs):
    ctr = native.Counter(prefix=b"", k=16, max_keys=1000)
    with pytest.raises(native.KmerError) as ei:
        ctr.count_buffer(inputs["test_short.fastq"])   # 1720 distinct keys > 1000
    assert ei.value.status == 5
    ctr.close()


def test_device_synth_matches_oracle_generator():
    import torch
    from kmerjs_amd import synth_fastq_device
    from oracle import oracle
    n = 4096
    buf = torch.empty(n * 317, dtype=torch.uint8, device="cuda")
    synth_fastq_device(buf.data_ptr(), 5, 1_000_000, n)
    torch.cuda.synchronize()
    assert buf.cpu().numpy().tobytes() == oracle.synth_fastq(5, 1_000_000, n)


@pytest.mark.parametrize("k,prefix", [(16, b"ATGAC"), (21, b"ATGAC"), (31, b"ATGAC"), (12, b"ACG")])
def test_synthetic_vs_oracle(native, k, prefix):
    import torch
    from kmerjs_amd import synth_fastq_device
    from oracle import oracle
    n = 200_000
    buf = torch.empty(n * 317, dtype=torch.uint8, device="cuda")
    synth_fastq_device(buf.data_ptr(), 1, 0, n)
    torch.cuda.synchronize()
    host = buf.cpu().numpy().tobytes()
    want = oracle.count_buffer(host, prefix, k, 1)
    ctr = native.Counter(k=k, prefix=prefix)
    ctr.reset()
    ctr.feed_device(buf.data_ptr(), len(host))
    got = ctr.finish().entries()
    ctr.close()
    assert len(got) == len(want)
    assert first_diff(got, want) is None


def test_realistic_reads_with_n(native):
    # SURVEY.md §8d realistic variant: N with p=0.001 and N at base 0 of 80% of reads
    from oracle import oracle
    rng = np.random.default_rng(11)
    raw = bytearray(oracle.synth_fastq(2, 0, 20000))
    arr = np.frombuffer(raw, dtype=np.uint8).reshape(-1, 317).copy()
    seq = arr[:, 13:163]
    seq[rng.random(seq.shape) < 0.001] = ord("N")
    seq[rng.random(len(seq)) < 0.8, 0] = ord("N")
    arr[:, 13:163] = seq
    data = arr.tobytes()
    for k, p in ((16, b"ATGAC"), (16, b""), (21, b"GT")):
        want = oracle.count_buffer(data, p, k, 1)
        ctr = native.Counter(k=k, prefix=p)
        got = ctr.count_buffer(data).entries()
        ctr.close()
        assert first_diff(got, want) is None, (k, p)


def test_determinism_and_repeat(native, inputs):
    ctr = native.Counter(k=16, prefix=b"ATGAC")
    a = ctr.count_buffer(inputs["test_long.kmer.fastq"]).entries()
    b = ctr.count_buffer(inputs["test_long.kmer.fastq"]).entries()
    ctr.close()
    assert a == b and len(a) == 401


def _shard_and_merge(native, data, k, prefix, world, batch_bytes=0):
    """Count `data` as `world` record-aligned shards (one context each, as one
    rank each would) and merge the partials in context 0 (multi.merge_to's
    exchange, done in-process)."""
    import torch
    from kmerjs_amd.multi import device_u64, invalid_key, split_at_records
    shards = split_at_records(data, world)
    ctrs = [native.Counter(k=k, prefix=prefix, batch_bytes=batch_bytes) for _ in range(world)]
    try:
        keys, vals, recs = [], [], []
        total_lines = 0
        for ctr, (lo, hi, lines_before) in zip(ctrs, shards):
            ctr.reset()
            ctr.set_position(lines_before, lo)
            part = data[lo:hi]
            if part:
                t = torch.frombuffer(bytearray(part), dtype=torch.uint8).cuda()
                ctr.feed_device(t.data_ptr(), len(part))
                torch.cuda.synchronize()
            total_lines = max(total_lines, ctr.lines())
            d_k, d_v, n = ctr.partial_device()
            if n:
                keys.append(device_u64(d_k, n, torch.device("cuda")).clone())
                vals.append(device_u64(d_v, 2 * n, torch.device("cuda")).view(n, 2).clone())
            recs.append(ctr.records_export())
        # pad like gather_partials does
        pad = torch.full((7,), invalid_key(k, len(prefix)), dtype=torch.int64, device="cuda")
        padv = torch.tensor([[-1, 0]] * 7, dtype=torch.int64, device="cuda")
        gk = torch.cat(keys + [pad])
        gv = torch.cat(vals + [padv])
        for r in recs[1:]:
            ctrs[0].records_import(*r)
        torch.cuda.synchronize()
        return ctrs[0].finish_merged(gk.data_ptr(), gv.data_ptr(), gk.numel(), total_lines)
    finally:
        for c in ctrs:
            c.close()


def _shard_and_exchange(native, data, k, prefix, world, device_merge=False):
    """Count `data` as `world` record-aligned shards (one context per rank) and
    finish with the hit exchange (multi.finish_exchange, done in-process): each
    owner counts the runs every rank sent it.  Returns the whole ordered Map
    (the owners' lists merged by first occurrence: on the host, or with
    device_merge by kmer_merge_ordered on rank 0 as multi.collect_ordered_device
    does after its gather) and the line count."""
    import torch
    from kmerjs_amd.multi import _CudaArray, device_u64, key_owner, split_at_records
    shards = split_at_records(data, world)
    ctrs = [native.Counter(k=k, prefix=prefix) for _ in range(world)]
    dev = torch.device("cuda")
    try:
        runs, recs, total_lines = [], [], 0
        for ctr, (lo, hi, lines_before) in zip(ctrs, shards):
            ctr.reset()
            ctr.set_position(lines_before, lo)
            part = data[lo:hi]
            if part:
                t = torch.frombuffer(bytearray(part), dtype=torch.uint8).cuda()
                ctr.feed_device(t.data_ptr(), len(part))
                torch.cuda.synchronize()
            total_lines = max(total_lines, ctr.lines())
            d_x, counts = ctr.exchange_prepare(world)
            x = device_u64(d_x, 2 * sum(counts), dev).clone() if sum(counts) else torch.empty(0, dtype=torch.int64,
                                                                                               device=dev)
            offs = np.cumsum([0] + counts)
            runs.append([x[2 * offs[o]:2 * offs[o + 1]] for o in range(world)])
            recs.append(ctr.records_export())
        for c, r in zip(ctrs[1:], recs[1:]):
            ctrs[0].records_import(*r)
            c.records_clear()                      # moved to rank 0 (multi.gather_records)
        kbits = 2 * (k - len(prefix))
        merged = []
        for o in range(world):
            recv = torch.cat([runs[src][o] for src in range(world)])
            if recv.numel():
                keys = recv.view(-1, 2)[:, 1]
                assert bool((key_owner(keys, kbits, world) == o).all())     # only this owner's key range
                fo = recv.view(-1, 2)[:, 0]
                assert bool((fo[1:] > fo[:-1]).all())                     # in first-occurrence order
            if device_merge:
                ctrs[o].finish_exchanged(recv.data_ptr(), recv.numel() // 2, total_lines)
                dk, dc, df, n = ctrs[o].result_device()
                if n:
                    kb = torch.as_tensor(_CudaArray(dk, n * k, "|u1"), device=dev).clone()
                    merged.append((kb, device_u64(dc, n, dev).clone(), device_u64(df, n, dev).clone()))
                continue
            r = ctrs[o].finish_exchanged(recv.data_ptr(), recv.numel() // 2, total_lines, want_result=True)
            merged += [(int(f), kk, c) for f, (kk, c) in zip(r.firsts.tolist(), r.entries())]
        if device_merge:
            # the owners' lists gathered to rank 0 (any order) and re-ordered there
            if merged:
                gk = torch.cat([m[0] for m in reversed(merged)])
                gc = torch.cat([m[1] for m in reversed(merged)])
                gf = torch.cat([m[2] for m in reversed(merged)])
            else:
                gk = torch.empty(0, dtype=torch.uint8, device=dev)
                gc = gf = torch.empty(0, dtype=torch.int64, device=dev)
            torch.cuda.synchronize()
            r = ctrs[0].merge_ordered(gk.data_ptr(), gc.data_ptr(), gf.data_ptr(), gc.numel(), total_lines,
                                      want_result=True)
            fs = r.firsts.tolist()
            assert all(a < b for a, b in zip(fs, fs[1:]))
            return r.entries(), r.lines
        merged.sort(key=lambda t: t[0])
        return [(kk, c) for _, kk, c in merged], total_lines
    finally:
        for c in ctrs:
            c.close()


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_hit_exchange_matches_oracle(native, world):
    # default multi-GPU finish: hits partitioned by owner, exchanged, counted per owner
    from oracle import oracle
    rng = np.random.default_rng(100 + world)
    arr = np.frombuffer(bytearray(oracle.synth_fastq(9, 0, 20000)), dtype=np.uint8).reshape(-1, 317).copy()
    seq = arr[:, 13:163]
    seq[rng.random(seq.shape) < 0.002] = ord("N")
    arr[:, 13:163] = seq
    data = arr.tobytes()
    for k, p, n in ((16, b"ATGAC", 20000), (13, b"AC", 20000), (32, b"ATGAC", 20000), (21, b"", 3000)):
        part = data[:317 * n]
        want = oracle.count_buffer(part, p, k, 1)
        got, lines = _shard_and_exchange(native, part, k, p, world)
        assert lines == 4 * n
        assert first_diff(got, want) is None, (world, k, p)
        # the device-side collect (multi.collect_ordered_device's merge)
        got, lines = _shard_and_exchange(native, part, k, p, world, device_merge=True)
        assert lines == 4 * n
        assert first_diff(got, want) is None, ("device merge", world, k, p)


@pytest.mark.parametrize("world", [2, 3, 5])
def test_sharded_merge_matches_oracle(native, world):
    # multi-GPU exchange: per-shard partials + merged finish == whole count
    from oracle import oracle
    rng = np.random.default_rng(world)
    arr = np.frombuffer(bytearray(oracle.synth_fastq(7, 0, 30000)), dtype=np.uint8).reshape(-1, 317).copy()
    seq = arr[:, 13:163]
    seq[rng.random(seq.shape) < 0.002] = ord("N")
    arr[:, 13:163] = seq
    data = arr.tobytes()
    for k, p in ((16, b"ATGAC"), (13, b"AC"), (32, b"ATGAC")):
        want = oracle.count_buffer(data, p, k, 1)
        r = _shard_and_merge(native, data, k, p, world)
        assert r.lines == 4 * 30000
        assert first_diff(r.entries(), want) is None, (world, k, p)


def test_long_lines_and_dense_hits(native):
    # lines spanning many tiles (every hit on the cross path, > one-workgroup sort)
    # and hit-dense prefixes (tiles overflowing their hit slots)
    from oracle import oracle
    rng = np.random.default_rng(5)
    recs = []
    for i, L in enumerate((300_000, 70_000, 151, 250_000)):
        seq = bytes(rng.choice(np.frombuffer(b"ACGT", dtype=np.uint8), L))
        recs.append(b"@c%d\n" % i + seq + b"\n+\n" + b"I" * L + b"\n")
    data = b"".join(recs)
    short = oracle.synth_fastq(9, 0, 3000)
    for buf, k, p in ((data, 16, b"AC"), (data, 21, b"ATGAC"), (short, 8, b"A"), (short, 12, b"AC"),
                      (data, 32, b"G")):
        want = oracle.count_buffer(buf, p, k, 1)
        ctr = native.Counter(k=k, prefix=p)
        got = ctr.count_buffer(buf).entries()
        ctr.close()
        assert len(got) == len(want), (k, p)
        assert first_diff(got, want) is None, (k, p)


@pytest.mark.parametrize("k,prefix", [(31, b""), (21, b""), (16, b"AC"), (12, b"G"), (32, b"AT")])
def test_dense_hit_path_vs_oracle(native, k, prefix):
    # empty / 1-3 base prefixes: every window ranked directly (SURVEY.md C3 shape)
    import torch
    from kmerjs_amd import synth_fastq_device
    from oracle import oracle
    n = 20_000
    buf = torch.empty(n * 317, dtype=torch.uint8, device="cuda")
    synth_fastq_device(buf.data_ptr(), 3, 0, n)
    torch.cuda.synchronize()
    host = buf.cpu().numpy().tobytes()
    want = oracle.count_buffer(host, prefix, k, 1)
    ctr = native.Counter(k=k, prefix=prefix)
    ctr.reset()
    ctr.feed_device(buf.data_ptr(), 317 * 7000)          # two record-aligned chunks
    ctr.feed_device(buf.data_ptr() + 317 * 7000, len(host) - 317 * 7000)
    got = ctr.finish().entries()
    ctr.close()
    assert len(got) == len(want)
    assert first_diff(got, want) is None


def test_gzip_input_and_result_writers(native, tmp_path, inputs, golden):
    # gzip FASTQ is read through zlib (count = that of the decompressed bytes);
    # the native writers match JSON.stringify(mapToJSON(map)) (lib/kmers.js:46-54)
    # and the npm main's text dump (lib/index.js:381-388)
    import gzip
    import json
    for name in ("test_kmers.fastq", "edge_crlf.fastq", "test_long.kmer.fastq"):
        plain = tmp_path / name
        plain.write_bytes(inputs[name])
        gz = tmp_path / (name + ".gz")
        gz.write_bytes(gzip.compress(inputs[name]))
        for p in (b"ATGAC", b""):
            ctr = native.Counter(k=16, prefix=p)
            a = ctr.count_file(str(plain), write=str(tmp_path / "a.json"), fmt=native.WRITE_JSON)
            b = ctr.count_file(str(gz), write=str(tmp_path / "b.txt"), fmt=native.WRITE_LEGACY)
            ctr.close()
            assert a.entries() == b.entries() and a.lines == b.lines
            obj = {k.decode("latin-1"): v for k, v in a.entries()}
            assert (tmp_path / "a.json").read_bytes().decode("latin-1") == \
                json.dumps(obj, separators=(",", ":"), ensure_ascii=False)
            legacy = "{\n" + "".join("%s: %d," % (k.decode("latin-1"), v) for k, v in a.entries()) + "}\n"
            assert (tmp_path / "b.txt").read_bytes().decode("latin-1") == legacy   # (keys may hold '\r')


@pytest.mark.parametrize("devs", [[0, 0], [0, 0, 0]])
def test_device_group_through_the_c_abi(native, golden, inputs, devs, tmp_path):
    # kmer_params.ndev: line-aligned shards counted on a device group (an
    # ordinal repeated on a one-GPU box), partials merged on devices[0] --
    # the same ordered Map as one device (goldens: ordered digest + lines)
    sel = lambda c: c["step"] == 1 and c["k"] in (5, 16, 31) and c["prefix"] in ("ATGAC", "", "A", "N")
    by_cfg = collections.defaultdict(list)
    for c in golden["cases"]:
        if sel(c):
            by_cfg[(c["prefix"], c["k"])].append(c)
    bad = []
    for (p, k), cases in by_cfg.items():
        ctr = native.Counter(k=k, prefix=p.encode(), devices=devs)
        try:
            for c in cases:
                r = ctr.count_buffer(inputs[c["input"]])
                if digest(r.entries()) != c["digest"] or r.lines != c["lines"]:
                    bad.append((c["input"], p, k, len(r), c["size"], r.lines, c["lines"]))
        finally:
            ctr.close()
    assert not bad, bad[:5]
    # a larger synthetic input (many tiles per shard) and a gzip file
    from oracle import oracle
    import gzip
    data = oracle.synth_fastq(7, 0, 150_000)
    want = oracle.count_buffer(data, b"ATGAC", 16, 1)
    ctr = native.Counter(k=16, prefix=b"ATGAC", devices=devs)
    assert first_diff(ctr.count_buffer(data).entries(), want) is None
    f = tmp_path / "s.fastq.gz"
    f.write_bytes(gzip.compress(data))
    assert ctr.count_file(str(f)).entries() == want
    with pytest.raises(native.KmerError):          # device-resident calls are single-device only
        ctr.reset()
    ctr.close()


def test_bucket_finish_repeated_after_table_counts(native):
    """Regression for the round-5 intermittent lost counts (DESIGN §8, round 6:
    an LDS race in bucket_scatter_kernel -- a wave rewrote a bucket's local
    start while slower waves still placed keys by it).  The failing sequences
    of the records: ordered k = 3 (one bucket) right after table-mode counts in
    the same process (gpurun_out/abtab/r8.txt: one count of CTT and the key CGT
    lost), and C2's finish shape (k = 16, ATGAC: 256 buckets); each repeated on
    the same reused buffers, every repeat exact against the oracle
    (lib/kmers.js:95: Map counts are exact)."""
    from oracle import oracle
    rng = np.random.default_rng(3)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    recs = []
    for i in range(12000):
        L = 9 if i % 5 else 150
        s = acgt[rng.integers(0, 4, L)].tobytes()
        recs.append(b"@r%d\n%s\n+\n%s\n" % (i, s, b"I" * L))
    short = b"".join(recs)
    reads = oracle.synth_fastq(11, 0, 100_000)
    tab = native.Counter(k=16, prefix=b"", flags=native.FLAG_UNORDERED)
    tab.count_buffer(short)
    tab.close()
    for data, k, prefix in ((short, 3, b""), (short, 8, b"A"), (reads, 16, b"ATGAC"), (reads, 3, b"")):
        want = oracle.count_buffer(data, prefix, k, 1)
        ctr = native.Counter(k=k, prefix=prefix)
        try:
            for rep in range(6):
                got = ctr.count_buffer(data).entries()
                assert got == want, (k, prefix, rep, first_diff(got, want))
        finally:
            ctr.close()
