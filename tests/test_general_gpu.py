"""The general path with the device merge (step 1: k > 64 with any prefix,
unprefixed k > 31, non-ACGT prefix bytes beyond the tile kernels): the
windows kernel finds every accepted window (lib/kmers.js:88-100 on both
strands: the reference's loop has no k limit), a chunk's windows become
session entries on the device, and a merge groups them by a 128-bit hash of
their bytes (neighbours with equal hashes compared byte for byte), sums the
counts, keeps the first occurrence, and orders the result by it (Map
insertion order).  Bit-exact against the oracle; no host record merge."""
import numpy as np
import pytest

from tests.util import first_diff

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    from kmerjs_amd import _native
    return _native


def _reads_with_n(seed, n, p_n=0.002):
    from oracle import oracle
    rng = np.random.default_rng(seed)
    arr = np.frombuffer(bytearray(oracle.synth_fastq(seed, 0, n)), dtype=np.uint8).reshape(-1, 317).copy()
    seq = arr[:, 13:163]
    seq[rng.random(seq.shape) < p_n] = ord("N")
    arr[:, 13:163] = seq
    return arr.tobytes()


@pytest.mark.parametrize("k,prefix", [(65, b"ATGAC"), (80, b"A"), (150, b""), (100, b"ATG"), (70, b"NNA"),
                                      (40, b""), (64, b""), (70, b"ATGACGTTCA"), (66, b"GTCAT")])
def test_general_device_merge_vs_oracle(native, k, prefix):
    # synthetic reads with N bytes (non-ACGT windows are keys like any other:
    # the merge works on bytes); one feed, then batches of 1 MiB.  An A/C/G/T
    # prefix takes the plane-candidate windows kernel, FLAG_BYTE_SCAN the
    # flattened one (both against the oracle)
    from oracle import oracle
    data = _reads_with_n(k, 12000)
    want = oracle.count_buffer(data, prefix, k, 1)
    for batch, flags in ((0, 0), (1 << 20, 0), (0, native.FLAG_BYTE_SCAN)):
        ctr = native.Counter(k=k, prefix=prefix, batch_bytes=batch, flags=flags)
        res = ctr.count_buffer(data)
        got = res.entries()
        ctr.close()
        assert len(got) == len(want), (k, prefix, batch, flags)
        assert first_diff(got, want) is None, (k, prefix, batch, flags)
        assert res.lines == data.count(b"\n")


def test_general_device_merge_reference_inputs(native, inputs):
    # the reference's own fixtures (test_long.kmer.fastq, test_kmers.fastq with
    # its X runs) and the edge inputs at k > 64 and unprefixed k > 31
    from oracle import oracle
    for name in ("test_long.kmer.fastq", "test_kmers.fastq", "test_short.fastq", "edge_blank.fastq",
                 "edge_contigs.fsa"):
        data = inputs[name]
        for k, p in ((66, b""), (90, b"A"), (35, b""), (70, b"ATGAC")):
            want = oracle.count_buffer(data, p, k, 1)
            ctr = native.Counter(k=k, prefix=p)
            got = ctr.count_buffer(data).entries()
            ctr.close()
            assert first_diff(got, want) is None, (name, k, p)


def test_general_device_merge_repeats_and_device_feeds(native):
    # many copies of few keys (poly-A / repeated reads: long groups in the
    # merge), fed as device chunks; the result equals the oracle's, and the
    # host records path (FLAG_NO_DENSE) gives the same Map
    import torch
    from oracle import oracle
    rep = b"".join(b"@r%d\n%s\n+\n%s\n" % (i, (b"A" * 150) if i % 3 else (b"ACGT" * 38)[:150], b"I" * 150)
                   for i in range(3000))
    data = rep + _reads_with_n(3, 3000)
    k = 70
    want = oracle.count_buffer(data, b"", k, 1)
    dev = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    ctr = native.Counter(k=k, prefix=b"")
    ctr.reset()
    ctr.feed_device(dev.data_ptr(), len(rep))
    ctr.feed_device(dev.data_ptr() + len(rep), len(data) - len(rep))
    got = ctr.finish().entries()
    ctr.close()
    assert first_diff(got, want) is None
    ctr = native.Counter(k=k, prefix=b"", flags=native.FLAG_NO_DENSE)
    assert first_diff(ctr.count_buffer(data).entries(), want) is None
    ctr.close()


def test_general_records_export_then_more_chunks(native):
    # kmer_records_export folds the device entries into host records (the
    # multi-rank gather); chunks fed after it and the finish still give every
    # key once (host records of k bytes rejoin the device merge)
    import torch
    from oracle import oracle
    data = _reads_with_n(9, 6000)
    half = 317 * 3000
    k, p = 72, b"AC"
    want = oracle.count_buffer(data, p, k, 1)
    dev = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    ctr = native.Counter(k=k, prefix=p)
    ctr.reset()
    ctr.feed_device(dev.data_ptr(), half)
    kb, off, cnt, fst = ctr.records_export()
    assert len(cnt) > 0
    ctr.feed_device(dev.data_ptr() + half, len(data) - half)
    got = ctr.finish().entries()
    ctr.close()
    assert first_diff(got, want) is None


def test_general_max_keys(native):
    # more distinct keys than max_keys: the reference Map's RangeError
    # (lib/kmers.js:95) as KMER_E_TOO_MANY_KEYS
    from oracle import oracle
    data = oracle.synth_fastq(4, 0, 2000)
    ctr = native.Counter(k=80, prefix=b"", max_keys=1000)
    with pytest.raises(native.KmerError) as e:
        ctr.count_buffer(data)
    assert e.value.status == 5
    ctr.close()


def test_general_long_prefix_and_forced_collision_retry(native):
    """Two routes the other cases miss: an A/C/G/T prefix longer than 16 bytes
    (gen_cand_kernel verifies candidates byte for byte in global memory,
    gen_bytes_eq, instead of in LDS), and the merge's collision retry (the
    (h2, h1) LSD sort + gather of h2), forced on the first attempt by
    KMER_FLAG_GEN_COLLIDE_TEST.  Both against the oracle (lib/kmers.js:88-100)."""
    from oracle import oracle
    data = bytearray(_reads_with_n(17, 12000))
    arr = np.frombuffer(data, dtype=np.uint8).reshape(-1, 317)
    p20 = bytes(arr[5, 13 + 10:13 + 30])
    assert all(ch in b"ACGT" for ch in p20)
    rc20 = oracle.complement(p20)
    for i in range(0, 12000, 37):                 # the prefix and its complement planted in many reads
        arr[i, 13 + 40:13 + 60] = np.frombuffer(p20 if i % 2 else rc20, dtype=np.uint8)
    data = bytes(data)
    for k, prefix, flags in ((70, p20, 0), (66, p20[:18], 0), (70, b"ATGAC", native.FLAG_GEN_COLLIDE_TEST),
                             (40, b"", native.FLAG_GEN_COLLIDE_TEST)):
        want = oracle.count_buffer(data, prefix, k, 1)
        assert len(want) > 100
        ctr = native.Counter(k=k, prefix=prefix, flags=flags)
        got = ctr.count_buffer(data).entries()
        ctr.close()
        assert first_diff(got, want) is None, (k, prefix, flags)
