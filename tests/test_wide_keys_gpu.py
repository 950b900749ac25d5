"""k in 33..64 on the packed path (SURVEY.md §8 verdict item: 128-bit window
codes).  A window's code is two words (the first k - 32 bases, the last 32);
keys of 2(k - |P|) >= 64 bits are ranked as (hi, lo) pairs and sorted by two
stable radix passes.  Bit-exact against the oracle (lib/kmers.js:88-100 on
both strands, Map insertion order), including non-ACGT windows (records),
reads cut across tiles, dense prefixes and the records path (NO_DENSE)."""
import numpy as np
import pytest

from tests.util import first_diff

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    from kmerjs_amd import _native
    return _native


@pytest.fixture(scope="module")
def synth():
    import torch
    from kmerjs_amd import synth_fastq_device
    n = 60_000
    buf = torch.empty(n * 317, dtype=torch.uint8, device="cuda")
    synth_fastq_device(buf.data_ptr(), 5, 0, n)
    torch.cuda.synchronize()
    return buf, buf.cpu().numpy().tobytes()


# (k, prefix): wide keys (k - |P| >= 32), 64-bit keys of k > 32, narrow ones
CASES = [(40, b"ATGAC"), (64, b"ATGAC"), (48, b"ACG"), (33, b"A"), (36, b"ATGA"), (63, b"GT"),
         (33, b"ATGAC"), (40, b"ATGACGTACGTAGCTAGCTAGCTAGCTAGCTAGC")]


@pytest.mark.parametrize("k,prefix", CASES)
def test_wide_synthetic_vs_oracle(native, synth, k, prefix):
    from oracle import oracle
    buf, host = synth
    want = oracle.count_buffer(host, prefix, k, 1)
    ctr = native.Counter(k=k, prefix=prefix)
    ctr.reset()
    ctr.feed_device(buf.data_ptr(), len(host))
    got = ctr.finish().entries()
    ctr.close()
    assert len(got) == len(want)
    assert first_diff(got, want) is None


def test_wide_with_n_batches_and_records_path(native):
    from oracle import oracle
    rng = np.random.default_rng(12)
    arr = np.frombuffer(bytearray(oracle.synth_fastq(3, 0, 20000)), dtype=np.uint8).reshape(-1, 317).copy()
    seq = arr[:, 13:163]
    seq[rng.random(seq.shape) < 0.002] = ord("N")
    arr[:, 13:163] = seq
    data = arr.tobytes()
    for k, p in ((40, b"ATGAC"), (56, b"AC"), (64, b"TTT")):
        want = oracle.count_buffer(data, p, k, 1)
        for flags, batch in ((0, 0), (0, 1 << 20), (native.FLAG_NO_DENSE, 0)):
            ctr = native.Counter(k=k, prefix=p, flags=flags, batch_bytes=batch)
            got = ctr.count_buffer(data).entries()
            ctr.close()
            assert first_diff(got, want) is None, (k, p, flags, batch)


def test_long_prefix_present_in_the_data(native, synth):
    # a 34-byte prefix cut from the input (so that it occurs): the emitted keys
    # carry all of it (|P| > 32)
    from oracle import oracle
    buf, host = synth
    line = host.split(b"\n")[1]
    for k, p in ((40, line[10:44]), (64, line[20:60]), (36, line[5:37])):
        want = oracle.count_buffer(host, p, k, 1)
        ctr = native.Counter(k=k, prefix=p)
        got = ctr.count_buffer(host).entries()
        ctr.close()
        assert len(want) > 0 and first_diff(got, want) is None, (k, p)


def test_non_acgt_prefixes_on_the_packed_path(native):
    # the key is P + the suffix's 2-bit code, so a prefix of any bytes stays on
    # the device (non-ACGT suffixes are records); reads with N at p = 0.02
    from oracle import oracle
    rng = np.random.default_rng(21)
    arr = np.frombuffer(bytearray(oracle.synth_fastq(4, 0, 20000)), dtype=np.uint8).reshape(-1, 317).copy()
    seq = arr[:, 13:163]
    seq[rng.random(seq.shape) < 0.02] = ord("N")
    arr[:, 13:163] = seq
    data = arr.tobytes()
    for k, p in ((16, b"N"), (16, b"NA"), (21, b"AN"), (40, b"NAC"), (12, b"GNT"), (16, b"X"), (8, b"NNNN"),
                 (33, b"N"), (16, b"@s")):
        want = oracle.count_buffer(data, p, k, 1)
        ctr = native.Counter(k=k, prefix=p)
        got = ctr.count_buffer(data).entries()
        ctr.close()
        assert first_diff(got, want) is None, (k, p, len(got), len(want))


def test_wide_group_and_partials(native):
    from oracle import oracle
    data = oracle.synth_fastq(8, 0, 30000)
    want = oracle.count_buffer(data, b"ATGAC", 40, 1)
    # a device group keeps the record path for k > 32 (its merge takes packed partials)
    ctr = native.Counter(k=40, prefix=b"ATGAC", devices=[0, 0])
    assert first_diff(ctr.count_buffer(data).entries(), want) is None
    ctr.close()
    # one context: keys of >= 64 bits have no packed partial (refused, not wrong)
    ctr = native.Counter(k=40, prefix=b"ATGAC")
    ctr.count_buffer(data)
    with pytest.raises(native.KmerError):
        ctr.partial_device()
    ctr.close()
