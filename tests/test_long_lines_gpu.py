"""Sequence lines longer than 2^23 bytes on the ordered paths (long-line
mode, KMER_FLAG_LONG_LINES / the automatic retry of kmer_count_file and
kmer_count_buffer): the reference has no line limit (lib/kmers.js:88-100), so
a 12 MB contig must count exactly like the oracle, in Map order, on every
ordered path (tile scan + packed keys, dense hits, tile records, general)."""
import numpy as np
import pytest

from tests.util import first_diff

pytestmark = pytest.mark.gpu


def _contig_input(seed, n_big=12_000_000):
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    big = acgt[rng.integers(0, 4, size=n_big)]
    big[rng.integers(0, n_big, size=50)] = ord("N")            # a few exotic windows
    small = acgt[rng.integers(0, 4, size=150)].tobytes()
    return (b">contig1\n" + big.tobytes() + b"\n+\nIIII\n" + b"@r2\n" + small + b"\n+\n" + b"I" * 150 + b"\n")


@pytest.fixture(scope="module")
def data():
    return _contig_input(21)


@pytest.mark.parametrize("k,prefix,step", [(21, b"ATGAC", 1), (21, b"AT", 1), (21, b"", 1), (21, b"ANG", 1),
                                           (21, b"ACG", 2)])
def test_long_contig_matches_oracle(data, k, prefix, step, tmp_path):
    import numpy as np
    from kmerjs_amd import _native
    from oracle import oracle
    c = _native.Counter(k=k, prefix=prefix, step=step)
    p = tmp_path / "contig.fastq"
    p.write_bytes(data)
    if step == 1:                                        # ordered keys + counts as arrays (Map order)
        keys, cnt = oracle.count_arrays(data, prefix, k)
        for r in (c.count_buffer(data), c.count_file(str(p))):   # (retried in long-line mode)
            assert r.keybuf == keys.tobytes() and np.array_equal(r.counts, cnt)
    else:
        want = oracle.count_buffer(data, prefix, k, step)
        got = c.count_buffer(data).entries()
        assert len(got) == len(want)
        assert first_diff(got, want) is None
        assert first_diff(c.count_file(str(p)).entries(), want) is None
    c.close()


def test_device_feed_needs_the_flag(data):
    import torch
    from kmerjs_amd import _native
    from oracle import oracle
    buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    c = _native.Counter(k=21, prefix=b"ATGAC")
    c.reset()
    with pytest.raises(_native.KmerError) as e:
        c.feed_device(buf.data_ptr(), buf.numel())
        c.finish()
    assert e.value.status == 7
    c.close()
    c = _native.Counter(k=21, prefix=b"ATGAC", flags=_native.FLAG_LONG_LINES)
    c.reset()
    c.feed_device(buf.data_ptr(), buf.numel())
    got = c.finish().entries()
    c.close()
    assert first_diff(got, oracle.count_buffer(data, b"ATGAC", 21, 1)) is None


@pytest.mark.parametrize("prefix", [b"ATGAC", b"", b"NNA"])
def test_group_context_retries_long_lines(data, prefix, tmp_path):
    """A device group meets a > 2^23-byte line: the count is redone in long-line
    mode on every device, as a single-device count is (group_count
    had no retry).  The W == 1 path (k > 64 would be the general path; NNA is
    the byte-SWAR packed path) and the sharded ordered paths."""
    from kmerjs_amd import _native
    from oracle import oracle
    want = oracle.count_buffer(data, prefix, 21, 1)
    p = tmp_path / "contig.fastq"
    p.write_bytes(data)
    c = _native.Counter(k=21, prefix=prefix, devices=[0, 0], batch_bytes=4 << 20)
    assert first_diff(c.count_buffer(data).entries(), want) is None
    assert first_diff(c.count_file(str(p)).entries(), want) is None
    c.close()


def test_progress_stays_monotone_across_the_long_line_retry(data, tmp_path):
    """The retry re-reads the input from the start; the progress callback must
    not go backwards (readFile()'s 'progress' events)."""
    from kmerjs_amd import _native
    p = tmp_path / "contig.fastq"
    p.write_bytes(data)
    for devices in (None, [0, 0]):
        seen = []
        c = _native.Counter(k=21, prefix=b"ATGAC", batch_bytes=1 << 20, devices=devices,
                            progress=lambda d, t: seen.append((d, t)))
        c.count_buffer(data)
        assert seen and all(b[0] >= a[0] for a, b in zip(seen, seen[1:])), seen[:8]
        assert seen[-1][0] == len(data)
        seen.clear()
        c.count_file(str(p))
        assert seen and all(b[0] >= a[0] for a, b in zip(seen, seen[1:])), seen[:8]
        assert seen[-1] == (len(data), len(data))
        c.close()
