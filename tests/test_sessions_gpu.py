"""Sessions on one counter whose hit density jumps (tiles overflowing their
hit slots: the chunk is redone with larger lists) or that turn on
long-segment cross sorting (40 kb reads) must each equal the oracle
(lib/kmers.js:88-100 semantics, restated in oracle/kmer_oracle.c): no state
of one session leaks into the next."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _reads(seed, n, body):
    rng = np.random.default_rng(seed)
    out = bytearray()
    for i in range(n):
        seq = body(rng)
        out += b"@r%d\n" % i + seq + b"\n+\n" + b"I" * len(seq) + b"\n"
    return bytes(out)


def _random(rng):
    return np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, size=150)].tobytes()


def _dense(rng):
    # the prefix every 5 bases on both strands: ~60 hits per read
    return (b"ATGAC" * 15 + b"GTCAT" * 15)[:150]


def _long(rng):
    return np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, size=40_000)].tobytes()


def _device_count(c, data):
    import torch
    buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    c.reset()
    c.feed_device(buf.data_ptr(), buf.numel())
    return c.finish()


def test_density_and_long_lines_across_sessions():
    from kmerjs_amd import _native
    from oracle import oracle
    k, prefix = 16, b"ATGAC"
    inputs = [_reads(1, 20_000, _random), _reads(2, 20_000, _dense), _reads(3, 20_000, _random),
              _reads(4, 40, _long), _reads(5, 20_000, _dense), _reads(6, 20_000, _random)]
    c = _native.Counter(k=k, prefix=prefix)
    for data in inputs:
        keys, cnt = oracle.count_arrays(data, prefix, k)
        r = _device_count(c, data)
        assert r.keybuf == keys.tobytes() and np.array_equal(r.counts, cnt)
    c.close()
