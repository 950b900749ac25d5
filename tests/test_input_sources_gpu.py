"""kmer_count_file on inputs that are not regular files: a FIFO (as
`<(zcat reads.fastq.gz)` or /dev/stdin give), plain and gzip-compressed.
fs.createReadStream in the reference reads those too (lib/kmers.js:139);
ADVICE r3 found the pread-based reader failing them with KMER_E_IO."""
import gzip
import os
import threading

import pytest

from tests.conftest import REPO

pytestmark = pytest.mark.gpu

GOLD = os.path.join(REPO, "tests", "golden", "inputs")


def _fifo_count(tmp_path, payload, **kw):
    from kmerjs_amd import _native
    path = str(tmp_path / "in.fifo")
    os.mkfifo(path)

    def writer():
        with open(path, "wb") as f:
            for i in range(0, len(payload), 65536):       # (a stream: many small writes)
                f.write(payload[i:i + 65536])

    t = threading.Thread(target=writer)
    t.start()
    c = _native.Counter(**kw)
    try:
        return c.count_file(path)
    finally:
        c.close()
        t.join(timeout=60)


@pytest.mark.parametrize("compress", [False, True])
@pytest.mark.parametrize("name,prefix,k", [("test_short.fastq", b"ATGAC", 16), ("test_long.kmer.fastq", b"", 21),
                                           ("test_kmers.fastq", b"ATGAC", 16)])
def test_fifo_input_matches_the_regular_file(tmp_path, name, prefix, k, compress):
    from kmerjs_amd import _native
    with open(os.path.join(GOLD, name), "rb") as f:
        data = f.read()
    c = _native.Counter(k=k, prefix=prefix)
    want = c.count_file(os.path.join(GOLD, name))
    c.close()
    got = _fifo_count(tmp_path, gzip.compress(data) if compress else data, k=k, prefix=prefix, batch_bytes=100000)
    assert got.entries() == want.entries() and got.lines == want.lines


def test_fifo_input_device_group(tmp_path):
    from oracle import oracle
    data = oracle.synth_fastq(7, 0, 20000)
    got = _fifo_count(tmp_path, data, k=16, prefix=b"ATGAC", devices=[0, 0], batch_bytes=1 << 20)
    assert got.entries() == oracle.count_buffer(data, b"ATGAC", 16, 1)
