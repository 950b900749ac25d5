"""step > 1 on the device (lib/kmers.js:88-100: `ini += this.step` over the line
and, separately, over its complement).  The dense-hit path ranks the stepped
windows of each strand (2 ceil(W / step) per sequence line); bit-exact against
the oracle, with non-ACGT windows (records), batches and both prefix kinds."""
import numpy as np
import pytest

from tests.util import first_diff

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    from kmerjs_amd import _native
    return _native


@pytest.fixture(scope="module")
def reads():
    from oracle import oracle
    rng = np.random.default_rng(31)
    arr = np.frombuffer(bytearray(oracle.synth_fastq(6, 0, 30000)), dtype=np.uint8).reshape(-1, 317).copy()
    seq = arr[:, 13:163]
    seq[rng.random(seq.shape) < 0.002] = ord("N")
    arr[:, 13:163] = seq
    return arr.tobytes()


@pytest.mark.parametrize("k,prefix,step", [(16, b"ATGAC", 2), (16, b"ATGAC", 3), (21, b"", 2), (31, b"", 7),
                                           (12, b"AC", 5), (32, b"T", 4), (16, b"ATGACGTA", 150)])
def test_step_vs_oracle(native, reads, k, prefix, step):
    from oracle import oracle
    want = oracle.count_buffer(reads, prefix, k, step)
    for batch in (0, 1 << 20):
        ctr = native.Counter(k=k, prefix=prefix, step=step, batch_bytes=batch)
        got = ctr.count_buffer(reads).entries()
        ctr.close()
        assert first_diff(got, want) is None, (k, prefix, step, batch)


def test_step_device_feed_and_lines(native):
    import torch
    from kmerjs_amd import synth_fastq_device
    from oracle import oracle
    n = 100_000
    buf = torch.empty(n * 317, dtype=torch.uint8, device="cuda")
    synth_fastq_device(buf.data_ptr(), 9, 0, n)
    torch.cuda.synchronize()
    host = buf.cpu().numpy().tobytes()
    want = oracle.count_buffer(host, b"AT", 16, 2)
    ctr = native.Counter(k=16, prefix=b"AT", step=2)
    ctr.reset()
    ctr.feed_device(buf.data_ptr(), len(host))
    r = ctr.finish()
    ctr.close()
    assert r.lines == 4 * n and first_diff(r.entries(), want) is None
