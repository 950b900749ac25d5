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


def test_every_golden_case(native, golden, inputs):
    bad = _run_cases(native, golden, inputs)
    assert not bad, bad[:5]


def test_two_pass_mode_matches(native, golden, inputs):
    bad = _run_cases(native, golden, inputs, flags=native.FLAG_TWO_PASS,
                     select=lambda c: c["step"] == 1 and c["k"] in (16, 31))
    assert not bad, bad[:5]


def test_record_path_matches(native, golden, inputs):
    bad = _run_cases(native, golden, inputs, flags=native.FLAG_NO_DENSE,
                     select=lambda c: c["prefix"] == "ATGAC" and c["step"] == 1)
    assert not bad, bad[:5]


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
