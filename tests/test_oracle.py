"""The CPU restatement (oracle/) against the reference's golden vectors.

Goldens come from running the unmodified reference lib/kmers.js
(tests/golden/gen_golden.py); the KATs are the reference's own tests
(test/kmers.js:12-52).
"""
import hashlib

from oracle import oracle
from tests.util import digest, js_stringify


def test_oracle_matches_every_golden(golden, inputs):
    bad = []
    for c in golden["cases"]:
        e, st = oracle.count_buffer(inputs[c["input"]], c["prefix"].encode(), c["k"], c["step"], stats=True)
        if digest(e) != c["digest"] or st["lines"] != c["lines"]:
            bad.append((c["input"], c["prefix"], c["k"], c["step"]))
    assert not bad, bad[:10]


def test_inputs_match_golden_sha(golden, inputs):
    for name, sha in golden["inputs"].items():
        assert hashlib.sha256(inputs[name]).hexdigest() == sha, name


def test_kat_first_key_kmersInLine():
    # test/kmers.js:12-19 — the template literal keeps its newline + indentation
    seq = ("NTTTATGACGCAATACTCCTCTCTCCTTCGTGGTCTTGCAGCGGGTTCTGC\n"
           "                   ATTTTTATTCCTTTTTGCCCCAACGGCATTCGCGGCGGAACAAACCGTTG")
    e = oracle.kmers_in_line(seq.encode())
    assert e[0][0] == b"ATGACGCAATACTCCT"
    assert e == [(b"ATGACGCAATACTCCT", 1)]


def test_kat_complement():
    # test/kmers.js:21-26
    assert oracle.complement(b"ATGACCTGAGAGCCTT") == b"AAGGCTCTCAGGTCAT"
    assert oracle.complement(b"acgtNX\r") == b"\rXNtgca"


def test_kat_read_file_sizes(inputs):
    # test/kmers.js:28-35 and :45-52
    short = oracle.count_buffer(inputs["test_short.fastq"])
    assert short == [(b"ATGACGCAATACTCCT", 1), (b"ATGACCTGAGAGCCTT", 1)]
    assert len(oracle.count_buffer(inputs["test_long.kmer.fastq"])) == 401


def test_appendix_c_digests(golden):
    # SURVEY.md Appendix C (first 16 hex of the ordered digest)
    want = {("test_short.fastq", "ATGAC", 16): "14056308710d569d",
            ("test_short.fastq", "", 31): "6c9b4d7ab7bda846",
            ("test_long.kmer.fastq", "ATGAC", 16): "05444cfc9ac76c53",
            ("test_long.kmer.fastq", "", 16): "f2884dd21ecdceaa",
            ("test_kmers.fastq", "ATGAC", 16): "060076d7e1acea40",
            ("test_kmers.fastq", "", 31): "f5b2531dc2f77941"}
    got = {(c["input"], c["prefix"], c["k"]): c["digest"][:16] for c in golden["cases"] if c["step"] == 1}
    for key, d in want.items():
        assert got[key] == d, key


def test_synth_generator_twins():
    from tests.golden.make_inputs import synth_fastq
    assert oracle.synth_fastq(7, 123, 50) == synth_fastq(7, 123, 50)
    b = oracle.synth_fastq(1, 0, 3)
    assert len(b) == 3 * 317 and b.startswith(b"@r0000000000\n")


def test_kmers_long_json_subset(inputs):
    # test_data/kmers_long.json is the golden Map of the missing test_long.fastq;
    # test_long.kmer.fastq's 401 keys are a subset with counts <=
    import json
    import os
    here = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(here, "golden", "kmers_long.json")) as f:
        big = json.load(f)
    assert len(big) == 6191 and sum(big.values()) == 9301
    for k, v in oracle.count_buffer(inputs["test_long.kmer.fastq"]):
        assert k.decode() in big and v <= big[k.decode()]


def test_js_stringify_format():
    assert js_stringify([(b"A\rC", 2)]) == '[["A\\rC",2]]'


def test_fasta_oracle_matches_python_restatement():
    """oracle_count_fasta (the FASTA-mode checker; parity unpinned by the
    reference, which has no FASTA parser) against an independent Python
    restatement, on edge-rich inputs: CRLF, blank lines, wrapped and 1-base
    lines, empty records, headerless first record, exotic bytes, no trailing
    newline; and against hand-computed cases."""
    from oracle import oracle
    from tests.fasta_util import fasta_reference_py, make_fasta
    cases = [make_fasta(1, 20, 400), make_fasta(2, 20, 300, crlf=True, blank=0.2),
             make_fasta(3, 15, 200, headerless=True, exotic=0.05), make_fasta(4, 10, 100, width=1),
             make_fasta(5, 12, 150, tail_newline=False), b"", b">only header", b"ACGTACGT", b">a\n>b\n\n>c\nAC\nGT\n"]
    for data in cases:
        for prefix, k, step in ((b"", 4, 1), (b"A", 5, 1), (b"AC", 3, 2), (b"", 1, 1)):
            want, lines = fasta_reference_py(data, prefix, k, step)
            got, st = oracle.count_buffer(data, prefix, k, step, stats=True, fasta=True)
            assert got == want, (data[:40], prefix, k, step)
            assert st["lines"] == lines
    # hand-computed: windows cross the line break of one record
    got = oracle.count_buffer(b">r\nAC\nGT\n", b"", 4, 1, fasta=True)
    assert got == [(b"ACGT", 2)]
    # ... and do not cross records
    assert oracle.count_buffer(b">r\nAC\n>s\nGT\n", b"", 4, 1, fasta=True) == []


def test_streamed_count_equals_buffer_count():
    # oracle_count_synth (blocks of generated records, the line state carried)
    # == oracle_count_buffer over the same bytes; its digest helper == digest()
    import numpy as np
    from tests.util import map_digest_arrays
    data = oracle.synth_fastq(7, 1000, 20000)
    keys, cnt = oracle.count_arrays(data, b"ATGAC", 16)
    k2, c2, f2, lines = oracle.count_synth_arrays(7, 1000, 20000, b"ATGAC", 16)
    assert np.array_equal(keys, k2) and np.array_equal(cnt, c2) and lines == 80000
    assert bool(np.all(f2[1:] > f2[:-1]))
    ents = oracle.count_buffer(data, b"ATGAC", 16)
    assert map_digest_arrays(keys, cnt) == digest(ents)[:16]


def test_streamed_table_digest_equals_map_digest():
    # oracle_table_digest (a sum over forward windows, no map) == the table
    # digest derived from the oracle's Map (canonical classes counted once per
    # forward window, App. A.6), with N bytes (records, outside the digest),
    # odd / even k (palindromes) and k = 1
    import numpy as np
    from tests.util import canonical_summary
    for k in (31, 16, 21, 2, 1):
        rng = np.random.default_rng(k)
        arr = np.frombuffer(bytearray(oracle.synth_fastq(8, 0, 3000)), dtype=np.uint8).reshape(-1, 317).copy()
        seq = arr[:, 13:163]
        seq[rng.random(seq.shape) < 0.002] = ord("N")
        arr[:, 13:163] = seq
        data = arr.tobytes()
        keys, cnt = oracle.count_arrays(data, b"", k)
        acgt = ~(keys == ord("N")).any(axis=1)
        _, fwd, dig = canonical_summary(keys[acgt], cnt[acgt], k)
        got, win = oracle.table_digest(data, k)
        assert got == dig and win == 3000 * (150 - k + 1), k
    clean = oracle.synth_fastq(3, 500, 4000)
    assert oracle.table_digest_synth(3, 500, 4000, 31, 1) == oracle.table_digest(clean, 31)
    assert oracle.table_digest_synth(3, 500, 4000, 31, 3) == oracle.table_digest(clean, 31)


def test_streamed_fasta_table_digest_equals_fasta_map_digest():
    # oracle_table_digest_fasta (C5 .fsa contigs, records joined) == the table
    # digest of oracle_count_fasta's Map, on wrapped, CRLF, blank-line and
    # headerless inputs; and the single-line contig file read as FASTQ (the
    # reference's rule, lib/kmers.js:151) through oracle_table_digest
    import bench
    from tests.fasta_util import make_fasta
    from tests.util import table_digest_from_map
    cases = [make_fasta(1, 20, 400), make_fasta(2, 20, 300, crlf=True, blank=0.2),
             make_fasta(3, 15, 200, headerless=True), make_fasta(4, 10, 100, width=1), b"", b">h\nA\nC\n"]
    contigs60, _ = bench.make_contigs(5, 300_000, 21, width=60)
    cases.append(contigs60)
    for data in cases:
        for k in (21, 4, 1):
            ents = oracle.count_buffer(data, b"", k, 1, fasta=True)
            got, _ = oracle.table_digest_fasta(data, k)
            assert got == table_digest_from_map(ents, k), (data[:30], k)
    single, _ = bench.make_contigs(5, 300_000, 21)
    got, _ = oracle.table_digest(single, 21)
    assert got == table_digest_from_map(oracle.count_buffer(single, b"", 21, 1), 21)


def test_fullsize_golden_c2_is_the_reference_digest():
    # tests/golden/fullsize.json's C2 answer (the oracle, streamed and merged
    # over shards) equals the reference's own readFile() run on the same bytes
    # (profiles/ref_js_c2.json)
    import json
    import os
    from tests.util import fullsize_golden
    ref = json.load(open(os.path.join(os.path.dirname(__file__), "..", "profiles", "ref_js_c2.json")))
    run = ref["runs"][0]
    g = fullsize_golden()
    assert (g["c2"]["digest"], g["c2"]["size"], g["c2"]["sum"]) == (run["digest"], run["size"], run["sum"])
    assert g["c4"]["lines"] == 4 * 125_000_000 and g["c3"]["forward_windows"] == 100_000_000 * 120
