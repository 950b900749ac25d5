"""bench.py's workload helpers (CPU): the k-mer (window) count that `value`
is quoted in, against the oracle's own enumeration."""
import sys

import pytest

from tests.conftest import REPO

sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_count_windows_matches_oracle_on_contigs():
    from oracle import oracle
    data, lens = bench.make_contigs(5, 1, 21)          # one contig: header + sequence line
    assert data.count(b"\n") == len(lens)
    want = sum(c for _, c in oracle.count_buffer(data, b"", 21, 1))
    assert bench.count_windows(lens, 0, 21) == want
    # a shard starting at line 1 sees the header (10 bytes < k) as its sequence line
    assert bench.count_windows(lens, 1, 21) == 0


def test_windows_per_read_matches_synthetic_reads():
    from oracle import oracle
    data = oracle.synth_fastq(1, 0, 50)
    for k in (16, 21, 31):
        want = sum(c for _, c in oracle.count_buffer(data, b"", k, 1))
        assert want == 50 * bench.windows_per_read(k)


@pytest.mark.parametrize("first_line", [0, 1, 2, 3])
def test_count_windows_line_phase(first_line):
    lens = [5, 30, 2, 30, 1, 40]
    got = bench.count_windows(lens, first_line, 4)
    want = sum(2 * (L - 4 + 1) for i, L in enumerate(lens) if (first_line + i) % 4 == 1 and L >= 4)
    assert got == want
