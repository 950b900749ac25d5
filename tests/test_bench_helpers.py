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


def test_gpus_n_launches_n_ranks_dry_run():
    """`bench.py --gpus N` with no launcher starts ranks 0..N-1 itself (VERDICT r3
    weak #1): the dry run prints the environment of each rank it would start."""
    import json
    import subprocess
    env = {k: v for k, v in __import__("os").environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, bench.__file__, "--gpus", "4", "--dry-run-launch"], env=env,
                       capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    rows = [json.loads(x) for x in p.stdout.strip().splitlines()]
    assert [r["env"]["RANK"] for r in rows] == ["0", "1", "2", "3"]
    assert [r["env"]["LOCAL_RANK"] for r in rows] == ["0", "1", "2", "3"]
    assert {r["env"]["WORLD_SIZE"] for r in rows} == {"4"}
    assert {r["env"]["MASTER_ADDR"] for r in rows} == {"127.0.0.1"}
    assert len({r["env"]["MASTER_PORT"] for r in rows}) == 1
    assert all("--dry-run-launch" not in r["cmd"] and r["cmd"][-2:] == ["--gpus", "4"] for r in rows)


def test_launch_ranks_runs_children_and_propagates_failure(tmp_path):
    """The launcher really starts N processes (no exec), each sees its rank, and
    one failing rank ends the job with its status (the others are stopped)."""
    script = tmp_path / "child.py"
    out = tmp_path / "seen"
    out.mkdir()
    script.write_text(
        "import os, sys, time\n"
        "r = int(os.environ['RANK'])\n"
        "open(os.path.join(%r, os.environ['RANK'] + '_' + os.environ['WORLD_SIZE']), 'w').close()\n"
        "if 'fail' in sys.argv and r == 1:\n"
        "    sys.exit(3)\n"
        "if 'fail' in sys.argv:\n"
        "    time.sleep(60)\n" % str(out))
    assert bench.launch_ranks(3, [], script=str(script)) == 0
    assert sorted(x.name for x in out.iterdir()) == ["0_3", "1_3", "2_3"]
    import time
    t0 = time.time()
    assert bench.launch_ranks(2, ["fail"], script=str(script)) == 3
    assert time.time() - t0 < 30                    # rank 0 was stopped, not waited for


def test_world_size_must_equal_gpus():
    import os
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, bench.__file__, "--gpus", "4"], env=env, capture_output=True, text=True,
                       timeout=60)
    assert p.returncode != 0 and "WORLD_SIZE=2 but --gpus 4" in p.stderr


@pytest.mark.parametrize("config", ["c2", "c4", "c3"])
def test_dry_run_plans_record_aligned_shards(config):
    """`bench.py --gpus 8 --dry-run` (no GPU): 8 ranks, each holding a
    record-aligned shard whose line / byte offsets are multi.shard_plan's --
    rank r starts at read r * n (line 4 r n, byte 317 r n), the shards tile the
    job without overlap; C3 splits its 100 M reads (strong scaling), C2 / C4
    hold a fixed share per GPU (weak)."""
    import json
    import os
    import subprocess
    from kmerjs_amd.multi import shard_plan
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, bench.__file__, "--gpus", "8", "--dry-run", "--config", config], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    rows = [json.loads(x) for x in p.stdout.strip().splitlines()]
    assert [r["rank"] for r in rows] == list(range(8))
    n = {"c2": 10_000_000, "c4": 125_000_000, "c3": 100_000_000 // 8}[config]
    for r in rows:
        want = shard_plan(n, r["rank"])
        assert {x: r[x] for x in want} == want
        assert r["lines_before"] == 4 * n * r["rank"] and r["byte_offset"] == 317 * n * r["rank"]
        assert r["scaling"] == ("strong" if config == "c3" else "weak")
    for a, b in zip(rows, rows[1:]):
        assert a["first_read"] + a["n_reads"] == b["first_read"]
    assert rows[0]["merge"] == ("dense" if config == "c4" else "hits")
