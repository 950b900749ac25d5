"""The Node.js drop-in (kmerjs_amd/node/kmers.js over the N-API addon)."""
import json
import os
import shutil
import subprocess

import pytest

from tests.conftest import REPO

NODE = shutil.which("node")
RUNNER = os.path.join(REPO, "tests", "node", "run_node_tests.js")
pytestmark = pytest.mark.skipif(NODE is None, reason="node not installed")


def _run(mode, timeout):
    # (KMERHIP_SEGV_TRACE: the addon prints a backtrace on a fatal signal)
    p = subprocess.run([NODE, RUNNER, mode], capture_output=True, text=True, timeout=timeout,
                       env=dict(os.environ, KMERHIP_SEGV_TRACE="1"))
    assert p.returncode == 0, (p.returncode, p.stderr[-4000:])
    res = json.loads(p.stdout.strip().splitlines()[-1])
    bad = [r for r in res if not r["ok"]]
    assert res and not bad, bad[:5]
    return res


def test_node_dropin_cpu():
    _run("cpu", 60)


@pytest.mark.gpu
def test_c1_readfile_pins_reference_digest():
    """BASELINE configs[0] through the reference's entry point: readFile() of
    test_data/test_short.fastq with preffix 'ATGAC', k = 16 (test/kmers.js:28-35)
    resolves to the reference's Map: 2 keys, the ordered digest of SURVEY.md
    App. C (sha256 of JSON.stringify([...map]) = 14056308710d569d...), lines 40."""
    path = os.path.join(REPO, "tests", "golden", "inputs", "test_short.fastq")
    p = subprocess.run([NODE, os.path.join(REPO, "tests", "node", "run_readfile.js"), path, "ATGAC", "16"],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r.get("error") is None, r
    assert r["digest"].startswith("14056308710d569d") and r["size"] == 2 and r["lines"] == 40


@pytest.mark.gpu
def test_node_dropin_gpu_parity(golden):
    res = _run("gpu", 600)
    assert len(res) > 20


KF_RUNNER = os.path.join(REPO, "tests", "node", "run_kmerfinder.js")


def _kf(mode, spec, tmp_path, timeout):
    f = tmp_path / "spec.json"
    f.write_text(json.dumps(spec))
    p = subprocess.run([NODE, KF_RUNNER, mode, str(f)], capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


def _pairs(r):
    return None if r is None else [list(x) for x in r]


def test_node_match_summary_matches_oracle(tmp_path):
    # kmerfinder.js's BigInt decimals (bignumber.js 2.x semantics) against the
    # oracle's Fraction restatement of lib/stats.js + matchSummary, no GPU
    import random
    from oracle import kmerfinder_oracle as ko
    rng = random.Random(17)
    summary = {"templates": 5030, "totalLen": 16525500, "uniqueLens": 8076292}   # test_data/summary.json
    cases = []
    for _ in range(300):
        ul = rng.randint(1, 20000)
        u = rng.randint(1, ul)
        ts = u * rng.randint(1, 9)
        cases.append({"u": u, "ts": ts, "lengths": ul * 2 + rng.randint(0, 99), "ulength": ul,
                      "fu": u + rng.randint(0, 50), "ft": ts + rng.randint(0, 500),
                      "hits": u + rng.randint(0, 10 ** 6), "qsize": rng.randint(u, 2 * 10 ** 6), "summary": summary})
    got = _kf("stats", {"cases": cases}, tmp_path, 60)
    seen = 0
    for c, g in zip(cases, got):
        m = {"uScore": c["u"], "tScore": c["ts"], "lengths": c["lengths"], "ulength": c["ulength"], "species": "s"}
        want = ko.match_summary(c["qsize"], "NC_1", m, {"uScore": c["fu"], "tScore": c["ft"]}, c["hits"], summary)
        assert _pairs(g) == _pairs(want), c
        seen += want is not None
    assert seen > 40


@pytest.mark.gpu
def test_node_kmerfinder_matches_oracle(tmp_path):
    """KmerFinderServer.findMatches through Node on the GPU matcher against the
    oracle (lib/kmerFinderServer.js:736-874): winner and standard scoring, the
    exhausted-hits rejection, and a query Map that comes from readFile()
    (a KmerMap: the winners' k-mers are deleted from it, by index)."""
    from oracle import kmerfinder_oracle as ko
    from oracle import oracle
    import numpy as np
    from tests.match_util import kmer_codes, kmer_strings, make_db, make_query

    def summ(db):
        return {"templates": len(db), "totalLen": sum(t["lengths"] for t in db),
                "uniqueLens": sum(t["ulength"] for t in db)}
    cases, want = [], []
    for seed, method, bg in ((31, "winner", 0.03), (32, "winner", 0.0), (33, "standard", 0.03)):
        db = make_db(seed, 50, 400)
        q = make_query(seed + 1, db, [3, 17, 40], background=bg)
        s = summ(db)
        spec_db = [{"sequence": t["sequence"], "lengths": t["lengths"], "ulenght": t["ulength"],
                    "species": t["species"], "reads": t["kmers"]} for t in db]       # the ETL's document shape
        cases.append({"templates": spec_db, "summary": s, "method": method, "query": list(q.items())})
        qo = dict(q)
        try:
            r = (ko.winner_scoring(qo, db, s, len(q)) if method == "winner" else
                 ko.standard_scoring(qo, db, s, len(q)))
            want.append({"results": [_pairs(x) for x in r], "remaining": [list(x) for x in qo.items()]})
        except ko.NoHits as e:
            want.append({"error": str(e), "remaining": [list(x) for x in qo.items()]})
    # a readFile() query: templates made of the file's own k-mers
    path = os.path.join(REPO, "tests", "golden", "inputs", "test_long.kmer.fastq")
    ents = oracle.count_buffer(open(path, "rb").read(), b"ATGAC", 16, 1)
    q = {k.decode("latin-1"): v for k, v in ents}
    keys = list(q)
    # T0 holds most of the file's k-mers, T1 a few more, T2.. k-mers the file lacks
    other = kmer_strings(kmer_codes(np.random.default_rng(5), 400, 16, "CCCCC"), 16)
    lists = [keys[:250], keys[250:330]] + [other[i * 40:(i + 1) * 40] + keys[330 + i * 10:340 + i * 10]
                                          for i in range(5)]
    db = [{"sequence": "T%d" % t, "lengths": 2 * len(l), "ulength": len(l), "species": "x", "kmers": l}
          for t, l in enumerate(lists)]
    s = summ(db)
    cases.append({"templates": db, "summary": s, "method": "winner", "maxHits": 3,
                  "file": {"path": path, "prefix": "ATGAC", "k": 16}})
    qo = dict(q)
    r = ko.winner_scoring(qo, db, s, len(q), max_hits=3)
    assert len(r) >= 2
    want.append({"results": [_pairs(x) for x in r], "remaining": [list(x) for x in qo.items()]})
    got = _kf("match", {"cases": cases}, tmp_path, 300)
    for g, w in zip(got, want):
        if "error" in w:
            assert g.get("error") == w["error"]
        else:
            assert g.get("error") is None, g.get("error")
            assert [_pairs(x) for x in g["results"]] == w["results"]
        assert g["remaining"] == w["remaining"]


@pytest.mark.gpu
def test_node_readfile_long_contig(tmp_path):
    """readFile() on a FASTA-like file with a 9 MB sequence line (beyond the
    default order key's 2^23 bytes): kmer_count_file redoes the count in
    long-line mode and the Map equals the oracle's (lib/kmers.js has no line
    limit, :88-100)."""
    import numpy as np
    from oracle import oracle
    from tests.util import digest
    rng = np.random.default_rng(9)
    big = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, size=9_000_000)].tobytes()
    data = b">contig\n" + big + b"\n+\nIIII\n@r2\nACGTATGACGTTAGCATGACCATGACAAAT\n+\nIIII\n"
    f = tmp_path / "contig.fa"
    f.write_bytes(data)
    want = oracle.count_buffer(data, b"ATGAC", 21, 1)
    p = subprocess.run([NODE, os.path.join(REPO, "tests", "node", "run_readfile.js"), str(f), "ATGAC", "21"],
                       capture_output=True, text=True, timeout=300)
    got = json.loads(p.stdout.strip().splitlines()[-1])
    assert got.get("digest") == digest(want), got
    assert got["size"] == len(want)
