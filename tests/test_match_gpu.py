"""GPU parity of the k-mer -> template matcher (include/kmer_match.h,
kmerjs_amd/kmerfinder.py) against the oracle restatement of kmerFinder's
findKmersMatchesRedis / winnerScoring / standardScoring
(oracle/kmerfinder_oracle.py; lib/kmerFinderServer.js:171-226, :452-522,
:625-874).  Everything integer is compared exactly; the statistics are the
same decimal arithmetic, compared as the JS numbers the reference returns."""
import numpy as np
import pytest

from oracle import kmerfinder_oracle as ko
from tests.match_util import kmer_codes, kmer_strings, make_db, make_query

pytestmark = pytest.mark.gpu


def _summary(db):
    return {"templates": len(db), "totalLen": sum(t["lengths"] for t in db),
            "uniqueLens": sum(t["ulength"] for t in db)}


@pytest.fixture(scope="module")
def kf():
    from kmerjs_amd import kmerfinder
    return kmerfinder


def _round1(kf, tdb, q, order=0):
    m = kf.Match(tdb, list(q.keys()), list(q.values()))
    try:
        return m.templates(order), m.winner()
    finally:
        m.close()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_first_round_matches_oracle(kf, seed):
    db = make_db(seed, 60, 500)
    tdb = kf.TemplateDB(db, 16)
    info = tdb.info()
    assert info["entries"] == sum(len(set(t["kmers"])) for t in db)
    assert info["distinct"] == len({km for t in db for km in t["kmers"]})
    q = make_query(seed + 100, db, [3, 20, 41])
    tpls, hits = ko.first_round(dict(q), db, ko.build_index(db))
    got, w = _round1(kf, tdb, q)
    assert [db[t]["sequence"] for t, _, _ in got] == list(tpls.keys())
    for t, u, s in got:
        o = tpls[db[t]["sequence"]]
        assert (u, s) == (o["uScore"], o["tScore"])
    assert w.hits == hits
    best = sorted(tpls.items(), key=lambda kv: -kv[1]["uScore"])[0][0]
    assert db[w.tmpl]["sequence"] == best
    dbo, _ = _round1(kf, tdb, q, order=1)
    assert [t for t, _, _ in dbo] == sorted(t for t, _, _ in got)


@pytest.mark.parametrize("seed,background", [(4, 0.03), (5, 0.05), (6, 0.02)])
def test_winner_scoring_matches_oracle(kf, seed, background):
    db = make_db(seed, 80, 600)
    summary = _summary(db)
    tdb = kf.TemplateDB(db, 16, summary)
    q = make_query(seed + 200, db, [1, 9, 33, 70], frac=0.5, background=background)
    size = len(q)
    qo = dict(q)
    want = ko.winner_scoring(qo, db, summary, size)
    got = kf.KmerFinder(tdb, "winner").find_matches(q)
    assert got == want
    assert list(q.items()) == list(qo.items())          # the same k-mers deleted, order kept
    assert len(want) >= 4


def test_winner_scoring_exhausted_hits_raises_like_reference(kf):
    # no background: the winners consume every hit and getMatches throws
    db = make_db(7, 30, 400)
    summary = _summary(db)
    tdb = kf.TemplateDB(db, 16, summary)
    q = make_query(8, db, [2, 11], background=0.0)
    qo = dict(q)
    with pytest.raises(ko.NoHits) as e1:
        ko.winner_scoring(qo, db, summary, len(q))
    with pytest.raises(kf.NoHits) as e2:
        kf.KmerFinder(tdb, "winner").find_matches(q)
    assert str(e1.value) == str(e2.value) == "No hits were found! (nHits === 0)"
    assert list(q.items()) == list(qo.items())


def test_max_hits_and_no_hits(kf):
    db = make_db(9, 40, 400)
    summary = _summary(db)
    tdb = kf.TemplateDB(db, 16, summary)
    q = make_query(10, db, [4, 8, 15, 16, 23], frac=0.6)
    want = ko.winner_scoring(dict(q), db, summary, len(q), max_hits=2)
    assert kf.KmerFinder(tdb, "winner", max_hits=2).find_matches(dict(q)) == want and len(want) == 2
    miss = {km: 1 for km in kmer_strings(kmer_codes(np.random.default_rng(1), 50, 16, "CCCCC"), 16)}
    for method in ("winner", "standard"):
        with pytest.raises(kf.NoHits, match=r"^No hits were found!$"):
            kf.KmerFinder(tdb, method).find_matches(dict(miss))


@pytest.mark.parametrize("seed", [11, 12])
def test_standard_scoring_matches_oracle(kf, seed):
    db = make_db(seed, 50, 500)
    summary = _summary(db)
    tdb = kf.TemplateDB(db, 16, summary)
    q = make_query(seed + 300, db, [0, 25, 49])
    want = ko.standard_scoring(q, db, summary, len(q))
    got = kf.KmerFinder(tdb, "standard").find_matches(dict(q))
    assert got == want
    assert got[-1] is None and got[0] is not None


def test_db_edge_cases(kf):
    from kmerjs_amd._native import KmerError
    # duplicates inside a template count once; empty templates; k = 32; k = 1
    rng = np.random.default_rng(3)
    for k in (32, 1, 5):
        pool = kmer_strings(kmer_codes(rng, 300, k, ""), k)
        db = []
        for t in range(12):
            kms = [pool[i] for i in rng.integers(0, len(pool), size=0 if t == 5 else 60)]
            db.append({"sequence": "T%d" % t, "lengths": 100, "ulength": max(1, len(set(kms))), "species": "x",
                       "kmers": kms})
        tdb = kf.TemplateDB(db, k)
        q = {km: int(c) for km, c in zip(pool[::3], rng.integers(1, 9, size=len(pool[::3])))}
        tpls, hits = ko.first_round(dict(q), db, ko.build_index(db))
        got, w = _round1(kf, tdb, q)
        assert [db[t]["sequence"] for t, _, _ in got] == list(tpls.keys())
        assert [(u, s) for _, u, s in got] == [(v["uScore"], v["tScore"]) for v in tpls.values()]
        assert w.hits == hits
    with pytest.raises(KmerError) as e:
        kf.TemplateDB([{"sequence": "x", "lengths": 1, "ulength": 1, "species": "", "kmers": ["ACGN"]}], 4)
    assert e.value.status == 2
    # an empty query and an empty DB
    tdb = kf.TemplateDB(make_db(1, 3, 50), 16)
    got, w = _round1(kf, tdb, {})
    assert got == [] and w.hits == 0 and w.tmpl == 0xFFFFFFFF
    empty = kf.TemplateDB([], 16)
    got, w = _round1(kf, empty, {"ATGACAAAAAAAAAAA": 2})
    assert got == [] and w.hits == 0


def test_large_first_round_vs_numpy(kf):
    rng = np.random.default_rng(21)
    k, nt, per = 16, 400, 3000
    codes = [kmer_codes(rng, per, k) for _ in range(nt)]
    starts = np.zeros(nt + 1, dtype=np.uint64)
    starts[1:] = np.cumsum([len(c) for c in codes])
    allc = np.concatenate(codes)
    tix = np.repeat(np.arange(nt), [len(c) for c in codes])
    keys = "".join(kmer_strings(allc, k)).encode()
    meta = [{"sequence": "T%d" % i, "lengths": per * 2, "ulength": per, "species": ""} for i in range(nt)]
    tdb = kf.TemplateDB.from_arrays(k, keys, starts, meta, {"templates": nt, "totalLen": 0, "uniqueLens": nt * per})
    qc = np.unique(kmer_codes(rng, 300000, k))
    rng.shuffle(qc)
    qn = rng.integers(1, 100, size=len(qc)).astype(np.uint64)
    m = kf.Match(tdb, kmer_strings(qc, k), qn)
    got = m.templates()
    w = m.winner()
    m.close()
    pairs = np.unique(np.stack([allc, tix.astype(np.uint64)], 1), axis=0)
    u, t, first, hits = ko.numpy_first_round(qc, qn, pairs[:, 0], pairs[:, 1].astype(np.int64))
    order = sorted(np.nonzero(u)[0], key=lambda i: (first[i], i))
    assert [x[0] for x in got] == [int(i) for i in order]
    assert [(x[1], x[2]) for x in got] == [(int(u[i]), int(t[i])) for i in order]
    assert w.hits == hits


def test_device_result_query_equals_host_keys(kf):
    # the counter's device result joins without a host round trip
    from kmerjs_amd._native import Counter
    from oracle import oracle
    data = oracle.synth_fastq(5, 0, 20000)
    c = Counter(k=16, prefix=b"ATGAC")
    ents = c.count_buffer(data).entries()
    d_keys, d_cnt, _, n = c.result_device()
    assert n == len(ents)
    kms = [e[0].decode("latin-1") for e in ents][:: 7]
    db = [{"sequence": "T%d" % t, "lengths": 10, "ulength": len(kms[t::5]), "species": "", "kmers": kms[t::5]}
          for t in range(5)]
    tdb = kf.TemplateDB(db, 16)
    md = kf.Match(tdb, device_result=(d_keys, 16, d_cnt, n))
    mh = kf.Match(tdb, [e[0].decode("latin-1") for e in ents], [e[1] for e in ents])
    assert md.templates() == mh.templates()
    assert (md.winner().tmpl, md.winner().hits) == (mh.winner().tmpl, mh.winner().hits)
    md.close()
    mh.close()
    c.close()
