"""CPU checks of the template matcher's host logic (no GPU): the product's
decimal statistics (kmerjs_amd/kmerfinder.py, bignumber.js 2.x semantics)
against the oracle's Fraction restatement, and the oracle's vectorised round 1
against its loop version."""
import random
from fractions import Fraction

import numpy as np

from oracle import kmerfinder_oracle as ko
from tests.match_util import make_db, make_query


def test_decimal_ops_match_fraction_restatement():
    from kmerjs_amd.kmerfinder import Dec
    rng = random.Random(5)
    for _ in range(3000):
        a = rng.randint(-10 ** 12, 10 ** 12)
        sa = rng.randint(0, 30)
        b = rng.randint(1, 10 ** 9) * rng.choice([1, -1])
        sb = rng.randint(0, 12)
        da, db = Dec(a, sa), Dec(b, sb)
        fa, fb = Fraction(a, 10 ** sa), Fraction(b, 10 ** sb)
        q = da.div(db)
        assert Fraction(q.n, 10 ** q.s) == ko.bn_div(fa, fb)
        for dp in (0, 2, 5):
            for he in (False, True):
                r = da.round(dp, he)
                assert Fraction(r.n, 10 ** r.s) == ko.bn_round(fa, dp, he)
        x = abs(fa)
        s = Dec(abs(a), sa).sqrt()
        assert Fraction(s.n, 10 ** s.s) == ko.bn_sqrt(x)
        assert Dec(a, sa).to_number() == ko.to_number(fa)


def test_round_ties():
    from kmerjs_amd.kmerfinder import Dec
    assert Dec(125, 3).round(2, True).to_number() == 0.12         # half-even
    assert Dec(135, 3).round(2, True).to_number() == 0.14
    assert Dec(121, 3).round(2).to_number() == 0.13               # ROUND_CEIL (lib/kmerFinderServer.js:7)
    assert Dec(-129, 3).round(2).to_number() == -0.12             # towards +infinity
    assert Dec(2, 0).div(3).n == 66666666666666666667


def test_match_summary_matches_oracle():
    from kmerjs_amd.kmerfinder import match_summary
    rng = random.Random(9)
    summary = {"templates": 5030, "totalLen": 16525500, "uniqueLens": 8076292}   # test_data/summary.json
    seen = 0
    for _ in range(400):
        ul = rng.randint(1, 20000)
        u = rng.randint(1, ul)
        t = {"lengths": ul * 2 + rng.randint(0, 99), "ulength": ul, "species": "s"}
        ts = u * rng.randint(1, 9)
        fu, ft = u + rng.randint(0, 50), ts + rng.randint(0, 500)
        hits = u + rng.randint(0, 10 ** 6)
        qsize = rng.randint(u, 2 * 10 ** 6)
        got = match_summary(qsize, "NC_1", t, u, ts, fu, ft, hits, summary)
        m = dict(t, uScore=u, tScore=ts)
        want = ko.match_summary(qsize, "NC_1", m, {"uScore": fu, "tScore": ft}, hits, summary)
        assert got == want
        seen += got is not None
    assert seen > 50


def test_fastp_thresholds():
    from kmerjs_amd.kmerfinder import Dec, fastp
    for thr, p in ko.FASTP:
        z = Dec(thr.numerator * 10 ** 6 // thr.denominator, 6)      # thr exactly (<= 6 dp)
        nxt = fastp(z)
        assert Fraction(nxt.n, 10 ** nxt.s) == ko.fastp(Fraction(z.n, 10 ** z.s))
        up = fastp(z + Dec(1, 9))
        assert Fraction(up.n, 10 ** up.s) == p


def test_numpy_first_round_matches_loop():
    db = make_db(3, 24, 300)
    q = make_query(4, db, [2, 7, 11], extras=False)
    tpls, hits = ko.first_round(dict(q), db, ko.build_index(db))
    code = {c: i for i, c in enumerate("ACGT")}

    def enc(s):
        v = 0
        for ch in s:
            v = v * 4 + code[ch]
        return v
    qk = list(q.keys())
    qc = np.array([enc(x) for x in qk], dtype=np.uint64)
    qn = np.array([q[x] for x in qk], dtype=np.uint64)
    pairs = sorted({(enc(km), ti) for ti, t in enumerate(db) for km in t["kmers"]})
    tc = np.array([p[0] for p in pairs], dtype=np.uint64)
    ti = np.array([p[1] for p in pairs], dtype=np.int64)
    u, t, first, h = ko.numpy_first_round(qc, qn, tc, ti)
    assert h == hits
    order = [i for i in sorted(np.nonzero(u)[0], key=lambda i: (first[i], i))]
    assert [db[i]["sequence"] for i in order] == list(tpls.keys())
    for i in order:
        s = tpls[db[i]["sequence"]]
        assert (int(u[i]), int(t[i])) == (s["uScore"], s["tScore"])


def test_oracle_winner_loop_finds_present_templates():
    db = make_db(11, 40, 400)
    q = make_query(12, db, [5, 17, 30], frac=0.7)
    size = len(q)
    summary = {"templates": len(db), "totalLen": sum(t["lengths"] for t in db),
               "uniqueLens": sum(t["ulength"] for t in db)}
    res = ko.winner_scoring(q, db, summary, size)
    names = [dict(r)["template"] for r in res]
    assert set(names[:3]) == {"NC_000005", "NC_000017", "NC_000030"}, names
    assert len(q) < size
