"""CPU restatement of kmerFinder's k-mer -> template matching (SURVEY.md §8f
row 3) -- TEST INFRASTRUCTURE ONLY: imported by tests/ and bench.py's
cpu_baseline leg, never by the product package (kmerjs_amd/).

What it restates (file:line in the reference tree):
* the template DB: a k-mer -> [template] index built from per-template k-mer
  lists (src/kmerPyToMongo.py:21-24, `list(set(...))` per k-mer: one entry per
  (k-mer, template)); each template carries sequence (its id), lengths,
  ulength, species (:36-42); a summary {templates, totalLen, uniqueLens}
  (test_data/summary.json; Redis hash 'Summary', lib/kmerFinderServer.js:712-727);
* 'winner' scoring (Redis): firstMatch -> findKmersMatchesRedis
  (lib/kmerFinderServer.js:171-226), findWinner / matchSummary / removeWinnerKmers
  / getMatches / loop (:736-849, :625-676, :684-709);
* 'standard' scoring (Mongo aggregation, :452-522, :857-874): every template
  with hits, in DB order, summarised and sorted by score;
* lib/stats.js zScore (:19-45) and fastp (:52-115) on bignumber.js 2.x
  (package.json:61 "^2.3.0"; absent from this image) as the reference
  configures it: lib/kmerFinderServer.js:7 runs BN.config({ROUNDING_MODE: 2})
  on the constructor lib/stats.js shares, so dividedBy and sqrt round to
  DECIMAL_PLACES = 20 with ROUND_CEIL (towards +infinity) and a bare round(dp)
  is a ceiling; plus / minus / times are exact, round(dp, 6) is half-even,
  toNumber parses the decimal string.  Restated here with exact Fractions.

Choices the reference leaves open (documented in DESIGN.md): the template list
of a k-mer is in ascending template (DB) order (the reference's is Redis list
order, set by the DB loader); Mongo's natural order is DB order.

Parity: the matching needs a live Redis / MongoDB and bignumber.js, neither of
which exists here, so it was not run against the reference: "parity unpinned"
against the reference itself; the GPU matcher is checked against this
restatement (tests/test_match_gpu.py).  numpy_first_round is a vectorised
restatement of round 1 for large cases, checked against the loop version.
"""
from fractions import Fraction
import math

DP = 20                                   # bignumber.js DECIMAL_PLACES
ETTA = Fraction(1, 10 ** 8)               # lib/stats.js:6
EVALUE = Fraction(5, 100)                 # lib/kmers.js:75 (new BN(0.05))
HALF = Fraction(1, 2)

# lib/stats.js:56-111: (z threshold, p)
FASTP = [("10.7016", "1e-26"), ("10.4862", "1e-25"), ("10.2663", "1e-24"), ("10.0416", "1e-23"),
         ("9.81197", "1e-22"), ("9.5769", "1e-21"), ("9.33604", "1e-20"), ("9.08895", "1e-19"),
         ("8.83511", "1e-18"), ("8.57394", "1e-17"), ("8.30479", "1e-16"), ("8.02686", "1e-15"),
         ("7.73926", "1e-14"), ("7.4409", "1e-13"), ("7.13051", "1e-12"), ("6.8065", "1e-11"),
         ("6.46695", "1e-10"), ("6.10941", "1e-9"), ("5.73073", "1e-8"), ("5.32672", "1e-7"),
         ("4.89164", "1e-6"), ("4.41717", "1e-5"), ("3.89059", "1e-4"), ("3.29053", "1e-3"),
         ("2.57583", "0.01"), ("1.95996", "0.05"), ("1.64485", "0.1")]
FASTP = [(Fraction(a), Fraction(b)) for a, b in FASTP]


class NoHits(Exception):
    """The reference's `throw new Error('No hits were found!...')`."""


# -- bignumber.js 2.x arithmetic ---------------------------------------------
def bn_round(x, dp, half_even=False):
    """round(dp, 6) when half_even, else ROUND_CEIL (the configured mode)."""
    s = 10 ** dp
    v = Fraction(x) * s
    if not half_even:
        return Fraction(math.ceil(v), s)
    neg = v < 0
    a = -v if neg else v
    fl = a.numerator // a.denominator
    rem = a - fl
    if rem > HALF or (rem == HALF and fl % 2 == 1):
        fl += 1
    return Fraction(-fl if neg else fl, s)


def bn_div(a, b):
    return bn_round(Fraction(a) / Fraction(b), DP)


def bn_sqrt(x):
    """sqrt rounded to 20 dp, ROUND_CEIL (x >= 0)."""
    y = Fraction(x) * 10 ** (2 * DP)
    t = math.isqrt(y.numerator // y.denominator)         # floor(sqrt(y))
    if t * t != y:                                         # not exact: round up
        t += 1
    return Fraction(t, 10 ** DP)


def to_number(x):
    return float(x)        # correctly rounded, like Number(decimal string)


def fastp(z):
    for thr, p in FASTP:
        if z > thr:
            return p
    return Fraction(1)


def zscore(r1, n1, r2, n2):
    """lib/stats.js:19-45."""
    p1 = bn_div(r1, n1) + ETTA
    p2 = bn_div(r2, n2) + ETTA
    p = bn_div(Fraction(r1) + r2, Fraction(n1) + n2 + ETTA)
    q = 1 - p
    square = bn_sqrt(p * q * (bn_div(1, Fraction(n1) + ETTA) + bn_div(1, Fraction(n2) + ETTA)) + ETTA)
    return bn_div(p1 - p2, square)


def match_summary(query_size, seq, match, first, hits, summary):
    """matchSummary (lib/kmerFinderServer.js:625-676): a list of (key, value)
    pairs (the reference's Map), or None when rejected."""
    u = match["uScore"]
    if not u > 0:
        return None
    z = zscore(u, match["ulength"], hits, summary["uniqueLens"])
    prob = fastp(z) * summary["templates"]
    if not EVALUE >= prob:
        return None
    qs = Fraction(query_size) + ETTA
    frac_q = bn_div(200 * u, qs)
    frac_d = bn_div(100 * u, Fraction(match["ulength"]) + ETTA)
    tot_q = bn_div(200 * first["uScore"], qs)
    tot_d = bn_div(100 * first["uScore"], Fraction(match["ulength"]) + ETTA)
    tot_cov = to_number(bn_round(bn_div(first["tScore"], match["lengths"]), 2, True))
    expected = bn_div(Fraction(hits) * match["ulength"], summary["uniqueLens"])
    return [("template", seq), ("score", u), ("expected", to_number(bn_round(expected, 0, True))),
            ("z", to_number(bn_round(z, 2))), ("probability", to_number(prob)),
            ("frac-q", to_number(bn_round(frac_q, 2, True))), ("frac-d", to_number(bn_round(frac_d, 2, True))),
            ("depth", to_number(bn_round(bn_div(match["tScore"], match["lengths"]), 2, True))),
            ("kmers-template", match["ulength"]), ("total-frac-q", to_number(bn_round(tot_q, 2, True))),
            ("total-frac-d", to_number(bn_round(tot_d, 2, True))), ("total-temp-cover", tot_cov),
            ("species", match["species"])]


# -- the DB --------------------------------------------------------------------
def build_index(templates):
    """templates: [{'sequence', 'lengths', 'ulength', 'species', 'kmers': [str]}]
    -> {kmer: [template index, ascending, unique]} (src/kmerPyToMongo.py:21-24)."""
    idx = {}
    for ti, t in enumerate(templates):
        for km in t["kmers"]:
            lst = idx.setdefault(km, [])
            if not lst or lst[-1] != ti:
                lst.append(ti)
    return idx


def _new_template(t, cov, kmer):
    return {"tScore": cov, "uScore": 1, "lengths": t["lengths"], "ulength": t["ulength"], "species": t["species"],
            "kmers": {kmer: None}}


def first_round(query, templates, index):
    """findKmersMatchesRedis (lib/kmerFinderServer.js:171-226): query = ordered
    dict kmer -> count.  Returns (templates by name in first-hit order, hits)."""
    out = {}
    hits = 0
    for kmer in list(query.keys()):
        lst = index.get(kmer, [])
        hits += len(lst)
        cov = query[kmer]
        for ti in lst:
            name = templates[ti]["sequence"]
            s = out.get(name)
            if s is not None:
                s["tScore"] += cov
                s["uScore"] += 1
                s["kmers"][kmer] = None
            else:
                out[name] = _new_template(templates[ti], cov, kmer)
    if hits == 0:
        raise NoHits("No hits were found!")
    return out, hits


def get_matches(first, query):
    """getMatches (lib/kmerFinderServer.js:791-830); deletes hit-less entries of `first`."""
    out = {}
    hits = 0
    for name in list(first.keys()):
        hit = first[name]
        tpl = out.get(name)
        for kmer in hit["kmers"]:
            if kmer in query:
                cov = query[kmer]
                if tpl is not None:
                    tpl["tScore"] += cov
                    tpl["uScore"] += 1
                    tpl["kmers"][kmer] = None
                else:
                    out[name] = {"tScore": cov, "uScore": 1, "lengths": hit["lengths"], "ulength": hit["ulength"],
                                 "species": hit["species"], "kmers": {kmer: None}}
                    tpl = out[name]
        if tpl is not None:
            hits += len(tpl["kmers"])
        else:
            del first[name]
    if hits == 0:
        raise NoHits("No hits were found! (nHits === 0)")
    return out, hits


def winner_scoring(query, templates, summary, query_size, max_hits=100, index=None):
    """winnerScoring (lib/kmerFinderServer.js:736-849).  query: dict kmer ->
    count in Map order, MUTATED like the reference's kmerMap (winners' k-mers
    deleted).  Returns the list of winner summaries (lists of pairs)."""
    if index is None:
        index = build_index(templates)
    results = []
    state = {"first": None}

    def find_winner(tpls, hits):
        items = sorted(tpls.items(), key=lambda kv: -kv[1]["uScore"])      # stable (sortKmerMatches)
        if state["first"] is None:
            state["first"] = tpls
        seq, match = items[0]
        w = match_summary(query_size, seq, match, state["first"][seq], hits, summary)
        if w is not None and EVALUE >= Fraction(repr(dict(w)["probability"])):
            results.append(w)
            return match["kmers"]
        return None

    def remove(kms):
        if kms is None:
            return False
        for km in kms:
            query.pop(km, None)
        return True

    tpls, hits = first_round(query, templates, index)
    going = remove(find_winner(tpls, hits))
    while going and len(results) < max_hits:
        tpls, hits = get_matches(state["first"], query)
        going = remove(find_winner(tpls, hits))
    if not results:
        raise NoHits("No hits were found! (kmerResults.length === 0)")
    return results


def standard_scoring(query, templates, summary, query_size):
    """standardScoring (lib/kmerFinderServer.js:857-874) over the Mongo
    aggregation (:452-522): templates with hits in DB order, each template's
    matched k-mers in its own k-mer order; summaries sorted by score (stable),
    rejected templates (None, JS `undefined`) last."""
    tpls = {}
    hits = 0
    for t in templates:
        filt = [km for km in dict.fromkeys(t["kmers"]) if km in query]
        hits += len(filt)
        for km in filt:
            s = tpls.get(t["sequence"])
            if s is not None:
                s["tScore"] += query[km]
                s["uScore"] += 1
            else:
                tpls[t["sequence"]] = {"tScore": query[km], "uScore": 1, "lengths": t["lengths"],
                                       "ulength": t["ulength"], "species": t["species"]}
    if hits == 0:
        raise NoHits("No hits were found!")
    out = [match_summary(query_size, seq, m, m, hits, summary) for seq, m in tpls.items()]
    kept = sorted([x for x in out if x is not None], key=lambda w: -dict(w)["score"])
    return kept + [None] * (len(out) - len(kept))


def numpy_first_round(q_codes, q_counts, t_codes, t_index):
    """Round-1 scores with numpy (large cases; CPU baseline): q_codes uint64[n]
    (query k-mers, one per Map key, -1 for keys that cannot match), q_counts,
    t_codes / t_index: the DB's (k-mer code, template) pairs, unique.
    Returns (uScore[n_t], tScore[n_t], first_hit_query[n_t], hits)."""
    import numpy as np
    n_t = int(t_index.max()) + 1 if t_index.size else 0
    order = np.argsort(q_codes, kind="stable")
    sq = q_codes[order]
    pos = np.searchsorted(sq, t_codes)
    pos_c = np.minimum(pos, max(sq.size - 1, 0))
    hit = (pos < sq.size) & (sq[pos_c] == t_codes) if sq.size else np.zeros(t_codes.size, bool)
    qi = order[pos_c[hit]]
    ti = t_index[hit]
    u = np.bincount(ti, minlength=n_t)
    t = np.bincount(ti, weights=q_counts[qi].astype(np.float64), minlength=n_t).astype(np.uint64)
    first = np.full(n_t, np.iinfo(np.int64).max, dtype=np.int64)
    np.minimum.at(first, ti, qi)
    return u, t, first, int(hit.sum())
