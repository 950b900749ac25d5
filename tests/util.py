"""Test helpers shared by CPU and GPU tests (not the oracle)."""
import hashlib
import json


def js_stringify(entries):
    """JSON.stringify([...map]) for (key_bytes, count) pairs of ASCII keys."""
    return json.dumps([[k.decode("latin-1"), int(v)] for k, v in entries], separators=(",", ":"),
                      ensure_ascii=False)


def digest(entries):
    return hashlib.sha256(js_stringify(entries).encode("utf-8")).hexdigest()


def map_digest_arrays(keys, counts):
    """digest()[:16] of a Map given as arrays in Map order -- keys (n, k) uint8
    of JSON-plain bytes (A/C/G/T), counts (n,) -- without building the list
    of pairs (full-size results: millions of entries)."""
    h = hashlib.sha256()
    h.update(b"[")
    kb = keys.tobytes()
    k = keys.shape[1] if keys.ndim == 2 else 0
    for i, c in enumerate(counts.tolist()):
        h.update(b'%s["%s",%d]' % (b"," if i else b"", kb[i * k:(i + 1) * k], c))
    h.update(b"]")
    return h.hexdigest()[:16]


def fullsize_golden():
    """tests/golden/fullsize.json: the oracle's answers at the BASELINE
    workloads' full sizes (tests/golden/gen_fullsize.py)."""
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize.json")) as f:
        return json.load(f)


def first_diff(a, b):
    for i, (x, y) in enumerate(zip(a, b)):
        if x != y:
            return i, x, y
    if len(a) != len(b):
        i = min(len(a), len(b))
        return i, a[i] if i < len(a) else None, b[i] if i < len(b) else None
    return None


_MUL = 0x9E3779B97F4A7C15


def _digest_mix(h):
    """splitmix64 finalizer on uint64 numpy arrays (kmer_table_digest's weight)."""
    import numpy as np
    with np.errstate(over="ignore"):
        h = h ^ (h >> np.uint64(30))
        h = h * np.uint64(0xBF58476D1CE4E5B9)
        h = h ^ (h >> np.uint64(27))
        h = h * np.uint64(0x94D049BB133111EB)
        return h ^ (h >> np.uint64(31))


def planar_codes(keys, k):
    """(n, k) uint8 A/C/G/T keys -> (code, rc code): code = hi_plane << k | lo_plane,
    base i at bit i of each plane, A/C/G/T = (hi, lo) 00/01/10/11 (kmer_api.h)."""
    import numpy as np
    n = keys.shape[0]
    flo = np.zeros(n, np.uint64)
    fhi = np.zeros(n, np.uint64)
    rlo = np.zeros(n, np.uint64)
    rhi = np.zeros(n, np.uint64)
    for i in range(k):
        b = keys[:, i]
        lo = (((b >> 1) ^ (b >> 2)) & 1).astype(np.uint64)
        hi = ((b >> 2) & 1).astype(np.uint64)
        flo |= lo << np.uint64(i)
        fhi |= hi << np.uint64(i)
        rlo |= (lo ^ np.uint64(1)) << np.uint64(k - 1 - i)      # rc: reversed, complemented
        rhi |= (hi ^ np.uint64(1)) << np.uint64(k - 1 - i)
    return (fhi << np.uint64(k)) | flo, (rhi << np.uint64(k)) | rlo


def canonical_summary(keys, cnt, k):
    """From an oracle Map counted with an empty prefix, as arrays (keys (n, k)
    A/C/G/T uint8, counts): (classes, forward windows, kmer_table_digest) of
    the table -- each class {c, rc c} counted once per forward window: Map(c),
    or Map(c) / 2 for a palindrome."""
    import numpy as np
    cf, cr = planar_codes(keys, k)
    rep = cf <= cr
    w = np.where(cf == cr, cnt // np.uint64(2), cnt)[rep]
    with np.errstate(over="ignore"):
        h = cf[rep] * np.uint64(_MUL)
        dig = int((w * _digest_mix(h)).sum(dtype=np.uint64))
    return int(rep.sum()), int(w.sum()), dig


def table_digest_from_map(entries, k):
    """kmer_table_digest of the table that holds a Map counted with an empty
    prefix (entries: (key bytes, count), A/C/G/T keys only): the table counts
    each class {c, rc c} once per forward window, i.e. Map(c), or Map(c) / 2 for
    a palindrome; h = min(code) * 0x9E3779B97F4A7C15."""
    import numpy as np
    if not entries:
        return 0
    keys = np.frombuffer(b"".join(kk for kk, _ in entries), dtype=np.uint8).reshape(-1, k)
    cnt = np.array([v for _, v in entries], dtype=np.uint64)
    cf, cr = planar_codes(keys, k)
    rep = cf <= cr                       # the class's entry under its smaller code
    w = np.where(cf == cr, cnt // np.uint64(2), cnt)[rep]
    with np.errstate(over="ignore"):
        h = cf[rep] * np.uint64(_MUL)
        return int((w * _digest_mix(h)).sum(dtype=np.uint64))


def packed_sorted(keys, cnt):
    """Rows of (n, k) uint8 keys (k <= 32) with counts -> (A/C/G/T rows as
    2-bit codes, first base most significant -- byte order -- sorted, their
    counts, {other row bytes: count}).  For comparing large table results."""
    import numpy as np
    n, k = keys.shape
    lut = np.full(256, 255, np.uint8)
    lut[list(b"ACGT")] = np.arange(4, dtype=np.uint8)
    v = lut[keys]
    ok = (v != 255).all(axis=1)
    code = np.zeros(n, np.uint64)
    for i in range(k):
        code = (code << np.uint64(2)) | (v[:, i] & 3).astype(np.uint64)
    o = np.argsort(code[ok], kind="stable")
    other = {keys[i].tobytes(): int(cnt[i]) for i in np.nonzero(~ok)[0]}
    return code[ok][o], cnt[ok][o], other


def result_packed_sorted(res, k):
    """packed_sorted of a kmer result whose keys all have length k."""
    import numpy as np
    keys = np.frombuffer(res.keybuf, dtype=np.uint8).reshape(-1, k) if len(res) else np.zeros((0, k), np.uint8)
    return packed_sorted(keys, res.counts)


def same_packed(a, b):
    import numpy as np
    return np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2] == b[2]
