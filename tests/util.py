"""Test helpers shared by CPU and GPU tests (not the oracle)."""
import hashlib
import json


def js_stringify(entries):
    """JSON.stringify([...map]) for (key_bytes, count) pairs of ASCII keys."""
    return json.dumps([[k.decode("latin-1"), int(v)] for k, v in entries], separators=(",", ":"),
                      ensure_ascii=False)


def digest(entries):
    return hashlib.sha256(js_stringify(entries).encode("utf-8")).hexdigest()


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
    b = keys.astype(np.uint64)
    lo = ((b >> np.uint64(1)) ^ (b >> np.uint64(2))) & np.uint64(1)
    hi = (b >> np.uint64(2)) & np.uint64(1)
    w = np.uint64(1) << np.arange(k, dtype=np.uint64)
    wr = w[::-1]
    flo, fhi = (lo * w).sum(1), (hi * w).sum(1)
    rlo, rhi = ((np.uint64(1) - lo) * wr).sum(1), ((np.uint64(1) - hi) * wr).sum(1)
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
