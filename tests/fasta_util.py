"""FASTA inputs for the FASTA-mode tests (KMER_FLAG_FASTA, an extension whose
parity is UNPINNED by the reference: it has no FASTA parser,
test/kmers.js:53-61, test/kmerFinderServer.js:158).  The checker is
oracle_count_fasta (oracle/kmer_oracle.c) and, for it, the small pure-Python
restatement below."""
import numpy as np


def make_fasta(seed, n_records=60, max_len=3000, width=None, crlf=False, headerless=False, exotic=0.0,
               blank=0.0, tail_newline=True):
    """Records with random sequence lengths wrapped at `width` (random widths
    when None), optional CRLF line ends, blank lines, N / lowercase bytes, a
    headerless first record, empty records, an unterminated last line."""
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    out = []
    eol = b"\r\n" if crlf else b"\n"
    for r in range(n_records):
        if r > 0 or not headerless:
            out.append(b">rec%d some description|x=%d" % (r, rng.integers(0, 1 << 30)) + eol)
        L = int(rng.integers(0, max_len + 1)) if rng.random() > 0.05 else int(rng.integers(0, 3))
        seq = acgt[rng.integers(0, 4, L)].copy()
        if exotic:
            m = rng.random(L) < exotic
            seq[m] = np.frombuffer(b"NnXa", dtype=np.uint8)[rng.integers(0, 4, int(m.sum()))]
        seq = seq.tobytes()
        w = width or int(rng.choice([1, 7, 60, 61, 70, 80, 1000]))
        for i in range(0, len(seq), w):
            out.append(seq[i:i + w] + eol)
            if blank and rng.random() < blank:
                out.append(eol)
    data = b"".join(out)
    if not tail_newline:
        data = data.rstrip(b"\r\n")
    return data


def fasta_reference_py(data, prefix, k, step=1):
    """Pure-Python restatement of oracle_count_fasta (small cases only)."""
    def comp(s):
        t = bytes.maketrans(b"ACGT", b"TGCA")
        return s.translate(t)[::-1]

    m = {}

    def kmers(t):
        L = len(t)
        if L < k:
            return
        ini = 0
        for _ in range(L - k + 1):
            key = t[min(ini, L):min(ini + k, L)]
            if key.startswith(prefix):
                m[key] = m.get(key, 0) + 1
            ini += step

    lines = data.split(b"\n")
    if lines and lines[-1] == b"":
        lines = lines[:-1]
    seq = []

    def flush():
        s = b"".join(seq)
        if len(s) > 1:
            kmers(s)
            kmers(comp(s))

    for ln in lines:
        if ln.endswith(b"\r"):
            ln = ln[:-1]
        if ln.startswith(b">"):
            flush()
            seq = []
        else:
            seq.append(ln)
    flush()
    return list(m.items()), len(lines)
