"""ctypes front-end of the CPU restatement (oracle/kmer_oracle.c).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package (kmerjs_amd/).
"""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class _Res(ctypes.Structure):
    _fields_ = [("keys", ctypes.POINTER(ctypes.c_uint8)),
                ("key_off", ctypes.POINTER(ctypes.c_uint64)),
                ("key_len", ctypes.POINTER(ctypes.c_uint32)),
                ("counts", ctypes.POINTER(ctypes.c_uint64)),
                ("first", ctypes.POINTER(ctypes.c_uint64)),
                ("n", ctypes.c_uint64),
                ("lines", ctypes.c_uint64),
                ("windows", ctypes.c_uint64),
                ("seq_lines", ctypes.c_uint64),
                ("cap", ctypes.c_uint64), ("keys_cap", ctypes.c_uint64), ("keys_used", ctypes.c_uint64),
                ("slots", ctypes.c_void_p), ("slot_mask", ctypes.c_uint64),
                ("hashes", ctypes.c_void_p), ("ordinal", ctypes.c_uint64)]


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        for fn in ("oracle_count_buffer", "oracle_kmers_in_line", "oracle_count_fasta"):
            f = getattr(L, fn)
            f.restype = ctypes.c_int
            f.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                          ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(_Res)]
        L.oracle_free.argtypes = [ctypes.POINTER(_Res)]
        L.oracle_complement.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
        L.oracle_synth_fastq.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
        L.oracle_count_synth.restype = ctypes.c_int
        L.oracle_count_synth.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_char_p,
                                         ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(_Res)]
        L.oracle_table_digest_buffer.restype = ctypes.c_int
        L.oracle_table_digest_buffer.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32,
                                                 ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_table_digest_fasta.restype = ctypes.c_int
        L.oracle_table_digest_fasta.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32,
                                                ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_table_digest_synth.restype = ctypes.c_int
        L.oracle_table_digest_synth.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                                ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64),
                                                ctypes.POINTER(ctypes.c_uint64)]
        _LIB = L
    return _LIB


class OracleError(RuntimeError):
    pass


def _collect(r):
    keys = ctypes.string_at(r.keys, int(r.key_off[r.n - 1] + r.key_len[r.n - 1])) if r.n else b""
    out = []
    for i in range(r.n):
        o = r.key_off[i]
        out.append((keys[o:o + r.key_len[i]], int(r.counts[i])))
    return out


def count_buffer(data: bytes, prefix: bytes = b"ATGAC", k: int = 16, step: int = 1, stats=False, fasta=False):
    """Ordered [(key_bytes, count)] exactly as the reference's Map iteration.
    fasta: the FASTA-mode extension (oracle_count_fasta: records by '>'
    header, sequence lines joined; parity unpinned by the reference)."""
    r = _Res()
    fn = lib().oracle_count_fasta if fasta else lib().oracle_count_buffer
    st = fn(data, len(data), prefix, len(prefix), k, step, ctypes.byref(r))
    try:
        if st:
            raise OracleError("oracle status %d" % st)
        out = _collect(r)
        if stats:
            return out, {"lines": int(r.lines), "windows": int(r.windows), "seq_lines": int(r.seq_lines)}
        return out
    finally:
        lib().oracle_free(ctypes.byref(r))


def count_arrays(data: bytes, prefix: bytes = b"ATGAC", k: int = 16):
    """count_buffer (step 1) as numpy arrays, for large cases: keys (n, k)
    uint8 in Map order, counts uint64 (n,)."""
    import numpy as np
    r = _Res()
    st = lib().oracle_count_buffer(data, len(data), prefix, len(prefix), k, 1, ctypes.byref(r))
    try:
        if st:
            raise OracleError("oracle status %d" % st)
        n = int(r.n)
        if n == 0:
            return np.zeros((0, k), np.uint8), np.zeros(0, np.uint64)
        off = np.ctypeslib.as_array(r.key_off, shape=(n,))
        assert int(off[-1]) == (n - 1) * k, "step-1 keys are k bytes, back to back"
        keys = np.ctypeslib.as_array(r.keys, shape=(n * k,)).reshape(n, k).copy()
        return keys, np.ctypeslib.as_array(r.counts, shape=(n,)).copy()
    finally:
        lib().oracle_free(ctypes.byref(r))


def count_synth_arrays(seed: int, first_read: int, n_reads: int, prefix: bytes = b"ATGAC", k: int = 16):
    """readFile() over the synthetic reads [first_read, first_read + n_reads)
    (oracle_count_synth: generated and counted in blocks, no input copy), as
    numpy arrays in Map order: keys (n, k) uint8, counts, first-occurrence
    ordinals (monotone), lines."""
    import numpy as np
    r = _Res()
    st = lib().oracle_count_synth(seed, first_read, n_reads, prefix, len(prefix), k, 1, ctypes.byref(r))
    try:
        if st:
            raise OracleError("oracle status %d" % st)
        n = int(r.n)
        if n == 0:
            return np.zeros((0, k), np.uint8), np.zeros(0, np.uint64), np.zeros(0, np.uint64), int(r.lines)
        off = np.ctypeslib.as_array(r.key_off, shape=(n,))
        assert int(off[-1]) == (n - 1) * k, "step-1 keys are k bytes, back to back"
        keys = np.ctypeslib.as_array(r.keys, shape=(n * k,)).reshape(n, k).copy()
        return (keys, np.ctypeslib.as_array(r.counts, shape=(n,)).copy(),
                np.ctypeslib.as_array(r.first, shape=(n,)).copy(), int(r.lines))
    finally:
        lib().oracle_free(ctypes.byref(r))


def table_digest(data: bytes, k: int):
    """kmer_table_digest's definition, streamed over a buffer (no map):
    (digest, windows examined per strand)."""
    d, w = ctypes.c_uint64(), ctypes.c_uint64()
    st = lib().oracle_table_digest_buffer(data, len(data), k, ctypes.byref(d), ctypes.byref(w))
    if st:
        raise OracleError("oracle status %d" % st)
    return d.value, w.value


def table_digest_fasta(data: bytes, k: int):
    """table_digest over FASTA records (KMER_FLAG_FASTA: a record's lines
    joined): (digest, windows examined per strand)."""
    d, w = ctypes.c_uint64(), ctypes.c_uint64()
    st = lib().oracle_table_digest_fasta(data, len(data), k, ctypes.byref(d), ctypes.byref(w))
    if st:
        raise OracleError("oracle status %d" % st)
    return d.value, w.value


def table_digest_synth(seed: int, first_read: int, n_reads: int, k: int, threads: int = 1):
    """table_digest of the synthetic reads [first_read, first_read + n_reads)
    on `threads` host threads: (digest, windows per strand)."""
    d, w = ctypes.c_uint64(), ctypes.c_uint64()
    st = lib().oracle_table_digest_synth(seed, first_read, n_reads, k, threads, ctypes.byref(d), ctypes.byref(w))
    if st:
        raise OracleError("oracle status %d" % st)
    return d.value, w.value


def kmers_in_line(line: bytes, prefix: bytes = b"ATGAC", k: int = 16, step: int = 1):
    r = _Res()
    st = lib().oracle_kmers_in_line(line, len(line), prefix, len(prefix), k, step, ctypes.byref(r))
    try:
        if st:
            raise OracleError("oracle status %d" % st)
        return _collect(r)
    finally:
        lib().oracle_free(ctypes.byref(r))


def complement(s: bytes) -> bytes:
    out = ctypes.create_string_buffer(len(s))
    lib().oracle_complement(s, len(s), out)
    return out.raw


def synth_fastq(seed: int, first_read: int, n_reads: int) -> bytes:
    buf = ctypes.create_string_buffer(317 * n_reads)
    lib().oracle_synth_fastq(seed, first_read, n_reads, buf)
    return buf.raw


def to_json(entries):
    """JSON.stringify([...map]) for ASCII keys (digest form of SURVEY.md App. C)."""
    import json
    return json.dumps([[k.decode("latin-1"), v] for k, v in entries], separators=(",", ":"), ensure_ascii=False)
