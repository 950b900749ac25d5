"""ctypes binding of libkmerhip.so (include/kmer_api.h).

The product path.  There is no CPU fallback: if the HIP library is missing
this module raises at import time, and every compute call goes to the GPU.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KMERHIP_LIB_EXPERIMENT") or os.path.join(HERE, "libkmerhip.so")   # (A/B builds only)

KMER_OK = 0
STATUS = {0: "ok", 1: "i/o error", 2: "bad parameter", 3: "out of memory", 4: "device error",
          5: "too many keys", 6: "non-ASCII input", 7: "line too long", 8: "bad call sequence"}
FLAG_TWO_PASS = 1
FLAG_NO_DENSE = 2
FLAG_BYTE_SCAN = 4
FLAG_SORT_FINISH = 8
FLAG_UNORDERED = 16
FLAG_TABLE_SPLIT_TEST = 32
FLAG_CANONICAL = 64
FLAG_LONG_LINES = 128
FLAG_FASTA = 1 << 16      # FASTA records (an extension; kmer_api.h)
FLAG_TABLE_FIXED_TEST = 1 << 17   # debug: table pass 1 always with fixed runs
FLAG_GEN_COLLIDE_TEST = 1 << 18   # debug: general-path merge takes the collision retry
TAB_PARTS = 1024    # table mode: pass-1 partitions (ownership unit across ranks)
WRITE_JSON = 0      # JSON.stringify(mapToJSON(map)), lib/kmers.js:46-54
WRITE_LEGACY = 1    # "{\nkey: count,...}\n", lib/index.js:381-388

# every symbol the header declares (tests/test_abi.py checks header <-> library)
EXPORTS = ["kmer_open", "kmer_close", "kmer_count_file", "kmer_count_buffer", "kmer_reset", "kmer_sync",
           "kmer_feed_device", "kmer_finish_device", "kmer_partial_device", "kmer_finish_merged",
           "kmer_exchange_prepare", "kmer_finish_exchanged", "kmer_merge_ordered",
           "kmer_records_export", "kmer_records_import", "kmer_records_clear", "kmer_result_device", "kmer_set_position",
           "kmer_lines", "kmer_result_size", "kmer_result_lines", "kmer_result_get",
           "kmer_result_arrays", "kmer_result_firsts", "kmer_result_write", "kmer_result_free",
           "kmer_synth_fastq_device",
           "kmer_last_timing", "kmer_phase_times", "kmer_table_stats", "kmer_table_digest", "kmer_table_routes", "kmer_table_device",
           "kmer_table_exchange_prepare", "kmer_table_finish_exchanged",
           "kmer_status_string", "kmer_last_error", "kmer_version"]
# include/kmer_match.h (the template matcher, same library)
MATCH_EXPORTS = ["kmer_db_open", "kmer_db_info", "kmer_db_close", "kmer_match_open", "kmer_match_open_device",
                 "kmer_match_info", "kmer_match_templates", "kmer_match_template_kmers", "kmer_match_winner", "kmer_match_remove",
                 "kmer_match_removed", "kmer_match_close", "kmer_match_last_error"]
EXPORTS = EXPORTS + MATCH_EXPORTS
ORDER_FIRST_HIT = 0    # kmer_match_templates: the Redis path's templates Map order
ORDER_DB = 1           # the Mongo aggregation's (DB) order


class Winner(ctypes.Structure):
    _fields_ = [("tmpl", ctypes.c_uint32), ("reserved", ctypes.c_uint32), ("uscore", ctypes.c_uint64),
                ("tscore", ctypes.c_uint64), ("hits", ctypes.c_uint64), ("first_uscore", ctypes.c_uint64),
                ("first_tscore", ctypes.c_uint64)]


class Params(ctypes.Structure):
    _fields_ = [("k", ctypes.c_uint32), ("step", ctypes.c_uint32),
                ("prefix", ctypes.c_char_p), ("prefix_len", ctypes.c_uint32),
                ("device", ctypes.c_int32), ("flags", ctypes.c_uint32),
                ("max_keys", ctypes.c_uint64), ("batch_bytes", ctypes.c_uint64),
                ("ndev", ctypes.c_uint32), ("devices", ctypes.POINTER(ctypes.c_int32)),
                ("progress", ctypes.c_void_p), ("progress_user", ctypes.c_void_p)]


# kmer_params.progress: void (*)(void *user, uint64_t done, uint64_t total)
PROGRESS_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64)


class KmerError(RuntimeError):
    def __init__(self, status, msg=""):
        super().__init__("%s: %s" % (STATUS.get(status, status), msg))
        self.status = status


def _load():
    # PyTorch-ROCm wheels bundle their own HIP runtime (libamdhip64.so, SONAME
    # libamdhip64.so.7).  Importing torch first makes the dynamic linker bind
    # libkmerhip.so to that same runtime, so one process never holds two HIP
    # runtimes (and device pointers from torch tensors are valid here).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError("libkmerhip.so not built (run `python -c 'import __graft_entry__ as g; g.build()'` "
                          "or `make -C kmerjs_amd/csrc`)")
    L = ctypes.CDLL(LIB_PATH)
    vp, u64, pu64 = ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)
    sig = {
        "kmer_open": (ctypes.c_int, [ctypes.POINTER(Params), ctypes.POINTER(vp)]),
        "kmer_close": (ctypes.c_int, [vp]),
        "kmer_count_file": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.POINTER(vp)]),
        "kmer_count_buffer": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(vp)]),
        "kmer_reset": (ctypes.c_int, [vp]),
        "kmer_sync": (ctypes.c_int, [vp]),
        "kmer_feed_device": (ctypes.c_int, [vp, vp, ctypes.c_size_t, vp]),
        "kmer_finish_device": (ctypes.c_int, [vp, ctypes.POINTER(vp)]),
        "kmer_partial_device": (ctypes.c_int, [vp, ctypes.POINTER(vp), ctypes.POINTER(vp), pu64]),
        "kmer_finish_merged": (ctypes.c_int, [vp, vp, vp, u64, u64, ctypes.POINTER(vp)]),
        "kmer_exchange_prepare": (ctypes.c_int, [vp, ctypes.c_uint32, ctypes.POINTER(vp), pu64]),
        "kmer_finish_exchanged": (ctypes.c_int, [vp, vp, u64, u64, vp, ctypes.POINTER(vp)]),
        "kmer_merge_ordered": (ctypes.c_int, [vp, vp, vp, vp, u64, u64, ctypes.POINTER(vp)]),
        "kmer_records_export": (ctypes.c_int, [vp, ctypes.POINTER(vp)]),
        "kmer_records_clear": (ctypes.c_int, [vp]),
        "kmer_records_import": (ctypes.c_int, [vp, ctypes.c_char_p, pu64, pu64, pu64, u64]),
        "kmer_result_device": (ctypes.c_int, [vp, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp), pu64]),
        "kmer_result_firsts": (ctypes.c_int, [vp, ctypes.POINTER(pu64)]),
        "kmer_set_position": (ctypes.c_int, [vp, u64, u64]),
        "kmer_lines": (ctypes.c_int, [vp, pu64]),
        "kmer_result_size": (u64, [vp]),
        "kmer_result_lines": (u64, [vp]),
        "kmer_result_get": (ctypes.c_int, [vp, u64, ctypes.POINTER(ctypes.c_char_p),
                                           ctypes.POINTER(ctypes.c_uint32), pu64]),
        "kmer_result_arrays": (ctypes.c_int, [vp, ctypes.POINTER(vp), ctypes.POINTER(pu64),
                                              ctypes.POINTER(pu64)]),
        "kmer_result_write": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_uint32]),
        "kmer_result_free": (None, [vp]),
        "kmer_synth_fastq_device": (ctypes.c_int, [vp, u64, u64, u64, vp]),
        "kmer_last_timing": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                            ctypes.POINTER(ctypes.c_double)]),
        "kmer_phase_times": (ctypes.c_int, [vp, ctypes.c_uint32, ctypes.POINTER(ctypes.c_char_p),
                                            ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint32)]),
        "kmer_table_stats": (ctypes.c_int, [vp, pu64, pu64, pu64]),
        "kmer_table_digest": (ctypes.c_int, [vp, pu64]),
        "kmer_table_routes": (ctypes.c_int, [vp, pu64, pu64, pu64, pu64]),
        "kmer_table_device": (ctypes.c_int, [vp, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp),
                                             ctypes.POINTER(vp), pu64]),
        "kmer_table_exchange_prepare": (ctypes.c_int, [vp, ctypes.c_uint32, ctypes.POINTER(vp), pu64, pu64]),
        "kmer_table_finish_exchanged": (ctypes.c_int, [vp, vp, u64, pu64, ctypes.c_uint32, ctypes.c_uint32, vp]),
        "kmer_status_string": (ctypes.c_char_p, [ctypes.c_int]),
        "kmer_last_error": (ctypes.c_char_p, [vp]),
        "kmer_version": (ctypes.c_char_p, []),
        "kmer_db_open": (ctypes.c_int, [ctypes.c_int32, ctypes.c_uint32, vp, u64, pu64, ctypes.c_uint32,
                                        ctypes.POINTER(vp)]),
        "kmer_db_info": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32), pu64,
                                        pu64]),
        "kmer_db_close": (ctypes.c_int, [vp]),
        "kmer_match_open": (ctypes.c_int, [vp, vp, pu64, pu64, u64, ctypes.POINTER(vp)]),
        "kmer_match_open_device": (ctypes.c_int, [vp, vp, ctypes.c_uint32, vp, u64, vp, ctypes.POINTER(vp)]),
        "kmer_match_info": (ctypes.c_int, [vp, pu64, ctypes.POINTER(ctypes.c_uint32)]),
        "kmer_match_templates": (ctypes.c_int, [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32),
                                                pu64, pu64, ctypes.POINTER(ctypes.c_uint32)]),
        "kmer_match_template_kmers": (ctypes.c_int, [vp, ctypes.c_uint32, u64, ctypes.POINTER(ctypes.c_uint32),
                                                     pu64]),
        "kmer_match_winner": (ctypes.c_int, [vp, ctypes.POINTER(Winner)]),
        "kmer_match_remove": (ctypes.c_int, [vp, ctypes.c_uint32, pu64]),
        "kmer_match_removed": (ctypes.c_int, [vp, vp]),
        "kmer_match_close": (ctypes.c_int, [vp]),
        "kmer_match_last_error": (ctypes.c_char_p, []),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


LIB = _load()


def version():
    return LIB.kmer_version().decode()


class Result:
    """Ordered (Map insertion order) result copied out of a kmer_result."""

    def __init__(self, handle):
        keys = ctypes.c_void_p()
        offs = ctypes.POINTER(ctypes.c_uint64)()
        cnts = ctypes.POINTER(ctypes.c_uint64)()
        n = LIB.kmer_result_size(handle)
        self.lines = LIB.kmer_result_lines(handle)
        LIB.kmer_result_arrays(handle, ctypes.byref(keys), ctypes.byref(offs), ctypes.byref(cnts))
        import numpy as np
        if n:
            firsts = ctypes.POINTER(ctypes.c_uint64)()
            LIB.kmer_result_firsts(handle, ctypes.byref(firsts))
            off = np.ctypeslib.as_array(offs, shape=(n + 1,)).copy()
            self.counts = np.ctypeslib.as_array(cnts, shape=(n,)).copy()
            self.firsts = np.ctypeslib.as_array(firsts, shape=(n,)).copy()
            nbytes = int(off[-1])
            # (ctypes.string_at takes a C int size: keys of > 2 GiB are copied through an array type)
            self.keybuf = ctypes.string_at(keys, nbytes) if nbytes < (1 << 31) else \
                (ctypes.c_char * nbytes).from_address(keys.value).raw
            self.offsets = off
        else:
            self.counts = np.zeros(0, dtype=np.uint64)
            self.firsts = np.zeros(0, dtype=np.uint64)
            self.keybuf = b""
            self.offsets = np.zeros(1, dtype=np.uint64)
        LIB.kmer_result_free(handle)

    def __len__(self):
        return len(self.counts)

    def keys(self):
        """[key_bytes] in first-occurrence order."""
        o = self.offsets.tolist()
        b = self.keybuf
        return [b[o[i]:o[i + 1]] for i in range(len(o) - 1)]

    def entries(self):
        """[(key_bytes, count)] in first-occurrence order."""
        o = self.offsets.tolist()
        c = self.counts.tolist()
        b = self.keybuf
        return [(b[o[i]:o[i + 1]], c[i]) for i in range(len(c))]


class Counter:
    """One kmer_ctx (device, configuration)."""

    def __init__(self, k=16, prefix=b"ATGAC", step=1, device=0, flags=0, max_keys=0, batch_bytes=0, devices=None,
                 progress=None):
        """devices: a list of HIP ordinals (ordinals may repeat) -> a multi-GPU
        group context: count_buffer / count_file shard the input over them and
        merge into one result (kmer_params.ndev).  progress(done, total): called
        after each input batch of count_file / count_buffer."""
        if isinstance(prefix, str):
            prefix = prefix.encode("latin-1")
        self._prefix = prefix
        p = Params(k=k, step=step, prefix=prefix, prefix_len=len(prefix), device=device, flags=flags,
                   max_keys=max_keys, batch_bytes=batch_bytes)
        if progress is not None:
            self._progress = PROGRESS_FN(lambda _u, done, total: progress(done, total))
            p.progress = ctypes.cast(self._progress, ctypes.c_void_p)
        if devices is not None and len(devices) > 1:
            self._devs = (ctypes.c_int32 * len(devices))(*devices)
            p.ndev = len(devices)
            p.devices = self._devs
        h = ctypes.c_void_p()
        st = LIB.kmer_open(ctypes.byref(p), ctypes.byref(h))
        if st != KMER_OK:
            raise KmerError(st, "kmer_open(k=%d, step=%d, prefix=%r)" % (k, step, prefix))
        self.h = h
        self.k, self.step = k, step

    def _check(self, st, what):
        if st != KMER_OK:
            raise KmerError(st, "%s: %s" % (what, LIB.kmer_last_error(self.h).decode()))

    def close(self):
        if self.h:
            LIB.kmer_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def count_buffer(self, data: bytes) -> Result:
        r = ctypes.c_void_p()
        self._check(LIB.kmer_count_buffer(self.h, data, len(data), ctypes.byref(r)), "count_buffer")
        return Result(r)

    def count_file(self, path, write=None, fmt=WRITE_JSON) -> Result:
        """Count a FASTQ file (plain or gzip).  write: also serialise the result
        to this path (natively, in Map order; fmt WRITE_JSON or WRITE_LEGACY)."""
        r = ctypes.c_void_p()
        self._check(LIB.kmer_count_file(self.h, os.fsencode(path), ctypes.byref(r)), "count_file")
        if write is not None:
            st = LIB.kmer_result_write(r, os.fsencode(write), fmt)
            if st != KMER_OK:
                LIB.kmer_result_free(r)
                raise KmerError(st, "kmer_result_write(%s)" % write)
        return Result(r)

    # ---- device-resident streaming ----
    def reset(self):
        self._check(LIB.kmer_reset(self.h), "reset")

    def sync(self):
        """Settle the chunk in flight (feed_device returns once it is queued)."""
        self._check(LIB.kmer_sync(self.h), "sync")

    def set_position(self, lines_before, byte_offset):
        self._check(LIB.kmer_set_position(self.h, lines_before, byte_offset), "set_position")

    def feed_device(self, ptr: int, nbytes: int, stream: int = 0):
        self._check(LIB.kmer_feed_device(self.h, ctypes.c_void_p(ptr), nbytes, ctypes.c_void_p(stream)),
                    "feed_device")

    def finish(self, want_result=True):
        r = ctypes.c_void_p()
        self._check(LIB.kmer_finish_device(self.h, ctypes.byref(r) if want_result else None), "finish")
        return Result(r) if want_result else None

    # ---- multi-GPU merge ----
    def partial_device(self):
        """(d_keys, d_vals, n): this session's unique packed keys (uint64[n]) and
        {first, count} pairs (uint64[n, 2]) in device memory."""
        k, v, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
        self._check(LIB.kmer_partial_device(self.h, ctypes.byref(k), ctypes.byref(v), ctypes.byref(n)),
                    "partial_device")
        return k.value or 0, v.value or 0, n.value

    def finish_merged(self, d_keys, d_vals, n, total_lines, want_result=True):
        r = ctypes.c_void_p()
        self._check(LIB.kmer_finish_merged(self.h, ctypes.c_void_p(d_keys), ctypes.c_void_p(d_vals), n, total_lines,
                                           ctypes.byref(r) if want_result else None), "finish_merged")
        return Result(r) if want_result else None

    def exchange_prepare(self, world):
        """(d_send, counts): this session's counting hits partitioned by owning
        rank (16-byte {order key, packed key} records, owner-major, each run in
        first-occurrence order) and the number of records per owner."""
        d = ctypes.c_void_p()
        cnt = (ctypes.c_uint64 * world)()
        self._check(LIB.kmer_exchange_prepare(self.h, world, ctypes.byref(d), cnt), "exchange_prepare")
        return d.value or 0, list(cnt)

    def finish_exchanged(self, d_recv, n, total_lines, stream=0, want_result=False):
        r = ctypes.c_void_p()
        self._check(LIB.kmer_finish_exchanged(self.h, ctypes.c_void_p(d_recv), n, total_lines, ctypes.c_void_p(stream),
                                              ctypes.byref(r) if want_result else None), "finish_exchanged")
        return Result(r) if want_result else None

    def merge_ordered(self, d_keys, d_counts, d_firsts, n, total_lines, want_result=False):
        """One Map-order result from gathered per-rank ordered lists (device
        pointers: n * k key bytes, uint64 counts, uint64 first-occurrence keys)."""
        r = ctypes.c_void_p()
        self._check(LIB.kmer_merge_ordered(self.h, ctypes.c_void_p(d_keys), ctypes.c_void_p(d_counts),
                                           ctypes.c_void_p(d_firsts), n, total_lines,
                                           ctypes.byref(r) if want_result else None), "merge_ordered")
        return Result(r) if want_result else None

    def records_export(self):
        """Host-side record keys (non-ACGT windows) as (keys, offsets, counts, firsts)."""
        r = ctypes.c_void_p()
        self._check(LIB.kmer_records_export(self.h, ctypes.byref(r)), "records_export")
        res = Result(r)
        return res.keybuf, res.offsets, res.counts, res.firsts

    def records_import(self, keybuf, offsets, counts, firsts):
        import numpy as np
        n = len(counts)
        if n == 0:
            return
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        cnt = np.ascontiguousarray(counts, dtype=np.uint64)
        fst = np.ascontiguousarray(firsts, dtype=np.uint64)
        P = ctypes.POINTER(ctypes.c_uint64)
        self._check(LIB.kmer_records_import(self.h, keybuf, off.ctypes.data_as(P), cnt.ctypes.data_as(P),
                                            fst.ctypes.data_as(P), n), "records_import")

    def records_clear(self):
        """Drop the host-side record keys (they were moved to another rank)."""
        self._check(LIB.kmer_records_clear(self.h), "records_clear")

    def result_device(self):
        """(d_keys, d_counts, d_firsts, n) of the last finish, in device memory."""
        k, c, f, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
        self._check(LIB.kmer_result_device(self.h, ctypes.byref(k), ctypes.byref(c), ctypes.byref(f),
                                           ctypes.byref(n)), "result_device")
        return k.value or 0, c.value or 0, f.value or 0, n.value

    def phase_times(self):
        """{phase: device ms since the last reset} (table mode: lines, hist1, scatter1, hist2, scatter2, final)."""
        names = (ctypes.c_char_p * 16)()
        ms = (ctypes.c_double * 16)()
        n = ctypes.c_uint32()
        self._check(LIB.kmer_phase_times(self.h, 16, names, ms, ctypes.byref(n)), "phase_times")
        return {names[i].decode(): ms[i] for i in range(min(n.value, 16))}

    def table_stats(self):
        """Table mode: (distinct canonical k-mers, distinct Map keys, sum of Map counts)."""
        a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        self._check(LIB.kmer_table_stats(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)), "table_stats")
        return a.value, b.value, c.value

    def table_digest(self):
        """kmer_table_digest: linear digest of the table (sum of count x mix(h))."""
        d = ctypes.c_uint64()
        self._check(LIB.kmer_table_digest(self.h, ctypes.byref(d)), "table_digest")
        return d.value

    def table_routes(self):
        """Table mode routes since the last reset: pass-1 chunks {fixed, merged, counted}, and
        finishes whose pass 2 ran with fixed bucket capacities (p2_fixed)."""
        a, b, c, d = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        self._check(LIB.kmer_table_routes(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c), ctypes.byref(d)),
                    "table_routes")
        return {"fixed": a.value, "merged": b.value, "counted": c.value, "p2_fixed": d.value}

    def table_device(self):
        """Table mode: (d_entries, d_bucket_start, d_bucket_len, d_big, n_big) in device memory."""
        e, st, ln, bg, nb = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
        self._check(LIB.kmer_table_device(self.h, ctypes.byref(e), ctypes.byref(st), ctypes.byref(ln),
                                          ctypes.byref(bg), ctypes.byref(nb)), "table_device")
        return e.value or 0, st.value or 0, ln.value or 0, bg.value or 0, nb.value

    def table_exchange_prepare(self, world):
        """Table mode across ranks: (d_send, counts, parts) -- this session's
        pass-1 keys as per-owner runs (uint64, owner-major), the keys per
        owner, and the keys per pass-1 partition (TAB_PARTS of them)."""
        d = ctypes.c_void_p()
        cnt = (ctypes.c_uint64 * world)()
        parts = (ctypes.c_uint64 * TAB_PARTS)()
        self._check(LIB.kmer_table_exchange_prepare(self.h, world, ctypes.byref(d), cnt, parts),
                    "table_exchange_prepare")
        return d.value or 0, list(cnt), list(parts)

    def table_finish_exchanged(self, d_recv, n, parts, world, rank, stream=0):
        """Pass 2 + final over the received keys (runs by source rank); parts =
        world x TAB_PARTS partition counts by source rank.  The table is
        written over d_recv: keep it alive until the next reset."""
        import numpy as np
        pa = np.ascontiguousarray(np.asarray(parts, dtype=np.uint64).reshape(-1))
        assert pa.size == world * TAB_PARTS
        self._check(LIB.kmer_table_finish_exchanged(self.h, ctypes.c_void_p(d_recv), n,
                                                    pa.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), world, rank,
                                                    ctypes.c_void_p(stream)), "table_finish_exchanged")

    def lines(self):
        n = ctypes.c_uint64()
        self._check(LIB.kmer_lines(self.h, ctypes.byref(n)), "lines")
        return n.value

    def last_timing(self, finish=True):
        """(scan_kernel_ms, feed_ms, finish_ms) device times since the last reset.
        finish=False: do not wait for a finish still running (finish_ms is None)."""
        a, b, c = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        self._check(LIB.kmer_last_timing(self.h, ctypes.byref(a), ctypes.byref(b),
                                         ctypes.byref(c) if finish else None), "last_timing")
        return a.value, b.value, (c.value if finish else None)


def synth_fastq_device(ptr: int, seed: int, first_read: int, n_reads: int, stream: int = 0):
    st = LIB.kmer_synth_fastq_device(ctypes.c_void_p(ptr), seed, first_read, n_reads, ctypes.c_void_p(stream))
    if st != KMER_OK:
        raise KmerError(st, "synth_fastq_device")
