// kmer_feed.hip — chunk feeds: device buffers, the packed path's chunk launch and settle,
// the line-array paths (general, dense hits), the FASTA rewrite, feed / reset.
#include "kmer_host.hpp"

namespace kmerhip {

kmer_status ensure_tiles(kmer_ctx *c, uint64_t n_tiles) {
    if (n_tiles <= c->tile_cap) return KMER_OK;
    const uint64_t cap = std::max<uint64_t>(n_tiles, 1024);
    hipStream_t s = c->stream;
    if (c->mode == MODE_TABLE) {
        // (table mode keeps no per-tile state beyond the newline counts)
    } else if (c->mode == MODE_GENERAL || c->mode == MODE_WINDOWS) {
        HIPCHK(c, c->lb_cnt.ensure(cap, s));
        HIPCHK(c, c->lb_lnl.ensure(cap, s));
        HIPCHK(c, c->tp_cnt.ensure(cap, s));
        HIPCHK(c, c->tp_lnl.ensure(cap, s));
    } else {
        HIPCHK(c, c->tsum.ensure(cap, s));
        HIPCHK(c, c->tscan.ensure(cap, s));
        HIPCHK(c, c->bsum.ensure(cap / TSCAN_BLOCK + 2, s));
        HIPCHK(c, c->bscan.ensure(cap / TSCAN_BLOCK + 2, s));
        HIPCHK(c, c->hits.ensure(cap * HMAX, s));
        if (c->p.k > 32) HIPCHK(c, c->hits_hi.ensure(cap * HMAX, s));
    }
    c->tile_cap = cap;
    return KMER_OK;
}

// the overflow hit list (and, k > 32, its high code words)
kmer_status ensure_ovf(kmer_ctx *c, uint64_t n, hipStream_t s) {
    HIPCHK(c, c->ovf.ensure(n, s));
    if (c->p.k > 32) HIPCHK(c, c->ovf_hi.ensure(c->ovf.cap, s));
    return KMER_OK;
}

// Host -> device upload through the context's pinned arena (kmer_host.hpp):
// the caller's buffer may go out of scope as soon as this returns.
kmer_status upload(kmer_ctx *c, void *dst, const void *src, size_t n, hipStream_t s) {
    if (n == 0) return KMER_OK;
    const size_t need = (n + 255) & ~(size_t)255;
    if (c->up_used + need > c->up_cap || c->up_streams.size() >= 8) {
        for (hipStream_t us : c->up_streams) HIPCHK(c, hipStreamSynchronize(us));
        c->up_streams.clear();
        c->up_used = 0;
        if (need > c->up_cap) {
            if (c->up_p) HIPCHK(c, hipHostFree(c->up_p));
            c->up_p = nullptr;
            c->up_cap = 0;
            const size_t cap = std::max<size_t>(need, 4u << 20);
            HIPCHK(c, hipHostMalloc((void **)&c->up_p, cap, hipHostMallocDefault));
            c->up_cap = cap;
        }
    }
    uint8_t *h = c->up_p + c->up_used;
    memcpy(h, src, n);
    c->up_used += need;
    if (std::find(c->up_streams.begin(), c->up_streams.end(), s) == c->up_streams.end()) c->up_streams.push_back(s);
    HIPCHK(c, hipMemcpyAsync(dst, h, n, hipMemcpyHostToDevice, s));
    return KMER_OK;
}

kmer_status ensure_records(kmer_ctx *c, uint64_t n) {
    HIPCHK(c, c->recs.ensure(n, c->stream));
    HIPCHK(c, c->rec_keys.ensure(c->recs.cap * (uint64_t)c->p.k, c->stream));
    return KMER_OK;
}

// Pull the records of the chunk just processed to the host and fold them into
// the ordered host map (count, first occurrence).  Keys are gathered on the
// device (rc applied there) at a fixed stride of k bytes.
kmer_status drain_records(kmer_ctx *c, const uint8_t *d_data, uint64_t n, hipStream_t s) {
    if (n == 0) return KMER_OK;
    const uint64_t k = c->p.k;
    kmer_status st = ensure_records(c, n);
    if (st) return st;
    HIPCHK(c, launch_gather_records(c->recs.p, k, n, d_data, c->rec_keys.p, s));
    std::vector<Record> recs(n);
    std::vector<char> keys(n * k);
    HIPCHK(c, hipMemcpyAsync(recs.data(), c->recs.p, n * sizeof(Record), hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(keys.data(), c->rec_keys.p, n * k, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    std::string key;
    for (uint64_t i = 0; i < n; ++i) {
        key.assign(keys.data() + i * k, recs[i].len);
        auto it = c->exotic.find(key);
        if (it == c->exotic.end()) {
            c->exotic.emplace(key, Ent{1, recs[i].order});
        } else {
            it->second.count += 1;
            it->second.first = std::min(it->second.first, recs[i].order);
        }
    }
    return KMER_OK;
}

// Wait for the chunk tail (hit_overflow_kernel's last block) to publish the
// chunk's counters: spin on the sequence word it writes last to mapped host
// memory, instead of a stream-synchronize round trip.  The stream is polled
// now and then, so that a failed or finished stream ends the wait.
kmer_status wait_tail(kmer_ctx *c, uint64_t seq, hipStream_t qs) {
    volatile uint64_t *flag = c->h_tail + 9;
    for (uint32_t i = 1;; ++i) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) break;
        if ((i & 1023) == 0) {
            const hipError_t e = hipStreamQuery(qs);
            if (e == hipSuccess) {
                if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) break;
                return fail(c, KMER_E_DEVICE, "chunk counters were not published");
            }
            if (e != hipErrorNotReady) HIPCHK(c, e);
        }
        __builtin_ia32_pause();
    }
    memcpy(c->h_small, (const void *)c->h_tail, 8 * 8);
    return KMER_OK;
}

// Read the scan / feed kernel times of the last chunk (lazily: the chunk's
// host wait returns before its closing event).
kmer_status resolve_feed_timing(kmer_ctx *c) {
    if (!c->feed_timing_pending) return KMER_OK;
    float ms = 0.f, ms_all = 0.f;
    HIPCHK(c, hipEventSynchronize(c->ev4));
    HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
    HIPCHK(c, hipEventElapsedTime(&ms_all, c->ev0, c->ev4));
    c->scan_ms += ms;
    c->feed_ms += ms_all;
    c->feed_timing_pending = false;
    return KMER_OK;
}

// Apply a pending reset / set_position (and `extra` PREP_* work) on the device.
kmer_status flush_prep(kmer_ctx *c, hipStream_t s, uint32_t extra) {
    const uint32_t f = c->prep_flags | extra;
    if (!f) return KMER_OK;
    HIPCHK(c, launch_prep(c->d_pos, c->d_pos_saved, c->d_err, c->d_scal, f, c->prep_lines, s));
    c->prep_flags = 0;
    return KMER_OK;
}

kmer_status check_err(kmer_ctx *c, uint32_t e) {
    if (e & ERR_NONASCII) return fail(c, KMER_E_NONASCII, "input contains a byte >= 0x80 (non-ASCII)");
    if (e & ERR_LINE_TOO_LONG)
        return fail(c, KMER_E_LINE_TOO_LONG,
                    c->pbits == PBITS_DEFAULT ? "sequence line longer than 2^23 bytes (KMER_FLAG_LONG_LINES)"
                                              : "long-line mode: a line longer than 2^40 bytes or more than 2^23 lines");
    if (e & ERR_LOOKBACK_TIMEOUT) return fail(c, KMER_E_DEVICE, "tile look-back timed out");
    if (e & ERR_DENSE_RANK) return fail(c, KMER_E_DEVICE, "dense-hit path: rank slot past the counted hits");
    return KMER_OK;
}

// ---------------------------------------------------------------------------
// fast path feed
// ---------------------------------------------------------------------------
struct TileSumOp {
    __host__ __device__ TileSum operator()(const TileSum &x, const TileSum &y) const { return tile_sum_op(x, y); }
};

// Grow the session rank arrays (preserving the first `keep` entries).
kmer_status ensure_rank_arrays(kmer_ctx *c, uint64_t need, uint64_t keep, hipStream_t s) {
    if (need >= (1ull << 32)) return fail(c, KMER_E_TOO_MANY_KEYS, "more than 2^32 prefix hits in one session");
    if (c->narrow) HIPCHK(c, c->rkey32.ensure(need, s, true, keep));
    else HIPCHK(c, c->rkey.ensure(need, s, true, keep));
    if (c->wide) HIPCHK(c, c->rkeyh.ensure(need, s, true, keep));
    HIPCHK(c, c->rord.ensure(need, s, true, keep));
    HIPCHK(c, c->ridx.ensure(need, s, true, keep));
    return KMER_OK;
}

kmer_status ensure_cross(kmer_ctx *c, uint64_t need, hipStream_t s) {
    HIPCHK(c, c->xord.ensure(need, s, true, c->n_cross));
    HIPCHK(c, c->xkey.ensure(need, s, true, c->n_cross));
    HIPCHK(c, c->xslot.ensure(need, s, true, c->n_cross));
    if (c->wide) {
        HIPCHK(c, c->xkeyl.ensure(need, s, true, c->n_cross));
        HIPCHK(c, c->xkeyh.ensure(need, s, true, c->n_cross));
    }
    return KMER_OK;
}

// session arrays the hit kernels write (they move when grown)
void bind_hits(kmer_ctx *c, HitArgs &h) {
    h.rkey = c->rkey.p;
    h.rkey32 = c->narrow ? c->rkey32.p : nullptr;
    h.rord = c->rord.p;
    h.xord = c->xord.p;
    h.xkey = c->xkey.p;
    h.xslot = c->xslot.p;
    h.rkeyh = c->rkeyh.p;
    h.xkeyl = c->xkeyl.p;
    h.xkeyh = c->xkeyh.p;
    h.xbase = c->n_cross;
    h.xcap = c->xord.cap;
    uint64_t rcap = c->narrow ? c->rkey32.cap : c->rkey.cap;
    rcap = std::min<uint64_t>(rcap, c->rord.cap);
    if (c->wide) rcap = std::min<uint64_t>(rcap, c->rkeyh.cap);
    h.rcap = rcap;
}

// One attempt at the pending chunk: scan, tile scan, hit resolution and the
// chunk tail (position, counters -> mapped host memory), all on the stream.
kmer_status launch_chunk(kmer_ctx *c) {
    auto &p = c->pend;
    const hipStream_t s = p.s;
    HIPCHK(c, hipEventRecord(c->ev0, s));
    if (c->planes) HIPCHK(c, launch_scan_planes(p.a, c->pargs, s));
    else HIPCHK(c, launch_scan_tiles(p.a, s));
    HIPCHK(c, hipEventRecord(c->ev1, s));
    HIPCHK(c, launch_tile_reduce(c->tsum.p, p.n_tiles, c->bsum.p, s));
    if (p.n_blocks > TSCAN_INLINE_MAX) {
        TileSum zero;
        memset(&zero, 0, sizeof(zero));
        ROCPRIM_RUN(c, rocprim::exclusive_scan(t, b, c->bsum.p, c->bscan.p, zero, (size_t)p.n_blocks, TileSumOp(), s));
        HIPCHK(c, launch_tile_scan(c->tsum.p, p.n_tiles, c->bscan.p, true, p.init, c->tscan.p, s));
    } else {
        HIPCHK(c, launch_tile_scan(c->tsum.p, p.n_tiles, c->bsum.p, false, p.init, c->tscan.p, s));
    }
    p.h.seq = ++c->tail_seq;
    HIPCHK(c, launch_hits(p.h, s));          // (+ the chunk tail: position, counters -> h_tail)
    HIPCHK(c, hipEventRecord(c->ev4, s));
    if (s != c->stream) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev4, 0));   // later work follows the chunk
    c->feed_timing_pending = true;
    return KMER_OK;
}

// Launch one chunk on the packed path and return: the host does not wait
// for it.  settle() (called by the next use of the context) reads its tail,
// redoes it after an overflow and applies its counters, so a caller can
// queue work elsewhere -- e.g. another context's finish -- meanwhile.
kmer_status scan_feed(kmer_ctx *c, const uint8_t *d, uint64_t len, uint32_t n_tiles, hipStream_t s) {
    const bool packed = c->mode == MODE_PACKED;
    kmer_status st;
    // rank capacity for every hit this chunk can produce: its tile slots + the overflow list
    if (packed) {
        st = ensure_rank_arrays(c, c->n_hits + (uint64_t)n_tiles * HMAX + c->ovf.cap, c->n_hits, s);
        if (st) return st;
        st = ensure_cross(c, c->n_cross + std::max<uint64_t>(n_tiles / 4, 4096), s);
        if (st) return st;
    }
    auto &p = c->pend;
    ScanArgs &a = p.a;
    memset(&a, 0, sizeof(a));
    a.data = d;
    a.len = len;
    a.abs_offset = c->abs_offset;
    a.n_tiles = n_tiles;
    a.k = c->p.k;
    a.plen = (uint32_t)c->prefix.size();
    a.p4 = pack4(c->prefix);
    a.r4 = pack4(c->rprefix);
    a.pmask = a.plen >= 4 ? 0xFFFFFFFFu : ((1u << (8 * a.plen)) - 1u);
    a.PR = c->d_PR;
    a.tsum = c->tsum.p;
    a.hits = c->hits.p;
    a.ovf = c->ovf.p;
    a.ovf_count = c->d_ovf_count;
    a.ovf_cap = c->ovf.cap;
    a.err = c->d_err;
    a.ablate = KH_EXPERIMENTS ? (c->p.flags & KMERHIP_XFLAG_MASK) >> 8 : 0u;   // (experiments only)
    a.hits_hi = c->hits_hi.p;
    a.ovf_hi = c->ovf_hi.p;

    HitArgs &h = p.h;
    memset(&h, 0, sizeof(h));
    h.hits = c->hits.p;
    h.tsum = c->tsum.p;
    h.tscan = c->tscan.p;
    h.ovf = c->ovf.p;
    h.ovf_count = c->d_ovf_count;
    h.ovf_cap = c->ovf.cap;
    h.n_tiles = n_tiles;
    h.k = a.k;
    h.plen = a.plen;
    h.abs_offset = c->abs_offset;
    h.pos = c->d_pos;
    h.packed = packed;
    h.pbits = c->pbits;
    h.smask = (c->kbits >= 64) ? ~0ull : ((1ull << c->kbits) - 1ull);
    h.invalid_key = c->kbits >= 63 ? ~0ull : (1ull << c->kbits);
    h.hits_hi = c->hits_hi.p;
    h.ovf_hi = c->ovf_hi.p;
    h.wide = c->wide ? 1u : 0u;
    h.ablate = a.ablate;
    if (c->wide) {                               // (high word: kbits - 64 < 64 bits, then the invalid bit)
        h.smask_hi = (1ull << (c->kbits - 64)) - 1ull;
        h.invalid_key = 1ull << (c->kbits - 64);
    }
    h.out_base = c->n_hits;
    h.recs = c->recs.p;
    h.rec_count = c->d_rec_count;
    h.rec_cap = c->recs.cap;
    h.err = c->d_err;
    bind_hits(c, h);
    h.data = d;
    h.len = len;
    h.scal = c->d_scal;
    h.ticket = c->d_hticket;
    h.chunk_hits = c->d_chunk_hits;
    h.chunk_cross = c->d_xcount;
    h.ends_open = c->d_ends_open;
    h.host_out = c->d_tail;
    p.init.cnt = 0;
    p.init.nh = 0;
    p.init.nx = 0;
    p.init.lnl = c->abs_offset;
    p.n_tiles = n_tiles;
    p.n_blocks = (n_tiles + TSCAN_BLOCK - 1) / TSCAN_BLOCK;
    p.d = d;
    p.len = len;
    // the chunk runs on the caller's stream (the context's own for the C-ABI
    // feeds), after everything queued so far: no cross-stream event waits
    // between the previous finish, the chunk and its finish (C2: 1.009 ->
    // 0.981 ms per step; two sessions in rotation still overlap, one's finish
    // with the other's chunk).  KMERHIP_ONE_STREAM=0: the chunk on a separate
    // low-priority stream (A/B experiments)
    static const bool one_stream = [] {
        const char *e = exp_env("KMERHIP_ONE_STREAM");
        return !(e && strcmp(e, "0") == 0);
    }();
    p.s = one_stream ? s : c->sstream;
    if (p.s != s) {
        HIPCHK(c, hipEventRecord(c->evq, s));
        HIPCHK(c, hipStreamWaitEvent(p.s, c->evq, 0));
    }
    // prologue: pending reset / position, position snapshot, zeroed chunk counters
    st = resolve_feed_timing(c);
    if (st) return st;
    st = flush_prep(c, p.s, PREP_SAVE | PREP_ZERO);
    if (st) return st;
    p.active = true;
    c->abs_offset += len;
    return launch_chunk(c);
}

// Settle the pending chunk: wait for its tail (published to mapped host
// memory, no stream sync), check errors; after an overflow grow the lists
// and redo it from the saved position (hit placement is idempotent: rank
// slots are rewritten, lists restart at this chunk's base); then apply its
// hit / cross counts and drain its records.
kmer_status settle(kmer_ctx *c) {
    auto &p = c->pend;
    if (!p.active) return KMER_OK;
    p.active = false;                            // (an error abandons the chunk)
    const bool packed = c->mode == MODE_PACKED;
    const hipStream_t s = p.s;
    kmer_status st;
    for (int attempt = 0;; ++attempt) {
        st = wait_tail(c, p.h.seq, s);
        if (st) return st;
        const uint32_t e = (uint32_t)c->h_small[5];
        st = check_err(c, e);
        if (st) return st;
        if (!(e & (ERR_OVF_OVERFLOW | ERR_REC_OVERFLOW | ERR_CROSS_OVERFLOW))) break;
        if (attempt == 7) return fail(c, KMER_E_OOM, "hit lists kept overflowing");
        st = resolve_feed_timing(c);
        if (st) return st;
        HIPCHK(c, hipMemsetAsync(c->d_err, 0, 4, s));
        HIPCHK(c, hipMemcpyAsync(c->d_pos, c->d_pos_saved, sizeof(StreamPos), hipMemcpyDeviceToDevice, s));
        if (e & ERR_OVF_OVERFLOW) {
            st = ensure_ovf(c, c->h_small[1] + 1024, s);
            if (st) return st;
            p.a.ovf = c->ovf.p;
            p.h.ovf = c->ovf.p;
            p.a.ovf_hi = c->ovf_hi.p;
            p.h.ovf_hi = c->ovf_hi.p;
            p.a.ovf_cap = p.h.ovf_cap = c->ovf.cap;
            if (packed) {
                st = ensure_rank_arrays(c, c->n_hits + (uint64_t)p.n_tiles * HMAX + c->ovf.cap, c->n_hits, s);
                if (st) return st;
            }
        }
        if (e & ERR_CROSS_OVERFLOW) {
            st = ensure_cross(c, c->n_cross + c->h_small[2] + 1024, s);
            if (st) return st;
        }
        if (e & ERR_REC_OVERFLOW) {
            st = ensure_records(c, c->h_small[0] + 1024);
            if (st) return st;
            p.h.recs = c->recs.p;
            p.h.rec_cap = c->recs.cap;
        }
        bind_hits(c, p.h);
        HIPCHK(c, hipMemsetAsync(c->d_scal, 0, 3 * 8, s));   // rec, ovf, cross counts of this chunk
        st = launch_chunk(c);
        if (st) return st;
    }
    if (packed) {
        c->n_hits += c->h_small[3];
        c->n_cross += c->h_small[2];
        c->long_seg |= (c->h_small[5] & INFO_LONGSEG) != 0;
    }
    c->chunk_open = c->h_small[7] != 0;
    const uint64_t nrec = c->h_small[0];
    if (nrec) {
        st = drain_records(c, p.d, nrec, s);
        if (st) return st;
    }
    return KMER_OK;
}


// ---------------------------------------------------------------------------
// general path feed
// ---------------------------------------------------------------------------
// Two-pass prefixes (debug mode): per-tile aggregates -> host scan -> arrays.
kmer_status two_pass_prefix(kmer_ctx *c, const uint8_t *d, uint64_t len, uint32_t n_tiles, hipStream_t s) {
    HIPCHK(c, launch_tile_aggregate(d, len, n_tiles, c->tp_cnt.p, c->tp_lnl.p, c->d_err, s));
    std::vector<uint64_t> cnt(n_tiles), last(n_tiles);
    StreamPos pos;
    HIPCHK(c, hipMemcpyAsync(cnt.data(), c->tp_cnt.p, n_tiles * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(last.data(), c->tp_lnl.p, n_tiles * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(&pos, c->d_pos, sizeof(pos), hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    uint64_t lines = pos.lines, lnl = c->abs_offset;
    for (uint32_t t = 0; t < n_tiles; ++t) {
        const uint64_t tc = cnt[t], tl = last[t];
        cnt[t] = lines;
        last[t] = lnl;
        lines += tc;
        if (tl) lnl = c->abs_offset + tl;
    }
    pos.lines = lines;
    uint8_t lastb = '\n';
    HIPCHK(c, hipMemcpyAsync(&lastb, d + len - 1, 1, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    pos.ends_open = lastb != '\n';
    kmer_status st = upload(c, c->tp_cnt.p, cnt.data(), n_tiles * 8, s);
    if (!st) st = upload(c, c->tp_lnl.p, last.data(), n_tiles * 8, s);
    if (!st) st = upload(c, c->d_pos, &pos, sizeof(pos), s);
    if (st) return st;
    return KMER_OK;
}

kmer_status read_pos(kmer_ctx *c, StreamPos *pos);

// Sequence-line descriptors of a chunk (lines kernel: decoupled look-back, or
// the two-pass debug mode); *nlines = descriptors written.
kmer_status collect_lines(kmer_ctx *c, const uint8_t *d, uint64_t len, uint32_t n_tiles, hipStream_t s,
                          uint64_t *nlines_out) {
    const bool lookback = !(c->p.flags & KMER_FLAG_TWO_PASS);
    HIPCHK(c, c->lines.ensure(1 << 16, s));
    TileArgs a;
    memset(&a, 0, sizeof(a));
    a.data = d;
    a.len = len;
    a.n_tiles = n_tiles;
    a.k = c->p.k;
    a.plen = (uint32_t)c->prefix.size();
    a.abs_offset = c->abs_offset;
    a.emit_lines = 1;
    a.lines_out = c->lines.p;
    a.line_count = c->d_line_count;
    a.line_cap = c->lines.cap;
    a.lb_cnt = c->lb_cnt.p;
    a.lb_lnl = c->lb_lnl.p;
    a.ticket = c->d_ticket;
    a.pos = c->d_pos;
    a.tp_cnt = c->tp_cnt.p;
    a.tp_lnl = c->tp_lnl.p;
    a.err = c->d_err;
    kmer_status st;
    HIPCHK(c, hipMemcpyAsync(c->d_pos_saved, c->d_pos, sizeof(StreamPos), hipMemcpyDeviceToDevice, s));
    for (int attempt = 0; attempt < 8; ++attempt) {
        HIPCHK(c, hipMemsetAsync(c->lb_cnt.p, 0, n_tiles * 8ull, s));
        HIPCHK(c, hipMemsetAsync(c->lb_lnl.p, 0, n_tiles * 8ull, s));
        HIPCHK(c, hipMemsetAsync(c->d_ticket, 0, 16, s));
        HIPCHK(c, hipMemsetAsync(c->d_line_count, 0, 8, s));
        if (!lookback) {
            st = two_pass_prefix(c, d, len, n_tiles, s);
            if (st) return st;
        }
        HIPCHK(c, hipEventRecord(c->ev0, s));
        HIPCHK(c, launch_lines(a, lookback, s));
        HIPCHK(c, hipEventRecord(c->ev1, s));
        HIPCHK(c, hipMemcpyAsync(c->h_small, c->d_scal, 8 * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        const uint32_t e = (uint32_t)c->h_small[5];
        st = check_err(c, e);
        if (st) return st;
        float ms = 0.f;
        HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
        c->scan_ms += ms;
        c->feed_ms += ms;
        if (e & ERR_LINE_OVERFLOW) {
            HIPCHK(c, hipMemsetAsync(c->d_err, 0, 4, s));
            HIPCHK(c, hipMemcpyAsync(c->d_pos, c->d_pos_saved, sizeof(StreamPos), hipMemcpyDeviceToDevice, s));
            HIPCHK(c, c->lines.ensure(c->h_small[6] + 1024, s));
            a.lines_out = c->lines.p;
            a.line_cap = c->lines.cap;
            continue;
        }
        break;
    }
    *nlines_out = c->h_small[6];
    return KMER_OK;
}

// General path with the device merge (step 1): the chunk's sequence lines
// (chunk_lines, as the dense path), the windows flattened over them
// (gen_windows_kernel), the accepted ones appended to the session's entries.
kmer_status general_feed_dev(kmer_ctx *c, const uint8_t *d, uint64_t len, uint32_t n_tiles, hipStream_t s) {
    const uint64_t li0 = c->host_lines;
    HIPCHK(c, hipEventRecord(c->ev0, s));
    uint64_t n_nl = 0, n_seq = 0;
    kmer_status st = chunk_lines(c, d, len, n_tiles, s, true, &n_nl, &n_seq);
    if (st) return st;
    uint64_t total = 0;
    if (n_seq) {
        HIPCHK(c, c->wbase.ensure(n_seq, s));
        ROCPRIM_RUN(c, rocprim::exclusive_scan(t, b, c->wcount.p, c->wbase.p, (uint64_t)0, (size_t)n_seq,
                                               rocprim::plus<uint64_t>(), s));
        HIPCHK(c, hipMemcpyAsync(c->h_small + 14, c->wbase.p + n_seq - 1, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(c->h_small + 15, c->wcount.p + n_seq - 1, 8, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(c, launch_pos_after(c->d_pos, li0 + n_nl, d, len, c->d_ends_open, s));
    HIPCHK(c, hipStreamSynchronize(s));
    if (n_seq) total = c->h_small[14] + c->h_small[15];
    c->host_lines = li0 + n_nl;
    uint64_t nrec = 0;
    if (total) {
        if (c->prefix.empty()) {                // (every window is a record)
            st = ensure_records(c, total);
            if (st) return st;
        }
        GenWinArgs w;
        memset(&w, 0, sizeof(w));
        w.data = d;
        w.len = len;
        w.lines = c->lines.p;
        w.wbase = c->wbase.p;
        w.tbase = c->tbase.p;
        w.first = (1u - (uint32_t)li0) & 3u;
        w.n_lines = n_seq;
        w.total = total;
        w.k = c->p.k;
        w.plen = (uint32_t)c->prefix.size();
        w.pbits = c->pbits;
        w.P = c->d_PR + 2 * KMAX_TILE;
        w.RP = w.P + c->prefix.size();
        w.err = c->d_err;
        // A/C/G/T prefix: candidates from the planes (gen_cand), then the
        // windows that fit their lines (gen_fix); else the flattened windows
        DBuf<Record> &out = c->gen_planes ? c->gcand : c->recs;
        for (int attempt = 0;; ++attempt) {
            w.recs = out.p;
            w.rec_count = c->d_rec_count;
            w.rec_cap = out.cap;
            HIPCHK(c, hipMemsetAsync(c->d_rec_count, 0, 8, s));
            if (c->gen_planes) HIPCHK(c, launch_gen_cand(w, c->pargs, s));
            else HIPCHK(c, launch_gen_windows(w, s));
            HIPCHK(c, hipMemcpyAsync(c->h_small, c->d_scal, 8 * 8, hipMemcpyDeviceToHost, s));
            HIPCHK(c, hipStreamSynchronize(s));
            const uint32_t e = (uint32_t)c->h_small[5];
            st = check_err(c, e);
            if (st) return st;
            if (!(e & ERR_REC_OVERFLOW)) break;
            if (attempt == 7) return fail(c, KMER_E_OOM, "record list kept overflowing");
            HIPCHK(c, hipMemsetAsync(c->d_err, 0, 4, s));
            if (c->gen_planes) HIPCHK(c, c->gcand.ensure(c->h_small[0] + 1024, s));
            else st = ensure_records(c, c->h_small[0] + 1024);
            if (st) return st;
        }
        nrec = c->h_small[0];
        if (c->gen_planes && nrec) {
            st = ensure_records(c, nrec);       // (records <= candidates: no overflow)
            if (st) return st;
            HIPCHK(c, hipMemsetAsync(c->d_rec_count, 0, 8, s));
            HIPCHK(c, launch_gen_fix(c->gcand.p, nrec, c->lines.p, w.k, w.plen, w.pbits, c->recs.p, c->d_rec_count,
                                     c->recs.cap, c->d_err, s));
            HIPCHK(c, hipMemcpyAsync(c->h_small, c->d_scal, 8 * 8, hipMemcpyDeviceToHost, s));
            HIPCHK(c, hipStreamSynchronize(s));
            st = check_err(c, (uint32_t)c->h_small[5]);
            if (st) return st;
            nrec = c->h_small[0];
        }
    }
    if (nrec) {
        st = general_append(c, d, nrec, s);
        if (st) return st;
    }
    HIPCHK(c, hipEventRecord(c->ev1, s));
    HIPCHK(c, hipEventSynchronize(c->ev1));
    float ms = 0.f;
    HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
    c->scan_ms += ms;
    c->feed_ms += ms;
    c->abs_offset += len;
    return KMER_OK;
}

kmer_status general_feed(kmer_ctx *c, const uint8_t *d, uint64_t len, uint32_t n_tiles, hipStream_t s) {
    if (c->gm_on) return general_feed_dev(c, d, len, n_tiles, s);
    uint64_t nlines = 0;
    kmer_status st = collect_lines(c, d, len, n_tiles, s, &nlines);
    if (st) return st;
    uint64_t nrec = 0;
    if (nlines) {
        WindowArgs w;
        memset(&w, 0, sizeof(w));
        w.data = d;
        w.lines = c->lines.p;
        w.n_lines = c->d_line_count;
        w.k = c->p.k;
        w.step = c->p.step;
        w.pbits = c->pbits;
        w.plen = (uint32_t)c->prefix.size();
        w.P = c->d_PR + 2 * KMAX_TILE;
        w.err = c->d_err;
        for (int attempt = 0; attempt < 8; ++attempt) {
            w.recs = c->recs.p;
            w.rec_count = c->d_rec_count;
            w.rec_cap = c->recs.cap;
            HIPCHK(c, hipMemsetAsync(c->d_rec_count, 0, 8, s));
            HIPCHK(c, hipEventRecord(c->ev0, s));
            HIPCHK(c, launch_windows(w, (uint32_t)std::min<uint64_t>(nlines, 65536), s));
            HIPCHK(c, hipEventRecord(c->ev1, s));
            HIPCHK(c, hipMemcpyAsync(c->h_small, c->d_scal, 8 * 8, hipMemcpyDeviceToHost, s));
            HIPCHK(c, hipStreamSynchronize(s));
            const uint32_t e = (uint32_t)c->h_small[5];
            st = check_err(c, e);
            if (st) return st;
            float ms = 0.f;
            HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
            c->feed_ms += ms;
            if (e & ERR_REC_OVERFLOW) {
                HIPCHK(c, hipMemsetAsync(c->d_err, 0, 4, s));
                st = ensure_records(c, c->h_small[0] + 1024);
                if (st) return st;
                continue;
            }
            break;
        }
        nrec = c->h_small[0];
    }
    if (nrec) {
        st = drain_records(c, d, nrec, s);
        if (st) return st;
    }
    c->abs_offset += len;
    return KMER_OK;
}

// Sequence lines of a chunk: newline positions (two streaming passes, no
// look-back), then one descriptor per sequence ordinal (c->lines, window
// counts in c->wcount).  check_len: lines whose windows exceed the order
// key's 2^23 positions are an error (ordered paths only).
kmer_status chunk_lines(kmer_ctx *c, const uint8_t *d, uint64_t len, uint32_t n_tiles, hipStream_t s, bool check_len,
                        uint64_t *n_nl_out, uint64_t *n_seq_out) {
    const uint64_t li0 = c->host_lines;
    // one pass over the input: per-tile counts + positions in per-tile slots
    // (KMERHIP_NL=two: the count pass + a second, writing pass; A/B experiments)
    static const bool two = [] {
        const char *e = exp_env("KMERHIP_NL");
        return e && strcmp(e, "two") == 0;
    }();
    HIPCHK(c, c->tcount.ensure(n_tiles, s));
    HIPCHK(c, c->tbase.ensure(n_tiles, s));
    if (two) {
        HIPCHK(c, launch_nl_count(d, len, n_tiles, c->tcount.p, c->d_err, s));
    } else {
        HIPCHK(c, c->nlslots.ensure((uint64_t)n_tiles * NL_SLOTS, s));
        HIPCHK(c, launch_nl_slots(d, len, n_tiles, NL_SLOTS, c->nlslots.p, c->tcount.p, c->d_err, s));
    }
    ROCPRIM_RUN(c, rocprim::exclusive_scan(t, b, c->tcount.p, c->tbase.p, (uint64_t)0, (size_t)n_tiles,
                                           rocprim::plus<uint64_t>(), s));
    HIPCHK(c, hipMemcpyAsync(c->h_small + 14, c->tbase.p + n_tiles - 1, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(c->h_small + 15, c->tcount.p + n_tiles - 1, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(c->h_small, c->d_scal, 8 * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    const uint32_t e = (uint32_t)c->h_small[5];
    kmer_status st = check_err(c, e);
    if (st) return st;
    const bool slots = !two && !(e & ERR_LINE_OVERFLOW);
    if (e & ERR_LINE_OVERFLOW)                   // (short lines: two passes; other bits kept)
        HIPCHK(c, hipMemsetD32Async((hipDeviceptr_t)c->d_err, (int)(e & ~ERR_LINE_OVERFLOW), 1, s));
    const uint64_t n_nl = c->h_small[14] + (uint32_t)c->h_small[15];
    if (!slots) {
        HIPCHK(c, c->nlpos.ensure(n_nl + 1, s));
        HIPCHK(c, launch_nl_write(d, len, n_tiles, c->tbase.p, c->nlpos.p, s));
    }
    const uint64_t first = (1u - (uint32_t)li0) & 3u;
    const uint64_t n_seq = n_nl >= first ? (n_nl - first) / 4 + 1 : 0;
    if (n_seq) {
        HIPCHK(c, c->lines.ensure(n_seq, s));
        HIPCHK(c, c->wcount.ensure(n_seq, s));
        unsigned int *lerr = check_len ? c->d_err : nullptr;
        const uint64_t maxrel = (1ull << c->pbits) - 1ull;
        if (slots) {
            HIPCHK(c, launch_seq_lines_slots(c->nlslots.p, c->tcount.p, c->tbase.p, n_tiles, NL_SLOTS, len, li0, first,
                                             n_nl, n_seq, c->p.k, c->p.step, c->lines.p, c->wcount.p, lerr, maxrel,
                                             s));
        } else {
            HIPCHK(c, launch_seq_lines(c->nlpos.p, n_nl, len, li0, n_seq, c->p.k, c->p.step, c->lines.p,
                                       c->wcount.p, lerr, maxrel, s));
        }
    }
    *n_nl_out = n_nl;
    *n_seq_out = n_seq;
    return KMER_OK;
}

// Dense-hit path, step 1, k <= 64 (kmer_dense.hip): a count pass over the
// lines, a scan of the per-line counts, then the accepted windows written at
// their rank slots -- the rank arrays hold only accepted windows.
kmer_status dense_windows_feed(kmer_ctx *c, const uint8_t *d, uint64_t len, uint64_t n_seq, uint64_t n_nl,
                               uint64_t li0, hipStream_t s) {
    DenseArgs g;
    memset(&g, 0, sizeof(g));
    g.data = d;
    g.len = len;
    g.lines = c->lines.p;
    g.n_lines = n_seq;
    g.lpw = std::max<uint64_t>(1, (n_seq + (1u << 17) - 1) >> 17);   // (<= 128 K waves)
    g.k = c->p.k;
    g.plen = (uint32_t)c->prefix.size();
    g.pbits = c->pbits;
    auto code = [](char ch) -> uint64_t { return ch == 'A' ? 0u : ch == 'C' ? 1u : ch == 'G' ? 2u : 3u; };
    for (char ch : c->prefix) g.pcode = (g.pcode << 2) | code(ch);
    g.smask = (c->kbits >= 64) ? ~0ull : ((1ull << c->kbits) - 1ull);
    g.smask_hi = c->kbits <= 64 ? 0ull : c->kbits >= 128 ? ~0ull : ((1ull << (c->kbits - 64)) - 1ull);
    g.P = c->d_PR + 2 * KMAX_TILE;
    g.RP = c->d_PR + 2 * KMAX_TILE + c->prefix.size();
    g.err = c->d_err;
    uint64_t total = 0;
    if (n_seq) {
        HIPCHK(c, c->dcnt.ensure(n_seq, s));
        HIPCHK(c, c->dtot.ensure(n_seq, s));
        HIPCHK(c, c->wbase.ensure(n_seq, s));
        g.cnt = c->dcnt.p;
        g.tot = c->dtot.p;
        HIPCHK(c, launch_dense_windows(g, false, s));
        ROCPRIM_RUN(c, rocprim::exclusive_scan(t, b, c->dtot.p, c->wbase.p, (uint64_t)0, (size_t)n_seq,
                                               rocprim::plus<uint64_t>(), s));
        HIPCHK(c, hipMemcpyAsync(c->h_small + 14, c->wbase.p + n_seq - 1, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(c->h_small + 15, c->dtot.p + n_seq - 1, 4, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(c, launch_pos_after(c->d_pos, li0 + n_nl, d, len, c->d_ends_open, s));
    HIPCHK(c, hipEventRecord(c->ev1, s));
    HIPCHK(c, hipStreamSynchronize(s));
    if (n_seq) total = c->h_small[14] + (uint32_t)c->h_small[15];
    c->host_lines = li0 + n_nl;
    {
        float ms = 0.f;
        HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
        c->scan_ms += ms;
        c->feed_ms += ms;
    }
    kmer_status st = ensure_rank_arrays(c, c->n_hits + total, c->n_hits, s);
    if (st) return st;
    HIPCHK(c, hipEventRecord(c->ev0, s));
    g.hbase = c->wbase.p;
    g.out_base = c->n_hits;
    g.out_end = c->n_hits + total;
    HIPCHK(c, c->ddbg.ensure(8, s));
    HIPCHK(c, hipMemsetAsync(c->ddbg.p, 0, 64, s));
    g.dbg = (unsigned long long *)c->ddbg.p;
    g.rkey = c->rkey.p;
    g.rkey32 = c->narrow ? c->rkey32.p : nullptr;
    g.rkeyh = c->wide ? c->rkeyh.p : nullptr;
    g.rord = c->rord.p;
    for (int attempt = 0; attempt < 8; ++attempt) {
        g.recs = c->recs.p;
        g.rec_count = c->d_rec_count;
        g.rec_cap = c->recs.cap;
        HIPCHK(c, hipMemsetAsync(c->d_rec_count, 0, 8, s));
        HIPCHK(c, launch_dense_windows(g, true, s));
        HIPCHK(c, hipEventRecord(c->ev1, s));
        HIPCHK(c, hipMemcpyAsync(c->h_small, c->d_scal, 8 * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        const uint32_t e = (uint32_t)c->h_small[5];
        if (e & ERR_DENSE_RANK) {                   // (a defect, reported with its context)
            uint64_t d[8];
            HIPCHK(c, hipMemcpy(d, c->ddbg.p, 64, hipMemcpyDeviceToHost));
            char msg[256];
            snprintf(msg, sizeof(msg),
                     "dense-hit path: rank slot past the counted hits (line %llu s %llu strand %llu counts %llx "
                     "rank %llu slot %llu end %llu, lines %llu lpw %llu)",
                     (unsigned long long)d[1], (unsigned long long)d[2], (unsigned long long)d[3],
                     (unsigned long long)d[4], (unsigned long long)d[5], (unsigned long long)d[6],
                     (unsigned long long)d[7], (unsigned long long)n_seq, (unsigned long long)g.lpw);
            return fail(c, KMER_E_DEVICE, msg);
        }
        st = check_err(c, e);
        if (st) return st;
        float ms = 0.f;
        HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
        c->feed_ms += ms;
        if (e & ERR_REC_OVERFLOW) {                 // (the redo writes the same slots)
            HIPCHK(c, hipMemsetAsync(c->d_err, 0, 4, s));
            st = ensure_records(c, c->h_small[0] + 1024);
            if (st) return st;
            continue;
        }
        break;
    }
    c->n_hits += total;
    c->chunk_open = c->h_small[7] != 0;
    const uint64_t nrec = c->h_small[0];
    if (nrec) {
        st = drain_records(c, d, nrec, s);
        if (st) return st;
    }
    c->abs_offset += len;
    return KMER_OK;
}

// Dense-hit path: every window of every sequence line goes to its rank slot
// (step > 1; no prefix, where every ACGT window is accepted and the count
// pass would only repeat the line lengths: k 21 / 4 M reads 78.1 vs 97.0 ms,
// C5 ordered 78.9 vs 95.4 ms, profiles/r06_ab/dense_*; and KMERHIP_DENSE=slots
// in experiment builds); with a prefix (step 1), and always past k = 32, only
// the accepted windows are ranked (dense_windows_feed: k 16 / AT 15.6 vs 33.3 ms).
kmer_status windows_feed(kmer_ctx *c, const uint8_t *d, uint64_t len, uint32_t n_tiles, hipStream_t s) {
    const uint64_t li0 = c->host_lines;
    kmer_status st;
    HIPCHK(c, hipEventRecord(c->ev0, s));
    uint64_t n_nl = 0, n_seq = 0;
    st = chunk_lines(c, d, len, n_tiles, s, true, &n_nl, &n_seq);
    if (st) return st;
    static const bool slots_only = [] {
        const char *e = exp_env("KMERHIP_DENSE");
        return e && strcmp(e, "slots") == 0;
    }();
    if (c->p.step == 1 && (c->p.k > (uint32_t)KMAX_DENSE || (!slots_only && !c->prefix.empty())))
        return dense_windows_feed(c, d, len, n_seq, n_nl, li0, s);
    c->win_slots = true;                          // (the finish compacts the rejected windows' slots away)
    uint64_t total = 0;
    if (n_seq) {
        HIPCHK(c, c->wbase.ensure(n_seq, s));
        ROCPRIM_RUN(c, rocprim::exclusive_scan(t, b, c->wcount.p, c->wbase.p, (uint64_t)0, (size_t)n_seq,
                                               rocprim::plus<uint64_t>(), s));
        HIPCHK(c, hipMemcpyAsync(c->h_small + 14, c->wbase.p + n_seq - 1, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(c->h_small + 15, c->wcount.p + n_seq - 1, 8, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(c, launch_pos_after(c->d_pos, li0 + n_nl, d, len, c->d_ends_open, s));
    HIPCHK(c, hipEventRecord(c->ev1, s));
    HIPCHK(c, hipStreamSynchronize(s));
    if (n_seq) total = c->h_small[14] + c->h_small[15];
    c->host_lines = li0 + n_nl;
    {
        float ms = 0.f;
        HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
        c->scan_ms += ms;
        c->feed_ms += ms;
    }
    st = ensure_rank_arrays(c, c->n_hits + total, c->n_hits, s);
    if (st) return st;
    HIPCHK(c, hipEventRecord(c->ev0, s));
    WinArgs w;
    memset(&w, 0, sizeof(w));
    w.data = d;
    w.len = len;
    w.lines = c->lines.p;
    w.n_lines = n_seq;
    w.li0 = li0;
    w.wbase = c->wbase.p;
    w.k = c->p.k;
    w.pbits = c->pbits;
    w.plen = (uint32_t)c->prefix.size();
    auto code = [](char ch) -> uint64_t { return ch == 'A' ? 0u : ch == 'C' ? 1u : ch == 'G' ? 2u : 3u; };
    for (char ch : c->prefix) w.pcode = (w.pcode << 2) | code(ch);
    for (char ch : c->rprefix) w.rcode = (w.rcode << 2) | code(ch);
    w.step = c->p.step;
    w.smask = (c->kbits >= 64) ? ~0ull : ((1ull << c->kbits) - 1ull);
    w.invalid_key = c->kbits >= 63 ? ~0ull : (1ull << c->kbits);
    w.out_base = c->n_hits;
    w.block_lines = total > 1024 * n_seq ? 1u : 0u;   // (> 512 windows per strand and line on average)
    w.rkey = c->rkey.p;
    w.rkey32 = c->narrow ? c->rkey32.p : nullptr;
    w.rord = c->rord.p;
    w.err = c->d_err;
    w.empty = (unsigned long long *)(c->d_scal + 10);
    w.P = c->d_P;
    for (int attempt = 0; attempt < 8; ++attempt) {
        w.recs = c->recs.p;
        w.rec_count = c->d_rec_count;
        w.rec_cap = c->recs.cap;
        HIPCHK(c, hipMemsetAsync(c->d_rec_count, 0, 8, s));
        HIPCHK(c, hipMemsetAsync(c->d_scal + 10, 0, 8, s));
        HIPCHK(c, hipMemsetAsync(c->d_scal + 11, 0xFF, 8, s));
        HIPCHK(c, launch_windows_packed(w, s));
        HIPCHK(c, hipEventRecord(c->ev1, s));
        HIPCHK(c, hipMemcpyAsync(c->h_small, c->d_scal, 8 * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(c->h_small + 18, c->d_scal + 10, 2 * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        const uint32_t e = (uint32_t)c->h_small[5];
        st = check_err(c, e);
        if (st) return st;
        float ms = 0.f;
        HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
        c->feed_ms += ms;
        if (e & ERR_REC_OVERFLOW) {                 // rank slots are rewritten by the redo
            HIPCHK(c, hipMemsetAsync(c->d_err, 0, 4, s));
            st = ensure_records(c, c->h_small[0] + 1024);
            if (st) return st;
            continue;
        }
        break;
    }
    c->n_hits += total;
    c->chunk_open = c->h_small[7] != 0;
    if (c->h_small[18]) {                        // step > 1, no prefix: the empty substrings' key ""
        auto it = c->exotic.find(std::string());
        if (it == c->exotic.end()) {
            c->exotic.emplace(std::string(), Ent{c->h_small[18], c->h_small[19]});
        } else {
            it->second.count += c->h_small[18];
            it->second.first = std::min(it->second.first, c->h_small[19]);
        }
    }
    const uint64_t nrec = c->h_small[0];
    if (nrec) {
        st = drain_records(c, d, nrec, s);
        if (st) return st;
    }
    c->abs_offset += len;
    return KMER_OK;
}


struct FaTileOp {
    __host__ __device__ FaTile operator()(const FaTile &a, const FaTile &b) const { return fa_tile_compose(a, b); }
};

// FASTA: rewrite the chunk [d, d + len) into FASTQ-shaped lines on the device
// (kmer_fasta.hip) -> *od, *olen; counts the chunk's input lines.  One host
// wait (the rewritten size).
kmer_status fasta_rewrite(kmer_ctx *c, const uint8_t *d, uint64_t len, hipStream_t s, const uint8_t **od,
                          uint64_t *olen) {
    const uint64_t nt64 = (len + TILE - 1) / TILE;
    if (nt64 > 0x7FFFFFFFull) return fail(c, KMER_E_BAD_PARAM, "chunk too large");
    const uint32_t n_tiles = (uint32_t)nt64;
    HIPCHK(c, c->fa_t.ensure(n_tiles + 1ull, s));
    HIPCHK(c, c->fa_x.ensure(n_tiles + 1ull, s));
    HIPCHK(c, hipMemsetAsync(c->fa_t.p + n_tiles, 0, sizeof(FaTile), s));   // (the identity: the scan's total lands there)
    HIPCHK(c, hipEventRecord(c->fa_ev[0], s));
    HIPCHK(c, launch_fa_tiles(d, len, n_tiles, c->fa_t.p, s));
    FaTile id;
    memset(&id, 0, sizeof(id));
    ROCPRIM_RUN(c, rocprim::exclusive_scan(t, b, c->fa_t.p, c->fa_x.p, id, (size_t)n_tiles + 1, FaTileOp(), s));
    FaTile tot;
    uint8_t last = 0;
    HIPCHK(c, hipMemcpyAsync(&tot, c->fa_x.p + n_tiles, sizeof(FaTile), hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(&last, d + len - 1, 1, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    c->fa_flip ^= 1u;
    DBuf<uint8_t> &ob = c->fa_out[c->fa_flip];
    HIPCHK(c, ob.ensure(tot.c0 + 16, s));
    HIPCHK(c, launch_fa_write(d, len, n_tiles, c->fa_x.p, ob.p, s));
    HIPCHK(c, hipEventRecord(c->fa_ev[1], s));
    if (c->mode == MODE_TABLE) {             // (table_feed synchronises the stream before its own timing)
        HIPCHK(c, hipEventSynchronize(c->fa_ev[1]));
        c->t_ms[6] += ev_ms(c, c->fa_ev[0], c->fa_ev[1]);
    }
    c->fa_lines += tot.nl + (last != '\n' ? 1 : 0);
    *od = ob.p;
    *olen = tot.c0;
    return KMER_OK;
}

kmer_status feed(kmer_ctx *c, const uint8_t *d, uint64_t len, hipStream_t s) {
    kmer_status st0 = settle(c);
    if (st0) return st0;
    if (c->fasta && len) {
        st0 = fasta_rewrite(c, d, len, s, &d, &len);
        if (st0) return st0;
    }
    if (c->mode != MODE_PACKED && c->mode != MODE_TILE_REC) {
        kmer_status st = flush_prep(c, s, 0);
        if (st) return st;
    }
    if (len == 0) return KMER_OK;
    const uint64_t n_tiles64 = (len + TILE - 1) / TILE;
    if (n_tiles64 > 0x7FFFFFFFull) return fail(c, KMER_E_BAD_PARAM, "chunk too large");
    const uint32_t n_tiles = (uint32_t)n_tiles64;
    if (c->chunk_open)
        return fail(c, KMER_E_BAD_PARAM, "the previous chunk did not end with '\\n' (chunks must be cut at line ends)");
    kmer_status st = ensure_tiles(c, n_tiles);
    if (st) return st;
    if (c->mode == MODE_GENERAL) return general_feed(c, d, len, n_tiles, s);
    if (c->mode == MODE_WINDOWS) return windows_feed(c, d, len, n_tiles, s);
    if (c->mode == MODE_TABLE) return table_feed(c, d, len, n_tiles, s);
    return scan_feed(c, d, len, n_tiles, s);
}

// (device side deferred to the next feed's prologue kernel: flush_prep)
kmer_status reset(kmer_ctx *c) {
    (void)settle(c);                             // (a chunk abandoned by the reset: its errors do not matter)
    c->prep_flags = PREP_RESET;
    c->feed_timing_pending = false;
    c->exotic.clear();
    c->abs_offset = 0;
    c->n_hits = 0;
    c->n_cross = 0;
    c->host_lines = 0;
    c->fa_lines = 0;
    c->long_seg = false;
    c->chunk_open = false;
    c->out_pending = false;
    c->timing_pending = false;
    c->n_out = 0;
    c->t_keys = 0;
    c->t_fill = 0;
    c->win_slots = false;
    c->t_p1_fixed = c->t_p1_merged = c->t_p1_counted = 0;
    c->t_p2_fixed = 0;
    c->gm_n = 0;
    c->gm_last = 0;
    c->gm_merged = true;
    c->t_cbase.clear();
    c->t_coff.clear();
    c->t_done = false;
    c->t_ent = nullptr;
    for (double &x : c->t_ms) x = 0.0;
    c->scan_ms = c->feed_ms = c->finish_ms = 0.0;
    c->open_stream = true;
    return KMER_OK;
}


}  // namespace kmerhip
