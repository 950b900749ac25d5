// kmer_api.hip — host orchestration behind the C-ABI (include/kmer_api.h).
//
// One kmer_ctx = one device, one HIP stream, the device tables for one
// (k, preffix, step) configuration.  Input flows in chunks that start at a
// line start; every chunk is one launch of the single-pass tile kernel (or,
// for configurations the tile kernel does not cover, the line-list + window
// kernels).  finish() compacts the dense table, radix-sorts it by first
// occurrence (rocPRIM), decodes keys and merges the rare record keys, giving
// the reference Map's exact iteration order (lib/kmers.js:76,95).
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/kmer_api.h"
#include "kmer_internal.hpp"

using namespace kmerhip;

namespace {

enum Mode { MODE_DENSE, MODE_TILE_REC, MODE_GENERAL };

struct Ent {
    uint64_t count;
    uint64_t first;
};

}  // namespace

struct kmer_result {
    uint64_t lines = 0;
    std::vector<char> keys;
    std::vector<uint64_t> offsets{0};
    std::vector<uint64_t> counts;
};

struct kmer_ctx {
    kmer_params p{};
    std::string prefix, rprefix;
    Mode mode = MODE_GENERAL;
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;

    // dense table
    uint64_t n_dense = 0;
    unsigned long long *d_counts = nullptr, *d_first = nullptr;
    // look-back state
    uint64_t tile_cap = 0;
    unsigned long long *d_lb_cnt = nullptr, *d_lb_lnl = nullptr;
    uint64_t *d_tp_cnt = nullptr, *d_tp_lnl = nullptr;
    // streaming scan path: per-tile aggregates, their scans, hit slots
    uint64_t *d_agg_cnt = nullptr, *d_agg_lnl = nullptr, *d_cscan = nullptr, *d_lnl_before = nullptr;
    uint32_t *d_tile_nhits = nullptr;
    HitRec *d_hits = nullptr;
    HitRec *d_ovf = nullptr;
    uint64_t ovf_cap = 0;
    unsigned long long *d_ovf_count = nullptr;
    void *d_scan_tmp = nullptr;
    size_t scan_tmp_bytes = 0;
    // small device words
    unsigned int *d_ticket = nullptr, *d_err = nullptr;
    unsigned long long *d_rec_count = nullptr, *d_line_count = nullptr, *d_nout = nullptr;
    StreamPos *d_pos = nullptr, *d_pos_saved = nullptr;
    // records & lines
    uint64_t rec_cap = 0, line_cap = 0;
    Record *d_recs = nullptr;
    SeqLine *d_lines = nullptr;
    uint8_t *d_rec_keys = nullptr;
    uint64_t *d_rec_off = nullptr;
    // finish buffers (dense)
    uint64_t *d_order = nullptr, *d_order2 = nullptr, *d_idx = nullptr, *d_idx2 = nullptr;
    uint8_t *d_keys_out = nullptr;
    uint64_t *d_cnt_out = nullptr;
    uint8_t *d_P = nullptr;
    uint8_t *d_PR = nullptr;       // P[0..64) then rc(P)[0..64) (tile layout); long P copied after
    void *d_sort_tmp = nullptr;
    size_t sort_tmp_bytes = 0;
    uint64_t last_n = 0;
    // host side
    uint64_t abs_offset = 0;
    bool open_stream = false;      // reset called, not finished
    std::unordered_map<std::string, Ent> exotic;
    // pinned scratch
    uint64_t *h_small = nullptr;   // [0]=rec_count [1]=line_count [2]=err [3]=nout [4..7]=pos
    // batch staging for host input
    uint8_t *d_batch = nullptr;
    uint64_t batch_cap = 0;
    uint8_t *h_stage = nullptr;
    uint64_t stage_cap = 0;
    // timing
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr, ev3 = nullptr, ev4 = nullptr;
    double count_ms = 0.0, finish_ms = 0.0, feed_ms = 0.0;
};

namespace {

const uint64_t DEFAULT_BATCH = 1ull << 30;

#define HIPCHK(ctx, x)                                                                      \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            (ctx)->err = std::string("HIP error: ") + hipGetErrorString(e_) + " at " #x;    \
            return KMER_E_DEVICE;                                                           \
        }                                                                                   \
    } while (0)

kmer_status fail(kmer_ctx *c, kmer_status s, const std::string &msg) {
    c->err = msg;
    return s;
}

uint8_t comp(uint8_t c) {
    switch (c) {
    case 'A': return 'T';
    case 'T': return 'A';
    case 'G': return 'C';
    case 'C': return 'G';
    default: return c;
    }
}

uint32_t pack4(const std::string &s) {
    uint32_t v = 0;
    for (size_t i = 0; i < 4 && i < s.size(); ++i) v |= (uint32_t)(uint8_t)s[i] << (8 * i);
    return v;
}

template <typename T>
hipError_t dalloc(T **p, uint64_t n) {
    return hipMalloc((void **)p, std::max<uint64_t>(n, 1) * sizeof(T));
}

template <typename T>
void dfree(T *&p) {
    if (p) (void)hipFree((void *)p);
    p = nullptr;
}

kmer_status ensure_tiles(kmer_ctx *c, uint64_t n_tiles) {
    if (n_tiles <= c->tile_cap) return KMER_OK;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    dfree(c->d_lb_cnt);
    dfree(c->d_lb_lnl);
    dfree(c->d_tp_cnt);
    dfree(c->d_tp_lnl);
    dfree(c->d_agg_cnt); dfree(c->d_agg_lnl); dfree(c->d_cscan); dfree(c->d_lnl_before);
    dfree(c->d_tile_nhits); dfree(c->d_hits);
    if (c->d_scan_tmp) (void)hipFree(c->d_scan_tmp);
    c->d_scan_tmp = nullptr;
    uint64_t cap = std::max<uint64_t>(n_tiles, 1024);
    HIPCHK(c, dalloc(&c->d_lb_cnt, cap));
    HIPCHK(c, dalloc(&c->d_lb_lnl, cap));
    HIPCHK(c, dalloc(&c->d_tp_cnt, cap));
    HIPCHK(c, dalloc(&c->d_tp_lnl, cap));
    if (c->mode != MODE_GENERAL) {
        HIPCHK(c, dalloc(&c->d_agg_cnt, cap));
        HIPCHK(c, dalloc(&c->d_agg_lnl, cap));
        HIPCHK(c, dalloc(&c->d_cscan, cap));
        HIPCHK(c, dalloc(&c->d_lnl_before, cap));
        HIPCHK(c, dalloc(&c->d_tile_nhits, cap));
        HIPCHK(c, dalloc(&c->d_hits, cap * HMAX));
        size_t a = 0, b = 0;
        HIPCHK(c, rocprim::exclusive_scan(nullptr, a, c->d_agg_cnt, c->d_cscan, (uint64_t)0, (size_t)cap,
                                          rocprim::plus<uint64_t>(), c->stream));
        HIPCHK(c, rocprim::exclusive_scan(nullptr, b, c->d_agg_lnl, c->d_lnl_before, (uint64_t)0, (size_t)cap,
                                          rocprim::maximum<uint64_t>(), c->stream));
        c->scan_tmp_bytes = std::max(a, b);
        HIPCHK(c, hipMalloc(&c->d_scan_tmp, std::max<size_t>(c->scan_tmp_bytes, 16)));
    }
    c->tile_cap = cap;
    return KMER_OK;
}

kmer_status ensure_records(kmer_ctx *c, uint64_t n) {
    if (n <= c->rec_cap) return KMER_OK;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    dfree(c->d_recs);
    dfree(c->d_rec_keys);
    dfree(c->d_rec_off);
    uint64_t cap = std::max<uint64_t>(n, 1 << 16);
    HIPCHK(c, dalloc(&c->d_recs, cap));
    HIPCHK(c, dalloc(&c->d_rec_off, cap));
    HIPCHK(c, dalloc(&c->d_rec_keys, cap * (uint64_t)c->p.k));
    c->rec_cap = cap;
    return KMER_OK;
}

kmer_status ensure_lines(kmer_ctx *c, uint64_t n) {
    if (n <= c->line_cap) return KMER_OK;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    dfree(c->d_lines);
    uint64_t cap = std::max<uint64_t>(n, 1 << 16);
    HIPCHK(c, dalloc(&c->d_lines, cap));
    c->line_cap = cap;
    return KMER_OK;
}

kmer_status ensure_ovf(kmer_ctx *c, uint64_t n) {
    if (n <= c->ovf_cap) return KMER_OK;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    dfree(c->d_ovf);
    uint64_t cap = std::max<uint64_t>(n, 1 << 16);
    HIPCHK(c, dalloc(&c->d_ovf, cap));
    c->ovf_cap = cap;
    return KMER_OK;
}

// Pull the records of the chunk just processed to the host and fold them into
// the ordered host map (count, first occurrence).  Keys are gathered on the
// device (rc applied there) at a fixed stride of k bytes.
kmer_status drain_records(kmer_ctx *c, const uint8_t *d_data, uint64_t n, hipStream_t s) {
    if (n == 0) return KMER_OK;
    const uint64_t k = c->p.k;
    std::vector<uint64_t> off(n);
    for (uint64_t i = 0; i < n; ++i) off[i] = i * k;
    HIPCHK(c, hipMemcpyAsync(c->d_rec_off, off.data(), n * 8, hipMemcpyHostToDevice, s));
    HIPCHK(c, launch_gather_records(c->d_recs, c->d_rec_off, n, d_data, c->d_rec_keys, s));
    std::vector<Record> recs(n);
    std::vector<char> keys(n * k);
    HIPCHK(c, hipMemcpyAsync(recs.data(), c->d_recs, n * sizeof(Record), hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(keys.data(), c->d_rec_keys, n * k, hipMemcpyDeviceToHost, s));
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

kmer_status check_err(kmer_ctx *c, uint32_t e) {
    if (e & ERR_NONASCII) return fail(c, KMER_E_NONASCII, "input contains a byte >= 0x80 (non-ASCII)");
    if (e & ERR_LINE_TOO_LONG) return fail(c, KMER_E_LINE_TOO_LONG, "sequence line longer than 2^23 bytes");
    if (e & ERR_LOOKBACK_TIMEOUT) return fail(c, KMER_E_DEVICE, "tile look-back timed out");
    return KMER_OK;
}

// Two-pass prefixes (debug mode): per-tile aggregates -> host scan -> arrays.
kmer_status two_pass_prefix(kmer_ctx *c, const uint8_t *d, uint64_t len, uint32_t n_tiles, hipStream_t s) {
    HIPCHK(c, launch_tile_aggregate(d, len, n_tiles, c->d_tp_cnt, c->d_tp_lnl, c->d_err, s));
    std::vector<uint64_t> cnt(n_tiles), last(n_tiles);
    StreamPos pos;
    HIPCHK(c, hipMemcpyAsync(cnt.data(), c->d_tp_cnt, n_tiles * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(last.data(), c->d_tp_lnl, n_tiles * 8, hipMemcpyDeviceToHost, s));
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
    HIPCHK(c, hipMemcpyAsync(c->d_tp_cnt, cnt.data(), n_tiles * 8, hipMemcpyHostToDevice, s));
    HIPCHK(c, hipMemcpyAsync(c->d_tp_lnl, last.data(), n_tiles * 8, hipMemcpyHostToDevice, s));
    HIPCHK(c, hipMemcpyAsync(c->d_pos, &pos, sizeof(pos), hipMemcpyHostToDevice, s));
    HIPCHK(c, hipStreamSynchronize(s));
    return KMER_OK;
}

// Fast path (dense / tile-record modes): streaming tile scan -> scans of the
// per-tile aggregates -> hit resolution -> stream position update.
kmer_status scan_feed(kmer_ctx *c, const uint8_t *d, uint64_t len, uint32_t n_tiles, hipStream_t s) {
    ScanArgs a;
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
    a.agg_cnt = c->d_agg_cnt;
    a.agg_lnl = c->d_agg_lnl;
    a.hits = c->d_hits;
    a.tile_nhits = c->d_tile_nhits;
    a.ovf = c->d_ovf;
    a.ovf_count = c->d_ovf_count;
    a.ovf_cap = c->ovf_cap;
    a.err = c->d_err;
    a.ablate = (c->p.flags >> 8) & 0xFFu;   // KMER_FLAG_ABLATE_* (experiments only)

    HitArgs h;
    memset(&h, 0, sizeof(h));
    h.hits = c->d_hits;
    h.tile_nhits = c->d_tile_nhits;
    h.ovf = c->d_ovf;
    h.ovf_count = c->d_ovf_count;
    h.ovf_cap = c->ovf_cap;
    h.n_tiles = n_tiles;
    h.k = a.k;
    h.plen = a.plen;
    h.abs_offset = c->abs_offset;
    h.pos = c->d_pos;
    h.cscan = c->d_cscan;
    h.lnl_before = c->d_lnl_before;
    h.dense = c->mode == MODE_DENSE;
    h.dense_update = 1;
    h.smask = (2 * (a.k - std::min(a.plen, a.k)) >= 64) ? ~0ull : ((1ull << (2 * (a.k - std::min(a.plen, a.k)))) - 1ull);
    h.counts = c->d_counts;
    h.first = c->d_first;
    h.recs = c->d_recs;
    h.rec_count = c->d_rec_count;
    h.rec_cap = c->rec_cap;
    h.err = c->d_err;

    HIPCHK(c, hipMemcpyAsync(c->d_pos_saved, c->d_pos, sizeof(StreamPos), hipMemcpyDeviceToDevice, s));
    kmer_status st;
    for (int attempt = 0; attempt < 8; ++attempt) {
        HIPCHK(c, hipMemsetAsync(c->d_ovf_count, 0, 8, s));
        HIPCHK(c, hipMemsetAsync(c->d_rec_count, 0, 8, s));
        HIPCHK(c, hipEventRecord(c->ev0, s));
        HIPCHK(c, launch_scan_tiles(a, s));
        HIPCHK(c, hipEventRecord(c->ev1, s));
        size_t tmp = c->scan_tmp_bytes;
        HIPCHK(c, rocprim::exclusive_scan(c->d_scan_tmp, tmp, c->d_agg_cnt, c->d_cscan, (uint64_t)0, (size_t)n_tiles,
                                          rocprim::plus<uint64_t>(), s));
        tmp = c->scan_tmp_bytes;
        HIPCHK(c, rocprim::exclusive_scan(c->d_scan_tmp, tmp, c->d_agg_lnl, c->d_lnl_before, (uint64_t)c->abs_offset,
                                          (size_t)n_tiles, rocprim::maximum<uint64_t>(), s));
        HIPCHK(c, launch_hits(h, s));
        HIPCHK(c, launch_pos_update(c->d_pos, c->d_cscan, c->d_agg_cnt, n_tiles, d, len, s));
        HIPCHK(c, hipEventRecord(c->ev4, s));
        HIPCHK(c, hipMemcpyAsync(c->h_small + 0, c->d_rec_count, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(c->h_small + 1, c->d_ovf_count, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(c->h_small + 2, c->d_err, 4, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        const uint32_t e = (uint32_t)c->h_small[2];
        st = check_err(c, e);
        if (st) return st;
        float ms = 0.f, ms_all = 0.f;
        HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
        HIPCHK(c, hipEventElapsedTime(&ms_all, c->ev0, c->ev4));
        c->count_ms += ms;
        c->feed_ms += ms_all;
        if (e & (ERR_OVF_OVERFLOW | ERR_REC_OVERFLOW)) {
            HIPCHK(c, hipMemsetAsync(c->d_err, 0, 4, s));
            HIPCHK(c, hipMemcpyAsync(c->d_pos, c->d_pos_saved, sizeof(StreamPos), hipMemcpyDeviceToDevice, s));
            if (e & ERR_OVF_OVERFLOW) {
                // nothing was resolved: plain redo with a larger overflow list
                st = ensure_ovf(c, c->h_small[1] + 1024);
                if (st) return st;
                a.ovf = c->d_ovf;
                h.ovf = c->d_ovf;
                a.ovf_cap = c->ovf_cap;
                h.ovf_cap = c->ovf_cap;
            } else {
                // dense table already holds this chunk: redo for the records only
                st = ensure_records(c, c->h_small[0] + 1024);
                if (st) return st;
                h.recs = c->d_recs;
                h.rec_cap = c->rec_cap;
                h.dense_update = 0;
            }
            continue;
        }
        break;
    }
    const uint64_t nrec = c->h_small[0];
    if (nrec) {
        st = drain_records(c, d, nrec, s);
        if (st) return st;
    }
    c->abs_offset += len;
    return KMER_OK;
}

kmer_status feed(kmer_ctx *c, const uint8_t *d, uint64_t len, hipStream_t s) {
    if (len == 0) return KMER_OK;
    const uint64_t n_tiles64 = (len + TILE - 1) / TILE;
    if (n_tiles64 > 0x7FFFFFFFull) return fail(c, KMER_E_BAD_PARAM, "chunk too large");
    const uint32_t n_tiles = (uint32_t)n_tiles64;
    kmer_status st = ensure_tiles(c, n_tiles);
    if (st) return st;
    if (c->mode != MODE_GENERAL) return scan_feed(c, d, len, n_tiles, s);
    const bool lookback = !(c->p.flags & KMER_FLAG_TWO_PASS);

    TileArgs a;
    memset(&a, 0, sizeof(a));
    a.data = d;
    a.len = len;
    a.n_tiles = n_tiles;
    a.k = c->p.k;
    a.plen = (uint32_t)c->prefix.size();
    a.p4 = pack4(c->prefix);
    a.r4 = pack4(c->rprefix);
    a.pmask = a.plen >= 4 ? 0xFFFFFFFFu : ((1u << (8 * a.plen)) - 1u);
    a.dense = c->mode == MODE_DENSE;
    a.dense_update = 1;
    a.abs_offset = c->abs_offset;
    a.emit_lines = c->mode == MODE_GENERAL;
    a.PR = c->d_PR;
    a.counts = c->d_counts;
    a.first = c->d_first;
    a.recs = c->d_recs;
    a.rec_count = c->d_rec_count;
    a.rec_cap = c->rec_cap;
    a.lines_out = c->d_lines;
    a.line_count = c->d_line_count;
    a.line_cap = c->line_cap;
    a.lb_cnt = c->d_lb_cnt;
    a.lb_lnl = c->d_lb_lnl;
    a.ticket = c->d_ticket;
    a.pos = c->d_pos;
    a.tp_cnt = c->d_tp_cnt;
    a.tp_lnl = c->d_tp_lnl;
    a.err = c->d_err;

    HIPCHK(c, hipMemcpyAsync(c->d_pos_saved, c->d_pos, sizeof(StreamPos), hipMemcpyDeviceToDevice, s));
    for (int attempt = 0; attempt < 8; ++attempt) {
        HIPCHK(c, hipMemsetAsync(c->d_lb_cnt, 0, n_tiles * 8ull, s));
        HIPCHK(c, hipMemsetAsync(c->d_lb_lnl, 0, n_tiles * 8ull, s));
        HIPCHK(c, hipMemsetAsync(c->d_ticket, 0, 16, s));
        HIPCHK(c, hipMemsetAsync(c->d_rec_count, 0, 8, s));
        HIPCHK(c, hipMemsetAsync(c->d_line_count, 0, 8, s));
        if (!lookback) {
            st = two_pass_prefix(c, d, len, n_tiles, s);
            if (st) return st;
        }
        HIPCHK(c, hipEventRecord(c->ev0, s));
        HIPCHK(c, launch_lines(a, lookback, s));
        HIPCHK(c, hipEventRecord(c->ev1, s));
        HIPCHK(c, hipMemcpyAsync(c->h_small + 0, c->d_rec_count, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(c->h_small + 1, c->d_line_count, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(c->h_small + 2, c->d_err, 4, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        const uint32_t e = (uint32_t)c->h_small[2];
        st = check_err(c, e);
        if (st) return st;
        float ms = 0.f;
        HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
        c->count_ms += ms;
        if (e & (ERR_REC_OVERFLOW | ERR_LINE_OVERFLOW)) {
            // capacity exceeded: grow and redo the chunk from the saved position;
            // the dense table already holds this chunk, so the redo skips it
            HIPCHK(c, hipMemsetAsync(c->d_err, 0, 4, s));
            HIPCHK(c, hipMemcpyAsync(c->d_pos, c->d_pos_saved, sizeof(StreamPos), hipMemcpyDeviceToDevice, s));
            if (e & ERR_REC_OVERFLOW) {
                st = ensure_records(c, c->h_small[0] + 1024);
                if (st) return st;
                a.recs = c->d_recs;
                a.rec_cap = c->rec_cap;
                if (c->mode == MODE_DENSE) a.dense_update = 0;
            }
            if (e & ERR_LINE_OVERFLOW) {
                st = ensure_lines(c, c->h_small[1] + 1024);
                if (st) return st;
                a.lines_out = c->d_lines;
                a.line_cap = c->line_cap;
            }
            continue;
        }
        break;
    }
    uint64_t nrec = c->h_small[0];
    if (c->mode == MODE_GENERAL) {
        const uint64_t nlines = c->h_small[1];
        if (nlines) {
            WindowArgs w;
            memset(&w, 0, sizeof(w));
            w.data = d;
            w.lines = c->d_lines;
            w.n_lines = c->d_line_count;
            w.k = c->p.k;
            w.step = c->p.step;
            w.plen = (uint32_t)c->prefix.size();
            w.P = c->d_PR + 2 * KMAX_TILE;
            w.err = c->d_err;
            // upper bound on records: every window of every line on both strands
            // is not known cheaply; start from the capacity and grow on overflow
            for (int attempt = 0; attempt < 8; ++attempt) {
                w.recs = c->d_recs;
                w.rec_count = c->d_rec_count;
                w.rec_cap = c->rec_cap;
                HIPCHK(c, hipMemsetAsync(c->d_rec_count, 0, 8, s));
                HIPCHK(c, hipEventRecord(c->ev0, s));
                const uint32_t grid = (uint32_t)std::min<uint64_t>(nlines, 65536);
                HIPCHK(c, launch_windows(w, grid, s));
                HIPCHK(c, hipEventRecord(c->ev1, s));
                HIPCHK(c, hipMemcpyAsync(c->h_small + 0, c->d_rec_count, 8, hipMemcpyDeviceToHost, s));
                HIPCHK(c, hipMemcpyAsync(c->h_small + 2, c->d_err, 4, hipMemcpyDeviceToHost, s));
                HIPCHK(c, hipStreamSynchronize(s));
                const uint32_t e = (uint32_t)c->h_small[2];
                st = check_err(c, e);
                if (st) return st;
                float ms = 0.f;
                HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
                c->count_ms += ms;
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
    }
    if (nrec) {
        st = drain_records(c, d, nrec, s);
        if (st) return st;
    }
    c->abs_offset += len;
    return KMER_OK;
}

kmer_status reset(kmer_ctx *c) {
    hipStream_t s = c->stream;
    if (c->mode == MODE_DENSE) {
        HIPCHK(c, hipMemsetAsync(c->d_counts, 0, c->n_dense * 8, s));
        HIPCHK(c, hipMemsetAsync(c->d_first, 0xFF, c->n_dense * 8, s));
    }
    HIPCHK(c, hipMemsetAsync(c->d_pos, 0, sizeof(StreamPos), s));
    HIPCHK(c, hipMemsetAsync(c->d_err, 0, 4, s));
    c->exotic.clear();
    c->abs_offset = 0;
    c->count_ms = 0.0;
    c->finish_ms = 0.0;
    c->feed_ms = 0.0;
    c->open_stream = true;
    return KMER_OK;
}

kmer_status finish(kmer_ctx *c, kmer_result **out) {
    if (!c->open_stream) return fail(c, KMER_E_STATE, "finish without reset/feed");
    hipStream_t s = c->stream;
    StreamPos pos;
    HIPCHK(c, hipEventRecord(c->ev2, s));
    uint64_t n = 0;
    if (c->mode == MODE_DENSE) {
        HIPCHK(c, hipMemsetAsync(c->d_nout, 0, 8, s));
        HIPCHK(c, launch_dense_compact(c->d_counts, c->d_first, c->n_dense, c->d_order, c->d_idx, c->d_nout, s));
        HIPCHK(c, hipMemcpyAsync(c->h_small + 3, c->d_nout, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(c->h_small + 4, c->d_pos, sizeof(StreamPos), hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        n = c->h_small[3];
        memcpy(&pos, c->h_small + 4, sizeof(pos));
        // sort by first-occurrence order; only the bits the orders can use
        const uint64_t max_order = ((pos.lines + 1) << 24) | 0xFFFFFFull;
        int end_bit = 64 - __builtin_clzll(max_order);
        if (n) {
            rocprim::double_buffer<uint64_t> keys(c->d_order, c->d_order2);
            rocprim::double_buffer<uint64_t> vals(c->d_idx, c->d_idx2);
            size_t tmp = c->sort_tmp_bytes;
            HIPCHK(c, rocprim::radix_sort_pairs(c->d_sort_tmp, tmp, keys, vals, (size_t)n, 0, end_bit, s));
            HIPCHK(c, launch_dense_decode(vals.current(), c->d_nout, n, c->p.k, (uint32_t)c->prefix.size(), c->d_P,
                                          c->d_counts, c->d_keys_out, c->d_cnt_out, s));
            if (keys.current() != c->d_order) {
                HIPCHK(c, hipMemcpyAsync(c->d_order, keys.current(), n * 8, hipMemcpyDeviceToDevice, s));
            }
        }
    } else {
        HIPCHK(c, hipMemcpyAsync(c->h_small + 4, c->d_pos, sizeof(StreamPos), hipMemcpyDeviceToHost, s));
    }
    HIPCHK(c, hipEventRecord(c->ev3, s));
    HIPCHK(c, hipStreamSynchronize(s));
    memcpy(&pos, c->h_small + 4, sizeof(pos));
    float ms = 0.f;
    HIPCHK(c, hipEventElapsedTime(&ms, c->ev2, c->ev3));
    c->finish_ms = ms;
    c->last_n = n;
    c->open_stream = false;

    const uint64_t total = n + c->exotic.size();
    if (c->p.max_keys && total > c->p.max_keys)
        return fail(c, KMER_E_TOO_MANY_KEYS, "more distinct keys than max_keys (reference Map limit)");
    if (!out) return KMER_OK;

    kmer_result *r = new (std::nothrow) kmer_result();
    if (!r) return fail(c, KMER_E_OOM, "host allocation failed");
    r->lines = pos.lines + pos.ends_open;
    const uint64_t k = c->p.k;
    std::vector<uint64_t> order(n), cnt(n);
    std::vector<char> dkeys(n * k);
    if (n) {
        HIPCHK(c, hipMemcpy(order.data(), c->d_order, n * 8, hipMemcpyDeviceToHost));
        HIPCHK(c, hipMemcpy(cnt.data(), c->d_cnt_out, n * 8, hipMemcpyDeviceToHost));
        HIPCHK(c, hipMemcpy(dkeys.data(), c->d_keys_out, n * k, hipMemcpyDeviceToHost));
    }
    // records (exotic / general) sorted by first occurrence
    std::vector<std::pair<uint64_t, const std::pair<const std::string, Ent> *>> ex;
    ex.reserve(c->exotic.size());
    for (auto &kv : c->exotic) ex.emplace_back(kv.second.first, &kv);
    std::sort(ex.begin(), ex.end(), [](const auto &x, const auto &y) { return x.first < y.first; });
    r->keys.reserve(n * k + ex.size() * k);
    r->offsets.reserve(total + 1);
    r->counts.reserve(total);
    uint64_t i = 0, j = 0;
    while (i < n || j < ex.size()) {
        if (j >= ex.size() || (i < n && order[i] < ex[j].first)) {
            r->keys.insert(r->keys.end(), dkeys.begin() + i * k, dkeys.begin() + (i + 1) * k);
            r->counts.push_back(cnt[i]);
            ++i;
        } else {
            const std::string &key = ex[j].second->first;
            r->keys.insert(r->keys.end(), key.begin(), key.end());
            r->counts.push_back(ex[j].second->second.count);
            ++j;
        }
        r->offsets.push_back(r->keys.size());
    }
    *out = r;
    return KMER_OK;
}

// Feed host bytes through the device in batches cut at '\n' boundaries.
kmer_status feed_host(kmer_ctx *c, const uint8_t *bytes, uint64_t len) {
    uint64_t batch = c->p.batch_bytes ? c->p.batch_bytes : DEFAULT_BATCH;
    uint64_t pos = 0;
    while (pos < len) {
        uint64_t end = std::min(len, pos + batch);
        if (end < len) {
            // cut after the last '\n' in [pos, end); a line longer than the batch extends it
            const uint8_t *p = bytes + pos;
            uint64_t cut = end - pos;
            while (cut > 0 && p[cut - 1] != '\n') --cut;
            if (cut == 0) {
                const void *nl = memchr(bytes + end, '\n', len - end);
                end = nl ? (uint64_t)((const uint8_t *)nl - bytes) + 1 : len;
            } else {
                end = pos + cut;
            }
        }
        const uint64_t n = end - pos;
        if (n > c->batch_cap) {
            HIPCHK(c, hipStreamSynchronize(c->stream));
            dfree(c->d_batch);
            HIPCHK(c, dalloc(&c->d_batch, n));
            c->batch_cap = n;
        }
        HIPCHK(c, hipMemcpyAsync(c->d_batch, bytes + pos, n, hipMemcpyHostToDevice, c->stream));
        kmer_status st = feed(c, c->d_batch, n, c->stream);
        if (st) return st;
        pos = end;
    }
    return KMER_OK;
}

}  // namespace

extern "C" {

const char *kmer_version(void) { return "kmerhip 0.1 (gfx950)"; }

const char *kmer_status_string(kmer_status s) {
    switch (s) {
    case KMER_OK: return "ok";
    case KMER_E_IO: return "i/o error";
    case KMER_E_BAD_PARAM: return "bad parameter";
    case KMER_E_OOM: return "out of memory";
    case KMER_E_DEVICE: return "device error";
    case KMER_E_TOO_MANY_KEYS: return "too many keys";
    case KMER_E_NONASCII: return "non-ASCII input";
    case KMER_E_LINE_TOO_LONG: return "line too long";
    case KMER_E_STATE: return "bad call sequence";
    }
    return "unknown";
}

const char *kmer_last_error(const kmer_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

kmer_status kmer_open(const kmer_params *pp, kmer_ctx **out) {
    if (!pp || !out) return KMER_E_BAD_PARAM;
    if (pp->k == 0 || pp->step == 0 || (pp->prefix_len && !pp->prefix)) return KMER_E_BAD_PARAM;
    kmer_ctx *c = new (std::nothrow) kmer_ctx();
    if (!c) return KMER_E_OOM;
    *out = nullptr;
    c->p = *pp;
    c->prefix.assign((const char *)pp->prefix, pp->prefix_len);
    c->rprefix.resize(c->prefix.size());
    for (size_t i = 0; i < c->prefix.size(); ++i)
        c->rprefix[c->prefix.size() - 1 - i] = (char)comp((uint8_t)c->prefix[i]);
    c->p.prefix = nullptr;
    for (unsigned char ch : c->prefix)
        if (ch >= 0x80) {
            delete c;
            return KMER_E_NONASCII;
        }
    c->device = pp->device;
    auto cleanup = [&](kmer_status s) {
        kmer_close(c);
        return s;
    };
    if (hipSetDevice(c->device) != hipSuccess) return cleanup(KMER_E_DEVICE);
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return cleanup(KMER_E_DEVICE);

    const uint32_t k = pp->k, plen = (uint32_t)c->prefix.size();
    bool acgt = plen > 0;
    for (char ch : c->prefix) acgt &= ch == 'A' || ch == 'C' || ch == 'G' || ch == 'T';
    if (pp->step == 1 && acgt && plen <= k && k <= (uint32_t)KMAX_DENSE && k - plen <= (uint32_t)DENSE_MAX_SUFFIX &&
        !(pp->flags & KMER_FLAG_NO_DENSE))
        c->mode = MODE_DENSE;
    else if (pp->step == 1 && plen > 0 && k <= (uint32_t)KMAX_TILE)
        c->mode = MODE_TILE_REC;
    else
        c->mode = MODE_GENERAL;

    bool ok = true;
    if (c->mode == MODE_DENSE) {
        c->n_dense = 1ull << (2 * (k - plen));
        ok &= dalloc(&c->d_counts, c->n_dense) == hipSuccess;
        ok &= dalloc(&c->d_first, c->n_dense) == hipSuccess;
        ok &= dalloc(&c->d_order, c->n_dense) == hipSuccess;
        ok &= dalloc(&c->d_order2, c->n_dense) == hipSuccess;
        ok &= dalloc(&c->d_idx, c->n_dense) == hipSuccess;
        ok &= dalloc(&c->d_idx2, c->n_dense) == hipSuccess;
        ok &= dalloc(&c->d_keys_out, c->n_dense * k) == hipSuccess;
        ok &= dalloc(&c->d_cnt_out, c->n_dense) == hipSuccess;
        ok &= dalloc(&c->d_P, std::max<uint32_t>(plen, 1)) == hipSuccess;
        if (ok && plen) ok &= hipMemcpy(c->d_P, c->prefix.data(), plen, hipMemcpyHostToDevice) == hipSuccess;
        if (ok) {
            rocprim::double_buffer<uint64_t> keys(c->d_order, c->d_order2);
            rocprim::double_buffer<uint64_t> vals(c->d_idx, c->d_idx2);
            size_t tmp = 0;
            ok &= rocprim::radix_sort_pairs(nullptr, tmp, keys, vals, (size_t)c->n_dense, 0, 64, c->stream) ==
                  hipSuccess;
            c->sort_tmp_bytes = tmp;
            ok &= dalloc((uint8_t **)&c->d_sort_tmp, tmp) == hipSuccess;
        }
    }
    {
        // [0,64) P and [64,128) rc(P) (tile kernel, truncated), [128, 128+|P|) full P (general kernel)
        std::vector<uint8_t> pr(2 * KMAX_TILE + c->prefix.size(), 0);
        memcpy(pr.data(), c->prefix.data(), std::min<size_t>(c->prefix.size(), KMAX_TILE));
        memcpy(pr.data() + KMAX_TILE, c->rprefix.data(), std::min<size_t>(c->rprefix.size(), KMAX_TILE));
        memcpy(pr.data() + 2 * KMAX_TILE, c->prefix.data(), c->prefix.size());
        ok &= dalloc(&c->d_PR, pr.size()) == hipSuccess;
        if (ok) ok &= hipMemcpy(c->d_PR, pr.data(), pr.size(), hipMemcpyHostToDevice) == hipSuccess;
    }
    ok &= dalloc(&c->d_ticket, 4) == hipSuccess;
    ok &= dalloc(&c->d_err, 1) == hipSuccess;
    ok &= dalloc(&c->d_rec_count, 1) == hipSuccess;
    ok &= dalloc(&c->d_line_count, 1) == hipSuccess;
    ok &= dalloc(&c->d_nout, 1) == hipSuccess;
    ok &= dalloc(&c->d_pos, 1) == hipSuccess;
    ok &= dalloc(&c->d_pos_saved, 1) == hipSuccess;
    ok &= hipHostMalloc((void **)&c->h_small, 16 * sizeof(uint64_t), hipHostMallocDefault) == hipSuccess;
    ok &= hipEventCreate(&c->ev0) == hipSuccess && hipEventCreate(&c->ev1) == hipSuccess &&
          hipEventCreate(&c->ev2) == hipSuccess && hipEventCreate(&c->ev3) == hipSuccess &&
          hipEventCreate(&c->ev4) == hipSuccess;
    ok &= dalloc(&c->d_ovf_count, 1) == hipSuccess;
    if (!ok) return cleanup(KMER_E_OOM);
    if (ensure_records(c, 1 << 16) || ensure_lines(c, 1 << 16) || ensure_tiles(c, 1 << 12) ||
        ensure_ovf(c, 1 << 16))
        return cleanup(KMER_E_OOM);
    if (hipMemset(c->d_err, 0, 4) != hipSuccess) return cleanup(KMER_E_DEVICE);
    if (reset(c) != KMER_OK) return cleanup(KMER_E_DEVICE);
    c->open_stream = false;
    if (hipStreamSynchronize(c->stream) != hipSuccess) return cleanup(KMER_E_DEVICE);
    *out = c;
    return KMER_OK;
}

kmer_status kmer_close(kmer_ctx *c) {
    if (!c) return KMER_E_BAD_PARAM;
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    dfree(c->d_counts); dfree(c->d_first);
    dfree(c->d_lb_cnt); dfree(c->d_lb_lnl); dfree(c->d_tp_cnt); dfree(c->d_tp_lnl);
    dfree(c->d_ticket); dfree(c->d_err); dfree(c->d_rec_count); dfree(c->d_line_count); dfree(c->d_nout);
    dfree(c->d_pos); dfree(c->d_pos_saved);
    dfree(c->d_recs); dfree(c->d_lines); dfree(c->d_rec_keys); dfree(c->d_rec_off);
    dfree(c->d_order); dfree(c->d_order2); dfree(c->d_idx); dfree(c->d_idx2);
    dfree(c->d_keys_out); dfree(c->d_cnt_out); dfree(c->d_P); dfree(c->d_PR);
    if (c->d_sort_tmp) (void)hipFree(c->d_sort_tmp);
    dfree(c->d_batch);
    dfree(c->d_agg_cnt); dfree(c->d_agg_lnl); dfree(c->d_cscan); dfree(c->d_lnl_before);
    dfree(c->d_tile_nhits); dfree(c->d_hits); dfree(c->d_ovf); dfree(c->d_ovf_count);
    if (c->d_scan_tmp) (void)hipFree(c->d_scan_tmp);
    if (c->h_small) (void)hipHostFree(c->h_small);
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    for (hipEvent_t e : {c->ev0, c->ev1, c->ev2, c->ev3, c->ev4})
        if (e) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return KMER_OK;
}

kmer_status kmer_reset(kmer_ctx *c) {
    if (!c) return KMER_E_BAD_PARAM;
    if (hipSetDevice(c->device) != hipSuccess) return KMER_E_DEVICE;
    return reset(c);
}

kmer_status kmer_feed_device(kmer_ctx *c, const void *d_bytes, size_t len, void *stream) {
    if (!c || (!d_bytes && len)) return KMER_E_BAD_PARAM;
    if (!c->open_stream) return fail(c, KMER_E_STATE, "feed without reset");
    if (hipSetDevice(c->device) != hipSuccess) return KMER_E_DEVICE;
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    if (s != c->stream) {
        // order the context's own stream after the caller's work
        hipEvent_t ev;
        HIPCHK(c, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        HIPCHK(c, hipEventRecord(ev, s));
        HIPCHK(c, hipStreamWaitEvent(c->stream, ev, 0));
        HIPCHK(c, hipEventDestroy(ev));
    }
    return feed(c, (const uint8_t *)d_bytes, len, c->stream);
}

kmer_status kmer_finish_device(kmer_ctx *c, kmer_result **out) {
    if (!c) return KMER_E_BAD_PARAM;
    if (hipSetDevice(c->device) != hipSuccess) return KMER_E_DEVICE;
    if (out) *out = nullptr;
    return finish(c, out);
}

kmer_status kmer_count_buffer(kmer_ctx *c, const uint8_t *bytes, size_t len, kmer_result **out) {
    if (!c || !out || (!bytes && len)) return KMER_E_BAD_PARAM;
    *out = nullptr;
    if (hipSetDevice(c->device) != hipSuccess) return KMER_E_DEVICE;
    kmer_status st = reset(c);
    if (st) return st;
    st = feed_host(c, bytes, len);
    if (st) {
        c->open_stream = false;
        return st;
    }
    return finish(c, out);
}

kmer_status kmer_count_file(kmer_ctx *c, const char *path, kmer_result **out) {
    if (!c || !path || !out) return KMER_E_BAD_PARAM;
    *out = nullptr;
    FILE *f = fopen(path, "rb");
    if (!f) return fail(c, KMER_E_IO, std::string("cannot open ") + path);
    if (hipSetDevice(c->device) != hipSuccess) {
        fclose(f);
        return KMER_E_DEVICE;
    }
    kmer_status st = reset(c);
    const uint64_t batch = c->p.batch_bytes ? c->p.batch_bytes : DEFAULT_BATCH;
    std::vector<uint8_t> buf;
    uint64_t carry = 0;
    bool eof = false;
    while (!st && !eof) {
        buf.resize(carry + batch);
        size_t got = fread(buf.data() + carry, 1, batch, f);
        if (got < batch) {
            if (ferror(f)) {
                st = fail(c, KMER_E_IO, std::string("read error on ") + path);
                break;
            }
            eof = true;
        }
        uint64_t have = carry + got;
        uint64_t cut = have;
        if (!eof) {
            while (cut > 0 && buf[cut - 1] != '\n') --cut;
            if (cut == 0) {   // one line longer than the batch: keep reading
                carry = have;
                continue;
            }
        }
        st = feed_host(c, buf.data(), cut);
        carry = have - cut;
        if (carry) memmove(buf.data(), buf.data() + cut, carry);
    }
    fclose(f);
    if (st) {
        c->open_stream = false;
        return st;
    }
    return finish(c, out);
}

kmer_status kmer_table_view(kmer_ctx *c, void **d_counts, void **d_first, uint64_t *n) {
    if (!c || !d_counts || !d_first || !n) return KMER_E_BAD_PARAM;
    if (c->mode != MODE_DENSE) return fail(c, KMER_E_STATE, "configuration does not use the dense table");
    *d_counts = c->d_counts;
    *d_first = c->d_first;
    *n = c->n_dense;
    return KMER_OK;
}

kmer_status kmer_set_position(kmer_ctx *c, uint64_t lines_before, uint64_t byte_offset) {
    if (!c) return KMER_E_BAD_PARAM;
    StreamPos pos{};
    pos.lines = lines_before;
    HIPCHK(c, hipMemcpyAsync(c->d_pos, &pos, sizeof(pos), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->abs_offset = byte_offset;
    return KMER_OK;
}

kmer_status kmer_lines(kmer_ctx *c, uint64_t *lines) {
    if (!c || !lines) return KMER_E_BAD_PARAM;
    StreamPos pos;
    HIPCHK(c, hipMemcpyAsync(&pos, c->d_pos, sizeof(pos), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    *lines = pos.lines + pos.ends_open;
    return KMER_OK;
}

kmer_status kmer_last_timing(kmer_ctx *c, double *count_ms, double *feed_ms, double *finish_ms) {
    if (!c) return KMER_E_BAD_PARAM;
    if (count_ms) *count_ms = c->count_ms;
    if (feed_ms) *feed_ms = c->feed_ms > 0 ? c->feed_ms : c->count_ms;
    if (finish_ms) *finish_ms = c->finish_ms;
    return KMER_OK;
}

kmer_status kmer_synth_fastq_device(void *d_out, uint64_t seed, uint64_t first_read, uint64_t n_reads,
                                    void *stream) {
    if (!d_out && n_reads) return KMER_E_BAD_PARAM;
    hipError_t e = launch_synth_fastq((uint8_t *)d_out, seed, first_read, n_reads, (hipStream_t)stream);
    if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
    return e == hipSuccess ? KMER_OK : KMER_E_DEVICE;
}

uint64_t kmer_result_size(const kmer_result *r) { return r ? r->counts.size() : 0; }
uint64_t kmer_result_lines(const kmer_result *r) { return r ? r->lines : 0; }

kmer_status kmer_result_get(const kmer_result *r, uint64_t i, const char **key, uint32_t *klen, uint64_t *count) {
    if (!r || i >= r->counts.size()) return KMER_E_BAD_PARAM;
    if (key) *key = r->keys.data() + r->offsets[i];
    if (klen) *klen = (uint32_t)(r->offsets[i + 1] - r->offsets[i]);
    if (count) *count = r->counts[i];
    return KMER_OK;
}

kmer_status kmer_result_arrays(const kmer_result *r, const char **keys, const uint64_t **offsets,
                               const uint64_t **counts) {
    if (!r) return KMER_E_BAD_PARAM;
    if (keys) *keys = r->keys.data();
    if (offsets) *offsets = r->offsets.data();
    if (counts) *counts = r->counts.data();
    return KMER_OK;
}

void kmer_result_free(kmer_result *r) { delete r; }

}  // extern "C"
