// kmer_api.hip — host orchestration behind the C-ABI (include/kmer_api.h).
//
// One kmer_ctx = one device, one HIP stream, one (k, preffix, step)
// configuration.  Input flows in chunks cut at line ends.
//
// Packed path (step 1, ACGT prefix of >= 4 bases, k <= 32), per chunk:
//   scan_planes_kernel   one HBM pass: '\n' aggregates + verified prefix hits
//   tile reduce / scan   per-tile lines / line start / hits / cross hits before
//   hit_kernel           line rule + first-occurrence order; each packed hit
//                        goes to its RANK slot (or the cross list)
// Dense-hit path (empty or 1-3 base ACGT prefix): newline array -> sequence
//   lines by ordinal -> every window written at its rank slot.
// finish: place the cross list, radix-sort (key, rank), heads (first element
// of a key group = first occurrence), scan of heads over ranks -> output
// position, emit decoded keys in the reference Map's exact iteration order
// (lib/kmers.js:76,95).
// Tile-record path (non-ACGT prefix, or k in 33..64) and general path
// (step > 1, k > 64, ...): windows become records merged on the host.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include <algorithm>
#include <condition_variable>
#include <cstdio>
#include <deque>
#include <mutex>
#include <functional>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/kmer_api.h"
#include "kmer_internal.hpp"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

using namespace kmerhip;

// every KMER_FLAG_* of include/kmer_api.h
constexpr uint32_t KMER_FLAGS_PUBLIC = 0xFFu | KMER_FLAG_FASTA;

namespace {

// PACKED: tile scan, packed keys; TILE_REC: tile scan, records (host merge);
// WINDOWS: dense hits (no / 1-3 base prefix), every window ranked; GENERAL:
// lines + windows kernels, records (any k, step, prefix); TABLE: unordered
// canonical counts in a hash-partitioned table (KMER_FLAG_UNORDERED).
enum Mode { MODE_PACKED, MODE_TILE_REC, MODE_WINDOWS, MODE_GENERAL, MODE_TABLE };

struct Ent {
    uint64_t count;
    uint64_t first;
};

// growable device array; `keep` preserves the first `used` elements on growth
template <typename T>
struct DBuf {
    T *p = nullptr;
    uint64_t cap = 0;
    hipError_t ensure(uint64_t n, hipStream_t s, bool keep = false, uint64_t used = 0) {
        if (n <= cap) return hipSuccess;
        uint64_t nc = std::max<uint64_t>(n, cap + cap / 2);
        nc = std::max<uint64_t>(nc, 1024);
        T *q = nullptr;
        hipError_t e = hipMalloc((void **)&q, nc * sizeof(T));
        if (e != hipSuccess) return e;
        if (p) {
            if (keep && used) {
                e = hipMemcpyAsync(q, p, used * sizeof(T), hipMemcpyDeviceToDevice, s);
                if (e != hipSuccess) return e;
            }
            e = hipStreamSynchronize(s);
            if (e != hipSuccess) return e;
            (void)hipFree(p);
        }
        p = q;
        cap = nc;
        return hipSuccess;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

}  // namespace

struct kmer_result {
    uint64_t lines = 0;
    std::vector<char> keys;
    std::vector<uint64_t> offsets{0};
    std::vector<uint64_t> counts;
    std::vector<uint64_t> firsts;
};

struct kmer_ctx {
    kmer_params p{};
    std::string prefix, rprefix;
    Mode mode = MODE_GENERAL;
    int device = 0;
    uint32_t pbits = PBITS_DEFAULT;       // order-key position bits (PBITS_LONG: long-line mode)
    hipStream_t stream = nullptr;  // high priority: finish, exchange, copies, everything but the scan chain
    hipStream_t sstream = nullptr; // low priority: a packed-path chunk (scan, tile scan, hit resolution)
    hipEvent_t evq = nullptr;      // orders sstream after stream
    std::string err;
    uint32_t kbits = 0;            // packed key bits = 2*(k - |P|)
    bool wide = false;             // packed keys of >= 64 bits (k <= 64): two words, the high one in rkeyh

    // per tile
    uint64_t tile_cap = 0;
    DBuf<TileSum> tsum, tscan, bsum, bscan;
    DBuf<uint64_t> wcount, wbase;  // dense-hit path: windows / first rank per sequence line
    DBuf<uint32_t> tcount;         // dense-hit path: '\n' per tile
    DBuf<uint64_t> tbase, nlpos;   // ... exclusive scan, chunk-relative '\n' positions (or sequence-line bounds)
    DBuf<uint16_t> nlslots;        // tile-relative '\n' positions, NL_SLOTS per tile
    uint64_t host_lines = 0;       // StreamPos.lines as last seen by the host (dense-hit path)
    DBuf<HitRec> hits, ovf;
    DBuf<uint64_t> hits_hi, ovf_hi;   // k > 32: the first k - 32 bases of each hit record's window
    DBuf<unsigned long long> lb_cnt, lb_lnl;   // general path look-back
    DBuf<uint64_t> tp_cnt, tp_lnl;             // general path, two-pass debug mode
    // session packed hits, by rank (first-occurrence order of all hits)
    uint64_t n_hits = 0, n_cross = 0;
    DBuf<uint64_t> rkey, rkey2, rord, rord2, rcnt, csel;
    DBuf<uint64_t> rkeyh, whA, whB;    // wide keys: high words by rank; sort scratch
    DBuf<uint32_t> ridx3;
    DBuf<uint32_t> rkey32, rkey32b;   // narrow keys: 2(k-|P|) + 1 <= 32 bits
    bool narrow = false;
    bool planes = false;           // ACGT prefix: bit-plane scan kernel
    PlaneArgs pargs{};
    DBuf<uint32_t> ridx, ridx2, opos;
    DBuf<HeadRec> hrec;
    DBuf<uint32_t> hcnt;           // by rank: != 0 iff first occurrence of its key (bucket finish: count)
    DBuf<uint32_t> bH, bHs;        // bucket finish: per (bucket, block) counts, their scan
    DBuf<uint16_t> pkey16;         // bucket finish: low key bits, partitioned
    DBuf<XHit> xsend;              // hit exchange: valid hits partitioned by owner rank
    DBuf<uint32_t> xH, xHs;        // ... per (owner, block) counts, their scan
    DBuf<uint64_t> xcnt;           // ... per owner totals (device)
    uint64_t *h_xcnt = nullptr;    // ... pinned host copy (XP_MAXW)
    bool long_seg = false;         // INFO_LONGSEG seen this session
    bool chunk_open = false;       // the last chunk did not end with '\n'
    bool out_pending = false;      // unique count of the last finish not yet read back (h_tail[8])
    bool timing_pending = false;   // finish events not yet read
    DBuf<uint64_t> xord, xord2, xkey, xkey2;   // cross list
    DBuf<uint64_t> xkeyl, xkeyh;               // ... wide keys (xkey then holds the entry's index)
    DBuf<uint32_t> xslot;
    // finish outputs
    DBuf<uint64_t> ukey, first, cnt_out, roff;
    DBuf<Agg> uval;
    DBuf<uint8_t> keys_out;
    uint64_t n_out = 0;            // ordered entries of the last finish (device)
    // records & lines
    DBuf<Record> recs;
    DBuf<SeqLine> lines;
    DBuf<uint8_t> rec_keys;
    // scratch
    DBuf<uint8_t> tmp;
    // device scalars, one block so that a feed reads them back with one copy:
    // [0] rec_count [1] ovf_count [2] cross count [3] chunk hits [4] unique keys
    // [5] err (u32) [6] line count [7] chunk ends open
    uint64_t *d_scal = nullptr;
    unsigned int *d_ticket = nullptr, *d_err = nullptr;
    unsigned long long *d_rec_count = nullptr, *d_line_count = nullptr, *d_ovf_count = nullptr;
    unsigned long long *d_xcount = nullptr, *d_chunk_hits = nullptr, *d_ends_open = nullptr;
    uint64_t *d_nuniq = nullptr;
    StreamPos *d_pos = nullptr, *d_pos_saved = nullptr;
    uint8_t *d_P = nullptr;        // prefix bytes (decode)
    uint8_t *d_PR = nullptr;       // [0,64) P, [64,128) rc(P) (tile kernel), [128,..) full P (general kernel)
    // host side
    uint64_t abs_offset = 0;
    bool open_stream = false;      // reset called, not finished
    std::unordered_map<std::string, Ent> exotic;
    uint64_t *h_small = nullptr;   // pinned (24 words): [0..7] copy of d_scal, [8..11] pos, [12..16] table feed
    uint64_t *h_tail = nullptr;    // pinned, mapped, coherent: d_scal[0..7] written by the chunk tail kernel
    uint64_t *d_tail = nullptr;    // ... its device address
    unsigned int *d_hticket = nullptr;   // chunk tail last-block ticket (d_scal[8])
    uint64_t tail_seq = 0;         // last chunk sequence number handed to the chunk tail kernel
    bool feed_timing_pending = false;   // scan / feed events of the last chunk not yet read
    uint32_t prep_flags = 0;       // PREP_RESET / PREP_SETPOS pending for the next feed's prologue
    // the last packed-path chunk, launched but not yet settled (its tail read,
    // overflows redone, counters applied): settle() before any other use
    struct Pending {
        bool active = false;
        ScanArgs a;
        HitArgs h;
        uint32_t n_tiles = 0, n_blocks = 0;
        TileSum init;
        const uint8_t *d = nullptr;
        uint64_t len = 0;
        hipStream_t s = nullptr;
    } pend;
    uint64_t prep_lines = 0;
    DBuf<uint8_t> batch;
    // table mode (kmer_table.hip)
    DBuf<uint64_t> tb1, tb2;       // pass-1 keys (session, partition-major per chunk); final entries -> tb1
    DBuf<uint32_t> tH, tnd;        // pass-1 / pass-2 histograms; distinct entries per bucket
    DBuf<uint64_t> tHs, tstart;    // their scans; bucket starts (TAB_NQ + 1)
    DBuf<uint64_t> tp1;            // pass-1 partition starts of the last chunk (TAB_NB)
    DBuf<TabUnit> tunits;          // pass-2 units, then TAB_NB partition heads
    DBuf<TabBig> tbig;             // entries with counts >= TAB_CMAX
    DBuf<uint32_t> tpc;            // pieces per sequence line (long lines)
    DBuf<uint32_t> tleft;          // [0] count, then [q, qe) pairs: units the sort final kernel left
    DBuf<uint64_t> tpb;            // ... their scan
    DBuf<SeqLine> tpieces;         // long lines cut into pieces of <= TAB_PIECE windows
    DBuf<unsigned long long> tstats;   // [0..2] final statistics, [3] big-list count, [4] digest
    uint64_t t_keys = 0;           // pass-1 keys of the session
    std::vector<uint64_t> t_cbase; // per chunk: first key in tb1
    std::vector<std::vector<uint64_t>> t_coff;   // per chunk: TAB_NB + 1 partition starts (chunk-relative)
    uint64_t t_canon = 0, t_nkeys = 0, t_sum = 0, t_nbig = 0;   // last finish
    bool t_done = false;           // a table finish holds results
    uint64_t *t_ent = nullptr;     // the table's entries (tb1, or the received keys' buffer after an exchange)
    DBuf<uint64_t> tsend;          // table exchange: send runs (sessions of several chunks)
    DBuf<uint64_t> trecv;          // group table mode: the keys this child owns, received from every child
    DBuf<TabSeg> tseg;             // ... and their segment table
    hipEvent_t tev[8] = {};        // table phase events
    // multi-device group (kmer_params.ndev > 1): one child context per device;
    // the group itself owns no device state beyond the merge buffers on
    // devices[0] (allocated through child 0)
    std::vector<kmer_ctx *> group;
    DBuf<uint64_t> gkeys, gkeys2;
    DBuf<Agg> gvals, gvals2;
    double t_ms[6] = {};           // table phase times since the reset: lines, hist1, scatter1, hist2, scatter2, final
    int n_cu = 0;
    // timing (HIP events on the context stream)
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr, ev3 = nullptr, ev4 = nullptr;
    hipEvent_t evw = nullptr;      // cross-stream wait (no timing)
    double scan_ms = 0.0, feed_ms = 0.0, finish_ms = 0.0;
    // FASTA input (KMER_FLAG_FASTA, kmer_fasta.hip): each chunk is rewritten
    // into FASTQ-shaped lines before it is counted
    bool fasta = false;
    DBuf<FaTile> fa_t, fa_x;       // per-tile functions, their exclusive scan (n_tiles + 1)
    DBuf<uint8_t> fa_out[2];       // rewritten chunks (alternating: the previous one may still be read)
    uint32_t fa_flip = 0;
    uint64_t fa_lines = 0;         // input lines of the session (kmerObj.lines)
    // progress of the current whole-input call (report_progress: monotone across a retry)
    bool progress_any = false;
    uint64_t progress_hw = 0;
};

namespace {

const uint64_t DEFAULT_BATCH = 1ull << 30;
const uint64_t FILE_BATCH = 256ull << 20;     // kmer_count_file read-ahead batch

#define HIPCHK(ctx, x)                                                                      \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            (ctx)->err = std::string("HIP error: ") + hipGetErrorString(e_) + " at " #x;    \
            return KMER_E_DEVICE;                                                           \
        }                                                                                   \
    } while (0)

// rocPRIM call with context-owned temporary storage: size query, grow, run.
// `CALL` is an expression in the names t (storage) and b (its size).
#define ROCPRIM_RUN(ctx, CALL)                                                          \
    do {                                                                                \
        size_t b = 0;                                                                   \
        void *t = nullptr;                                                              \
        HIPCHK(ctx, CALL);                                                              \
        HIPCHK(ctx, (ctx)->tmp.ensure(b + 16, (ctx)->stream));                          \
        t = (ctx)->tmp.p;                                                               \
        HIPCHK(ctx, CALL);                                                              \
    } while (0)

// Progress callback of kmer_count_file / kmer_count_buffer: non-decreasing over
// the whole call, so a long-line retry (which reads the input again from the
// start) reports nothing until it is back at what was already reported.
void report_progress(kmer_ctx *c, uint64_t done, uint64_t total) {
    if (!c->p.progress) return;
    if (c->progress_any && done < c->progress_hw) return;
    c->progress_any = true;
    c->progress_hw = done;
    c->p.progress(c->p.progress_user, done, total);
}

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

int bit_width(uint64_t x) { return x ? 64 - __builtin_clzll(x) : 0; }

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
    HIPCHK(c, c->roff.ensure(n, s));
    std::vector<uint64_t> off(n);
    for (uint64_t i = 0; i < n; ++i) off[i] = i * k;
    HIPCHK(c, hipMemcpyAsync(c->roff.p, off.data(), n * 8, hipMemcpyHostToDevice, s));
    HIPCHK(c, launch_gather_records(c->recs.p, c->roff.p, n, d_data, c->rec_keys.p, s));
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
    return KMER_OK;
}

// ---------------------------------------------------------------------------
// fast path feed
// ---------------------------------------------------------------------------
struct IsHead {
    __host__ __device__ uint32_t operator()(uint32_t c) const { return c ? 1u : 0u; }
};

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
}

// One attempt at the pending chunk: scan, tile scan, hit resolution and the
// chunk tail (position, counters -> mapped host memory), all on the stream.
kmer_status launch_chunk(kmer_ctx *c) {
    auto &p = c->pend;
    const hipStream_t s = p.s;
    HIPCHK(c, hipEventRecord(c->ev0, s));
    if (c->planes) HIPCHK(c, launch_scan_planes(p.a, c->pargs, c->n_cu, s));
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

#define SETTLE(ctx)                                                                       \
    do {                                                                                  \
        if (!(ctx)->group.empty()) return fail(ctx, KMER_E_STATE, "single-device call on a group context"); \
        const kmer_status st_ = settle(ctx);                                              \
        if (st_) return st_;                                                              \
    } while (0)

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
    HIPCHK(c, hipMemcpyAsync(c->tp_cnt.p, cnt.data(), n_tiles * 8, hipMemcpyHostToDevice, s));
    HIPCHK(c, hipMemcpyAsync(c->tp_lnl.p, last.data(), n_tiles * 8, hipMemcpyHostToDevice, s));
    HIPCHK(c, hipMemcpyAsync(c->d_pos, &pos, sizeof(pos), hipMemcpyHostToDevice, s));
    HIPCHK(c, hipStreamSynchronize(s));
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

kmer_status general_feed(kmer_ctx *c, const uint8_t *d, uint64_t len, uint32_t n_tiles, hipStream_t s) {
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

// Dense-hit path: every window of every sequence line goes to its rank slot.
kmer_status windows_feed(kmer_ctx *c, const uint8_t *d, uint64_t len, uint32_t n_tiles, hipStream_t s) {
    const uint64_t li0 = c->host_lines;
    kmer_status st;
    HIPCHK(c, hipEventRecord(c->ev0, s));
    uint64_t n_nl = 0, n_seq = 0;
    st = chunk_lines(c, d, len, n_tiles, s, true, &n_nl, &n_seq);
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

// ---------------------------------------------------------------------------
// table mode feed (kernels: kmer_table.hip)
// ---------------------------------------------------------------------------
// Pass 1 of one chunk: its sequence lines, then per workgroup share of lines
// a histogram of keys by partition, a scan, and the scatter into tb1 after
// the session's earlier keys.  Non-ACGT windows go to the host map.
float ev_ms(kmer_ctx *c, hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) ms = 0.f;
    return ms;
}

kmer_status table_feed(kmer_ctx *c, const uint8_t *d, uint64_t len, uint32_t n_tiles, hipStream_t s) {
    const uint64_t li0 = c->host_lines;
    HIPCHK(c, hipEventRecord(c->ev0, s));
    HIPCHK(c, hipEventRecord(c->tev[0], s));
    uint64_t n_nl = 0, n_seq = 0;
    kmer_status st = chunk_lines(c, d, len, n_tiles, s, false, &n_nl, &n_seq);
    if (st) return st;
    HIPCHK(c, launch_pos_after(c->d_pos, li0 + n_nl, d, len, c->d_ends_open, s));
    c->host_lines = li0 + n_nl;
    // long lines -> pieces of <= TAB_PIECE windows (balance pass 1's shares)
    const SeqLine *plines = c->lines.p;
    uint64_t n_items = n_seq;
    if (n_seq) {
        HIPCHK(c, c->tpc.ensure(n_seq + 1, s));
        HIPCHK(c, c->tpb.ensure(n_seq, s));
        uint32_t *split = c->tpc.p + n_seq;             // set when a line is not exactly one piece
        HIPCHK(c, hipMemsetAsync(split, 0, 4, s));
        HIPCHK(c, launch_tab_piece_count(c->wcount.p, n_seq, c->tpc.p, split, s));
        HIPCHK(c, hipMemcpyAsync(c->h_small + 16, split, 4, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        uint64_t n_pieces = n_seq;                // (no split: one piece per line)
        if ((uint32_t)c->h_small[16]) {
            ROCPRIM_RUN(c, rocprim::exclusive_scan(t, b, c->tpc.p, c->tpb.p, (uint64_t)0, (size_t)n_seq,
                                                   rocprim::plus<uint64_t>(), s));
            HIPCHK(c, hipMemcpyAsync(c->h_small + 12, c->tpb.p + n_seq - 1, 8, hipMemcpyDeviceToHost, s));
            HIPCHK(c, hipMemcpyAsync(c->h_small + 13, c->tpc.p + n_seq - 1, 4, hipMemcpyDeviceToHost, s));
            HIPCHK(c, hipStreamSynchronize(s));
            n_pieces = c->h_small[12] + (uint32_t)c->h_small[13];
        }
        if (n_pieces == 0) {
            n_items = 0;                          // no line holds a window
        } else if ((uint32_t)c->h_small[16]) {    // long lines (or empty ones, dropped on the way)
            HIPCHK(c, c->tpieces.ensure(std::max<uint64_t>(n_pieces, 1), s));
            HIPCHK(c, launch_tab_piece_write(c->lines.p, c->wcount.p, c->tpb.p, n_seq, c->p.k, c->tpieces.p, s));
            plines = c->tpieces.p;
            n_items = n_pieces;
        }
    }
    HIPCHK(c, hipEventRecord(c->tev[1], s));
    if (n_items) {
        TabArgs a;
        memset(&a, 0, sizeof(a));
        a.data = d;
        a.len = len;
        a.lines = plines;
        a.n_lines = n_items;
        const uint64_t nwg0 = std::min<uint64_t>(8192, (n_items + 63) / 64);
        a.lpw = (n_items + nwg0 - 1) / nwg0;
        a.nwg = (uint32_t)((n_items + a.lpw - 1) / a.lpw);
        a.k = c->p.k;
        for (size_t i = 0; i < c->prefix.size(); ++i) {
            const uint8_t ch = (uint8_t)c->prefix[i];
            a.plo |= ((((uint32_t)ch >> 1) ^ ((uint32_t)ch >> 2)) & 1u) << i;
            a.phi |= (((uint32_t)ch >> 2) & 1u) << i;
        }
        a.pmask = c->prefix.size() >= 32 ? ~0u : ((1u << c->prefix.size()) - 1u);
        a.canonical = (c->p.flags & KMER_FLAG_CANONICAL) ? 1u : 0u;
        a.err = c->d_err;
        const uint64_t nh = (uint64_t)TAB_NB * a.nwg;
        HIPCHK(c, c->tH.ensure(nh, s));
        HIPCHK(c, c->tHs.ensure(nh, s));
        HIPCHK(c, c->tp1.ensure(TAB_NB, s));
        a.H1 = c->tH.p;
        HIPCHK(c, launch_tab_hist1(a, s));
        ROCPRIM_RUN(c, rocprim::exclusive_scan(t, b, c->tH.p, c->tHs.p, (uint64_t)0, (size_t)nh,
                                               rocprim::plus<uint64_t>(), s));
        HIPCHK(c, launch_tab_p1_offsets(c->tHs.p, a.nwg, c->tp1.p, s));
        std::vector<uint64_t> off(TAB_NB + 1);
        HIPCHK(c, hipMemcpyAsync(off.data(), c->tp1.p, TAB_NB * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(c->h_small + 14, c->tHs.p + nh - 1, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(c->h_small + 15, c->tH.p + nh - 1, 4, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipEventRecord(c->tev[2], s));
        HIPCHK(c, hipStreamSynchronize(s));
        c->t_ms[0] += ev_ms(c, c->tev[0], c->tev[1]);
        c->t_ms[1] += ev_ms(c, c->tev[1], c->tev[2]);
        const uint64_t n_c = c->h_small[14] + (uint32_t)c->h_small[15];
        off[TAB_NB] = n_c;
        HIPCHK(c, c->tb1.ensure(c->t_keys + n_c, s, true, c->t_keys));
        a.H1s = c->tHs.p;
        a.base = c->t_keys;
        a.B1 = c->tb1.p;
        for (int attempt = 0;; ++attempt) {
            a.recs = c->recs.p;
            a.rec_count = c->d_rec_count;
            a.rec_cap = c->recs.cap;
            HIPCHK(c, hipMemsetAsync(c->d_rec_count, 0, 8, s));
            HIPCHK(c, hipEventRecord(c->tev[2], s));
            HIPCHK(c, launch_tab_scatter1(a, s));
            HIPCHK(c, hipEventRecord(c->tev[3], s));
            HIPCHK(c, hipMemcpyAsync(c->h_small, c->d_scal, 8 * 8, hipMemcpyDeviceToHost, s));
            HIPCHK(c, hipStreamSynchronize(s));
            const float ms_s1 = ev_ms(c, c->tev[2], c->tev[3]);
            const uint32_t e = (uint32_t)c->h_small[5];
            st = check_err(c, e);
            if (st) return st;
            if (!(e & ERR_REC_OVERFLOW)) {         // (a redo rewrites the same key ranges)
                c->t_ms[2] += ms_s1;
                break;
            }
            if (attempt == 7) return fail(c, KMER_E_OOM, "record list kept overflowing");
            HIPCHK(c, hipMemsetAsync(c->d_err, 0, 4, s));
            st = ensure_records(c, c->h_small[0] + 1024);
            if (st) return st;
        }
        const uint64_t nrec = c->h_small[0];
        if (nrec) {
            st = drain_records(c, d, nrec, s);
            if (st) return st;
        }
        c->t_cbase.push_back(c->t_keys);
        c->t_coff.push_back(std::move(off));
        c->t_keys += n_c;
    }
    HIPCHK(c, hipEventRecord(c->ev1, s));
    HIPCHK(c, hipMemcpyAsync(c->h_small, c->d_scal, 8 * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    float ms = 0.f;
    HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
    c->scan_ms += ms;
    c->feed_ms += ms;
    c->chunk_open = c->h_small[7] != 0;
    c->abs_offset += len;
    return KMER_OK;
}

uint64_t inv_odd(uint64_t a) {   // inverse of an odd number mod 2^64 (Newton)
    uint64_t x = a;
    for (int i = 0; i < 5; ++i) x *= 2 - a * x;
    return x;
}

// Pass 2 + final of the session: pass-1 partitions (one run per chunk) are
// cut into units; each unit's keys go to their 2^20 buckets in tb2; the
// final kernel merges each bucket in LDS and writes its entries into tb1.
// B1: the pass-1 keys (default: this session's, tb1); [qlo, qhi): the buckets
// present (multi-GPU: this rank's partitions; the others are left empty).
kmer_status table_finish(kmer_ctx *c, const uint64_t *B1 = nullptr, uint32_t qlo = 0, uint32_t qhi = TAB_NQ) {
    hipStream_t s = c->stream;
    c->t_canon = c->t_nkeys = c->t_sum = c->t_nbig = 0;
    c->t_done = true;
    const uint64_t n = c->t_keys;
    if (n == 0) return KMER_OK;
    // the table is written over the pass-1 keys (dead after pass 2)
    if (!B1) B1 = c->tb1.p;
    c->t_ent = const_cast<uint64_t *>(B1);
    std::vector<TabUnit> units;
    std::vector<TabUnit> heads(TAB_NB);
    uint64_t ubase = 0;
    for (uint32_t p = 0; p < TAB_NB; ++p) {
        const size_t first = units.size();
        for (size_t ch = 0; ch < c->t_cbase.size(); ++ch) {
            const uint64_t a0 = c->t_coff[ch][p], a1 = c->t_coff[ch][p + 1];
            for (uint64_t o = a0; o < a1; o += TAB_UNIT) {
                TabUnit u{};
                u.start = c->t_cbase[ch] + o;
                u.len = (uint32_t)std::min<uint64_t>(TAB_UNIT, a1 - o);
                units.push_back(u);
            }
        }
        if (units.size() == first) units.push_back(TabUnit{});   // empty partition: zero histogram row
        const uint32_t nun = (uint32_t)(units.size() - first);
        for (size_t i = first; i < units.size(); ++i) {
            units[i].u = (uint32_t)(i - first);
            units[i].nunits = nun;
            units[i].hbase = ubase * TAB_NB;
        }
        heads[p] = units[first];
        ubase += nun;
    }
    const uint64_t n_units = units.size();
    if (n_units >= (1ull << 31)) return fail(c, KMER_E_BAD_PARAM, "too many table units");
    units.insert(units.end(), heads.begin(), heads.end());
    HIPCHK(c, c->tunits.ensure(units.size(), s));
    HIPCHK(c, hipMemcpyAsync(c->tunits.p, units.data(), units.size() * sizeof(TabUnit), hipMemcpyHostToDevice, s));
    const uint64_t nh = n_units * TAB_NB;
    HIPCHK(c, c->tH.ensure(nh, s));
    HIPCHK(c, c->tHs.ensure(nh, s));
    HIPCHK(c, c->tb2.ensure(n, s));
    HIPCHK(c, c->tstart.ensure(TAB_NQ + 1, s));
    HIPCHK(c, c->tnd.ensure(TAB_NQ, s));
    HIPCHK(c, c->tbig.ensure(1 << 16, s));
    HIPCHK(c, c->tstats.ensure(5, s));
    HIPCHK(c, hipEventRecord(c->tev[4], s));
    HIPCHK(c, launch_tab_hist2(B1, c->tunits.p, (uint32_t)n_units, c->tH.p, s));
    ROCPRIM_RUN(c, rocprim::exclusive_scan(t, b, c->tH.p, c->tHs.p, (uint64_t)0, (size_t)nh,
                                           rocprim::plus<uint64_t>(), s));
    HIPCHK(c, hipEventRecord(c->tev[5], s));
    HIPCHK(c, launch_tab_scatter2(B1, c->tunits.p, (uint32_t)n_units, c->tHs.p, c->tb2.p, s));
    HIPCHK(c, hipEventRecord(c->tev[6], s));
    HIPCHK(c, launch_tab_starts(c->tHs.p, c->tunits.p + n_units, n, c->tstart.p, s));
    HIPCHK(c, hipMemsetAsync(c->tstats.p, 0, 4 * sizeof(unsigned long long), s));
    TabFinal f;
    memset(&f, 0, sizeof(f));
    f.B2 = c->tb2.p;
    f.start = c->tstart.p;
    f.out = c->t_ent;
    f.nd = c->tnd.p;
    const uint64_t mean = n / TAB_NQ;
    uint64_t range_keys = 3000;               // mean keys per LDS range (load ~0.37: short probes; measured best at C3)
    if (const char *rk = exp_env("KMERHIP_TAB_RANGE")) range_keys = std::max<uint64_t>(64, strtoull(rk, nullptr, 10));
    while (f.sub_bits < 16 && (mean >> f.sub_bits) > range_keys) ++f.sub_bits;
    f.range_keys = (uint32_t)std::min<uint64_t>(range_keys, TAB_CAP);
    f.cap = (c->p.flags & KMER_FLAG_TABLE_SPLIT_TEST) ? 64 : TAB_CAP;
    if (const char *ab = exp_env("KMERHIP_TAB_ABLATE")) f.ablate = (uint32_t)atoi(ab);   // experiments only
    f.big = c->tbig.p;
    f.big_count = c->tstats.p + 3;
    f.big_cap = c->tbig.cap;
    f.err = c->d_err;
    f.k = c->p.k;
    for (size_t i = 0; i < c->prefix.size(); ++i) {
        const uint8_t ch = (uint8_t)c->prefix[i];
        f.plo |= ((((uint32_t)ch >> 1) ^ ((uint32_t)ch >> 2)) & 1u) << i;
        f.phi |= (((uint32_t)ch >> 2) & 1u) << i;
    }
    f.pmask = c->prefix.size() >= 32 ? ~0u : ((1u << c->prefix.size()) - 1u);
    f.inv = inv_odd(TAB_MUL);
    f.canonical = (c->p.flags & KMER_FLAG_CANONICAL) ? 1u : 0u;
    f.stats = c->tstats.p;
    f.qlo = qlo;
    f.qhi = qhi;
    if (qlo != 0 || qhi != TAB_NQ) HIPCHK(c, hipMemsetAsync(c->tnd.p, 0, TAB_NQ * sizeof(uint32_t), s));
    const uint32_t fgrid = (uint32_t)std::max(c->n_cu, 1);
    std::vector<uint64_t> hprof;
#ifdef TAB_PROF
    if (exp_env("KMERHIP_TAB_PROF")) {         // experiments (-DTAB_PROF build): per-phase clocks of the final kernel
#else
    if (false) {
#endif
        HIPCHK(c, hipMalloc((void **)&f.prof, fgrid * 64ull));
        HIPCHK(c, hipMemsetAsync(f.prof, 0, fgrid * 64ull, s));
        hprof.resize(fgrid * 8ull);
    }
    // the sort kernel (two workgroups per CU) takes every unit it can; the
    // general kernel (hash path, range splits) takes the ones it leaves
    // (crowded buckets, many copies of a key).  KMERHIP_TAB_FINAL=general: the
    // general kernel alone (A/B experiments).
    const char *fk = exp_env("KMERHIP_TAB_FINAL");
    const bool sort_first = !(fk && strcmp(fk, "general") == 0) && !f.prof &&
                            !(c->p.flags & KMER_FLAG_TABLE_SPLIT_TEST);
    HIPCHK(c, hipEventRecord(c->tev[2], s));
    if (sort_first) {
        HIPCHK(c, c->tleft.ensure(2ull * TAB_NQ + 1, s));
        f.left = c->tleft.p + 1;
        f.left_n = c->tleft.p;
        HIPCHK(c, hipMemsetAsync(c->tleft.p, 0, 4, s));
        HIPCHK(c, launch_tab_sort_final(f, 2 * fgrid, s));
    }
    HIPCHK(c, launch_tab_final(f, fgrid, s));
    HIPCHK(c, hipEventRecord(c->tev[7], s));
    if (f.prof) {
        HIPCHK(c, hipMemcpyAsync(hprof.data(), f.prof, fgrid * 64ull, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        (void)hipFree(f.prof);
        double ph[6] = {0, 0, 0, 0, 0, 0};
        uint64_t ranges = 0, buckets = 0;
        for (uint32_t g = 0; g < fgrid; ++g) {
            for (int i = 0; i < 6; ++i) ph[i] += i == 4 ? 0 : (double)hprof[g * 8 + i] * 0.01 / fgrid;   // us
            ranges += hprof[g * 8 + 4] >> 32;
            buckets += hprof[g * 8 + 4] & 0xFFFFFFFFull;
        }
        fprintf(stderr, "tab_final prof (us per workgroup): load+setup %.0f range-syncs %.0f insert %.0f emit %.0f "
                        "empty %.0f | buckets %llu ranges %llu sub_bits %u\n", ph[0], ph[1], ph[2], ph[3], ph[5],
                (unsigned long long)buckets, (unsigned long long)ranges, f.sub_bits);
    }
    HIPCHK(c, hipMemcpyAsync(c->h_small + 8, c->tstats.p, 4 * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(c->h_small, c->d_scal, 8 * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    c->t_ms[3] += ev_ms(c, c->tev[4], c->tev[5]);
    c->t_ms[4] += ev_ms(c, c->tev[5], c->tev[6]);
    c->t_ms[5] += ev_ms(c, c->tev[2], c->tev[7]);
    const uint32_t e = (uint32_t)c->h_small[5];
    if (e & ERR_COUNT_OVERFLOW) return fail(c, KMER_E_TOO_MANY_KEYS, "a k-mer count exceeds 2^32 - 1");
    if (e & ERR_BIG_OVERFLOW) return fail(c, KMER_E_OOM, "too many k-mers with counts >= 2^20");
    if (e & ERR_TAB_SPLIT) return fail(c, KMER_E_DEVICE, "table bucket could not be split");
    c->t_canon = c->h_small[8];
    c->t_nkeys = c->h_small[9];
    c->t_sum = c->h_small[10];
    c->t_nbig = c->h_small[11];
    c->n_out = c->t_nkeys;
    return KMER_OK;
}

// Canonical classes of the record keys (KMER_FLAG_CANONICAL: forward windows)
std::unordered_map<std::string, uint64_t> canonical_records(const kmer_ctx *c) {
    std::unordered_map<std::string, uint64_t> cls;
    for (auto &kv : c->exotic) {
        std::string r(kv.first.rbegin(), kv.first.rend());
        for (char &ch : r) ch = (char)comp((uint8_t)ch);
        cls[std::min(kv.first, r)] += kv.second.count;
    }
    return cls;
}

// Host result of a table finish: every canonical entry expanded into its Map
// keys (c and rc c, prefix-filtered; palindromes counted twice), plus the
// record keys; entries sorted by key bytes (the table has no order).
kmer_status build_table_result(kmer_ctx *c, uint64_t lines, kmer_result **out) {
    kmer_result *r = new (std::nothrow) kmer_result();
    if (!r) return fail(c, KMER_E_OOM, "host allocation failed");
    r->lines = lines;
    std::vector<std::pair<std::string, uint64_t>> ents;
    const uint32_t k = c->p.k;
    if (c->t_keys) {
        hipStream_t s = c->stream;
        std::vector<uint64_t> start(TAB_NQ + 1), ent(c->t_keys);
        std::vector<uint32_t> nd(TAB_NQ);
        std::vector<TabBig> big(c->t_nbig);
        bool ok = hipMemcpyAsync(start.data(), c->tstart.p, start.size() * 8, hipMemcpyDeviceToHost, s) == hipSuccess &&
                  hipMemcpyAsync(nd.data(), c->tnd.p, nd.size() * 4, hipMemcpyDeviceToHost, s) == hipSuccess &&
                  hipMemcpyAsync(ent.data(), c->t_ent, ent.size() * 8, hipMemcpyDeviceToHost, s) == hipSuccess;
        if (ok && !big.empty())
            ok = hipMemcpyAsync(big.data(), c->tbig.p, big.size() * sizeof(TabBig), hipMemcpyDeviceToHost, s) == hipSuccess;
        if (!ok || hipStreamSynchronize(s) != hipSuccess) {
            delete r;
            return fail(c, KMER_E_DEVICE, "result copy failed");
        }
        std::unordered_map<uint64_t, uint64_t> bigc;
        for (auto &b : big) bigc[b.h] = b.count;
        const uint64_t inv = inv_odd(TAB_MUL);
        const bool canon = (c->p.flags & KMER_FLAG_CANONICAL) != 0;
        const uint64_t kmask = k >= 32 ? 0xFFFFFFFFull : ((1ull << k) - 1);
        std::string key(k, 'A'), rkey(k, 'A');
        for (uint32_t q = 0; q < TAB_NQ; ++q) {
            for (uint32_t i = 0; i < nd[q]; ++i) {
                const uint64_t w = ent[start[q] + i];
                const uint64_t h = ((uint64_t)q << TAB_RBITS) | (w >> 20);
                uint64_t cnt = w & TAB_CMAX;
                if (cnt == TAB_CMAX) cnt = bigc[h];
                const uint64_t x = h * inv;          // tab_mix^-1
                const uint64_t lo = x & kmask, hi = (x >> k) & kmask;
                for (uint32_t j = 0; j < k; ++j) {
                    const uint32_t v = (uint32_t)(((hi >> j) & 1u) << 1 | ((lo >> j) & 1u));
                    key[j] = "ACGT"[v];
                    rkey[k - 1 - j] = "TGCA"[v];
                }
                const bool pal = key == rkey;
                if (canon) {                          // one key per class, counted once per window
                    const std::string &ck = key < rkey ? key : rkey;
                    if (ck.compare(0, c->prefix.size(), c->prefix) == 0) ents.emplace_back(ck, cnt);
                    continue;
                }
                if (key.compare(0, c->prefix.size(), c->prefix) == 0) ents.emplace_back(key, pal ? 2 * cnt : cnt);
                if (!pal && rkey.compare(0, c->prefix.size(), c->prefix) == 0) ents.emplace_back(rkey, cnt);
            }
        }
    }
    if (c->p.flags & KMER_FLAG_CANONICAL) {
        // record keys (non-ACGT windows; forward windows only, unfiltered):
        // classed under min(x, rc x), then the prefix is tested on that key
        for (auto &kv : canonical_records(c))
            if (kv.first.compare(0, c->prefix.size(), c->prefix) == 0) ents.emplace_back(kv.first, kv.second);
    } else {
        for (auto &kv : c->exotic) ents.emplace_back(kv.first, kv.second.count);
    }
    std::sort(ents.begin(), ents.end());
    r->keys.reserve(ents.size() * k);
    r->offsets.reserve(ents.size() + 1);
    r->counts.reserve(ents.size());
    for (auto &e : ents) {
        r->keys.insert(r->keys.end(), e.first.begin(), e.first.end());
        r->offsets.push_back(r->keys.size());
        r->counts.push_back(e.second);
        r->firsts.push_back(0);
    }
    *out = r;
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
    c->t_cbase.clear();
    c->t_coff.clear();
    c->t_done = false;
    c->t_ent = nullptr;
    for (double &x : c->t_ms) x = 0.0;
    c->scan_ms = c->feed_ms = c->finish_ms = 0.0;
    c->open_stream = true;
    return KMER_OK;
}

// ---------------------------------------------------------------------------
// finish
// ---------------------------------------------------------------------------
// Place the cross entries: sorted by order key they take the natural slots
// sorted ascending (the slots that tile-local ranking left to them).
kmer_status apply_cross(kmer_ctx *c) {
    hipStream_t s = c->stream;
    const uint64_t n = c->n_cross;
    if (n == 0) return KMER_OK;
    uint32_t *k32 = c->narrow ? c->rkey32.p : nullptr;
    if (!c->long_seg) {
        HIPCHK(c, launch_cross_segsort(c->xord.p, c->xkey.p, c->xslot.p, n, c->rkey.p, k32, c->rord.p, c->pbits, s));
    } else if (n <= XSMALL_MAX) {
        HIPCHK(c, launch_cross_sort_small(c->xslot.p, c->xord.p, c->xkey.p, n, c->rkey.p, k32, c->rord.p, s));
    } else {
        StreamPos pos;
        kmer_status st = read_pos(c, &pos);
        if (st) return st;
        HIPCHK(c, c->xord2.ensure(n, s));
        HIPCHK(c, c->xkey2.ensure(n, s));
        rocprim::double_buffer<uint64_t> ob(c->xord.p, c->xord2.p);
        rocprim::double_buffer<uint64_t> kb(c->xkey.p, c->xkey2.p);
        const int obits = std::min(64, bit_width(((pos.lines + 1) << (c->pbits + 1)) | ((2ull << c->pbits) - 1ull)));
        ROCPRIM_RUN(c, rocprim::radix_sort_pairs(t, b, ob, kb, (size_t)n, 0, obits, s));
        HIPCHK(c, launch_cross_scatter(c->xslot.p, ob.current(), kb.current(), n, c->rkey.p, k32, c->rord.p, s));
    }
    if (c->wide) HIPCHK(c, launch_cross_wide_fix(c->xslot.p, n, c->xkeyl.p, c->xkeyh.p, c->rkey.p, c->rkeyh.p, s));
    c->n_cross = 0;
    return KMER_OK;
}

// stable radix sort of (key, rank), then the heads.  Without per-entry
// counts the by-rank keys are kept (the sort writes a copy), hcnt is
// prefilled with 1 and only repeated / invalid keys are scattered
// (heads_sparse); merged partials (with_counts) sum u64 counts into HeadRecs.
template <typename K>
kmer_status sort_and_heads(kmer_ctx *c, K *keys, K *keys2, uint64_t n, bool with_counts) {
    hipStream_t s = c->stream;
    const uint64_t invalid = c->kbits >= 63 ? ~0ull : (1ull << c->kbits);
    const int end_bit = std::min<int>(8 * (int)sizeof(K), (int)c->kbits + 1);   // + the invalid-key bit
    if (!with_counts) {
        rocprim::counting_iterator<uint32_t> iota(0u);
        ROCPRIM_RUN(c, rocprim::radix_sort_pairs(t, b, keys, keys2, iota, c->ridx2.p, (size_t)n, 0, end_bit, s));
        HIPCHK(c, hipMemsetD32Async((hipDeviceptr_t)c->hcnt.p, 1, n, s));
        if (sizeof(K) == 4)
            HIPCHK(c, launch_heads_sparse(nullptr, (const uint32_t *)keys2, c->ridx2.p, n, invalid, c->hcnt.p, s));
        else
            HIPCHK(c, launch_heads_sparse((const uint64_t *)keys2, nullptr, c->ridx2.p, n, invalid, c->hcnt.p, s));
        return KMER_OK;
    }
    rocprim::double_buffer<K> kb(keys, keys2);
    rocprim::double_buffer<uint32_t> vb(c->ridx.p, c->ridx2.p);
    ROCPRIM_RUN(c, rocprim::radix_sort_pairs(t, b, kb, vb, (size_t)n, 0, end_bit, s));
    const uint64_t *rcnt = c->rcnt.p;
    if (sizeof(K) == 4)
        HIPCHK(c, launch_heads32((const uint32_t *)kb.current(), vb.current(), n, (uint32_t)invalid, rcnt, c->hrec.p, c->hcnt.p, s));
    else
        HIPCHK(c, launch_heads((const uint64_t *)kb.current(), vb.current(), n, invalid, rcnt, c->hrec.p, c->hcnt.p, s));
    return KMER_OK;
}

// wide keys (two words): stable (lo, rank) sort, then a stable sort of the
// high words by that order -> ranks ordered by (hi, lo), ascending within a
// key; heads over the pairs (hcnt prefilled with 1, as the sparse heads)
kmer_status sort_and_heads_wide(kmer_ctx *c, uint64_t n) {
    hipStream_t s = c->stream;
    HIPCHK(c, c->whA.ensure(n, s));
    HIPCHK(c, c->whB.ensure(n, s));
    HIPCHK(c, c->ridx3.ensure(n, s));
    rocprim::counting_iterator<uint32_t> iota(0u);
    ROCPRIM_RUN(c, rocprim::radix_sort_pairs(t, b, c->rkey.p, c->rkey2.p, iota, c->ridx2.p, (size_t)n, 0, 64, s));
    HIPCHK(c, launch_gather_u64(c->rkeyh.p, c->ridx2.p, n, c->whA.p, s));
    const int hbits = (int)c->kbits - 64 + 1;    // + the invalid bit
    ROCPRIM_RUN(c, rocprim::radix_sort_pairs(t, b, c->whA.p, c->whB.p, c->ridx2.p, c->ridx3.p, (size_t)n, 0, hbits, s));
    HIPCHK(c, launch_gather_u64(c->rkey.p, c->ridx3.p, n, c->rkey2.p, s));
    HIPCHK(c, hipMemsetD32Async((hipDeviceptr_t)c->hcnt.p, 1, n, s));
    HIPCHK(c, launch_heads_wide(c->whB.p, c->rkey2.p, c->ridx3.p, n, 1ull << (c->kbits - 64), c->hcnt.p, s));
    return KMER_OK;
}

// bucket partition + per-bucket LDS tables (keys of <= 24 bits)
kmer_status bucket_heads(kmer_ctx *c, uint64_t n) {
    hipStream_t s = c->stream;
    const uint32_t shift = std::min<uint32_t>(c->kbits, BKT_LOW);
    const uint32_t nb = 1u << (c->kbits - shift);
    const uint64_t nblk64 = (n + BKT_EPB_HOST - 1) / BKT_EPB_HOST;
    if (nblk64 > 0x7FFFFFFFull) return fail(c, KMER_E_BAD_PARAM, "too many hits");
    const uint32_t nblk = (uint32_t)nblk64;
    const uint32_t invalid = 1u << c->kbits;
    HIPCHK(c, c->bH.ensure((uint64_t)nb * nblk, s));
    HIPCHK(c, c->bHs.ensure((uint64_t)nb * nblk, s));
    HIPCHK(c, c->pkey16.ensure(n, s));
    HIPCHK(c, c->ridx2.ensure(n, s));
    HIPCHK(c, launch_bucket_hist(c->rkey32.p, n, invalid, shift, nb, nblk, c->bH.p, c->hcnt.p, s));
    ROCPRIM_RUN(c, rocprim::exclusive_scan(t, b, c->bH.p, c->bHs.p, 0u, (size_t)nb * nblk, rocprim::plus<uint32_t>(), s));
    HIPCHK(c, launch_bucket_scatter(c->rkey32.p, n, invalid, shift, nb, nblk, c->bHs.p, c->pkey16.p, c->ridx2.p, s));
    HIPCHK(c, launch_bucket_heads(c->pkey16.p, c->ridx2.p, c->bHs.p, c->bH.p, nb, nblk, shift, c->hcnt.p, s));
    return KMER_OK;
}

struct KeyValid32 {
    uint32_t inv;
    __host__ __device__ bool operator()(uint32_t k) const { return k != inv; }
};
struct KeyValid64 {
    uint64_t inv;
    __host__ __device__ bool operator()(uint64_t k) const { return k != inv; }
};

// Dense-hit path with a prefix: every window of a sequence line holds a rank
// slot and the windows that do not start with the prefix (or its reverse
// complement) carry the invalid key.  The matching ones are compacted, in
// rank order, before the finish sorts them -- a 1-3-base prefix rejects most
// windows (C2 input, prefix ACG: 37.5 M of 2.7 G).
kmer_status compact_windows(kmer_ctx *c) {
    hipStream_t s = c->stream;
    const uint64_t n = c->n_hits;
    if (n == 0) return KMER_OK;
    const uint64_t invalid = c->kbits >= 63 ? ~0ull : (1ull << c->kbits);
    HIPCHK(c, c->ridx2.ensure(n, s));
    HIPCHK(c, c->csel.ensure(1, s));
    rocprim::counting_iterator<uint32_t> iota(0u);
    if (c->narrow) {
        auto fl = rocprim::make_transform_iterator(c->rkey32.p, KeyValid32{(uint32_t)invalid});
        ROCPRIM_RUN(c, rocprim::select(t, b, iota, fl, c->ridx2.p, c->csel.p, (size_t)n, s));
    } else {
        auto fl = rocprim::make_transform_iterator(c->rkey.p, KeyValid64{invalid});
        ROCPRIM_RUN(c, rocprim::select(t, b, iota, fl, c->ridx2.p, c->csel.p, (size_t)n, s));
    }
    HIPCHK(c, hipMemcpyAsync(c->h_small + 20, c->csel.p, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    const uint64_t n2 = c->h_small[20];
    if (n2 >= n) return KMER_OK;
    // gathered into the second buffers, copied back (the session buffers keep their size)
    if (c->narrow) {
        HIPCHK(c, c->rkey32b.ensure(n2 + 1, s));
        HIPCHK(c, launch_gather_u32(c->rkey32.p, c->ridx2.p, n2, c->rkey32b.p, s));
        HIPCHK(c, hipMemcpyAsync(c->rkey32.p, c->rkey32b.p, n2 * 4, hipMemcpyDeviceToDevice, s));
    } else {
        HIPCHK(c, c->rkey2.ensure(n2 + 1, s));
        HIPCHK(c, launch_gather_u64(c->rkey.p, c->ridx2.p, n2, c->rkey2.p, s));
        HIPCHK(c, hipMemcpyAsync(c->rkey.p, c->rkey2.p, n2 * 8, hipMemcpyDeviceToDevice, s));
    }
    HIPCHK(c, c->rord2.ensure(n2 + 1, s));
    HIPCHK(c, launch_gather_u64(c->rord.p, c->ridx2.p, n2, c->rord2.p, s));
    HIPCHK(c, hipMemcpyAsync(c->rord.p, c->rord2.p, n2 * 8, hipMemcpyDeviceToDevice, s));
    c->n_hits = n2;
    return KMER_OK;
}

// resolve a deferred unique count (finish without a host result)
kmer_status resolve_out(kmer_ctx *c) {
    kmer_status st = resolve_feed_timing(c);
    if (st) return st;
    if (c->out_pending) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        c->n_out = c->h_tail[8];
        c->out_pending = false;
    }
    if (c->timing_pending) {
        float ms = 0.f;
        HIPCHK(c, hipEventSynchronize(c->ev3));
        HIPCHK(c, hipEventElapsedTime(&ms, c->ev2, c->ev3));
        c->finish_ms = ms;
        c->timing_pending = false;
    }
    return KMER_OK;
}

// Rank arrays (rkey / rord / ridx [/ rcnt]) of n hits -> unique keys in
// first-occurrence order: stable radix sort of (key, rank); group heads flag
// their rank; a scan of the flags gives each unique key its output position.
// partial: (code, {first, count}) into ukey/uval; else decoded keys, counts
// and firsts into keys_out / cnt_out / first.  Returns the unique count.
// sync = false: the unique count is copied back asynchronously (resolve_out).
kmer_status rank_finish(kmer_ctx *c, uint64_t n, bool partial, bool with_counts, uint64_t *nu_out, bool sync = true) {
    hipStream_t s = c->stream;
    *nu_out = 0;
    if (n == 0) return KMER_OK;
    if (c->narrow) HIPCHK(c, c->rkey32b.ensure(n, s));
    else HIPCHK(c, c->rkey2.ensure(n, s));
    HIPCHK(c, c->ridx2.ensure(n, s));
    if (with_counts) HIPCHK(c, c->hrec.ensure(n, s));
    HIPCHK(c, c->hcnt.ensure(n + 4, s));
    HIPCHK(c, c->opos.ensure(n, s));
    if (partial) {
        HIPCHK(c, c->ukey.ensure(n, s));
        HIPCHK(c, c->uval.ensure(n, s));
    } else {
        HIPCHK(c, c->keys_out.ensure(n * c->p.k, s));
        HIPCHK(c, c->cnt_out.ensure(n, s));
        HIPCHK(c, c->first.ensure(n, s));
    }
    const uint64_t invalid = c->kbits >= 63 ? ~0ull : (1ull << c->kbits);
    kmer_status st;
    // (merged partials carry counts: the sort finish sums them in 64 bits)
    const bool bucket = c->narrow && c->kbits <= BKT_LOW + 11 && !with_counts && !(c->p.flags & KMER_FLAG_SORT_FINISH);
    if (c->wide)
        st = sort_and_heads_wide(c, n);          // (no partials / merged counts: refused for wide keys)
    else if (bucket)
        st = bucket_heads(c, n);
    else if (c->narrow)
        st = sort_and_heads<uint32_t>(c, c->rkey32.p, c->rkey32b.p, n, with_counts);
    else
        st = sort_and_heads<uint64_t>(c, c->rkey.p, c->rkey2.p, n, with_counts);
    if (st) return st;
    auto is_head = rocprim::make_transform_iterator(c->hcnt.p, IsHead());
    ROCPRIM_RUN(c, rocprim::exclusive_scan(t, b, is_head, c->opos.p, 0u, (size_t)n, rocprim::plus<uint32_t>(), s));
    EmitArgs e;
    memset(&e, 0, sizeof(e));
    e.hcnt = c->hcnt.p;
    e.hrec = with_counts ? c->hrec.p : nullptr;
    e.rkey32 = c->narrow ? c->rkey32.p : nullptr;
    e.rkey64 = c->narrow ? nullptr : c->rkey.p;
    e.rkeyh = c->wide ? c->rkeyh.p : nullptr;
    e.opos = c->opos.p;
    e.rord = c->rord.p;
    e.n = n;
    e.invalid_key = invalid;
    e.nuniq = c->d_nuniq;
    e.nuniq_host = c->d_tail + 8;
    e.k = c->p.k;
    e.plen = (uint32_t)c->prefix.size();
    e.partial = partial ? 1u : 0u;
    memcpy(e.P, c->prefix.data(), std::min<size_t>(c->prefix.size(), sizeof(e.P)));
    e.keys_out = c->keys_out.p;
    e.cnt_out = c->cnt_out.p;
    e.first_out = c->first.p;
    e.ukey = c->ukey.p;
    e.uval = c->uval.p;
    HIPCHK(c, launch_emit(e, s));
    if (!sync) {
        c->out_pending = true;
        return KMER_OK;
    }
    HIPCHK(c, hipStreamSynchronize(s));
    *nu_out = c->h_tail[8];
    return KMER_OK;
}

// ordered device entries + host records -> host result
kmer_status build_result(kmer_ctx *c, uint64_t lines, kmer_result **out) {
    kmer_result *r = new (std::nothrow) kmer_result();
    if (!r) return fail(c, KMER_E_OOM, "host allocation failed");
    r->lines = lines;
    const uint64_t n = c->n_out, k = c->p.k;
    std::vector<uint64_t> order(n), cnt(n);
    std::vector<char> dkeys(n * k);
    if (n) {
        hipStream_t s = c->stream;
        if (hipMemcpyAsync(order.data(), c->first.p, n * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipMemcpyAsync(cnt.data(), c->cnt_out.p, n * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipMemcpyAsync(dkeys.data(), c->keys_out.p, n * k, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            delete r;
            return fail(c, KMER_E_DEVICE, "result copy failed");
        }
    }
    std::vector<std::pair<uint64_t, const std::pair<const std::string, Ent> *>> ex;
    ex.reserve(c->exotic.size());
    for (auto &kv : c->exotic) ex.emplace_back(kv.second.first, &kv);
    std::sort(ex.begin(), ex.end(), [](const auto &x, const auto &y) { return x.first < y.first; });
    const uint64_t total = n + ex.size();
    r->keys.reserve(n * k + ex.size() * k);
    r->offsets.reserve(total + 1);
    r->counts.reserve(total);
    r->firsts.reserve(total);
    uint64_t i = 0, j = 0;
    while (i < n || j < ex.size()) {
        if (j >= ex.size() || (i < n && order[i] < ex[j].first)) {
            r->keys.insert(r->keys.end(), dkeys.begin() + i * k, dkeys.begin() + (i + 1) * k);
            r->counts.push_back(cnt[i]);
            r->firsts.push_back(order[i]);
            ++i;
        } else {
            const std::string &key = ex[j].second->first;
            r->keys.insert(r->keys.end(), key.begin(), key.end());
            r->counts.push_back(ex[j].second->second.count);
            r->firsts.push_back(ex[j].first);
            ++j;
        }
        r->offsets.push_back(r->keys.size());
    }
    *out = r;
    return KMER_OK;
}

kmer_status read_pos(kmer_ctx *c, StreamPos *pos) {
    kmer_status st = settle(c);
    if (st) return st;
    st = flush_prep(c, c->stream, 0);
    if (st) return st;
    HIPCHK(c, hipMemcpyAsync(c->h_small + 8, c->d_pos, sizeof(StreamPos), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    memcpy(pos, c->h_small + 8, sizeof(StreamPos));
    return KMER_OK;
}

// Without a host result (`out` NULL) and without max_keys, nothing here waits
// for the device: the unique count and the timing are read back lazily.
kmer_status finish(kmer_ctx *c, kmer_result **out) {
    if (!c->open_stream) return fail(c, KMER_E_STATE, "finish without reset/feed");
    kmer_status st = settle(c);
    if (st) return st;
    HIPCHK(c, hipEventRecord(c->ev2, c->stream));
    uint64_t nu = 0;
    c->n_out = 0;
    const bool sync = out || c->p.max_keys;
    if (c->mode == MODE_PACKED || c->mode == MODE_WINDOWS) {
        st = apply_cross(c);
        if (st) return st;
        if (c->mode == MODE_WINDOWS && !c->prefix.empty()) {
            st = compact_windows(c);
            if (st) return st;
        }
        st = rank_finish(c, c->n_hits, false, false, &nu, sync);
        if (st) return st;
        c->n_out = nu;
    } else if (c->mode == MODE_TABLE) {
        st = table_finish(c);
        if (st) return st;
    }
    HIPCHK(c, hipEventRecord(c->ev3, c->stream));
    c->timing_pending = true;
    c->open_stream = false;
    if (!sync) return KMER_OK;
    st = resolve_out(c);
    if (st) return st;
    const uint64_t total = c->n_out + c->exotic.size();
    if (c->p.max_keys && total > c->p.max_keys)
        return fail(c, KMER_E_TOO_MANY_KEYS, "more distinct keys than max_keys (reference Map limit)");
    if (!out) return KMER_OK;
    StreamPos pos;
    st = read_pos(c, &pos);
    if (st) return st;
    const uint64_t lines = c->fasta ? c->fa_lines : pos.lines + pos.ends_open;
    if (c->mode == MODE_TABLE) return build_table_result(c, lines, out);
    return build_result(c, lines, out);
}

// Where a batch of input may end (chunks are cut at line ends; FASTA chunks
// before a header line, so that no record spans two chunks).
// batch_cut: the last cut inside [p, p + n), 0 = none;
// batch_extend: the first cut at or after b + from, else len.
uint64_t batch_cut(const uint8_t *p, uint64_t n, bool fasta) {
    if (!fasta) {
        const void *q = n ? memrchr(p, '\n', n) : nullptr;
        return q ? (uint64_t)((const uint8_t *)q - p) + 1 : 0;
    }
    uint64_t e = n ? n - 1 : 0;                  // a '\n' at j < n - 1 with p[j + 1] == '>'
    while (e > 0) {
        const void *q = memrchr(p, '\n', e);
        if (!q) return 0;
        const uint64_t j = (uint64_t)((const uint8_t *)q - p);
        if (p[j + 1] == '>') return j + 1;
        e = j;
    }
    return 0;
}

uint64_t batch_extend(const uint8_t *b, uint64_t from, uint64_t len, bool fasta) {
    uint64_t i = from;
    while (i < len) {
        const void *q = memchr(b + i, '\n', len - i);
        if (!q) return len;
        i = (uint64_t)((const uint8_t *)q - b) + 1;
        if (!fasta || (i < len && b[i] == '>')) return i;
    }
    return len;
}

// Feed host bytes through the device in batches cut at '\n' boundaries.
kmer_status feed_host(kmer_ctx *c, const uint8_t *bytes, uint64_t len, bool report = false) {
    const uint64_t batch = c->p.batch_bytes ? c->p.batch_bytes : DEFAULT_BATCH;
    uint64_t pos = 0;
    while (pos < len) {
        uint64_t end = std::min(len, pos + batch);
        if (end < len) {
            // cut after the last '\n' in [pos, end) (FASTA: before the last header
            // line); a line (record) longer than the batch extends it
            const uint64_t cut = batch_cut(bytes + pos, end - pos, c->fasta);
            end = cut ? pos + cut : batch_extend(bytes, end, len, c->fasta);
        }
        const uint64_t n = end - pos;
        kmer_status st0 = settle(c);            // the previous batch is done with the staging buffer
        if (st0) return st0;
        HIPCHK(c, c->batch.ensure(n, c->stream));
        HIPCHK(c, hipMemcpyAsync(c->batch.p, bytes + pos, n, hipMemcpyHostToDevice, c->stream));
        kmer_status st = feed(c, c->batch.p, n, c->stream);
        if (st) return st;
        pos = end;
        if (report) report_progress(c, pos, len);
    }
    if (report && len == 0) report_progress(c, 0, 0);
    return KMER_OK;
}

// ---------------------------------------------------------------------------
// multi-device group (kmer_params.ndev > 1)
// ---------------------------------------------------------------------------
// The input is read as a stream of batches cut at '\n' (lib/kmers.js:114-139
// reads the file in chunks too; here a batch is up to batch_bytes, default
// 256 MiB for files) and the batches are dealt round robin to the children,
// one host thread per child: each sets its position (lines and bytes before
// the batch, from a running newline count on the reading thread) and feeds the
// batch, while the next batches are read.  Memory: a pool of batch buffers,
// not the whole file.  Then, by configuration:
//  * ordered (packed keys): each child reduces its session to unique packed
//    keys {first, count} (kmer_partial_device); the partials are copied to
//    devices[0] (peer copies over xGMI) and finished there (min first, sum
//    counts, Map order);
//  * table / canonical mode: each child's pass-1 keys go to the child that
//    owns their slice of the hash space (kmer_table_exchange_prepare, peer
//    copies), and every child runs pass 2 + final over its own buckets, all
//    at once; statistics and digests add up over the children;
//  * anything else (records only): every batch on devices[0].
// Record keys (non-ACGT windows) move from every child to child 0 on the host.
struct GroupSrc {
    virtual ~GroupSrc() {}
    virtual void progress(uint64_t *done, uint64_t *total) = 0;
    // the next batch (valid until release()); false at the end of the input
    virtual bool next(const uint8_t **p, uint64_t *n, kmer_status *st, std::string *err) = 0;
    virtual void release(const uint8_t *) {}
};

// batches of a caller's buffer
struct MemSrc : GroupSrc {
    const uint8_t *b;
    uint64_t len, batch, pos = 0;
    bool fasta;
    MemSrc(const uint8_t *b_, uint64_t len_, uint64_t batch_, bool fasta_)
        : b(b_), len(len_), batch(std::max<uint64_t>(batch_, 1)), fasta(fasta_) {}
    void progress(uint64_t *d, uint64_t *t) override {
        *d = pos;
        *t = len;
    }
    bool next(const uint8_t **p, uint64_t *n, kmer_status *, std::string *) override {
        if (pos >= len) return false;
        uint64_t end = std::min(len, pos + batch);
        if (end < len) {                             // (a line / record longer than the batch extends it)
            const uint64_t cut = batch_cut(b + pos, end - pos, fasta);
            end = cut ? pos + cut : batch_extend(b, end, len, fasta);
        }
        *p = b + pos;
        *n = end - pos;
        pos = end;
        return true;
    }
};

// Batches of a file cut at '\n', read ahead: a reader thread fills a ring of
// host buffers with the next raw ranges of the file (plain files: several
// preads in parallel per range; gzip: zlib) while the caller counts the
// batches it already has, so the file read overlaps the device work
// (lib/kmers.js:108-139 streams the file in chunks too).  A batch is the
// carry of the previous range (the bytes after its last '\n', copied into the
// headroom in front of the next range) plus this range up to its last '\n'.
// Several batches may be outstanding (group counts); each is released when
// its bytes have been consumed.
struct FileBatches : GroupSrc {
    static constexpr uint64_t HEAD = 1ull << 20;     // headroom for the carry
    struct Slot {
        std::unique_ptr<uint8_t[]> buf;
        uint64_t cap = 0, len = 0;
        uint64_t zoff = 0;                           // gzip: compressed bytes read when the slot was filled
        int state = 0;                               // 0 free, 1 filled, 2 in use
        bool last = false;
    };
    int fd = -1;
    gzFile gz = nullptr;
    uint64_t batch = 0, size = 0, rd_off = 0;
    int threads = 1;
    std::vector<Slot> ring;
    std::mutex m;
    std::condition_variable cv;
    std::thread reader;
    bool stop = false, rd_eof = false;
    kmer_status rd_st = KMER_OK;
    std::string rd_err;
    uint64_t next_fill = 0, next_take = 0, consumed = 0;
    uint64_t consumed_z = 0;                         // gzip: compressed offset of the last batch taken
    std::vector<uint8_t> carry;
    std::unordered_map<const uint8_t *, std::unique_ptr<uint8_t[]>> big;   // batches of lines longer than HEAD
    std::unordered_map<const uint8_t *, size_t> slot_of;
    bool done = false;
    bool fasta = false;                              // batches cut before header lines

    ~FileBatches() override {
        {
            std::lock_guard<std::mutex> lk(m);
            stop = true;
        }
        cv.notify_all();
        if (reader.joinable()) reader.join();
        if (gz) gzclose(gz);
        if (fd >= 0) close(fd);
    }

    kmer_status open(const char *path, uint64_t batch_, size_t nslots, std::string *err) {
        fd = ::open(path, O_RDONLY);
        if (fd < 0) {
            *err = std::string("cannot open ") + path;
            return KMER_E_IO;
        }
        struct stat sb;
        const bool regular = fstat(fd, &sb) == 0 && S_ISREG(sb.st_mode);
        if (regular) size = (uint64_t)sb.st_size;
        unsigned char magic[2] = {0, 0};
        // a pipe, FIFO, socket or terminal (fs.createReadStream reads those too)
        // cannot be pread: zlib reads it sequentially on the reader thread, and
        // passes it through unchanged when it is not gzip (transparent mode)
        const bool gzip = !regular || (pread(fd, magic, 2, 0) == 2 && magic[0] == 0x1f && magic[1] == 0x8b);
        batch = std::max<uint64_t>(batch_, 1);
        if (gzip) {
            gz = gzdopen(dup(fd), "rb");
            if (!gz) {
                *err = std::string("cannot read gzip stream ") + path;
                return KMER_E_IO;
            }
            gzbuffer(gz, 1 << 20);
        } else if (size) {
            batch = std::min<uint64_t>(batch, size);  // a small file takes one small buffer
        }
        const unsigned hc = std::thread::hardware_concurrency();
        threads = gzip ? 1 : (int)std::max(1u, std::min(8u, hc ? hc / 2 : 1u));
        ring.resize(std::max<size_t>(nslots, 2));
        reader = std::thread([this] { read_loop(); });
        return KMER_OK;
    }

    // raw range r into slot r % R (plain: `threads` preads in parallel)
    void read_loop() {
        while (true) {
            size_t si;
            {
                std::unique_lock<std::mutex> lk(m);
                si = (size_t)(next_fill % ring.size());
                cv.wait(lk, [&] { return stop || ring[si].state == 0; });
                if (stop) return;
            }
            Slot &S = ring[si];
            if (S.cap < HEAD + batch) {
                S.buf.reset(new (std::nothrow) uint8_t[HEAD + batch]);
                S.cap = S.buf ? HEAD + batch : 0;
            }
            kmer_status st = S.buf ? KMER_OK : KMER_E_OOM;
            uint64_t got = 0;
            bool eof = false;
            if (!st && gz) {
                while (got < batch) {
                    const unsigned want = (unsigned)std::min<uint64_t>(batch - got, 1u << 30);
                    const int r = gzread(gz, S.buf.get() + HEAD + got, want);
                    if (r < 0) {
                        st = KMER_E_IO;
                        break;
                    }
                    got += (uint64_t)r;
                    if ((unsigned)r < want) break;
                }
                int zerr = 0;
                gzerror(gz, &zerr);
                if (zerr != Z_OK && zerr != Z_BUF_ERROR) st = KMER_E_IO;
                eof = got < batch;
                S.zoff = (uint64_t)std::max<z_off_t>(gzoffset(gz), 0);   // (gz is this thread's alone)
            } else if (!st) {
                // parallel preads of [rd_off, rd_off + batch); a short read (end of
                // file, or a file that is not regular) ends the input
                const int T = threads;
                const uint64_t piece = (batch + T - 1) / T;
                std::vector<uint64_t> gotv(T, 0);
                std::vector<int> errv(T, 0);
                auto job = [&](int t) {
                    const uint64_t a = (uint64_t)t * piece, b = std::min<uint64_t>(batch, a + piece);
                    uint64_t o = a;
                    while (o < b) {
                        const ssize_t r = pread(fd, S.buf.get() + HEAD + o, (size_t)(b - o), (off_t)(rd_off + o));
                        if (r < 0) {
                            errv[t] = 1;
                            break;
                        }
                        if (r == 0) break;
                        o += (uint64_t)r;
                    }
                    gotv[t] = o - a;
                };
                std::vector<std::thread> th;
                for (int t = 1; t < T; ++t) th.emplace_back(job, t);
                job(0);
                for (auto &x : th) x.join();
                for (int t = 0; t < T; ++t) {
                    if (errv[t]) st = KMER_E_IO;
                    const uint64_t a = (uint64_t)t * piece, b = std::min<uint64_t>(batch, a + piece);
                    got += gotv[t];
                    if (gotv[t] < b - a) {               // the file ends inside this piece
                        eof = true;
                        break;
                    }
                }
                rd_off += got;
            }
            std::lock_guard<std::mutex> lk(m);
            S.len = got;
            S.last = eof || st;
            S.state = 1;
            if (st) {
                rd_st = st;
                rd_err = "read error";
            }
            ++next_fill;
            cv.notify_all();
            if (S.last) return;
        }
    }

    bool next(const uint8_t **p, uint64_t *n, kmer_status *st, std::string *err) override {
        while (!done) {
            size_t si;
            {
                std::unique_lock<std::mutex> lk(m);
                si = (size_t)(next_take % ring.size());
                cv.wait(lk, [&] { return ring[si].state == 1; });
                ring[si].state = 2;
                ++next_take;
                if (rd_st) {
                    *st = rd_st;
                    *err = rd_err;
                    done = true;
                    return false;
                }
            }
            Slot &S = ring[si];
            consumed += S.len;
            consumed_z = S.zoff;
            const bool last = S.last;
            uint8_t *start;
            uint64_t have;
            std::unique_ptr<uint8_t[]> own;
            if (carry.size() <= HEAD) {
                start = S.buf.get() + HEAD - carry.size();
                if (!carry.empty()) memcpy(start, carry.data(), carry.size());
                have = carry.size() + S.len;
            } else {                                      // a line longer than the headroom
                own.reset(new (std::nothrow) uint8_t[carry.size() + S.len]);
                if (!own) {
                    *st = KMER_E_OOM;
                    *err = "host batch buffer";
                    done = true;
                    return false;
                }
                memcpy(own.get(), carry.data(), carry.size());
                memcpy(own.get() + carry.size(), S.buf.get() + HEAD, S.len);
                start = own.get();
                have = carry.size() + S.len;
            }
            const uint64_t cut = last ? have : batch_cut(start, have, fasta);
            carry.assign(start + cut, start + have);
            if (last) done = true;
            if (cut == 0) {                               // (no '\n' yet: all of it is carry)
                release_slot(si);
                if (last) return false;
                continue;
            }
            *p = start;
            *n = cut;
            std::lock_guard<std::mutex> lk(m);
            if (own) {
                release_slot_locked(si);
                big[start] = std::move(own);
            } else {
                slot_of[start] = si;
            }
            return true;
        }
        return false;
    }

    void release_slot_locked(size_t si) {
        ring[si].state = 0;
        cv.notify_all();
    }
    void release_slot(size_t si) {
        std::lock_guard<std::mutex> lk(m);
        release_slot_locked(si);
    }
    void release(const uint8_t *q) override {
        std::lock_guard<std::mutex> lk(m);
        auto b = big.find(q);
        if (b != big.end()) {
            big.erase(b);
            return;
        }
        auto it = slot_of.find(q);
        if (it != slot_of.end()) {
            release_slot_locked(it->second);
            slot_of.erase(it);
        }
    }
    // progress: (bytes taken, file size) -- for gzip the compressed offset of the
    // batches taken and the compressed size.  Called on the consuming thread
    // only (never touches the gzFile, which the reader thread owns)
    void progress(uint64_t *d, uint64_t *t) override {
        *d = gz ? consumed_z : consumed;
        *t = size;
        if (*d > *t && *t) *d = *t;
    }
};

// group partials, concatenated by child: each child's partial is in
// first-occurrence order but the children's batches interleave, so the
// concatenation is re-ordered by first occurrence (radix sort of first ->
// index, then a gather) before kmer_finish_merged, which takes index = rank
__global__ __launch_bounds__(256) void partial_firsts_kernel(const Agg *vals, uint64_t n, uint64_t *firsts,
                                                             uint32_t *idx) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        firsts[i] = vals[i].first;
        idx[i] = (uint32_t)i;
    }
}

__global__ __launch_bounds__(256) void partial_gather_kernel(const uint64_t *keys, const Agg *vals, const uint32_t *idx,
                                                             uint64_t n, uint64_t *okeys, Agg *ovals) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t j = idx[i];
        okeys[i] = keys[j];
        ovals[i] = vals[j];
    }
}

// records a FASTA batch holds (kmer_fasta.hip's rewrite: one per header line,
// plus a headerless one when the batch does not start with a header)
uint64_t fasta_records(const uint8_t *p, uint64_t n) {
    if (!n) return 0;
    uint64_t r = p[0] != '>' ? 1 : 0;
    const uint8_t *e = p + n;
    for (const uint8_t *q = p; q < e;) {
        if (*q == '>' && (q == p || q[-1] == '\n')) ++r;
        const void *nl = memchr(q, '\n', (size_t)(e - q));
        if (!nl) break;
        q = (const uint8_t *)nl + 1;
    }
    return r;
}

uint64_t count_newlines(const uint8_t *p, uint64_t n) {
    uint64_t c = 0;
    const uint8_t *e = p + n;
    while (p < e) {
        const void *q = memchr(p, '\n', (size_t)(e - p));
        if (!q) break;
        ++c;
        p = (const uint8_t *)q + 1;
    }
    return c;
}

// records (non-ACGT windows) of children 1.. -> child 0
kmer_status group_gather_records(kmer_ctx *g) {
    kmer_ctx *c0 = g->group[0];
    for (size_t i = 1; i < g->group.size(); ++i) {
        kmer_result *r = nullptr;
        kmer_status st = kmer_records_export(g->group[i], &r);
        if (st) return fail(g, st, "records export");
        const uint64_t m = kmer_result_size(r);
        if (m) {
            const char *kb = nullptr;
            const uint64_t *off = nullptr, *cnt = nullptr, *fst = nullptr;
            kmer_result_arrays(r, &kb, &off, &cnt);
            kmer_result_firsts(r, &fst);
            st = kmer_records_import(c0, kb, off, cnt, fst, m);
            if (!st) st = kmer_records_clear(g->group[i]);
        }
        kmer_result_free(r);
        if (st) return fail(g, st, "records import");
    }
    return KMER_OK;
}

// run f(i) for every child i on its own thread (device selected); first error wins
kmer_status group_each(kmer_ctx *g, size_t n, const std::function<kmer_status(size_t)> &f) {
    std::vector<kmer_status> sts(n, KMER_OK);
    std::vector<std::thread> th;
    for (size_t i = 0; i < n; ++i)
        th.emplace_back([&, i]() {
            if (hipSetDevice(g->group[i]->device) != hipSuccess) {
                sts[i] = KMER_E_DEVICE;
                return;
            }
            sts[i] = f(i);
        });
    for (auto &t : th) t.join();
    for (size_t i = 0; i < n; ++i)
        if (sts[i]) return fail(g, sts[i], "device " + std::to_string(g->group[i]->device) + ": " + g->group[i]->err);
    return KMER_OK;
}

kmer_status group_count(kmer_ctx *g, GroupSrc &src, kmer_result **out) {
    const size_t N = g->group.size();
    kmer_ctx *c0 = g->group[0];
    const int mode = c0->mode;
    // (keys of >= 64 bits have no packed partials: devices[0] counts alone)
    const bool ordered = (mode == MODE_PACKED && !c0->wide) || mode == MODE_WINDOWS;
    const size_t W = (ordered || mode == MODE_TABLE) ? N : 1;    // children that take batches
    g->t_done = false;
    // -- the batch stream, dealt round robin over W worker threads
    struct Job {
        const uint8_t *p;
        uint64_t n, lines, off;
    };
    struct Worker {
        std::deque<Job> q;
        std::mutex m;
        std::condition_variable cv;
        bool end = false;
        kmer_status st = KMER_OK;
    };
    std::vector<std::unique_ptr<Worker>> wk;
    for (size_t i = 0; i < W; ++i) wk.emplace_back(new Worker());
    std::vector<std::thread> th;
    for (size_t i = 0; i < W; ++i)
        th.emplace_back([&, i]() {
            Worker &w = *wk[i];
            kmer_ctx *c = g->group[i];
            kmer_status st = hipSetDevice(c->device) == hipSuccess ? reset(c) : KMER_E_DEVICE;
            while (true) {
                Job j;
                {
                    std::unique_lock<std::mutex> lk(w.m);
                    w.cv.wait(lk, [&] { return !w.q.empty() || w.end; });
                    if (w.q.empty()) break;
                    j = w.q.front();
                    w.q.pop_front();
                }
                if (!st) st = kmer_set_position(c, j.lines, j.off);
                if (!st) st = feed_host(c, j.p, j.n);
                if (!st) st = settle(c);
                if (!st && hipStreamSynchronize(c->stream) != hipSuccess) st = KMER_E_DEVICE;   // bytes consumed
                src.release(j.p);
                if (st) {
                    c->open_stream = false;
                    std::lock_guard<std::mutex> lk(w.m);
                    w.st = st;
                }
            }
            std::lock_guard<std::mutex> lk(w.m);
            if (st) w.st = st;
        });
    uint64_t lines = 0, off = 0, nb = 0, in_lines = 0;
    uint8_t last = '\n';
    const bool fasta = (g->p.flags & KMER_FLAG_FASTA) != 0;
    kmer_status rst = KMER_OK;
    std::string rerr;
    const uint8_t *p = nullptr;
    uint64_t n = 0;
    while (src.next(&p, &n, &rst, &rerr)) {
        bool failed = false;
        for (auto &w : wk) {
            std::lock_guard<std::mutex> lk(w->m);
            failed |= w->st != KMER_OK;
        }
        if (failed) {
            src.release(p);
            break;
        }
        // positions are counted in the lines the devices see: FASTA batches are
        // rewritten into four lines per record (kmer_fasta.hip)
        const uint64_t in_nl = count_newlines(p, n);
        const uint64_t nl = fasta ? 4 * fasta_records(p, n) : in_nl;
        in_lines += in_nl;
        last = p[n - 1];
        Worker &w = *wk[nb % W];
        {
            std::lock_guard<std::mutex> lk(w.m);
            w.q.push_back(Job{p, n, lines, off});
        }
        w.cv.notify_one();
        lines += nl;
        off += n;
        ++nb;
        if (g->p.progress) {                          // (batches handed to the devices)
            uint64_t d = 0, t = 0;
            src.progress(&d, &t);
            report_progress(g, d, t);
        }
    }
    if (nb == 0 && g->p.progress) {                   // (an empty input: one event)
        uint64_t d = 0, t = 0;
        src.progress(&d, &t);
        report_progress(g, d, t);
    }
    for (auto &w : wk) {
        {
            std::lock_guard<std::mutex> lk(w->m);
            w->end = true;
        }
        w->cv.notify_one();
    }
    for (auto &t : th) t.join();
    if (rst) return fail(g, rst, rerr);
    for (size_t i = 0; i < W; ++i)
        if (wk[i]->st) return fail(g, wk[i]->st, "device " + std::to_string(g->group[i]->device) + ": " + g->group[i]->err);
    const uint64_t total_lines = in_lines + (off > 0 && last != '\n' ? 1 : 0);
    if (hipSetDevice(c0->device) != hipSuccess) return fail(g, KMER_E_DEVICE, "hipSetDevice");
    if (!ordered && mode != MODE_TABLE) {            // every batch went to devices[0]
        kmer_status st = finish(c0, out);
        if (st) return fail(g, st, c0->err);
        return KMER_OK;
    }
    if (ordered) {
        std::vector<const void *> pk(N, nullptr), pv(N, nullptr);
        std::vector<uint64_t> pn(N, 0);
        kmer_status st = group_each(g, N, [&](size_t i) { return kmer_partial_device(g->group[i], &pk[i], &pv[i], &pn[i]); });
        if (st) return st;
        uint64_t tot = 0;
        for (size_t i = 0; i < N; ++i) tot += pn[i];
        if (hipSetDevice(c0->device) != hipSuccess) return fail(g, KMER_E_DEVICE, "hipSetDevice");
        hipStream_t s = c0->stream;
        HIPCHK(g, g->gkeys.ensure(tot, s));
        HIPCHK(g, g->gvals.ensure(tot, s));
        uint64_t o = 0;
        for (size_t i = 0; i < N; ++i) {                 // partials -> devices[0], in child order
            if (!pn[i]) continue;
            kmer_ctx *c = g->group[i];
            if (c->device == c0->device) {
                HIPCHK(g, hipMemcpyAsync(g->gkeys.p + o, pk[i], pn[i] * 8, hipMemcpyDeviceToDevice, s));
                HIPCHK(g, hipMemcpyAsync(g->gvals.p + o, pv[i], pn[i] * sizeof(Agg), hipMemcpyDeviceToDevice, s));
            } else {
                HIPCHK(g, hipMemcpyPeerAsync(g->gkeys.p + o, c0->device, pk[i], c->device, pn[i] * 8, s));
                HIPCHK(g, hipMemcpyPeerAsync(g->gvals.p + o, c0->device, pv[i], c->device, pn[i] * sizeof(Agg), s));
            }
            o += pn[i];
        }
        if (nb > N && tot > 1) {                     // (batches interleaved over the children)
            if (tot >= (1ull << 32)) return fail(g, KMER_E_TOO_MANY_KEYS, "more than 2^32 partial entries");
            HIPCHK(g, c0->xord.ensure(tot, s));
            HIPCHK(g, c0->xord2.ensure(tot, s));
            HIPCHK(g, c0->ridx.ensure(tot, s));
            HIPCHK(g, c0->ridx2.ensure(tot, s));
            const uint32_t grid = (uint32_t)std::min<uint64_t>((tot + 255) / 256, 16384);
            hipLaunchKernelGGL(partial_firsts_kernel, dim3(grid), dim3(256), 0, s, g->gvals.p, tot, c0->xord.p,
                               c0->ridx.p);
            HIPCHK(g, hipGetLastError());
            rocprim::double_buffer<uint64_t> kb(c0->xord.p, c0->xord2.p);
            rocprim::double_buffer<uint32_t> vb(c0->ridx.p, c0->ridx2.p);
            kmer_ctx *c = c0;                         // (ROCPRIM_RUN's scratch)
            ROCPRIM_RUN(c, rocprim::radix_sort_pairs(t, b, kb, vb, (size_t)tot, 0, 64, s));
            HIPCHK(g, g->gkeys2.ensure(tot, s));
            HIPCHK(g, g->gvals2.ensure(tot, s));
            hipLaunchKernelGGL(partial_gather_kernel, dim3(grid), dim3(256), 0, s, g->gkeys.p, g->gvals.p,
                               vb.current(), tot, g->gkeys2.p, g->gvals2.p);
            HIPCHK(g, hipGetLastError());
            std::swap(g->gkeys, g->gkeys2);
            std::swap(g->gvals, g->gvals2);
        }
        HIPCHK(g, hipStreamSynchronize(s));
        st = group_gather_records(g);
        if (st) return st;
        st = kmer_finish_merged(c0, g->gkeys.p, g->gvals.p, tot, total_lines, out);
        if (st) return fail(g, st, c0->err);
        return KMER_OK;
    }
    // table mode: pass-1 keys to their owners, then pass 2 + final on every child
    std::vector<const void *> snd(N, nullptr);
    std::vector<std::vector<uint64_t>> cnt(N, std::vector<uint64_t>(N, 0));
    std::vector<uint64_t> parts((uint64_t)N * TAB_NB, 0);
    kmer_status st = group_each(g, N, [&](size_t i) {
        return kmer_table_exchange_prepare(g->group[i], (uint32_t)N, &snd[i], cnt[i].data(), parts.data() + i * TAB_NB);
    });
    if (st) return st;
    std::vector<uint64_t> recv_n(N, 0);
    st = group_each(g, N, [&](size_t o) -> kmer_status {
        kmer_ctx *c = g->group[o];
        hipStream_t s = c->stream;
        uint64_t tot = 0;
        for (size_t i = 0; i < N; ++i) tot += cnt[i][o];
        recv_n[o] = tot;
        if (c->trecv.ensure(std::max<uint64_t>(tot, 1), s) != hipSuccess) return fail(c, KMER_E_OOM, "receive buffer");
        uint64_t at = 0;
        for (size_t i = 0; i < N; ++i) {                 // runs in source order
            uint64_t before = 0;
            for (size_t x = 0; x < o; ++x) before += cnt[i][x];
            if (cnt[i][o]) {
                const uint64_t *from = (const uint64_t *)snd[i] + before;
                const int sd = g->group[i]->device;
                const hipError_t e = sd == c->device
                                         ? hipMemcpyAsync(c->trecv.p + at, from, cnt[i][o] * 8, hipMemcpyDeviceToDevice, s)
                                         : hipMemcpyPeerAsync(c->trecv.p + at, c->device, from, sd, cnt[i][o] * 8, s);
                if (e != hipSuccess) return fail(c, KMER_E_DEVICE, std::string("HIP error: ") + hipGetErrorString(e));
            }
            at += cnt[i][o];
        }
        return hipStreamSynchronize(s) == hipSuccess ? KMER_OK : fail(c, KMER_E_DEVICE, "exchange copy");
    });
    if (st) return st;
    st = group_gather_records(g);
    if (st) return st;
    st = group_each(g, N, [&](size_t o) {
        kmer_ctx *c = g->group[o];
        return kmer_table_finish_exchanged(c, c->trecv.p, recv_n[o], parts.data(), (uint32_t)N, (uint32_t)o, c->stream);
    });
    if (st) return st;
    g->t_done = true;
    uint64_t keys = 0;
    for (size_t o = 0; o < N; ++o) {
        uint64_t kk = 0;
        st = kmer_table_stats(g->group[o], nullptr, &kk, nullptr);
        if (st) return fail(g, st, g->group[o]->err);
        keys += kk;
    }
    if (c0->p.max_keys && keys > c0->p.max_keys)
        return fail(g, KMER_E_TOO_MANY_KEYS, "more distinct keys than max_keys (reference Map limit)");
    if (!out) return KMER_OK;
    // one host result: the children's entries (disjoint canonical classes), sorted by key bytes
    std::vector<std::pair<std::string, uint64_t>> ents;
    for (size_t o = 0; o < N; ++o) {
        kmer_result *r = nullptr;
        if (hipSetDevice(g->group[o]->device) != hipSuccess) return fail(g, KMER_E_DEVICE, "hipSetDevice");
        st = build_table_result(g->group[o], total_lines, &r);
        if (st) return fail(g, st, g->group[o]->err);
        for (uint64_t i = 0; i + 1 < r->offsets.size(); ++i)
            ents.emplace_back(std::string(r->keys.data() + r->offsets[i], r->offsets[i + 1] - r->offsets[i]), r->counts[i]);
        kmer_result_free(r);
    }
    std::sort(ents.begin(), ents.end());
    kmer_result *r = new (std::nothrow) kmer_result();
    if (!r) return fail(g, KMER_E_OOM, "host allocation failed");
    r->lines = total_lines;
    for (auto &e : ents) {
        r->keys.insert(r->keys.end(), e.first.begin(), e.first.end());
        r->offsets.push_back(r->keys.size());
        r->counts.push_back(e.second);
        r->firsts.push_back(0);
    }
    *out = r;
    return KMER_OK;
}

constexpr uint64_t GROUP_FILE_BATCH = 256ull << 20;

kmer_status group_count_buffer(kmer_ctx *g, const uint8_t *bytes, uint64_t len, kmer_result **out) {
    const size_t N = g->group.size();
    // default: one batch per child (a buffer is already in host memory)
    const uint64_t batch = g->p.batch_bytes ? g->p.batch_bytes : std::max<uint64_t>(1, (len + N - 1) / N);
    MemSrc src(bytes, len, batch, (g->p.flags & KMER_FLAG_FASTA) != 0);
    return group_count(g, src, out);
}

kmer_status group_count_file(kmer_ctx *g, const char *path, kmer_result **out) {
    const size_t N = g->group.size();
    FileBatches src;
    src.fasta = (g->p.flags & KMER_FLAG_FASTA) != 0;
    std::string err;
    const kmer_status st = src.open(path, g->p.batch_bytes ? g->p.batch_bytes : GROUP_FILE_BATCH, N + 2, &err);
    if (st) return fail(g, st, err);
    return group_count(g, src, out);
}

}  // namespace

extern "C" {

const char *kmer_version(void) { return "kmerhip 0.2 (gfx950)"; }

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
    // reserved / experiment-only flag bits (KMERHIP_XFLAG_*, a -DKMERHIP_EXPERIMENTS build)
    if (!KH_EXPERIMENTS && (pp->flags & ~KMER_FLAGS_PUBLIC)) return KMER_E_BAD_PARAM;
    *out = nullptr;
    if (pp->ndev > 1) {
        if (pp->ndev > 64) return KMER_E_BAD_PARAM;
        kmer_ctx *g = new (std::nothrow) kmer_ctx();
        if (!g) return KMER_E_OOM;
        g->p = *pp;
        g->p.prefix = nullptr;
        g->p.devices = nullptr;
        g->prefix.assign((const char *)pp->prefix, pp->prefix_len);
        for (uint32_t i = 0; i < pp->ndev; ++i) {
            kmer_params cp = *pp;
            cp.ndev = 1;
            cp.devices = nullptr;
            cp.device = pp->devices ? pp->devices[i] : (int32_t)i;
            kmer_ctx *c = nullptr;
            const kmer_status st = kmer_open(&cp, &c);
            if (st) {
                kmer_close(g);
                return st;
            }
            g->group.push_back(c);
        }
        g->device = g->group[0]->device;
        g->mode = g->group[0]->mode;
        *out = g;
        return KMER_OK;
    }
    kmer_ctx *c = new (std::nothrow) kmer_ctx();
    if (!c) return KMER_E_OOM;
    c->p = *pp;
    c->fasta = (pp->flags & KMER_FLAG_FASTA) != 0;
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
    if (hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess) c->n_cu = 256;
    {
        // two priorities: another session's finish (short, latency-bound
        // kernels) is dispatched ahead of the remaining workgroups of a
        // running scan instead of queueing behind all of them
        int lo = 0, hi = 0;
        if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) lo = hi = 0;
        if (hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi) != hipSuccess ||
            hipStreamCreateWithPriority(&c->sstream, hipStreamNonBlocking, lo) != hipSuccess ||
            hipEventCreateWithFlags(&c->evq, hipEventDisableTiming) != hipSuccess)
            return cleanup(KMER_E_DEVICE);
    }

    c->pbits = (pp->flags & KMER_FLAG_LONG_LINES) ? PBITS_LONG : PBITS_DEFAULT;
    const uint32_t k = pp->k, plen = (uint32_t)c->prefix.size();
    bool acgt = plen > 0;
    for (char ch : c->prefix) acgt &= ch == 'A' || ch == 'C' || ch == 'G' || ch == 'T';
    const bool dense_ok = !(pp->flags & KMER_FLAG_NO_DENSE) && pp->step == 1 && plen <= k;
    const bool win_step = !(pp->flags & KMER_FLAG_NO_DENSE) && pp->step > 1 && plen <= k &&
                          (plen == 0 ? k <= 31 : (acgt && k <= (uint32_t)KMAX_DENSE));
    if ((pp->flags & KMER_FLAG_CANONICAL) &&
        !(pp->step == 1 && plen <= k && k <= (uint32_t)KMAX_PACKED && (plen == 0 || acgt))) {
        delete c;                               // (canonical counts exist in table mode only)
        return KMER_E_BAD_PARAM;
    }
    if ((pp->flags & (KMER_FLAG_UNORDERED | KMER_FLAG_CANONICAL)) && pp->step == 1 && plen <= k &&
        k <= (uint32_t)KMAX_PACKED && (plen == 0 || acgt))
        c->mode = MODE_TABLE;
    else if (dense_ok && (plen == 0 ? k <= 31 : (acgt && plen <= 3 && k <= (uint32_t)KMAX_DENSE)))
        c->mode = MODE_WINDOWS;
    else if (win_step)
        c->mode = MODE_WINDOWS;                 // step > 1: every stepped window ranked (the tile scan has no line ends)
    else if (dense_ok && plen > 0 && k <= (uint32_t)KMAX_TILE)
        c->mode = MODE_PACKED;                  // (k > 32: 128-bit window codes; any prefix bytes: key = P + suffix code)
    else if (pp->step == 1 && plen > 0 && k <= (uint32_t)KMAX_TILE)
        c->mode = MODE_TILE_REC;
    else
        c->mode = MODE_GENERAL;
    const bool packed_keys = c->mode == MODE_PACKED || c->mode == MODE_WINDOWS;
    c->kbits = packed_keys ? 2 * (k - plen) : 0;
    c->narrow = packed_keys && c->kbits <= 31;
    c->wide = packed_keys && c->kbits >= 64;
    c->planes = (c->mode == MODE_PACKED || c->mode == MODE_TILE_REC) && acgt && !(pp->flags & KMER_FLAG_BYTE_SCAN);
    if (c->planes) {
        // plane bits of a base: bit 1 (plane L) and bit 2 (plane H) of its ASCII byte
        auto code = [](char ch) -> uint32_t { return (((uint8_t)ch >> 1) & 1u) | ((((uint8_t)ch >> 2) & 1u) << 1); };
        c->pargs.pb = std::min<uint32_t>(plen, 5);
        for (uint32_t i = 0; i < 5; ++i) {
            const uint32_t cp = i < plen ? code(c->prefix[i]) : 0u, cr = i < plen ? code(c->rprefix[i]) : 0u;
            c->pargs.kl[i] = (cp & 1u) ? 0u : ~0u;
            c->pargs.kh[i] = (cp & 2u) ? 0u : ~0u;
            c->pargs.rl[i] = (cr & 1u) ? 0u : ~0u;
            c->pargs.rh[i] = (cr & 2u) ? 0u : ~0u;
        }
    }

    bool ok = true;
    ok &= dalloc(&c->d_P, std::max<uint32_t>(plen, 1)) == hipSuccess;
    if (ok && plen) ok &= hipMemcpy(c->d_P, c->prefix.data(), plen, hipMemcpyHostToDevice) == hipSuccess;
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
    ok &= dalloc(&c->d_scal, 16) == hipSuccess;
    if (ok) {
        ok &= hipMemset(c->d_scal, 0, 128) == hipSuccess;
        c->d_hticket = (unsigned int *)(c->d_scal + 8);
        c->d_rec_count = (unsigned long long *)(c->d_scal + 0);
        c->d_ovf_count = (unsigned long long *)(c->d_scal + 1);
        c->d_xcount = (unsigned long long *)(c->d_scal + 2);
        c->d_chunk_hits = (unsigned long long *)(c->d_scal + 3);
        c->d_nuniq = c->d_scal + 4;
        c->d_err = (unsigned int *)(c->d_scal + 5);
        c->d_line_count = (unsigned long long *)(c->d_scal + 6);
        c->d_ends_open = (unsigned long long *)(c->d_scal + 7);
    }
    ok &= dalloc(&c->d_pos, 1) == hipSuccess;
    ok &= dalloc(&c->d_pos_saved, 1) == hipSuccess;
    ok &= hipHostMalloc((void **)&c->h_small, 24 * sizeof(uint64_t), hipHostMallocDefault) == hipSuccess;
    ok &= hipHostMalloc((void **)&c->h_tail, 16 * sizeof(uint64_t), hipHostMallocMapped | hipHostMallocCoherent) ==
          hipSuccess;
    ok &= c->h_tail && hipHostGetDevicePointer((void **)&c->d_tail, c->h_tail, 0) == hipSuccess;
    if (c->h_tail) memset(c->h_tail, 0, 16 * sizeof(uint64_t));
    for (hipEvent_t &e : c->tev) ok &= hipEventCreate(&e) == hipSuccess;
    ok &= hipEventCreate(&c->ev0) == hipSuccess && hipEventCreate(&c->ev1) == hipSuccess &&
          hipEventCreate(&c->ev2) == hipSuccess && hipEventCreate(&c->ev3) == hipSuccess &&
          hipEventCreate(&c->ev4) == hipSuccess &&
          hipEventCreateWithFlags(&c->evw, hipEventDisableTiming) == hipSuccess;
    if (!ok) return cleanup(KMER_E_OOM);
    if (ensure_records(c, 1 << 16) || ensure_tiles(c, 1 << 12)) return cleanup(KMER_E_OOM);
    if (ensure_ovf(c, 1 << 16, c->stream) != KMER_OK) return cleanup(KMER_E_OOM);
    if (hipMemset(c->d_err, 0, 4) != hipSuccess) return cleanup(KMER_E_DEVICE);
    if (reset(c) != KMER_OK) return cleanup(KMER_E_DEVICE);
    c->open_stream = false;
    if (hipStreamSynchronize(c->stream) != hipSuccess) return cleanup(KMER_E_DEVICE);
    *out = c;
    return KMER_OK;
}

kmer_status kmer_close(kmer_ctx *c) {
    if (!c) return KMER_E_BAD_PARAM;
    if (!c->group.empty()) {
        if (hipSetDevice(c->group[0]->device) == hipSuccess) {
            c->gkeys.release();
            c->gvals.release();
            c->gkeys2.release();
            c->gvals2.release();
        }
        for (kmer_ctx *x : c->group) kmer_close(x);
        delete c;
        return KMER_OK;
    }
    (void)hipSetDevice(c->device);
    (void)settle(c);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    c->tcount.release();
    c->nlslots.release();
    c->fa_t.release();
    c->fa_x.release();
    c->fa_out[0].release();
    c->fa_out[1].release();
    for (auto *b : {&c->tbase, &c->nlpos, &c->wcount, &c->wbase, &c->tp_cnt, &c->tp_lnl, &c->rkey, &c->rkey2, &c->rord, &c->rord2, &c->csel, &c->rcnt, &c->xord, &c->xord2,
                    &c->xkey, &c->xkey2, &c->ukey, &c->first, &c->cnt_out, &c->roff})
        b->release();
    for (auto *b : {&c->ridx, &c->ridx2, &c->opos, &c->xslot, &c->rkey32, &c->rkey32b, &c->bH, &c->bHs}) b->release();
    c->pkey16.release();
    c->xsend.release();
    c->xH.release();
    c->xHs.release();
    c->xcnt.release();
    if (c->h_xcnt) (void)hipHostFree(c->h_xcnt);
    c->bsum.release();
    c->bscan.release();
    c->hrec.release();
    c->hcnt.release();
    c->tsum.release();
    c->tscan.release();
    c->hits.release();
    c->ovf.release();
    c->lb_cnt.release();
    c->lb_lnl.release();
    c->uval.release();
    c->keys_out.release();
    c->recs.release();
    c->lines.release();
    c->rec_keys.release();
    c->tmp.release();
    c->batch.release();
    for (auto *b : {&c->tb1, &c->tb2, &c->tHs, &c->tstart, &c->tp1, &c->tpb, &c->tsend}) b->release();
    c->tseg.release();
    c->tpc.release();
    c->tpieces.release();
    c->tH.release();
    c->tnd.release();
    c->tunits.release();
    c->tbig.release();
    c->tstats.release();
    c->tleft.release();
    c->trecv.release();
    dfree(c->d_ticket); dfree(c->d_scal); dfree(c->d_pos); dfree(c->d_pos_saved);
    dfree(c->d_P); dfree(c->d_PR);
    if (c->h_small) (void)hipHostFree(c->h_small);
    if (c->h_tail) (void)hipHostFree(c->h_tail);
    for (hipEvent_t e : {c->ev0, c->ev1, c->ev2, c->ev3, c->ev4, c->evw})
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->tev)
        if (e) (void)hipEventDestroy(e);
    if (c->sstream) (void)hipStreamSynchronize(c->sstream);
    if (c->evq) (void)hipEventDestroy(c->evq);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->sstream) (void)hipStreamDestroy(c->sstream);
    delete c;
    return KMER_OK;
}

kmer_status kmer_sync(kmer_ctx *c) {
    if (!c) return KMER_E_BAD_PARAM;
    if (!c->group.empty()) return fail(c, KMER_E_STATE, "single-device call on a group context");
    if (hipSetDevice(c->device) != hipSuccess) return KMER_E_DEVICE;
    return settle(c);
}

kmer_status kmer_reset(kmer_ctx *c) {
    if (!c) return KMER_E_BAD_PARAM;
    if (!c->group.empty()) return fail(c, KMER_E_STATE, "single-device call on a group context");
    if (hipSetDevice(c->device) != hipSuccess) return KMER_E_DEVICE;
    return reset(c);
}

kmer_status kmer_feed_device(kmer_ctx *c, const void *d_bytes, size_t len, void *stream) {
    if (!c || (!d_bytes && len)) return KMER_E_BAD_PARAM;
    SETTLE(c);
    if (!c->open_stream) return fail(c, KMER_E_STATE, "feed without reset");
    if (hipSetDevice(c->device) != hipSuccess) return KMER_E_DEVICE;
    hipStream_t s = (hipStream_t)stream;
    if (s != c->stream) {
        // order the context's own (non-blocking) stream after the caller's
        // work; NULL is the legacy default stream, which a non-blocking stream
        // does not otherwise wait for
        HIPCHK(c, hipEventRecord(c->evw, s));
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->evw, 0));
    }
    return feed(c, (const uint8_t *)d_bytes, len, c->stream);
}

kmer_status kmer_finish_device(kmer_ctx *c, kmer_result **out) {
    if (!c) return KMER_E_BAD_PARAM;
    SETTLE(c);
    if (hipSetDevice(c->device) != hipSuccess) return KMER_E_DEVICE;
    if (out) *out = nullptr;
    return finish(c, out);
}

namespace {

// A whole-input count that met a sequence line longer than the default
// order key's position field (2^23 bytes: a FASTA contig or chromosome) is
// redone once in long-line mode (2^40-byte lines, up to 2^23 lines).
// A group context redoes it on every device.
void set_pbits(kmer_ctx *c, uint32_t pbits) {
    c->pbits = pbits;
    for (kmer_ctx *x : c->group) x->pbits = pbits;
}

kmer_status with_long_line_retry(kmer_ctx *c, const std::function<kmer_status()> &count) {
    c->progress_any = false;
    c->progress_hw = 0;
    kmer_status st = count();
    if (st == KMER_E_LINE_TOO_LONG && c->pbits == PBITS_DEFAULT && c->mode != MODE_TABLE) {
        set_pbits(c, PBITS_LONG);
        st = count();
        set_pbits(c, PBITS_DEFAULT);
    }
    return st;
}

kmer_status count_buffer_once(kmer_ctx *c, const uint8_t *bytes, size_t len, kmer_result **out) {
    kmer_status st = reset(c);
    if (st) return st;
    st = feed_host(c, bytes, len, true);
    if (st) {
        c->open_stream = false;
        return st;
    }
    return finish(c, out);
}

kmer_status count_file_once(kmer_ctx *c, const char *path, kmer_result **out);

}  // namespace

kmer_status kmer_count_buffer(kmer_ctx *c, const uint8_t *bytes, size_t len, kmer_result **out) {
    if (!c || !out || (!bytes && len)) return KMER_E_BAD_PARAM;
    *out = nullptr;
    if (!c->group.empty()) return with_long_line_retry(c, [&] { return group_count_buffer(c, bytes, len, out); });
    if (hipSetDevice(c->device) != hipSuccess) return KMER_E_DEVICE;
    return with_long_line_retry(c, [&] { return count_buffer_once(c, bytes, len, out); });
}

kmer_status kmer_count_file(kmer_ctx *c, const char *path, kmer_result **out) {
    if (!c || !path || !out) return KMER_E_BAD_PARAM;
    *out = nullptr;
    if (!c->group.empty()) return with_long_line_retry(c, [&] { return group_count_file(c, path, out); });
    return with_long_line_retry(c, [&] { return count_file_once(c, path, out); });
}

namespace {

kmer_status count_file_once(kmer_ctx *c, const char *path, kmer_result **out) {
    if (hipSetDevice(c->device) != hipSuccess) return KMER_E_DEVICE;
    // the file is read ahead (FileBatches: a reader thread, parallel preads)
    // in batches of batch_bytes (default 256 MiB; no larger than the file),
    // while the device counts the batch before; gzip input (magic 1f 8b) is
    // read through zlib, the count being that of the decompressed FASTQ
    FileBatches src;
    src.fasta = c->fasta;
    std::string err;
    kmer_status st = src.open(path, c->p.batch_bytes ? c->p.batch_bytes : FILE_BATCH, 3, &err);
    if (st) return fail(c, st, err);
    st = reset(c);
    const uint8_t *p = nullptr;
    uint64_t n = 0;
    kmer_status rst = KMER_OK;
    while (!st && src.next(&p, &n, &rst, &err)) {
        st = feed_host(c, p, n);
        if (!st) st = settle(c);
        if (!st && hipStreamSynchronize(c->stream) != hipSuccess) st = fail(c, KMER_E_DEVICE, "stream sync");
        src.release(p);                           // (the batch's bytes are on the device)
        if (!st && c->p.progress) {
            uint64_t d = 0, t = 0;
            src.progress(&d, &t);
            report_progress(c, d, t);
        }
    }
    if (!st && rst) st = fail(c, rst, err + " on " + path);
    if (st) {
        c->open_stream = false;
        return st;
    }
    if (c->p.progress && src.consumed == 0) {        // (an empty file: one event, as progress-stream's end)
        uint64_t d = 0, t = 0;
        src.progress(&d, &t);
        report_progress(c, d, t);
    }
    return finish(c, out);
}

}  // namespace

kmer_status kmer_partial_device(kmer_ctx *c, const void **d_keys, const void **d_vals, uint64_t *n) {
    if (!c || !d_keys || !d_vals || !n) return KMER_E_BAD_PARAM;
    SETTLE(c);
    if (c->mode != MODE_PACKED && c->mode != MODE_WINDOWS)
        return fail(c, KMER_E_STATE, "configuration has no packed keys");
    if (c->wide) return fail(c, KMER_E_STATE, "keys of 64 bits or more (k - |P| >= 32) have no packed partials");
    if (hipSetDevice(c->device) != hipSuccess) return KMER_E_DEVICE;
    kmer_status st = apply_cross(c);
    if (st) return st;
    uint64_t nu = 0;
    st = rank_finish(c, c->n_hits, true, false, &nu);
    if (st) return st;
    c->n_hits = 0;           // the rank arrays were consumed by the sort
    *d_keys = c->ukey.p;
    *d_vals = c->uval.p;
    *n = nu;
    return KMER_OK;
}

kmer_status kmer_finish_merged(kmer_ctx *c, const void *d_keys, const void *d_vals, uint64_t n,
                               uint64_t total_lines, kmer_result **out) {
    if (!c || (n && (!d_keys || !d_vals))) return KMER_E_BAD_PARAM;
    SETTLE(c);
    if (c->mode != MODE_PACKED && c->mode != MODE_WINDOWS)
        return fail(c, KMER_E_STATE, "configuration has no packed keys");
    if (c->wide) return fail(c, KMER_E_STATE, "keys of 64 bits or more (k - |P| >= 32) have no packed partials");
    if (hipSetDevice(c->device) != hipSuccess) return KMER_E_DEVICE;
    if (out) *out = nullptr;
    hipStream_t s = c->stream;
    HIPCHK(c, hipEventRecord(c->ev2, s));
    // the partials, concatenated in shard order, are already in first-occurrence
    // order: their index is their rank
    kmer_status st = ensure_rank_arrays(c, n, 0, s);
    if (st) return st;
    HIPCHK(c, c->rcnt.ensure(n, s));
    HIPCHK(c, launch_merge_prep((const uint64_t *)d_keys, (const Agg *)d_vals, n, c->rkey.p,
                                c->narrow ? c->rkey32.p : nullptr, c->rord.p, c->rcnt.p, c->ridx.p, s));
    uint64_t nu = 0;
    const bool sync = out || c->p.max_keys;
    st = rank_finish(c, n, false, true, &nu, sync);
    if (st) return st;
    c->n_out = nu;
    HIPCHK(c, hipEventRecord(c->ev3, s));
    c->timing_pending = true;
    c->n_hits = 0;
    c->n_cross = 0;
    c->open_stream = false;
    if (!sync) return KMER_OK;
    st = resolve_out(c);
    if (st) return st;
    const uint64_t total = c->n_out + c->exotic.size();
    if (c->p.max_keys && total > c->p.max_keys)
        return fail(c, KMER_E_TOO_MANY_KEYS, "more distinct keys than max_keys (reference Map limit)");
    if (!out) return KMER_OK;
    return build_result(c, total_lines, out);
}

// One ordered result from the ranks' ordered key ranges (after
// kmer_finish_exchanged), gathered to one device: a stable radix sort of the
// first-occurrence keys (each list is sorted; their union is re-ordered),
// then keys / counts / firsts permuted into the context's result arrays.
kmer_status kmer_merge_ordered(kmer_ctx *c, const void *d_keys, const void *d_counts, const void *d_firsts,
                               uint64_t n, uint64_t total_lines, kmer_result **out) {
    if (!c || (n && (!d_keys || !d_counts || !d_firsts))) return KMER_E_BAD_PARAM;
    SETTLE(c);
    if (c->mode != MODE_PACKED && c->mode != MODE_WINDOWS)
        return fail(c, KMER_E_STATE, "configuration has no packed keys");
    if (n >= (1ull << 32)) return fail(c, KMER_E_TOO_MANY_KEYS, "more than 2^32 entries to merge");
    if (hipSetDevice(c->device) != hipSuccess) return KMER_E_DEVICE;
    if (out) *out = nullptr;
    hipStream_t s = c->stream;
    HIPCHK(c, hipEventRecord(c->ev2, s));
    const uint64_t k = c->p.k;
    if (n) {
        HIPCHK(c, c->xord.ensure(n, s));
        HIPCHK(c, c->xord2.ensure(n, s));
        HIPCHK(c, c->ridx.ensure(n, s));
        HIPCHK(c, c->ridx2.ensure(n, s));
        HIPCHK(c, c->keys_out.ensure(n * k, s));
        HIPCHK(c, c->cnt_out.ensure(n, s));
        HIPCHK(c, c->first.ensure(n, s));
        HIPCHK(c, hipMemcpyAsync(c->xord.p, d_firsts, n * 8, hipMemcpyDeviceToDevice, s));
        rocprim::counting_iterator<uint32_t> iota(0u);
        ROCPRIM_RUN(c, rocprim::radix_sort_pairs(t, b, c->xord.p, c->xord2.p, iota, c->ridx2.p, (size_t)n, 0, 64, s));
        HIPCHK(c, launch_permute_rows((const uint8_t *)d_keys, (const uint64_t *)d_counts, (const uint64_t *)d_firsts,
                                      c->ridx2.p, n, (uint32_t)k, c->keys_out.p, c->cnt_out.p, c->first.p, s));
    }
    c->n_out = n;
    c->out_pending = false;
    HIPCHK(c, hipEventRecord(c->ev3, s));
    c->timing_pending = true;
    c->open_stream = false;
    const bool sync = out || c->p.max_keys;
    if (!sync) return KMER_OK;
    kmer_status st = resolve_out(c);
    if (st) return st;
    const uint64_t total = c->n_out + c->exotic.size();
    if (c->p.max_keys && total > c->p.max_keys)
        return fail(c, KMER_E_TOO_MANY_KEYS, "more distinct keys than max_keys (reference Map limit)");
    if (!out) return KMER_OK;
    return build_result(c, total_lines, out);
}

kmer_status kmer_exchange_prepare(kmer_ctx *c, uint32_t world, const void **d_send, uint64_t *counts) {
    if (!c || !d_send || !counts || world == 0 || world > XP_MAXW) return KMER_E_BAD_PARAM;
    SETTLE(c);
    if (c->mode != MODE_PACKED && c->mode != MODE_WINDOWS)
        return fail(c, KMER_E_STATE, "configuration has no packed keys");
    if (c->wide) return fail(c, KMER_E_STATE, "keys of 64 bits or more (k - |P| >= 32) have no packed partials");
    if (!c->open_stream) return fail(c, KMER_E_STATE, "exchange without reset/feed");
    if (hipSetDevice(c->device) != hipSuccess) return KMER_E_DEVICE;
    hipStream_t s = c->stream;
    kmer_status st = apply_cross(c);
    if (st) return st;
    const uint64_t n = c->n_hits;
    *d_send = nullptr;
    for (uint32_t o = 0; o < world; ++o) counts[o] = 0;
    c->n_hits = 0;           // the rank arrays are handed over (finish_exchanged refills them)
    if (n == 0) return KMER_OK;
    const uint64_t nblk64 = (n + XP_EPB_HOST - 1) / XP_EPB_HOST;
    if ((uint64_t)world * nblk64 >= (1ull << 31)) return fail(c, KMER_E_BAD_PARAM, "too many hits to partition");
    const uint32_t nblk = (uint32_t)nblk64;
    const uint64_t invalid = c->kbits >= 63 ? ~0ull : (1ull << c->kbits);
    HIPCHK(c, c->xsend.ensure(n, s));
    HIPCHK(c, c->xH.ensure((uint64_t)world * nblk, s));
    HIPCHK(c, c->xHs.ensure((uint64_t)world * nblk, s));
    HIPCHK(c, c->xcnt.ensure(world, s));
    if (!c->h_xcnt) HIPCHK(c, hipHostMalloc((void **)&c->h_xcnt, XP_MAXW * sizeof(uint64_t), hipHostMallocDefault));
    const uint64_t *rk = c->narrow ? nullptr : c->rkey.p;
    const uint32_t *rk32 = c->narrow ? c->rkey32.p : nullptr;
    HIPCHK(c, launch_xpart_hist(rk, rk32, n, invalid, c->kbits, world, nblk, c->xH.p, s));
    ROCPRIM_RUN(c, rocprim::exclusive_scan(t, b, c->xH.p, c->xHs.p, 0u, (size_t)world * nblk,
                                           rocprim::plus<uint32_t>(), s));
    HIPCHK(c, launch_xpart_scatter(rk, rk32, c->rord.p, n, invalid, c->kbits, world, nblk, c->xH.p, c->xHs.p,
                                   c->xsend.p, c->xcnt.p, s));
    HIPCHK(c, hipMemcpyAsync(c->h_xcnt, c->xcnt.p, world * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    for (uint32_t o = 0; o < world; ++o) counts[o] = c->h_xcnt[o];
    *d_send = c->xsend.p;
    return KMER_OK;
}

kmer_status kmer_finish_exchanged(kmer_ctx *c, const void *d_recv, uint64_t n, uint64_t total_lines,
                                  void *wait_stream, kmer_result **out) {
    if (!c || (n && !d_recv)) return KMER_E_BAD_PARAM;
    SETTLE(c);
    if (c->mode != MODE_PACKED && c->mode != MODE_WINDOWS)
        return fail(c, KMER_E_STATE, "configuration has no packed keys");
    if (c->wide) return fail(c, KMER_E_STATE, "keys of 64 bits or more (k - |P| >= 32) have no packed partials");
    if (hipSetDevice(c->device) != hipSuccess) return KMER_E_DEVICE;
    if (out) *out = nullptr;
    hipStream_t s = c->stream;
    // the received buffer was written on the caller's stream (the collective);
    // NULL is the legacy default stream, which the context's non-blocking
    // stream does not otherwise wait for
    HIPCHK(c, hipEventRecord(c->evw, (hipStream_t)wait_stream));
    HIPCHK(c, hipStreamWaitEvent(s, c->evw, 0));
    HIPCHK(c, hipEventRecord(c->ev2, s));
    // the received hits, concatenated by source rank, are in rank order
    kmer_status st = ensure_rank_arrays(c, n, 0, s);
    if (st) return st;
    HIPCHK(c, launch_xprep((const XHit *)d_recv, n, c->rkey.p, c->narrow ? c->rkey32.p : nullptr, c->rord.p,
                           c->ridx.p, s));
    uint64_t nu = 0;
    const bool sync = out || c->p.max_keys;
    st = rank_finish(c, n, false, false, &nu, sync);
    if (st) return st;
    c->n_out = nu;
    HIPCHK(c, hipEventRecord(c->ev3, s));
    c->timing_pending = true;
    c->n_hits = 0;
    c->n_cross = 0;
    c->open_stream = false;
    if (!sync) return KMER_OK;
    st = resolve_out(c);
    if (st) return st;
    const uint64_t total = c->n_out + c->exotic.size();
    if (c->p.max_keys && total > c->p.max_keys)
        return fail(c, KMER_E_TOO_MANY_KEYS, "more distinct keys than max_keys (reference Map limit)");
    if (!out) return KMER_OK;
    return build_result(c, total_lines, out);
}

// Table mode across ranks: rank o owns the pass-1 partitions [o * TAB_NB /
// world, (o + 1) * TAB_NB / world), i.e. a contiguous slice of the hash space
// and its buckets.  The send buffer holds, per owner, that owner's
// partitions in partition order (one chunk: tb1 as it is).
uint32_t tab_part_lo(uint32_t o, uint32_t world) { return (uint32_t)((uint64_t)o * TAB_NB / world); }

kmer_status kmer_table_exchange_prepare(kmer_ctx *c, uint32_t world, const void **d_send, uint64_t *counts,
                                        uint64_t *parts) {
    if (!c || !d_send || !counts || !parts || world == 0 || world > TAB_NB) return KMER_E_BAD_PARAM;
    SETTLE(c);
    if (c->mode != MODE_TABLE) return fail(c, KMER_E_STATE, "not a table-mode context (KMER_FLAG_UNORDERED)");
    if (!c->open_stream) return fail(c, KMER_E_STATE, "exchange without reset/feed");
    if (hipSetDevice(c->device) != hipSuccess) return KMER_E_DEVICE;
    hipStream_t s = c->stream;
    const size_t nch = c->t_cbase.size();
    for (uint32_t p = 0; p < TAB_NB; ++p) {
        uint64_t x = 0;
        for (size_t ch = 0; ch < nch; ++ch) x += c->t_coff[ch][p + 1] - c->t_coff[ch][p];
        parts[p] = x;
    }
    for (uint32_t o = 0; o < world; ++o) {
        uint64_t x = 0;
        for (uint32_t p = tab_part_lo(o, world); p < tab_part_lo(o + 1, world); ++p) x += parts[p];
        counts[o] = x;
    }
    *d_send = nullptr;
    const uint64_t n = c->t_keys;
    if (n == 0) return KMER_OK;
    if (nch == 1 && c->t_cbase[0] == 0) {
        *d_send = c->tb1.p;
        return KMER_OK;
    }
    std::vector<TabSeg> segs;
    uint64_t dst = 0;
    for (uint32_t p = 0; p < TAB_NB; ++p)
        for (size_t ch = 0; ch < nch; ++ch) {
            const uint64_t a0 = c->t_coff[ch][p], a1 = c->t_coff[ch][p + 1];
            if (a1 > a0) segs.push_back(TabSeg{c->t_cbase[ch] + a0, dst, a1 - a0});
            dst += a1 - a0;
        }
    if (segs.size() >= (1ull << 31)) return fail(c, KMER_E_BAD_PARAM, "too many table segments");
    HIPCHK(c, c->tsend.ensure(n, s));
    HIPCHK(c, c->tseg.ensure(segs.size(), s));
    HIPCHK(c, hipMemcpyAsync(c->tseg.p, segs.data(), segs.size() * sizeof(TabSeg), hipMemcpyHostToDevice, s));
    HIPCHK(c, launch_tab_segcopy(c->tb1.p, c->tseg.p, (uint32_t)segs.size(), c->tsend.p, s));
    HIPCHK(c, hipStreamSynchronize(s));        // (segs is a host temporary; the caller's collective follows)
    *d_send = c->tsend.p;
    return KMER_OK;
}

kmer_status kmer_table_finish_exchanged(kmer_ctx *c, void *d_recv, uint64_t n, const uint64_t *parts,
                                        uint32_t world, uint32_t rank, void *wait_stream) {
    if (!c || (n && !d_recv) || !parts || world == 0 || world > TAB_NB || rank >= world) return KMER_E_BAD_PARAM;
    SETTLE(c);
    if (c->mode != MODE_TABLE) return fail(c, KMER_E_STATE, "not a table-mode context (KMER_FLAG_UNORDERED)");
    if (hipSetDevice(c->device) != hipSuccess) return KMER_E_DEVICE;
    const uint32_t plo = tab_part_lo(rank, world), phi = tab_part_lo(rank + 1, world);
    // the received runs, by source rank: source r's keys of this rank's
    // partitions, partition-major -- one "chunk" per source
    std::vector<uint64_t> cbase;
    std::vector<std::vector<uint64_t>> coff;
    uint64_t base = 0;
    for (uint32_t r = 0; r < world; ++r) {
        std::vector<uint64_t> off(TAB_NB + 1, 0);
        uint64_t x = 0;
        for (uint32_t p = 0; p < TAB_NB; ++p) {
            off[p] = x;
            if (p >= plo && p < phi) x += parts[(uint64_t)r * TAB_NB + p];
        }
        off[TAB_NB] = x;
        cbase.push_back(base);
        coff.push_back(std::move(off));
        base += x;
    }
    if (base != n) return fail(c, KMER_E_BAD_PARAM, "received key count does not match the partition counts");
    hipStream_t s = c->stream;
    HIPCHK(c, hipEventRecord(c->evw, (hipStream_t)wait_stream));
    HIPCHK(c, hipStreamWaitEvent(s, c->evw, 0));
    c->t_cbase = std::move(cbase);
    c->t_coff = std::move(coff);
    c->t_keys = n;
    HIPCHK(c, hipEventRecord(c->ev2, s));
    kmer_status st = table_finish(c, n ? (const uint64_t *)d_recv : nullptr, plo << TAB_L2, phi << TAB_L2);
    if (st) return st;
    HIPCHK(c, hipEventRecord(c->ev3, s));
    c->timing_pending = true;
    c->open_stream = false;
    return KMER_OK;
}

kmer_status kmer_records_export(kmer_ctx *c, kmer_result **out) {
    if (!c || !out) return KMER_E_BAD_PARAM;
    SETTLE(c);
    kmer_result *r = new (std::nothrow) kmer_result();
    if (!r) return KMER_E_OOM;
    std::vector<std::pair<uint64_t, const std::pair<const std::string, Ent> *>> ex;
    for (auto &kv : c->exotic) ex.emplace_back(kv.second.first, &kv);
    std::sort(ex.begin(), ex.end(), [](const auto &x, const auto &y) { return x.first < y.first; });
    for (auto &e : ex) {
        r->keys.insert(r->keys.end(), e.second->first.begin(), e.second->first.end());
        r->offsets.push_back(r->keys.size());
        r->counts.push_back(e.second->second.count);
        r->firsts.push_back(e.first);
    }
    *out = r;
    return KMER_OK;
}

kmer_status kmer_records_import(kmer_ctx *c, const char *keys, const uint64_t *offsets, const uint64_t *counts,
                                const uint64_t *firsts, uint64_t n) {
    if (!c || (n && (!keys || !offsets || !counts || !firsts))) return KMER_E_BAD_PARAM;
    SETTLE(c);
    for (uint64_t i = 0; i < n; ++i) {
        std::string key(keys + offsets[i], offsets[i + 1] - offsets[i]);
        auto it = c->exotic.find(key);
        if (it == c->exotic.end()) {
            c->exotic.emplace(key, Ent{counts[i], firsts[i]});
        } else {
            it->second.count += counts[i];
            it->second.first = std::min(it->second.first, firsts[i]);
        }
    }
    return KMER_OK;
}

kmer_status kmer_records_clear(kmer_ctx *c) {
    if (!c) return KMER_E_BAD_PARAM;
    SETTLE(c);
    c->exotic.clear();
    return KMER_OK;
}

kmer_status kmer_set_position(kmer_ctx *c, uint64_t lines_before, uint64_t byte_offset) {
    if (!c) return KMER_E_BAD_PARAM;
    SETTLE(c);
    if (hipSetDevice(c->device) != hipSuccess) return KMER_E_DEVICE;
    c->prep_flags |= PREP_SETPOS;      // applied by the next feed's prologue (flush_prep)
    c->prep_lines = lines_before;
    c->abs_offset = byte_offset;
    c->host_lines = lines_before;
    return KMER_OK;
}

kmer_status kmer_lines(kmer_ctx *c, uint64_t *lines) {
    if (!c || !lines) return KMER_E_BAD_PARAM;
    SETTLE(c);
    StreamPos pos;
    kmer_status st = read_pos(c, &pos);
    if (st) return st;
    *lines = c->fasta ? c->fa_lines : pos.lines + pos.ends_open;
    return KMER_OK;
}

kmer_status kmer_result_device(kmer_ctx *c, const void **d_keys, const void **d_counts, const void **d_firsts,
                               uint64_t *n) {
    if (!c || !n) return KMER_E_BAD_PARAM;
    SETTLE(c);
    if (c->mode == MODE_TABLE) return fail(c, KMER_E_STATE, "table mode: use kmer_table_device");
    kmer_status st = resolve_out(c);
    if (st) return st;
    if (d_keys) *d_keys = c->keys_out.p;
    if (d_counts) *d_counts = c->cnt_out.p;
    if (d_firsts) *d_firsts = c->first.p;
    *n = c->n_out;
    return KMER_OK;
}

kmer_status kmer_table_stats(kmer_ctx *c, uint64_t *canonical, uint64_t *keys, uint64_t *total) {
    if (!c) return KMER_E_BAD_PARAM;
    if (!c->group.empty()) {                         // a group: its children's shares add up
        if (c->mode != MODE_TABLE || !c->t_done) return fail(c, KMER_E_STATE, "no table finish on this group yet");
        uint64_t a[3] = {0, 0, 0};
        for (kmer_ctx *x : c->group) {
            uint64_t b[3] = {0, 0, 0};
            if (hipSetDevice(x->device) != hipSuccess) return KMER_E_DEVICE;
            const kmer_status st = kmer_table_stats(x, &b[0], &b[1], &b[2]);
            if (st) return fail(c, st, x->err);
            for (int i = 0; i < 3; ++i) a[i] += b[i];
        }
        if (canonical) *canonical = a[0];
        if (keys) *keys = a[1];
        if (total) *total = a[2];
        return KMER_OK;
    }
    SETTLE(c);
    if (c->mode != MODE_TABLE) return fail(c, KMER_E_STATE, "not a table-mode context (KMER_FLAG_UNORDERED)");
    if (!c->t_done) return fail(c, KMER_E_STATE, "no table finish yet");
    uint64_t rk = 0, rs = 0;
    if (c->p.flags & KMER_FLAG_CANONICAL) {
        for (auto &kv : canonical_records(c))
            if (kv.first.compare(0, c->prefix.size(), c->prefix) == 0) {
                rk += 1;
                rs += kv.second;
            }
    } else {
        for (auto &kv : c->exotic) {
            rk += 1;
            rs += kv.second.count;
        }
    }
    if (canonical) *canonical = c->t_canon;
    if (keys) *keys = c->t_nkeys + rk;
    if (total) *total = c->t_sum + rs;
    return KMER_OK;
}

kmer_status kmer_table_device(kmer_ctx *c, const void **d_entries, const void **d_bucket_start,
                              const void **d_bucket_len, const void **d_big, uint64_t *n_big) {
    if (!c) return KMER_E_BAD_PARAM;
    SETTLE(c);
    if (c->mode != MODE_TABLE) return fail(c, KMER_E_STATE, "not a table-mode context (KMER_FLAG_UNORDERED)");
    if (!c->t_done) return fail(c, KMER_E_STATE, "no table finish yet");
    const bool any = c->t_keys != 0;
    if (d_entries) *d_entries = any ? c->t_ent : nullptr;
    if (d_bucket_start) *d_bucket_start = any ? c->tstart.p : nullptr;
    if (d_bucket_len) *d_bucket_len = any ? c->tnd.p : nullptr;
    if (d_big) *d_big = any ? c->tbig.p : nullptr;
    if (n_big) *n_big = c->t_nbig;
    return KMER_OK;
}

kmer_status kmer_table_digest(kmer_ctx *c, uint64_t *digest) {
    if (!c || !digest) return KMER_E_BAD_PARAM;
    if (!c->group.empty()) {                         // a group: its children's digests add up
        if (c->mode != MODE_TABLE || !c->t_done) return fail(c, KMER_E_STATE, "no table finish on this group yet");
        uint64_t a = 0;
        for (kmer_ctx *x : c->group) {
            uint64_t d = 0;
            if (hipSetDevice(x->device) != hipSuccess) return KMER_E_DEVICE;
            const kmer_status st = kmer_table_digest(x, &d);
            if (st) return fail(c, st, x->err);
            a += d;
        }
        *digest = a;
        return KMER_OK;
    }
    SETTLE(c);
    if (c->mode != MODE_TABLE) return fail(c, KMER_E_STATE, "not a table-mode context (KMER_FLAG_UNORDERED)");
    if (!c->t_done) return fail(c, KMER_E_STATE, "no table finish yet");
    *digest = 0;
    if (!c->t_keys) return KMER_OK;
    hipStream_t s = c->stream;
    unsigned long long *d = c->tstats.p + 4;
    HIPCHK(c, hipMemsetAsync(d, 0, 8, s));
    HIPCHK(c, launch_tab_digest(c->t_ent, c->tstart.p, c->tnd.p, d, s));
    uint64_t acc = 0;
    std::vector<TabBig> big(c->t_nbig);
    HIPCHK(c, hipMemcpyAsync(&acc, d, 8, hipMemcpyDeviceToHost, s));
    if (!big.empty())
        HIPCHK(c, hipMemcpyAsync(big.data(), c->tbig.p, big.size() * sizeof(TabBig), hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    for (const TabBig &b : big) acc += (b.count - TAB_CMAX) * tab_digest_mix(b.h);   // entries hold TAB_CMAX
    *digest = acc;
    return KMER_OK;
}

kmer_status kmer_phase_times(kmer_ctx *c, uint32_t max, const char **names, double *ms, uint32_t *n) {
    if (!c || !n || (max && (!names || !ms))) return KMER_E_BAD_PARAM;
    SETTLE(c);
    static const char *tab_names[6] = {"lines", "hist1", "scatter1", "hist2", "scatter2", "final"};
    static const char *ord_names[3] = {"scan", "feed", "finish"};
    if (c->mode == MODE_TABLE) {
        *n = 6;
        for (uint32_t i = 0; i < 6 && i < max; ++i) {
            names[i] = tab_names[i];
            ms[i] = c->t_ms[i];
        }
        return KMER_OK;
    }
    kmer_status st = resolve_out(c);
    if (st) return st;
    const double v[3] = {c->scan_ms, c->feed_ms, c->finish_ms};
    *n = 3;
    for (uint32_t i = 0; i < 3 && i < max; ++i) {
        names[i] = ord_names[i];
        ms[i] = v[i];
    }
    return KMER_OK;
}

kmer_status kmer_last_timing(kmer_ctx *c, double *scan_ms, double *feed_ms, double *finish_ms) {
    if (!c) return KMER_E_BAD_PARAM;
    SETTLE(c);
    // (the finish is waited for only when its time is asked for)
    kmer_status st = finish_ms ? resolve_out(c) : resolve_feed_timing(c);
    if (st) return st;
    if (scan_ms) *scan_ms = c->scan_ms;
    if (feed_ms) *feed_ms = c->feed_ms;
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

kmer_status kmer_result_firsts(const kmer_result *r, const uint64_t **firsts) {
    if (!r || !firsts) return KMER_E_BAD_PARAM;
    *firsts = r->firsts.data();
    return KMER_OK;
}

// Serialise a result in Map order.  KMER_WRITE_JSON: JSON.stringify of
// mapToJSON(map) (lib/kmers.js:46-54): {"key":count,...}, keys escaped as
// JSON.stringify does (\" \\ \b \f \n \r \t, other bytes < 0x20 as \u00XX).
// KMER_WRITE_LEGACY: the npm main's dump (lib/index.js:381-388):
// "{\n" then "key: count," per entry, then "}\n".
kmer_status kmer_result_write(const kmer_result *r, const char *path, uint32_t format) {
    if (!r || !path || format > KMER_WRITE_LEGACY) return KMER_E_BAD_PARAM;
    FILE *f = fopen(path, "wb");
    if (!f) return KMER_E_IO;
    std::string out;
    out.reserve(1 << 22);
    const uint64_t n = r->counts.size();
    char num[32];
    auto flush = [&]() -> bool {
        const bool ok = fwrite(out.data(), 1, out.size(), f) == out.size();
        out.clear();
        return ok;
    };
    bool ok = true;
    out += format == KMER_WRITE_JSON ? "{" : "{\n";
    for (uint64_t i = 0; i < n && ok; ++i) {
        const char *k = r->keys.data() + r->offsets[i];
        const uint64_t kl = r->offsets[i + 1] - r->offsets[i];
        const int nl = snprintf(num, sizeof(num), "%llu", (unsigned long long)r->counts[i]);
        if (format == KMER_WRITE_JSON) {
            if (i) out += ',';
            out += '"';
            for (uint64_t j = 0; j < kl; ++j) {
                const unsigned char ch = (unsigned char)k[j];
                switch (ch) {
                case '"': out += "\\\""; break;
                case '\\': out += "\\\\"; break;
                case '\b': out += "\\b"; break;
                case '\f': out += "\\f"; break;
                case '\n': out += "\\n"; break;
                case '\r': out += "\\r"; break;
                case '\t': out += "\\t"; break;
                default:
                    if (ch < 0x20) {
                        char u[8];
                        snprintf(u, sizeof(u), "\\u%04x", ch);
                        out += u;
                    } else {
                        out += (char)ch;
                    }
                }
            }
            out += "\":";
            out.append(num, nl);
        } else {
            out.append(k, kl);
            out += ": ";
            out.append(num, nl);
            out += ',';
        }
        if (out.size() > (1u << 22)) ok = flush();
    }
    out += format == KMER_WRITE_JSON ? "}" : "}\n";
    ok = ok && flush();
    ok = (fclose(f) == 0) && ok;
    return ok ? KMER_OK : KMER_E_IO;
}

void kmer_result_free(kmer_result *r) { delete r; }

}  // extern "C"
