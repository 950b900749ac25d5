// kmer_host.hpp — host-side internals shared by the C-ABI translation units
// (kmer_api.hip: entry points; kmer_feed.hip: chunk feeds and the packed
// path's settle; kmer_finish.hip: ordered finish; kmer_tabhost.hip: table
// mode orchestration; kmer_io.hip: host input (buffers, files, FIFOs, gzip)
// and the whole-input counts; kmer_group.hip: multi-device groups).
// The kernels and their launchers are in kmer_internal.hpp.
#pragma once
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
constexpr uint32_t KMER_FLAGS_PUBLIC = 0xFFu | KMER_FLAG_FASTA | KMER_FLAG_TABLE_FIXED_TEST | KMER_FLAG_GEN_COLLIDE_TEST;

namespace kmerhip {


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
        hipError_t e;
        if (p && !(keep && used)) {               // nothing to keep: the old block goes first (peak = the new size)
            e = hipStreamSynchronize(s);
            if (e != hipSuccess) return e;
            (void)hipFree(p);
            p = nullptr;
            cap = 0;
        }
        T *q = nullptr;
        e = hipMalloc((void **)&q, nc * sizeof(T));
        if (e != hipSuccess) return e;
        if (exp_env("KMERHIP_POISON")) {           // (experiments build: every new buffer starts as 0xA5 bytes)
            e = hipMemsetAsync(q, 0xA5, nc * sizeof(T), s);
            if (e != hipSuccess) return e;
        }
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


}  // namespace kmerhip


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
    DBuf<uint64_t> dcnt;           // dense-hit path (kmer_dense.hip): accepted forward | reverse << 32 per line
    DBuf<uint32_t> dtot;           // ... their sum per line (scanned into wbase)
    DBuf<uint64_t> ddbg;           // ... a refused rank slot's context (diagnostics)
    bool win_slots = false;        // a chunk of this session ranked every window (the finish compacts)
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
    bool gen_planes = false;       // general path, A/C/G/T prefix: windows from the plane candidates (gen_cand_kernel)
    PlaneArgs pargs{};
    DBuf<uint32_t> ridx, ridx2, ecnt, bbase;
    DBuf<uint64_t> epre;
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
    DBuf<uint64_t> ukey, first, cnt_out;
    DBuf<Agg> uval;
    DBuf<uint8_t> keys_out;
    uint64_t n_out = 0;            // ordered entries of the last finish (device)
    // records & lines
    DBuf<uint32_t> cpcnt;          // dense-hit compaction: valid ranks per CP_BLOCK
    DBuf<uint64_t> cpoff;          // ... their offsets (+ total)
    DBuf<Record> recs;
    DBuf<Record> gcand;            // general path, A/C/G/T prefix: window candidates (gen_cand_kernel)
    DBuf<SeqLine> lines;
    DBuf<uint8_t> rec_keys;
    // scratch
    DBuf<uint8_t> tmp;
    // device scalars, one block so that a feed reads them back with one copy:
    // [0] rec_count [1] ovf_count [2] cross count [3] chunk hits [4] unique keys
    // [5] err (u32) [6] line count [7] chunk ends open
    uint64_t *d_scal = nullptr;
    unsigned int *d_ticket = nullptr, *d_err = nullptr;
    unsigned int *d_bticket = nullptr;   // bucket_offsets_kernel last-block ticket (returned to 0 by it)
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
    uint64_t *h_small = nullptr;   // pinned (24 words): [0..7] copy of d_scal, [8..11] pos, [12..17] table feed
    uint64_t *h_tail = nullptr;    // pinned, mapped, coherent: d_scal[0..7] written by the chunk tail kernel
    // pinned staging of every host -> device upload (upload()): a pageable
    // hipMemcpyAsync may read its host buffer after the call returns, so the
    // bytes are copied here first; a region is reused only after the streams
    // that read it have been synchronised (bump allocation, drained on wrap)
    uint8_t *up_p = nullptr;
    size_t up_cap = 0, up_used = 0;
    std::vector<hipStream_t> up_streams;
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
    DBuf<unsigned long long> tspc; // pass-1 spill-area cursors (TAB_NB) + overflow count
    DBuf<TabUnit> tunits;          // pass-2 units, then TAB_NB partition heads
    DBuf<TabBig> tbig;             // entries with counts >= TAB_CMAX
    DBuf<uint32_t> tpc;            // pieces per sequence line (long lines)
    DBuf<uint32_t> tleft;          // [0] count, then [q, qe) pairs: units the sort final kernel left
    DBuf<uint64_t> tpb;            // ... their scan
    DBuf<SeqLine> tpieces;         // long lines cut into pieces of <= TAB_PIECE windows
    DBuf<unsigned long long> tstats;   // [0..2] final statistics, [3] big-list count, [4] digest
    uint64_t t_keys = 0;           // pass-1 slots of the session (keys, plus filler of fixed runs)
    uint64_t t_p1_fixed = 0, t_p1_merged = 0, t_p1_counted = 0;   // pass-1 routes (kmer_table_routes)
    uint64_t t_p2_fixed = 0;       // finishes whose pass 2 ran with fixed bucket capacities (tab_scatter2f)
    uint64_t t_fill = 0;           // ... of which filler slots (an estimate: windows with non-ACGT bytes are not keys)
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
    uint32_t peer_staged = 0;      // device pairs of the group without peer access (copies staged by the runtime)
    // general path, device merge (step 1, kmer_finish.hip general_merge):
    // session entries -- key bytes at stride k, counts, first-occurrence keys
    bool gm_on = false;
    bool gm_merged = true;         // entries unique (merged since the last append)
    uint64_t gm_last = 0;          // entries after the last merge
    uint64_t gm_n = 0;
    DBuf<uint8_t> gm_keys, gm_keys2;
    DBuf<uint64_t> gm_cnt, gm_cnt2, gm_first, gm_first2, gm_h1, gm_h2, gm_h1b, gm_h2b;
    DBuf<uint32_t> gm_idx, gm_idx2, gm_head, gm_gid, gm_start;
    DBuf<unsigned int> gm_flag;
    DBuf<uint64_t> gkeys, gkeys2;
    DBuf<Agg> gvals, gvals2;
    double t_ms[7] = {};           // table phase times since the reset: lines, hist1, scatter1, hist2, scatter2, final, fasta
    hipEvent_t fa_ev[2] = {nullptr, nullptr};   // around a chunk's FASTA rewrite
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

namespace kmerhip {


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
inline void report_progress(kmer_ctx *c, uint64_t done, uint64_t total) {
    if (!c->p.progress) return;
    if (c->progress_any && done < c->progress_hw) return;
    c->progress_any = true;
    c->progress_hw = done;
    c->p.progress(c->p.progress_user, done, total);
}

inline kmer_status fail(kmer_ctx *c, kmer_status s, const std::string &msg) {
    c->err = msg;
    return s;
}

inline uint8_t comp(uint8_t c) {
    switch (c) {
    case 'A': return 'T';
    case 'T': return 'A';
    case 'G': return 'C';
    case 'C': return 'G';
    default: return c;
    }
}

inline uint32_t pack4(const std::string &s) {
    uint32_t v = 0;
    for (size_t i = 0; i < 4 && i < s.size(); ++i) v |= (uint32_t)(uint8_t)s[i] << (8 * i);
    return v;
}

template <typename T>
inline hipError_t dalloc(T **p, uint64_t n) {
    return hipMalloc((void **)p, std::max<uint64_t>(n, 1) * sizeof(T));
}

template <typename T>
inline void dfree(T *&p) {
    if (p) (void)hipFree((void *)p);
    p = nullptr;
}

inline int bit_width(uint64_t x) { return x ? 64 - __builtin_clzll(x) : 0; }

#define SETTLE(ctx)                                                                       \
    do {                                                                                  \
        if (!(ctx)->group.empty()) return fail(ctx, KMER_E_STATE, "single-device call on a group context"); \
        const kmer_status st_ = settle(ctx);                                              \
        if (st_) return st_;                                                              \
    } while (0)

// the input of a multi-device group count: batches of a buffer or a file
struct GroupSrc {
    virtual ~GroupSrc() {}
    virtual void progress(uint64_t *done, uint64_t *total) = 0;
    // the next batch (valid until release()); false at the end of the input
    virtual bool next(const uint8_t **p, uint64_t *n, kmer_status *st, std::string *err) = 0;
    virtual void release(const uint8_t *) {}
};

// ---- functions shared between the host translation units ----
kmer_status ensure_tiles(kmer_ctx *c, uint64_t n_tiles);
kmer_status upload(kmer_ctx *c, void *dst, const void *src, size_t n, hipStream_t s);
kmer_status general_append(kmer_ctx *c, const uint8_t *d, uint64_t nrec, hipStream_t s);
kmer_status general_merge(kmer_ctx *c);
kmer_status general_finish(kmer_ctx *c);
kmer_status general_to_host(kmer_ctx *c);
kmer_status ensure_ovf(kmer_ctx *c, uint64_t n, hipStream_t s);
kmer_status ensure_records(kmer_ctx *c, uint64_t n);
kmer_status drain_records(kmer_ctx *c, const uint8_t *d_data, uint64_t n, hipStream_t s);
kmer_status wait_tail(kmer_ctx *c, uint64_t seq, hipStream_t qs);
kmer_status resolve_feed_timing(kmer_ctx *c);
kmer_status flush_prep(kmer_ctx *c, hipStream_t s, uint32_t extra);
kmer_status check_err(kmer_ctx *c, uint32_t e);
kmer_status ensure_rank_arrays(kmer_ctx *c, uint64_t need, uint64_t keep, hipStream_t s);
kmer_status ensure_cross(kmer_ctx *c, uint64_t need, hipStream_t s);
void bind_hits(kmer_ctx *c, HitArgs &h);
kmer_status launch_chunk(kmer_ctx *c);
kmer_status scan_feed(kmer_ctx *c, const uint8_t *d, uint64_t len, uint32_t n_tiles, hipStream_t s);
kmer_status settle(kmer_ctx *c);
kmer_status two_pass_prefix(kmer_ctx *c, const uint8_t *d, uint64_t len, uint32_t n_tiles, hipStream_t s);
kmer_status collect_lines(kmer_ctx *c, const uint8_t *d, uint64_t len, uint32_t n_tiles, hipStream_t s,
                          uint64_t *nlines_out);
kmer_status general_feed(kmer_ctx *c, const uint8_t *d, uint64_t len, uint32_t n_tiles, hipStream_t s);
kmer_status chunk_lines(kmer_ctx *c, const uint8_t *d, uint64_t len, uint32_t n_tiles, hipStream_t s, bool check_len,
                        uint64_t *n_nl_out, uint64_t *n_seq_out);
kmer_status windows_feed(kmer_ctx *c, const uint8_t *d, uint64_t len, uint32_t n_tiles, hipStream_t s);
float ev_ms(kmer_ctx *c, hipEvent_t a, hipEvent_t b);
kmer_status table_feed(kmer_ctx *c, const uint8_t *d, uint64_t len, uint32_t n_tiles, hipStream_t s);
kmer_status table_finish(kmer_ctx *c, const uint64_t *B1 = nullptr, uint32_t qlo = 0, uint32_t qhi = TAB_NQ);
std::unordered_map<std::string, uint64_t> canonical_records(const kmer_ctx *c);
kmer_status build_table_result(kmer_ctx *c, uint64_t lines, kmer_result **out);
kmer_status fasta_rewrite(kmer_ctx *c, const uint8_t *d, uint64_t len, hipStream_t s, const uint8_t **od,
                          uint64_t *olen);
kmer_status feed(kmer_ctx *c, const uint8_t *d, uint64_t len, hipStream_t s);
kmer_status reset(kmer_ctx *c);
kmer_status apply_cross(kmer_ctx *c);
kmer_status sort_and_heads_wide(kmer_ctx *c, uint64_t n);
kmer_status bucket_heads(kmer_ctx *c, uint64_t n);
kmer_status compact_windows(kmer_ctx *c);
kmer_status resolve_out(kmer_ctx *c);
kmer_status rank_finish(kmer_ctx *c, uint64_t n, bool partial, bool with_counts, uint64_t *nu_out, bool sync = true);
kmer_status build_result(kmer_ctx *c, uint64_t lines, kmer_result **out);
kmer_status read_pos(kmer_ctx *c, StreamPos *pos);
kmer_status finish(kmer_ctx *c, kmer_result **out);
uint64_t batch_cut(const uint8_t *p, uint64_t n, bool fasta);
uint64_t batch_extend(const uint8_t *b, uint64_t from, uint64_t len, bool fasta);
kmer_status feed_host(kmer_ctx *c, const uint8_t *bytes, uint64_t len, bool report = false);
uint64_t fasta_records(const uint8_t *p, uint64_t n);
uint64_t count_newlines(const uint8_t *p, uint64_t n);
kmer_status group_gather_records(kmer_ctx *g);
kmer_status group_each(kmer_ctx *g, size_t n, const std::function<kmer_status(size_t)> &f);
kmer_status group_count(kmer_ctx *g, GroupSrc &src, kmer_result **out);
void set_pbits(kmer_ctx *c, uint32_t pbits);
kmer_status with_long_line_retry(kmer_ctx *c, const std::function<kmer_status()> &count);
kmer_status count_buffer_once(kmer_ctx *c, const uint8_t *bytes, size_t len, kmer_result **out);
kmer_status count_file_once(kmer_ctx *c, const char *path, kmer_result **out);
kmer_status group_count_buffer(kmer_ctx *g, const uint8_t *bytes, uint64_t len, kmer_result **out);
kmer_status group_count_file(kmer_ctx *g, const char *path, kmer_result **out);

}  // namespace kmerhip
