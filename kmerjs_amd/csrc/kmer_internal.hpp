// kmer_internal.hpp — shared definitions between the gfx950 kernels
// (kmer_kernels.hip) and the host orchestration (kmer_api.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

namespace kmerhip {

// ---- experiment switches ----------------------------------------------------
// A/B switches (KMERHIP_* environment variables) and ablations (the
// KMERHIP_XFLAG_ABLATE_* bits of kmer_params.flags; results are WRONG with
// them) exist only in a -DKMERHIP_EXPERIMENTS build of the library, made by
// tools/ for timing studies.  The shipping libkmerhip.so reads no environment
// variable, and kmer_open rejects the ablation bits (KMER_E_BAD_PARAM).
#ifdef KMERHIP_EXPERIMENTS
inline const char *exp_env(const char *name) { return getenv(name); }
#define KH_ABLATE(a) ((a).ablate)
constexpr bool KH_EXPERIMENTS = true;
#else
inline const char *exp_env(const char *) { return nullptr; }
#define KH_ABLATE(a) 0u
constexpr bool KH_EXPERIMENTS = false;
#endif
enum : uint32_t {
    KMERHIP_XFLAG_ABLATE_HITS = 1u << 8,   // drop every prefix candidate
    KMERHIP_XFLAG_ABLATE_SWAR = 1u << 9,   // skip the SWAR prefix scan
    KMERHIP_XFLAG_MASK = 0xFFu << 8,       // bits 8..15: tile-scan ablations (ScanArgs::ablate)
};

// ---- tile geometry (tile kernel) -------------------------------------------
// One workgroup owns one 16 KiB tile of the input.  The tile plus a front halo
// (rc windows whose start lies in the previous tile) and a back halo (forward
// windows that run into the next tile) is staged in LDS.
constexpr int TPB = 256;                 // threads per workgroup (4 waves)
constexpr int BPT = 64;                  // bytes scanned per thread
constexpr int TILE = TPB * BPT;          // 16384
constexpr int FH = 64;                   // front halo bytes
constexpr int BH = 80;                   // back halo bytes (>= KMAX_TILE - 1 + 3, x16)
constexpr int KMAX_PACKED = 32;          // longest k of a 2-bit packed (u64) key
constexpr int KMAX_TILE = 64;            // longest k handled by the tile kernel
constexpr int KMAX_DENSE = 32;           // longest k packed into 2-bit codes
constexpr uint32_t MAXREL = (1u << 23) - 1;  // longest sequence line (bytes - 1), default order-key layout
// Order key = line << (pbits + 1) | strand << pbits | position field (pbits
// bits).  Default 23 (lines up to 8 MiB, 2^40 lines); long-line mode 40
// (lines up to 1 TiB, 2^23 lines) -- KMER_FLAG_LONG_LINES, or the automatic
// retry of kmer_count_file / kmer_count_buffer.
constexpr uint32_t PBITS_DEFAULT = 23, PBITS_LONG = 40;
// newline positions kept per 16 KiB tile by the one-pass line split (lines of
// >= 16 bytes on average; denser tiles take the two-pass route)
constexpr uint32_t NL_SLOTS = 1024;

// error bits (device-side, OR-ed into ctx->d_err)
enum : uint32_t {
    ERR_NONASCII = 1u << 0,
    ERR_LINE_TOO_LONG = 1u << 1,
    ERR_LOOKBACK_TIMEOUT = 1u << 2,
    ERR_REC_OVERFLOW = 1u << 3,
    ERR_LINE_OVERFLOW = 1u << 4,
    ERR_OVF_OVERFLOW = 1u << 5,
    ERR_CROSS_OVERFLOW = 1u << 6,
    ERR_COUNT_OVERFLOW = 1u << 7,    // table mode: one key counted 2^32 times in one bucket
    ERR_BIG_OVERFLOW = 1u << 8,      // table mode: big-count list full
    ERR_TAB_SPLIT = 1u << 9,         // table mode: bucket range could not be split further
    ERR_DENSE_RANK = 1u << 10,       // dense-hit path: a rank slot past the counted hits (count / write disagree)
    ERR_TAB_CAP = 1u << 11,          // table mode: a bucket past its fixed pass-2 capacity (counted route redoes it)
    // not an error: a tile without '\n' had hits, or a tile overflowed its hit
    // slots -- cross segments may be long (finish sorts the whole cross list)
    INFO_LONGSEG = 1u << 16,
};

// look-back word: [63:62] status, [61:0] value
constexpr uint64_t LB_AGG = 1ull << 62;
constexpr uint64_t LB_INC = 2ull << 62;
constexpr uint64_t LB_VAL = (1ull << 62) - 1;

// Running position of the stream, kept in device memory so consecutive
// launches chain without host round trips.
struct StreamPos {
    uint64_t lines;        // newlines consumed before the next chunk (= its first line index)
    uint64_t unused;
    uint64_t ends_open;    // 1 if the last chunk did not end with '\n'
    uint64_t pad;
};

// A window that cannot take the dense path (non-ACGT byte, long key, or a
// non-dense configuration).  Its key bytes are gathered later:
// key = strand ? rc(data[pos, pos+len)) : data[pos, pos+len)   (pos is chunk-relative)
struct Record {
    uint64_t order;
    uint64_t pos;
    uint32_t len;
    uint32_t strand;
};

// A sequence line for the general (any k / any step) kernel.
struct SeqLine {
    uint64_t start;        // chunk-relative byte offset
    uint64_t len;
    uint64_t line_index;   // global line index
};

// A verified prefix hit from the tile scan with its tile-local line context.
struct HitRec {
    uint64_t code;         // 2-bit codes of the k-byte forward window (its last 32 bases when k > 32;
                           // the first k - 32 are in ScanArgs::hits_hi / ovf_hi at the same index)
    uint32_t tile;
    uint32_t qm;           // [13:0] pattern position q, [14] strand, [15] exotic, [16] line start in tile,
                           // [31:17] ordinal of the hit in its tile
    uint32_t c_local;      // '\n' count in the tile before the window start
    uint32_t lstart;       // tile-relative line start (when [16] is set)
};
constexpr int HMAX = 64;   // hit slots per tile (more go to the overflow list)

// Per-tile aggregates of the scan kernel, scanned (exclusive) across tiles
// with TileSumOp: lines before the tile, start of the line open at the tile
// start, hits before the tile.
struct TileSum {
    uint64_t cnt;                  // real '\n' count
    uint32_t nh;                   // prefix hits (stored + overflow)
    uint32_t nx;                   // ... of which cross hits (line crosses a tile edge; all if overflowed)
    uint64_t lnl;                  // absolute start of the line after its last '\n' (0 = none; scan: max)
};

__host__ __device__ inline TileSum tile_sum_op(const TileSum &x, const TileSum &y) {
    TileSum r;
    r.cnt = x.cnt + y.cnt;
    r.nh = x.nh + y.nh;
    r.nx = x.nx + y.nx;
    r.lnl = x.lnl > y.lnl ? x.lnl : y.lnl;
    return r;
}
constexpr uint32_t TSCAN_BLOCK = 1024;     // tiles per block of the tile scan
constexpr uint32_t TSCAN_INLINE_MAX = 2048; // block-sum prefixes computed in-kernel up to this many blocks

struct ScanArgs {
    const uint8_t *data;
    uint64_t len;
    uint64_t abs_offset;
    uint32_t n_tiles, k, plen;
    uint32_t p4, r4, pmask;
    const uint8_t *PR;
    TileSum *tsum;                 // per tile
    HitRec *hits;                  // n_tiles * HMAX slots
    HitRec *ovf;
    unsigned long long *ovf_count;
    uint64_t ovf_cap;
    unsigned int *err;
    uint32_t ablate;               // experiments only: bit0 = drop all candidates
    uint64_t *hits_hi, *ovf_hi;    // k > 32: code of the window's first k - 32 bases, per hit slot
};

// Bit-plane prefix test (ACGT prefixes): per prefix base i, xor masks that
// turn the plane bits into "code bit equals P_i's bit" (~0 where P_i's bit is 0).
struct PlaneArgs {
    uint32_t kl[5], kh[5];         // P (forward strand)
    uint32_t rl[5], rh[5];         // rc(P), as a forward-strand string
    uint32_t pb;                   // bases tested on the planes: min(|P|, 5); the rest byte-exact
};

// value of a unique packed key: first-occurrence order and count
struct Agg {
    uint64_t first;
    uint64_t count;
};

// Hit resolution.  Packed mode places every hit of the session at its RANK
// (position in first-occurrence order of all hits): a hit whose line lies
// inside one tile gets hits-before-tile + its rank among the tile's hits;
// hits of lines that cross a tile edge (or of overflowed tiles) go to the
// cross list with their natural slot and are placed by a sort at finish.
struct HitArgs {
    const HitRec *hits;
    const TileSum *tsum;
    const TileSum *tscan;          // exclusive scan of tsum (cnt: sum, lnl: max from abs_offset, nh: sum)
    const HitRec *ovf;
    const unsigned long long *ovf_count;
    uint64_t ovf_cap;
    uint32_t n_tiles, k, plen;
    uint64_t abs_offset;
    const StreamPos *pos;
    uint32_t packed;               // ACGT windows are ranked packed keys
    uint32_t pbits;                // order-key position bits (PBITS_*)
    uint64_t smask;                // suffix mask: 2*(k - |P|) bits (its low 64 when wide)
    uint64_t invalid_key;          // 2^(2*(k-|P|)): sorts after every real key (wide: in rkeyh)
    // k > 32: 128-bit window codes (hits_hi / ovf_hi); wide (2(k - |P|) >= 64):
    // keys of two words, the high one in rkeyh (cross list: xkeyh, and xkey
    // holds the entry's own index until apply_cross has moved it)
    const uint64_t *hits_hi, *ovf_hi;
    uint32_t wide;
    uint32_t ablate;               // experiments (KMER_FLAG_ABLATE_*): no line-length errors on unwritten records
    uint64_t smask_hi;             // wide: mask of the high word (2(k - |P|) - 64 bits)
    uint64_t *rkeyh;
    uint64_t *xkeyh, *xkeyl;
    uint64_t out_base;             // session hits before this chunk
    uint64_t rcap;                 // capacity of the rank arrays (a slot past it: the chunk overflowed and is redone)
    uint64_t *rkey;                // by rank: suffix code (invalid_key: filtered / record)
    uint32_t *rkey32;              // ... as u32 when 2(k-|P|) + 1 <= 32 (then rkey is unused)
    uint64_t *rord;                // by rank: first-occurrence order key
    uint64_t *xord, *xkey;         // cross list in natural-slot order (order, key, natural slot)
    uint32_t *xslot;
    uint64_t xbase, xcap;          // session cross entries before this chunk, capacity
    Record *recs;
    unsigned long long *rec_count;
    uint64_t rec_cap;
    unsigned int *err;
    // chunk tail (hit_overflow_kernel's last block): stream position update and
    // the chunk's counters published to host memory
    const uint8_t *data;
    uint64_t len;
    uint64_t *scal;                // device scalars [0..7] (see kmer_ctx::d_scal)
    unsigned int *ticket;          // last-block ticket (returned to 0 by the last block)
    unsigned long long *chunk_hits, *chunk_cross, *ends_open;
    uint64_t *host_out;            // mapped host memory: copy of scal[0..7], then [9] = seq
    uint64_t seq;                  // chunk sequence number (the host waits for it in host_out[9])
};

// By rank, after the key sort: the key and its total count if this rank is
// the key's first occurrence, count 0 otherwise.
struct HeadRec {
    uint64_t key;
    uint64_t count;
};

// Ordered output from the rank arrays after the key sort.
struct EmitArgs {
    const uint32_t *hcnt;          // by rank: the key's count at its first occurrence, else 0
    const HeadRec *hrec;           // merged finish (summed counts): by rank, key and u64 count of heads; else null
    const uint32_t *rkey32;        // hrec == null: key by rank (narrow keys) ...
    const uint64_t *rkey64;        // ... or (wider keys)
    const uint64_t *rkeyh;         // ... with, for keys of >= 64 bits, their high words
    const uint32_t *ecnt;          // heads per EMIT_RPB ranks (head_count_kernel)
    const uint64_t *epre;          // ... their exclusive scan, or null: each workgroup sums the earlier counts
    const uint64_t *rord;          // by rank: order key
    uint64_t n;
    uint64_t invalid_key;
    uint64_t *nuniq;
    uint64_t *nuniq_host;          // mapped host copy of *nuniq (or null)
    uint32_t k, plen, partial;
    uint8_t P[KMAX_TILE];          // the prefix (|P| <= k <= 64 on the packed paths)
    uint8_t *keys_out;             // decode: n * k bytes
    uint64_t *cnt_out, *first_out;
    uint64_t *ukey;                // partial: suffix codes
    Agg *uval;                     // partial: {first, count}
};

struct TileArgs {
    const uint8_t *data;
    uint64_t len;
    uint32_t n_tiles;
    uint32_t k;
    uint32_t plen;
    uint32_t p4, r4, pmask;        // first min(4,|P|) bytes of P and rc(P) (little-endian), byte mask
    uint32_t dense;                // 1: ACGT windows go to the dense table
    uint32_t dense_update;         // 0: skip dense atomics (record-overflow redo of a chunk)
    uint64_t abs_offset;           // absolute byte offset of data[0] in the whole input
    uint32_t emit_lines;           // 1: emit sequence-line descriptors instead of windows
    const uint8_t *PR;             // device: P[0..KMAX_TILE) then rc(P)[0..KMAX_TILE)
    // dense table
    unsigned long long *counts;
    unsigned long long *first;
    // records
    Record *recs;
    unsigned long long *rec_count;
    uint64_t rec_cap;
    // line list
    SeqLine *lines_out;
    unsigned long long *line_count;
    uint64_t line_cap;
    // look-back / positions
    unsigned long long *lb_cnt;
    unsigned long long *lb_lnl;
    unsigned int *ticket;
    StreamPos *pos;
    const uint64_t *tp_cnt;        // two-pass mode: exclusive newline count per tile (absolute line index)
    const uint64_t *tp_lnl;        // two-pass mode: line start before tile (absolute)
    unsigned int *err;
};

// General path with the device merge (step 1): sequence lines from
// chunk_lines, their windows flattened (wbase: exclusive scan of 2W per line)
struct GenWinArgs {
    const uint8_t *data;
    uint64_t len;
    const SeqLine *lines;
    const uint64_t *wbase;
    const uint64_t *tbase;         // newlines before each TILE of the chunk (chunk_lines)
    uint64_t first;                // line index (from the chunk start) of the first sequence line
    uint64_t n_lines, total;       // lines, windows of both strands
    uint32_t k, plen, pbits;
    const uint8_t *P, *RP;         // the prefix and its reverse complement (device)
    Record *recs;
    unsigned long long *rec_count;
    uint64_t rec_cap;
    unsigned int *err;
};
hipError_t launch_gen_windows(const GenWinArgs &a, hipStream_t s);
hipError_t launch_gen_cand(const GenWinArgs &a, const PlaneArgs &pa, hipStream_t s);   // A/C/G/T prefix
hipError_t launch_gen_fix(const Record *cand, uint64_t n, const SeqLine *lines, uint32_t k, uint32_t plen,
                          uint32_t pbits, Record *recs, unsigned long long *rec_count, uint64_t rec_cap,
                          unsigned int *err, hipStream_t s);

struct WindowArgs {
    const uint8_t *data;
    const SeqLine *lines;
    const unsigned long long *n_lines;
    uint32_t k, step, plen;
    uint32_t pbits;                // order-key position bits (PBITS_*)
    const uint8_t *P;              // device copy of the prefix
    Record *recs;
    unsigned long long *rec_count;
    uint64_t rec_cap;
    unsigned int *err;
};

// Dense-hit path (empty or 1-2 base ACGT prefix, step 1, k <= 32): every
// window of every sequence line gets a rank slot -- its position in the
// first-occurrence order: line base (scan of 2W per sequence line) + s for
// the forward window at s, + W + (W-1-s) for the reverse strand's.
struct WinArgs {
    const uint8_t *data;
    uint64_t len;
    const SeqLine *lines;          // by sequence ordinal (len 0: no windows)
    uint64_t n_lines;
    uint64_t li0;                  // line index of the chunk's first line
    const uint64_t *wbase;         // by sequence ordinal: rank of the line's first window (chunk-relative)
    uint32_t k, plen;
    uint32_t pbits;                // order-key position bits (PBITS_*)
    uint32_t step;                 // windows at 0, step, 2 step, ... of the line and of its complement
    unsigned long long *empty;     // step > 1, no prefix: [0] empty keys "" counted, [1] min order key of one
    const uint8_t *P;              // device copy of the prefix (cut-short windows of step > 1)
    uint64_t pcode, rcode;         // P and rc(P) as 2-bit codes (first base most significant)
    uint64_t smask, invalid_key;
    uint64_t out_base;
    uint32_t block_lines;          // lines of many windows (contigs): a workgroup per line, else a wave
    uint64_t *rkey;
    uint32_t *rkey32;
    uint64_t *rord;
    Record *recs;
    unsigned long long *rec_count;
    uint64_t rec_cap;
    unsigned int *err;
};

// dense-hit path, step 1, k <= 64 (kmer_dense.hip): only accepted windows,
// ranked by two passes over the lines
struct DenseArgs {
    const uint8_t *data;
    uint64_t len;
    const SeqLine *lines;          // by sequence ordinal (len 0: no windows)
    uint64_t n_lines;
    uint64_t lpw;                  // lines per wave
    uint32_t k, plen;
    uint32_t pbits;                // order-key position bits (PBITS_*)
    uint64_t pcode;                // P as 2-bit codes (first base most significant)
    uint64_t smask, smask_hi;      // the key: the low 2 (k - |P|) bits of the window code (hi: above bit 64)
    uint64_t *cnt;                 // count pass: per line accepted forward | reverse << 32
    uint32_t *tot;                 // count pass: per line forward + reverse
    const uint64_t *hbase;         // write pass: per line first slot (chunk-relative, exclusive scan of tot)
    uint64_t out_base;
    uint64_t out_end;              // write pass: out_base + the counted hits (slots past it are refused)
    unsigned long long *dbg;       // write pass: the first refused slot's context (8 words, [0] = taken)
    uint32_t *rkey32;              // narrow keys (2 (k - |P|) <= 31 bits), else rkey
    uint64_t *rkey;
    uint64_t *rkeyh;               // wide keys (2 (k - |P|) >= 64 bits): the bits above 64
    uint64_t *rord;
    const uint8_t *P, *RP;         // device: P and rc(P) (exotic windows' prefix bytes)
    Record *recs;
    unsigned long long *rec_count;
    uint64_t rec_cap;
    unsigned int *err;
};
hipError_t launch_dense_windows(const DenseArgs &a, bool write, hipStream_t s);

// ---- launchers (kmer_kernels.hip) ------------------------------------------
hipError_t launch_lines(const TileArgs &a, bool lookback, hipStream_t s);
hipError_t launch_scan_tiles(const ScanArgs &a, hipStream_t s);
hipError_t launch_scan_planes(const ScanArgs &a, const PlaneArgs &pa, hipStream_t s);
hipError_t launch_hits(const HitArgs &a, hipStream_t s);
// exclusive scan of the per-tile sums (init folded in); bsum / bscan: n_blocks scratch
hipError_t launch_tile_reduce(const TileSum *in, uint32_t n, TileSum *bsum, hipStream_t s);
hipError_t launch_tile_scan(const TileSum *in, uint32_t n, const TileSum *bsum, bool bsum_scanned, TileSum init,
                            TileSum *out, hipStream_t s);
enum : uint32_t { PREP_RESET = 1, PREP_SETPOS = 2, PREP_SAVE = 4, PREP_ZERO = 8 };
hipError_t launch_prep(StreamPos *pos, StreamPos *saved, unsigned int *err, uint64_t *scal, uint32_t flags,
                       uint64_t lines, hipStream_t s);
hipError_t launch_tile_aggregate(const uint8_t *data, uint64_t len, uint32_t n_tiles, uint64_t *agg_cnt,
                                 uint64_t *agg_lnl, unsigned int *err, hipStream_t s);
hipError_t launch_windows(const WindowArgs &a, uint32_t grid, hipStream_t s);
// rkey32 != NULL: keys are written as u32 (narrow mode), else to rkey
hipError_t launch_cross_scatter(const uint32_t *slot, const uint64_t *ord, const uint64_t *key, uint64_t n,
                                uint64_t *rkey, uint32_t *rkey32, uint64_t *rord, hipStream_t s);
hipError_t launch_cross_sort_small(const uint32_t *slot, const uint64_t *ord, const uint64_t *key, uint64_t n,
                                   uint64_t *rkey, uint32_t *rkey32, uint64_t *rord, hipStream_t s);
constexpr uint64_t XSMALL_MAX = 16384;   // cross lists up to this size: one-workgroup sort
hipError_t launch_cross_segsort(uint64_t *ord, uint64_t *key, const uint32_t *slot, uint64_t n, uint64_t *rkey,
                                uint32_t *rkey32, uint64_t *rord, uint32_t pbits, hipStream_t s);
hipError_t launch_heads(const uint64_t *skey, const uint32_t *srank, uint64_t n, uint64_t invalid_key,
                        const uint64_t *rcnt, HeadRec *hrec, uint32_t *hcnt, hipStream_t s);
// sort finish without per-entry counts: hcnt prefilled with 1, only groups of >= 2 and invalid keys written
hipError_t launch_heads_sparse(const uint64_t *skey64, const uint32_t *skey32, const uint32_t *srank, uint64_t n,
                               uint64_t invalid_key, uint32_t *hcnt, hipStream_t s);
hipError_t launch_heads32(const uint32_t *skey, const uint32_t *srank, uint64_t n, uint32_t invalid_key,
                          const uint64_t *rcnt, HeadRec *hrec, uint32_t *hcnt, hipStream_t s);
hipError_t launch_emit(const EmitArgs &a, hipStream_t s);
hipError_t launch_head_count(const uint32_t *hcnt, uint64_t n, uint32_t *ecnt, hipStream_t s);
uint64_t emit_blocks(uint64_t n);
constexpr uint64_t EMIT_DIRECT_MAX = 4096;   // emit workgroups that sum the earlier counts themselves (O(n^2) reads)
// wide keys (2(k - |P|) >= 64 bits, k <= 64): dst[i] = src[idx[i]]; the cross
// entries' keys after apply_cross; heads over (hi, lo) sorted ranks (hcnt
// prefilled with 1, as launch_heads_sparse)
hipError_t launch_gather_u64(const uint64_t *src, const uint32_t *idx, uint64_t n, uint64_t *dst, hipStream_t s);
hipError_t launch_gather_u32(const uint32_t *src, const uint32_t *idx, uint64_t n, uint32_t *dst, hipStream_t s);
constexpr uint64_t CP_BLOCK = 4096;   // ranks per compaction workgroup (compact_count / compact_write)
hipError_t launch_compact_count(const uint32_t *k32, const uint64_t *k64, uint64_t n, uint64_t invalid, uint32_t *bcnt,
                                hipStream_t s);
hipError_t launch_compact_write(const uint32_t *k32, const uint64_t *k64, const uint64_t *ord, uint64_t n,
                                uint64_t invalid, const uint64_t *boff, uint32_t *o32, uint64_t *o64, uint64_t *oord,
                                hipStream_t s);
hipError_t launch_cross_wide_fix(const uint32_t *xslot, uint64_t n, const uint64_t *xkeyl, const uint64_t *xkeyh,
                                 uint64_t *rkey, uint64_t *rkeyh, hipStream_t s);
hipError_t launch_heads_wide(const uint64_t *shi, const uint64_t *slo, const uint32_t *srank, uint64_t n,
                             uint64_t invalid_hi, uint32_t *hcnt, hipStream_t s);
// bucket finish (u32 keys of <= BKT_LOW + 11 bits)
constexpr uint32_t BKT_LOW = 14;             // keys per bucket table: 2^14 (128 KiB of LDS: min rank, count)
constexpr uint32_t BKT_MAX = 2048;           // buckets (keys of <= BKT_LOW + 11 bits)
constexpr uint32_t BKT_EPB_HOST = 4096;      // elements per partition block (= BKT_EPB)
hipError_t launch_bucket_hist(const uint32_t *key, uint64_t n, uint32_t invalid, uint32_t shift, uint32_t nb,
                              uint32_t nblk, uint32_t *H, uint32_t *hcnt, hipStream_t s);
hipError_t launch_bucket_offsets(const uint32_t *H, uint32_t nb, uint32_t nblk, uint32_t *Hs, uint32_t *btot,
                                 uint32_t *bbase, unsigned int *ticket, hipStream_t s);
hipError_t launch_bucket_scatter(const uint32_t *key, uint64_t n, uint32_t invalid, uint32_t shift, uint32_t nb,
                                 uint32_t nblk, const uint32_t *Hs, const uint32_t *bbase, uint16_t *pkey,
                                 uint32_t *prank, hipStream_t s);
hipError_t launch_bucket_heads(const uint16_t *pkey, const uint32_t *prank, const uint32_t *bbase, uint32_t nb,
                               uint32_t shift, uint32_t *hcnt, hipStream_t s);
// multi-GPU hit exchange (kmer_exchange_prepare / kmer_finish_exchanged)
struct XHit {
    uint64_t ord;                  // first-occurrence order key
    uint64_t key;                  // packed suffix code
};
constexpr uint32_t XP_MAXW = 256;            // most ranks of one exchange
constexpr uint32_t XP_EPB_HOST = 4096;       // rank slots per partition block (= XP_EPB)
hipError_t launch_xpart_hist(const uint64_t *rkey, const uint32_t *rkey32, uint64_t n, uint64_t invalid,
                             uint32_t kbits, uint32_t world, uint32_t nblk, uint32_t *H, hipStream_t s);
hipError_t launch_xpart_scatter(const uint64_t *rkey, const uint32_t *rkey32, const uint64_t *rord, uint64_t n,
                                uint64_t invalid, uint32_t kbits, uint32_t world, uint32_t nblk, const uint32_t *H,
                                const uint32_t *Hs, XHit *out, uint64_t *counts, hipStream_t s);
hipError_t launch_xprep(const XHit *x, uint64_t n, uint64_t *rkey, uint32_t *rkey32, uint64_t *rord, uint32_t *ridx,
                        hipStream_t s);
hipError_t launch_merge_prep(const uint64_t *keys, const Agg *vals, uint64_t n, uint64_t *rkey, uint32_t *rkey32,
                             uint64_t *rord, uint64_t *rcnt, uint32_t *ridx, hipStream_t s);
hipError_t launch_gather_records(const Record *recs, uint64_t stride, uint64_t n,
                                 const uint8_t *data, uint8_t *out, hipStream_t s);
hipError_t launch_nl_count(const uint8_t *data, uint64_t len, uint32_t n_tiles, uint32_t *tcount, unsigned int *err,
                           hipStream_t s);
hipError_t launch_nl_write(const uint8_t *data, uint64_t len, uint32_t n_tiles, const uint64_t *tbase, uint64_t *nl,
                           hipStream_t s);
// one pass: per-tile '\n' counts + tile-relative positions in `cap` u16 slots per
// tile (ERR_LINE_OVERFLOW: a tile had more; fall back to nl_write)
hipError_t launch_nl_slots(const uint8_t *data, uint64_t len, uint32_t n_tiles, uint32_t cap, uint16_t *slots,
                          uint32_t *tcount, unsigned int *err, hipStream_t s);
// sequence lines from the slots (tbase: exclusive scan of tcount)
hipError_t launch_seq_lines_slots(const uint16_t *slots, const uint32_t *tcount, const uint64_t *tbase,
                                  uint32_t n_tiles, uint32_t cap, uint64_t len, uint64_t li0, uint64_t first,
                                  uint64_t n_nl, uint64_t n_seq, uint32_t k, uint32_t step, SeqLine *lines,
                                  uint64_t *wcount, unsigned int *err, uint64_t maxrel, hipStream_t s);
// wcount = windows of both strands per sequence line: 2 ceil(W / step)
hipError_t launch_seq_lines(const uint64_t *nl, uint64_t n_nl, uint64_t len, uint64_t li0, uint64_t n_seq, uint32_t k,
                            uint32_t step, SeqLine *lines, uint64_t *wcount, unsigned int *err, uint64_t maxrel,
                            hipStream_t s);
hipError_t launch_pos_after(StreamPos *pos, uint64_t lines, const uint8_t *data, uint64_t len,
                            unsigned long long *ends_open, hipStream_t s);
hipError_t launch_windows_packed(const WinArgs &a, hipStream_t s);

// ---- table mode (kmer_table.hip): unordered canonical counts ---------------
// Every counted forward window w contributes its canonical planar code
// c = min(code(w), code(rc w)) (planar code: low plane bits of the k bases,
// then the high plane bits, base 0 least significant; A=00 C=01 G=10 T=11 as
// (hi, lo)); h = tab_mix(c) is a bijection.  h's top 10 bits pick the pass-1
// partition, the next 10 the bucket (2^20 buckets), the low 44 bits are the
// remainder kept in the table.  count(x) = C[c] for x in {c, rc c} when x
// starts with P (palindromes: 2 C[c]) -- SURVEY.md App. A.6.
constexpr uint32_t TAB_L1 = 10, TAB_L2 = 10;           // bits per partition level
constexpr uint32_t TAB_NB = 1u << 10;                  // bins per level
constexpr uint32_t TAB_NQ = 1u << (TAB_L1 + TAB_L2);   // buckets
constexpr uint32_t TAB_RBITS = 64 - TAB_L1 - TAB_L2;   // remainder bits (44)
constexpr uint64_t TAB_CMAX = 0xFFFFFull;              // entry count field (20 bits); larger -> big list
constexpr uint64_t TAB_UNIT = 1ull << 18;              // pass-2 keys per workgroup
constexpr uint32_t TAB_FWG = 1024;                     // final workgroup (16 waves, one per CU)
constexpr uint32_t TAB_SLOTS = 8192;                   // final LDS table slots (96 KiB)
constexpr uint32_t TAB_CAP = 7000;                     // distinct keys per range before it is split (+1024 in flight)

// multiplicative hash: a bijection of the 64-bit code (odd multiplier) whose
// top bits -- partition and bucket -- depend on every bit of the code
constexpr uint64_t TAB_MUL = 0x9E3779B97F4A7C15ull;
__host__ __device__ inline uint64_t tab_mix(uint64_t x) { return x * TAB_MUL; }
constexpr uint64_t tab_inv_odd(uint64_t a) {   // inverse of an odd number mod 2^64 (Newton: 3 -> 96 bits)
    uint64_t x = a;
    for (int i = 0; i < 5; ++i) x *= 2 - a * x;
    return x;
}
constexpr uint64_t TAB_INV = tab_inv_odd(TAB_MUL);
static_assert(TAB_INV * TAB_MUL == 1, "TAB_INV");
// NARROW keys (k <= 21).  The key code c' has 41 bits: odd k -- the
// orientation (w or rc w) whose middle base is A or C, with that base's zero
// high-plane bit taken out (exactly one orientation qualifies: complementing a
// base flips both its bits, and the middle base is its own mirror); even k --
// min(code(w), code(rc w)) (< 2^40).  h = f(c') << 23 with f(x) = (x ^ (x >>
// 21)) TAB_MUL mod 2^41, a bijection of [0, 2^41) (the xor-shift lets the
// bucket bits see every bit).  The remainder's low 23 bits are then 0, and a
// key below its partition fits 31 bits: (uint32_t)(h >> 23) = bucket offset
// << 21 | the remainder's top 21 bits -- the 32-bit keys of pass 1's runs
// (B1) and of pass 2's regions (B2), with TAB_SENT32 free for filler slots.
constexpr uint32_t TAB_NSH = 23;
constexpr uint32_t TAB_NARROW_K = 21;
constexpr uint32_t TAB_SENT32 = 0xFFFFFFFFu;
__host__ __device__ inline uint64_t tab_mix_n(uint64_t x) { return ((x ^ (x >> 21)) * TAB_MUL) << TAB_NSH; }
// pass 1: the narrow key code of a window from its two orientations' codes
__host__ __device__ inline uint64_t tab_canon_n(uint64_t cf, uint64_t cr, uint32_t k) {
    if (!(k & 1)) return cf < cr ? cf : cr;
    const uint32_t pos = k + (k - 1) / 2;             // the middle base's high-plane bit
    const uint64_t c = ((cf >> pos) & 1) ? cr : cf;
    return ((c >> (pos + 1)) << pos) | (c & ((1ull << pos) - 1));
}
// the planar code of h: the canonical code (wide keys) or an orientation of
// the window (narrow keys); inv = TAB_MUL^-1 mod 2^64
__host__ __device__ inline uint64_t tab_code(uint64_t h, uint32_t k, bool narrow, uint64_t inv) {
    if (!narrow) return h * inv;
    const uint64_t z = ((h >> TAB_NSH) * inv) & ((1ull << 41) - 1);
    const uint64_t x = z ^ (z >> 21);
    if (!(k & 1)) return x;
    const uint32_t pos = k + (k - 1) / 2;
    return ((x >> pos) << (pos + 1)) | (x & ((1ull << pos) - 1));
}
// reverse complement of a planar code (k <= 32)
__host__ __device__ inline uint64_t tab_rc_code(uint64_t code, uint32_t k) {
    const uint32_t km = k >= 32 ? ~0u : ((1u << k) - 1u);
    const uint32_t lo = (uint32_t)code & km, hi = (uint32_t)(code >> k) & km;
    const uint32_t rlo = __builtin_bitreverse32(~lo & km) >> (32 - k);
    const uint32_t rhi = __builtin_bitreverse32(~hi & km) >> (32 - k);
    return ((uint64_t)rhi << k) | rlo;
}
// the hash the table digest weighs: tab_mix(min(code(w), code(rc w))) for every k
__host__ __device__ inline uint64_t tab_digest_key(uint64_t h, uint32_t k, bool narrow) {
    if (!narrow) return h;
    const uint64_t c = tab_code(h, k, true, TAB_INV), r = tab_rc_code(c, k);
    return tab_mix(c < r ? c : r);
}
// Table digest weight of a key h: the splitmix64 finalizer (kmer_table_digest)
__host__ __device__ inline uint64_t tab_digest_mix(uint64_t h) {
    h ^= h >> 30;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 27;
    h *= 0x94D049BB133111EBull;
    return h ^ (h >> 31);
}

struct TabArgs {
    const uint8_t *data;
    uint64_t len;
    const SeqLine *lines;          // by sequence ordinal (len 0: no windows)
    uint64_t n_lines;
    uint64_t lpw;                  // sequence lines per pass-1 workgroup
    uint32_t nwg;                  // pass-1 workgroups
    uint32_t k;
    uint32_t plo, phi, pmask;      // prefix planes (base i at bit i), mask of |P| bits
    uint32_t canonical;            // non-ACGT windows: forward-strand records, unfiltered (KMER_FLAG_CANONICAL)
    uint32_t narrow;               // k <= 21: h = tab_mix_n(tab_canon_n(..)), and B1 holds 32-bit keys (h >> 23)
    uint32_t *H1;                  // hist: [p * nwg + g]
    const uint64_t *H1s;           // scatter: exclusive scan of H1 (chunk-relative)
    uint64_t base;                 // scatter: session keys before this chunk
    uint64_t *B1;                  // scatter: hashed keys, partition-major
    Record *recs;                  // non-ACGT windows
    unsigned long long *rec_count;
    uint64_t rec_cap;
    unsigned int *err;
    // pass 1 without the counting pass (tab_scatter1f): partition p owns
    // [base + p * PS, base + (p + 1) * PS), PS = R + S: workgroup w's run at
    // p * PS + pcw[w] (pcw[w + 1] - pcw[w] keys), then S spill slots for the
    // keys past their run (cursor pcur[p]; a full spill area counts in
    // pcur[TAB_NB] and the chunk is redone by the counted pass)
    const uint64_t *pcw;
    uint64_t R, S, PS;
    unsigned long long *pcur;
};

// Pass-1 filler of a run's unused tail (tab_scatter1f), skipped by pass 2:
// tab_mix(2^64 - 1), whose code is no k-mer of k <= 31 (codes < 2^62).
constexpr uint64_t TAB_SENT = 0ull - TAB_MUL;

struct TabUnit {                   // pass 2: a run of one pass-1 partition's keys
    uint64_t start;                // first key in B1
    uint64_t hbase;                // H2 index of (bin 0, unit 0) of the partition
    uint32_t len, u, nunits, part; // keys, unit index within the partition, units of the partition, the partition
};

struct TabBig {                    // entries whose count does not fit the 20-bit field
    uint64_t h, count;
};

struct TabFinal {
    const uint64_t *B2;            // keys by bucket
    const uint64_t *start;         // TAB_NQ + 1 bucket starts in B2 (and in out)
    uint64_t *out;                 // per bucket: nd[q] entries (rem << 20 | min(count, TAB_CMAX))
    uint32_t *nd;
    uint32_t sub_bits;             // (unused: ranges are sized per unit from range_keys)
    uint32_t range_keys;           // target keys per LDS range (small buckets are grouped up to it)
    uint32_t cap;                  // claims per range before it is split (<= TAB_CAP)
    uint32_t ablate;               // experiments only (results WRONG): 1 no insert, 2 no emit; sort kernel:
                                   // 8 no bin scan, 16 no statistics, 32 no entry stores
    TabBig *big;
    unsigned long long *big_count;
    uint64_t big_cap;
    unsigned int *err;
    uint32_t k, plo, phi, pmask;
    uint32_t canonical;            // statistics of the canonical-k-mer view (KMER_FLAG_CANONICAL)
    uint64_t inv;                  // inverse of TAB_MUL mod 2^64 (tab_code)
    uint32_t narrow;               // keys h = tab_mix_n(c) (k <= 21)
    uint32_t b2n;                  // (narrow, capq) B2 holds 32-bit keys: (uint32_t)(h >> 23) (bucket offset, remainder)
    unsigned long long *stats;     // [0] canonical entries [1] Map keys [2] sum of Map counts
    uint64_t *prof;                // experiments only (KMERHIP_TAB_PROF): per-workgroup phase clocks, 8 each
    uint32_t qlo, qhi;             // buckets [qlo, qhi) of this table (multi-GPU: the rank's partitions)
    // units the sort kernel (tab_sort_final) leaves to the general kernel: pairs
    // [q, qe) of buckets; the general kernel walks this list instead of
    // [qlo, qhi) when `left` is set
    uint32_t *left;
    unsigned int *left_n;
    // fixed-capacity pass 2 (tab_scatter2f): REGION r = tab_region(q) holds
    // the keys of qg consecutive buckets of one partition (1: one bucket) at
    // B2[r capq .. r capq + inlen[r]), in no order; rstart = the scan of inlen
    // (the compact OUTPUT layout: entries of region r from rstart[r]).  qg 1:
    // rstart is `start`; qg > 1: `start` holds rstart[tab_region(q)] (from
    // tab_region_starts) and the sort final writes each bucket's exact start
    // (wstart) from its counting sort.  capq 0: contiguous buckets, start for
    // both.
    uint64_t capq;
    const uint32_t *inlen;
    uint32_t qg, rpp, gmag;        // buckets per region, regions per partition, ceil(2^20 / qg)
    const uint64_t *rstart;
    uint64_t *wstart;
};

// fixed pass-2 region of bucket q (qg buckets per region, rpp regions per partition)
__host__ __device__ inline uint32_t tab_region(uint32_t q, uint32_t rpp, uint32_t gmag) {
    return (q >> TAB_L2) * rpp + (((q & (TAB_NB - 1)) * gmag) >> 20);
}

constexpr uint64_t TAB_PIECE = 4096;                   // windows per piece of a long line (pass 1)
hipError_t launch_tab_piece_count(const uint64_t *wcount, uint64_t n, uint32_t *pc, uint32_t *split, hipStream_t s);
hipError_t launch_tab_piece_write(const SeqLine *lines, const uint64_t *wcount, const uint64_t *pbase, uint64_t n,
                                  uint32_t k, SeqLine *out, hipStream_t s);
hipError_t launch_tab_hist1(const TabArgs &a, hipStream_t s);
hipError_t launch_tab_scatter1(const TabArgs &a, hipStream_t s);
hipError_t launch_tab_p1_offsets(const uint64_t *H1s, uint32_t nwg, uint64_t *out, hipStream_t s);
hipError_t launch_tab_hist2(const uint64_t *B1, const TabUnit *units, uint32_t n_units, uint32_t *H2, hipStream_t s);
hipError_t launch_tab_scatter2(const uint64_t *B1, const TabUnit *units, uint32_t n_units, const uint64_t *H2s,
                               uint64_t *B2, hipStream_t s);
hipError_t launch_tab_starts(const uint64_t *H2s, const uint32_t *H2, uint64_t nh, const TabUnit *pfirst,
                             uint64_t *start, hipStream_t s);
// pass 2 without its histogram: one workgroup per partition p in [p0, p0 +
// np), bucket q's keys at B2[q cap ..) (capacity cap, a multiple of 8);
// blen[q] = its keys; a bucket past its capacity sets ERR_TAB_CAP (the caller
// redoes pass 2 with the counted route)
hipError_t launch_tab_scatter2f(const uint64_t *B1, const TabUnit *units, const uint32_t *ufirst, uint32_t p0,
                                uint32_t np, uint64_t cap, uint32_t rpp, uint32_t gmag, bool narrow, bool b1n,
                                void *B2, uint32_t *blen, unsigned int *err, hipStream_t s);
// start[q] = rstart[tab_region(q)] for every bucket, start[TAB_NQ] = the total
hipError_t launch_tab_region_starts(const uint64_t *rstart, uint32_t rpp, uint32_t gmag, uint64_t *start,
                                    hipStream_t s);
hipError_t launch_tab_scatter1f(const TabArgs &a, hipStream_t s);
hipError_t launch_tab_wg_windows(const SeqLine *lines, uint64_t n, uint64_t lpw, uint32_t k, uint32_t nwg,
                                 uint64_t *W, hipStream_t s);
// pass-1 spill areas (tab_scatter1f): the unused slots of each partition's
// spill area filled with TAB_SENT
hipError_t launch_tab_spill_fill(bool narrow, uint64_t *B1, uint64_t base, uint64_t R, uint64_t S, uint64_t PS,
                                 const unsigned long long *pcur, hipStream_t s);
hipError_t launch_tab_final(const TabFinal &a, uint32_t grid, hipStream_t s);
hipError_t launch_tab_sort_final(const TabFinal &a, uint32_t grid, hipStream_t s);
constexpr uint32_t TAB_SWG = 512;
constexpr uint64_t TAB_SORT_KEYS = 12288;               // sort final: keys of a unit (one bucket, or narrow keys: TS_CAP1)
constexpr uint64_t TAB_SORT_KEYS_BIG = 12160;           // ... with 16,384 bins (fixed regions: tab_sort_final_kernel<14>)
constexpr uint64_t TAB_SORT_GROUP_KEYS = 6144;          // sort final: keys of a unit of several buckets (TS_CAPG)                      // sort-final workgroup (8 waves, two per CU)
hipError_t launch_tab_digest(const uint64_t *ent, const uint64_t *start, const uint32_t *nd, uint32_t k,
                            uint32_t narrow, unsigned long long *out,
                             hipStream_t s);
// multi-GPU table exchange: copy n segments {src offset, dst offset, length}
// of u64 keys (one workgroup per segment, grid-strided)
struct TabSeg {
    uint64_t src, dst, len;
    uint64_t part;                 // (tab_widen) the segment's pass-1 partition
};
hipError_t launch_tab_segcopy(const uint64_t *src, const TabSeg *segs, uint32_t n, uint64_t *dst, hipStream_t s);
// 32-bit pass-1 keys (narrow) -> 64-bit h (segment src/dst in keys; filler -> TAB_SENT)
hipError_t launch_tab_widen(const uint32_t *src, const TabSeg *segs, uint32_t n, uint64_t *dst, hipStream_t s);
// FASTA input (kmer_fasta.hip, KMER_FLAG_FASTA): a chunk of FASTA rewritten
// as FASTQ-shaped lines (header, joined sequence, "", "" per record).  A tile
// of 16 KiB is a function of the header state it inherits: kind 0 passes the
// state through, 1 / 2 leave it 0 / 1; c0 / c1 = output bytes for an incoming
// state 0 / 1; nl = input '\n' bytes.  Composed by an exclusive scan.
struct FaTile {
    uint32_t kind, pad;
    uint64_t c0, c1, nl;
};
__host__ __device__ inline FaTile fa_tile_compose(const FaTile &a, const FaTile &b) {
    FaTile r;
    const uint32_t s0 = a.kind ? a.kind - 1 : 0u, s1 = a.kind ? a.kind - 1 : 1u;
    r.kind = b.kind ? b.kind : a.kind;
    r.pad = 0;
    r.c0 = a.c0 + (s0 ? b.c1 : b.c0);
    r.c1 = a.c1 + (s1 ? b.c1 : b.c0);
    r.nl = a.nl + b.nl;
    return r;
}
hipError_t launch_fa_tiles(const uint8_t *data, uint64_t len, uint32_t n_tiles, FaTile *tiles, hipStream_t s);
hipError_t launch_fa_write(const uint8_t *data, uint64_t len, uint32_t n_tiles, const FaTile *tiles_x, uint8_t *out,
                           hipStream_t s);
hipError_t launch_synth_fastq(uint8_t *out, uint64_t seed, uint64_t first_read, uint64_t n_reads,
                              hipStream_t s);
hipError_t launch_gen_append(const Record *recs, uint64_t n, const uint8_t *data, uint32_t k, uint8_t *keys,
                             uint64_t *cnt, uint64_t *first, hipStream_t s);
hipError_t launch_gen_hash(const uint8_t *keys, uint64_t n, uint32_t k, uint64_t seed, uint64_t *h1, uint64_t *h2,
                           uint32_t *idx, hipStream_t s);
hipError_t launch_gen_heads(const uint64_t *h1, const uint64_t *h2, const uint32_t *idx, uint64_t n, const uint8_t *keys,
                            uint32_t k, uint32_t *head, unsigned int *collide, hipStream_t s);
hipError_t launch_gen_starts(const uint32_t *head, const uint32_t *gid, uint64_t n, uint32_t *start, hipStream_t s);
hipError_t launch_gen_reduce(const uint32_t *start, uint64_t ng, const uint32_t *idx, const uint8_t *keys,
                             const uint64_t *cnt, const uint64_t *first, uint32_t k, uint8_t *okeys, uint64_t *ocnt,
                             uint64_t *ofirst, hipStream_t s);
hipError_t launch_permute_rows(const uint8_t *keys, const uint64_t *cnt, const uint64_t *first, const uint32_t *idx,
                               uint64_t n, uint32_t k, uint8_t *okeys, uint64_t *ocnt, uint64_t *ofirst,
                               hipStream_t s);

}  // namespace kmerhip
