// kmer_kernels.hip — gfx950 (CDNA4) kernels for the kmerjs FASTQ k-mer loop.
//
// Reference semantics (lib/kmers.js, see oracle/kmer_oracle.c for the exact
// restatement): lines split on '\n' (:114-136); a line is a sequence line iff
// its 0-based index n has n % 4 == 1 and length > 1 (:151,:160); each sequence
// line s is scanned, then complement(s) (:152-155, :31-38); every k-window
// key = substring(ini, ini+k) that startsWith(preffix) is counted (:88-100);
// Map order = first occurrence (:95).
//
// Device pipeline:
//   scan_planes_kernel / scan_tile_kernel  one 16 KiB tile per workgroup,
//                 single pass over HBM: stage tile + halos in LDS, '\n'
//                 counts and block scan, prefix test of every window on both
//                 strands (bit-planes of 2-bit codes, or byte SWAR), exact
//                 verification, one hit record per verified window.
//   hit_kernel    global line index (after a scan of the tile sums), the
//                 sequence-line rule, order key, rank slot of each hit.
//   finish        cross-list placement, heads / emit after the key sort.
//   dense-hit path: newline array, sequence lines, windows_packed_kernel.
//   general path: lines_kernel (decoupled look-back) + windows_kernel ->
//                 records for the host merge.
//
// Canonical identity used by the tile kernel: the
// reverse-complement strand's window at j is rc of the forward window at
// p = L-k-j, so both strands are served by ONE forward scan: a forward window
// w at p yields key w if w starts with P, and key rc(w) if w ends with rc(P).
#include "kmer_internal.hpp"

#include <algorithm>
#include <cstring>

namespace kmerhip {

// ---------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t align4(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_alignbyte(hi, lo, sel);
}

// Set a rarely-changing info bit: read first, so that thousands of tiles do
// not serialise on one device-scope atomic (long contigs flag every tile).
__device__ __forceinline__ void set_info(unsigned int *err, unsigned int bit) {
    if (!(__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit)) atomicOr(err, bit);
}

// Inclusive wave64 prefix sum with DPP (row_shr 1/2/4/8 inside rows of 16,
// then row_bcast 15 / 31 across rows): no LDS round trips on the critical path.
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}

// '\n' bytes among four ASCII bytes (< 0x80): bit 7 of (x ^ "\n\n\n\n") +
// 0x7F per byte is set iff the byte is NOT '\n' (no carries: every byte < 0x80),
// so the count is 4 - popcount.  One v_xad_u32 + and + bcnt per word.
__device__ __forceinline__ uint32_t not_nl_bits(uint32_t x) {
    return ((x ^ 0x0A0A0A0Au) + 0x7F7F7F7Fu) & 0x80808080u;
}

// The same with the xor and the add in one v_xad_u32 (the compiler emits a
// v_xor / v_add pair for the expression above): 3 VALU per word with the and
// and the accumulating bcnt, not 4.  k0a / k7f hold 0x0A0A0A0A / 0x7F7F7F7F.
__device__ __forceinline__ uint32_t not_nl_bits_xad(uint32_t x, uint32_t k0a, uint32_t k7f) {
    uint32_t r;
    asm("v_xad_u32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(k0a), "s"(k7f));
    return r & 0x80808080u;
}

// per-byte 0x80 flag for bytes equal to '\n'; exact for ASCII bytes (< 0x80)
__device__ __forceinline__ uint32_t nl_flags(uint32_t x) {
    uint32_t t = x ^ 0x0A0A0A0Au;
    return ~(t + 0x7F7F7F7Fu) & 0x80808080u;
}


__device__ __forceinline__ uint8_t comp_byte(uint8_t c) {
    return c == 'A' ? 'T' : c == 'T' ? 'A' : c == 'G' ? 'C' : c == 'C' ? 'G' : c;
}

__device__ __forceinline__ uint64_t lb_load(unsigned long long *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(unsigned long long *p, uint64_t v) {
    __hip_atomic_store(p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr uint32_t SPIN_LIMIT = 1u << 22;

// Decoupled look-back over one of the two per-tile words (wave 0 only).
// SUM: exclusive prefix sum of aggregates (line index of the tile start).
// !SUM: nearest non-zero value (line start before the tile: positions grow
// with the tile index, so the nearest predecessor that saw a '\n' holds the max).
template <bool SUM>
__device__ uint64_t look_back(unsigned long long *words, uint32_t tile, unsigned int *err) {
    const int lane = threadIdx.x & 63;
    uint64_t acc = 0;
    int64_t top = (int64_t)tile - 1;
    uint32_t spins = 0;
    while (true) {
        int64_t idx = top - lane;
        uint64_t v = 0;
        bool valid = idx >= 0;
        // spin until every predecessor in the window has published something
        while (true) {
            v = valid ? lb_load(words + idx) : LB_INC;
            bool ready = (v >> 62) != 0;
            if (__all(ready)) break;
            if (++spins > SPIN_LIMIT) {
                if (lane == 0) atomicOr(err, ERR_LOOKBACK_TIMEOUT);
                return acc;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        const uint64_t val = valid ? (v & LB_VAL) : 0;
        const bool inc = (v >> 62) == 2;
        if (SUM) {
            unsigned long long incmask = __ballot(inc);
            int stop = incmask ? __ffsll((long long)incmask) - 1 : 64;
            uint64_t contrib = lane <= stop ? val : 0;
            // wave reduce
            for (int d = 32; d >= 1; d >>= 1) contrib += __shfl_xor(contrib, d);
            acc += contrib;
            if (incmask) return acc;
        } else {
            unsigned long long hit = __ballot(inc || val != 0);
            if (hit) {
                int stop = __ffsll((long long)hit) - 1;
                return __shfl(val, stop);
            }
        }
        top -= 64;
    }
}

// ---------------------------------------------------------------------------
// tile kernel
// ---------------------------------------------------------------------------
constexpr int NCH_MAIN = TILE / 16;          // 1024 16-byte chunks
constexpr int NCH_FRONT = FH / 16;           // 4
constexpr int NCH_BACK = BH / 16;            // 5
constexpr int BUFSZ = FH + TILE + BH;

// bytes outside [0, len) read as '\n' (a line boundary that is never a window byte)
__device__ __noinline__ uint4 load_chunk_edge(const uint8_t *data, int64_t g, uint64_t len) {
    uint32_t w[4];
#pragma unroll 1
    for (int i = 0; i < 4; ++i) {
        uint32_t x = 0;
        for (int b = 0; b < 4; ++b) {
            const int64_t p = g + i * 4 + b;
            const uint32_t c = (p >= 0 && (uint64_t)p < len) ? data[p] : (uint32_t)'\n';
            x |= c << (8 * b);
        }
        w[i] = x;
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ uint4 load_chunk(const uint8_t *data, int64_t g, uint64_t len) {
    if (g >= 0 && (uint64_t)g + 16 <= len) return *(const uint4 *)(data + g);
    return load_chunk_edge(data, g, len);
}


struct TileShared {
    uint32_t tpre[TPB + 1];      // exclusive '\n' count per thread inside the tile; [TPB] = total
    uint32_t wsum[TPB / 64];
    int32_t last_thr;            // highest thread owning a '\n'
    uint32_t tile;
    uint64_t line_base;          // global line index of the tile's first byte
    uint64_t lnl_before;         // absolute start of the line containing the tile's first byte
    uint64_t lnl_tile;           // absolute line start after the tile's last '\n' (0 = none)
    int32_t lastpos;             // tile-relative position of the tile's last real '\n' (-1 = none)
    uint32_t nh;                 // hit records written by this tile
    uint32_t qn;                 // hit queue fill
    uint32_t more;               // a lane could not queue all its hits this round
    uint32_t q[1024];            // verified hits: (tile position << 1) | strand
};

// newline count in [64*thr, q) for tile-relative q within thread thr's range
__device__ __forceinline__ uint32_t nl_before_in_thread(const uint8_t *buf, int thr, int q) {
    const uint32_t *lw = (const uint32_t *)(buf + FH + 64 * thr);
    int n = q - 64 * thr;        // bytes to count, 0..64
    uint32_t c = 0;
#pragma unroll 1
    for (int i = 0; i < 16 && n > 0; ++i, n -= 4) {
        uint32_t z = nl_flags(lw[i]);
        if (n < 4) z &= (1u << (8 * n)) - 1u;
        c += __popc(z);
    }
    return c;
}

// unaligned 32-bit read of tile bytes at tile-relative position p (p >= -FH)
__device__ __forceinline__ uint32_t lds_word(const uint8_t *buf, int p) {
    const int a = FH + p;
    const uint32_t *w = (const uint32_t *)(buf + (a & ~3));
    return align4(w[1], w[0], (uint32_t)(a & 3));
}


// reverse complement of a 2-bit code of k bases (A=0 C=1 G=2 T=3)
__device__ __forceinline__ uint64_t revcomp_code(uint64_t x, uint32_t k) {
    x = ~x;
    x = ((x >> 2) & 0x3333333333333333ull) | ((x & 0x3333333333333333ull) << 2);
    x = ((x >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((x & 0x0F0F0F0F0F0F0F0Full) << 4);
    x = __builtin_bswap64(x);
    return k >= 32 ? x : (x >> (64 - 2 * k));
}

// the same for a 128-bit code of 32 < k <= 64 bases (hi: the first k - 32)
__device__ __forceinline__ void revcomp_code128(uint64_t hi, uint64_t lo, uint32_t k, uint64_t *rhi, uint64_t *rlo) {
    const uint64_t h = revcomp_code(lo, 32), l = revcomp_code(hi, 32);   // the 128 bits reversed
    const uint32_t s = 128 - 2 * k;                                     // garbage bits at the bottom (< 64)
    *rlo = s ? (l >> s) | (h << (64 - s)) : l;
    *rhi = s ? h >> s : h;
}

// Shared tile prologue: stage tile + halos in LDS, per-thread words, '\n'
// count, block exclusive scan (sh.tpre), tile's last '\n' (sh.lastpos).
// Returns the tile's '\n' count (bytes < len only).
__device__ __forceinline__ uint32_t tile_prologue(const uint8_t *data, uint64_t len, int64_t g0, uint8_t *buf,
                                                  TileShared &sh, uint32_t (&w)[17], unsigned int *err) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // ---- stage tile + halos into LDS (16 B per lane, coalesced) ----
    uint4 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = load_chunk(data, g0 + (int64_t)(tid + TPB * i) * 16, len);
    uint4 vh = make_uint4(0, 0, 0, 0);
    const bool halo = tid < NCH_FRONT + NCH_BACK;
    const int hc = tid < NCH_FRONT ? tid : NCH_FRONT + NCH_MAIN + (tid - NCH_FRONT);
    if (halo) vh = load_chunk(data, g0 - FH + (int64_t)hc * 16, len);
    uint32_t orall = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        orall |= v[i].x | v[i].y | v[i].z | v[i].w;
        *(uint4 *)(buf + FH + (tid + TPB * i) * 16) = v[i];
    }
    if (halo) *(uint4 *)(buf + hc * 16) = vh;
    if (orall & 0x80808080u) atomicOr(err, ERR_NONASCII);
    __syncthreads();

    // ---- per-thread view: bytes [64*tid, 64*tid + 68) ----
    {
        const uint4 *lp = (const uint4 *)(buf + FH + 64 * tid);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint4 x = lp[i];
            w[4 * i] = x.x; w[4 * i + 1] = x.y; w[4 * i + 2] = x.z; w[4 * i + 3] = x.w;
        }
        w[16] = *(const uint32_t *)(buf + FH + 64 * tid + 64);
    }
    // ---- '\n' count of the bytes this thread owns (only real bytes < len) ----
    uint32_t cnt = 0;
    const int64_t gt = g0 + 64 * tid;
    if (gt + 64 <= (int64_t)len) {
#pragma unroll
        for (int i = 0; i < 16; ++i) cnt += __popc(nl_flags(w[i]));
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int64_t n = (int64_t)len - (gt + 4 * i);
            uint32_t z = nl_flags(w[i]);
            if (n <= 0) z = 0; else if (n < 4) z &= (1u << (8 * n)) - 1u;
            cnt += __popc(z);
        }
    }
    // ---- block exclusive scan of cnt ----
    uint32_t incl = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d);
        if (lane >= d) incl += y;
    }
    if (lane == 63) sh.wsum[wid] = incl;
    if (cnt) atomicMax(&sh.last_thr, tid);
    __syncthreads();
    uint32_t woff = 0, total = 0;
#pragma unroll
    for (int i = 0; i < TPB / 64; ++i) {
        woff += i < wid ? sh.wsum[i] : 0;
        total += sh.wsum[i];
    }
    sh.tpre[tid] = woff + incl - cnt;
    if (tid == 0) sh.tpre[TPB] = total;
    if (tid == sh.last_thr) {
        // last real '\n' of this thread's bytes (word-wise, from the end)
        int lastpos = -1;
#pragma unroll 1
        for (int i = 15; i >= 0 && lastpos < 0; --i) {
            const int64_t n = (int64_t)len - (gt + 4 * i);
            uint32_t z = nl_flags(*(const uint32_t *)(buf + FH + 64 * tid + 4 * i));
            if (n <= 0) z = 0; else if (n < 4) z &= (1u << (8 * n)) - 1u;
            if (z) lastpos = 64 * tid + 4 * i + ((31 - __clz(z)) >> 3);
        }
        sh.lastpos = lastpos;
    }
    if (sh.last_thr < 0 && tid == 0) sh.lastpos = -1;
    __syncthreads();
    return total;
}

// ---------------------------------------------------------------------------
// General path, step 1: sequence-line descriptors (decoupled look-back over
// tiles for the line index / line start of each tile).
// ---------------------------------------------------------------------------
template <bool LOOKBACK>
__global__ __launch_bounds__(TPB) void lines_kernel(TileArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[BUFSZ];
    __shared__ TileShared sh;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    if (tid == 0) {
        sh.tile = LOOKBACK ? atomicAdd(a.ticket, 1u) : blockIdx.x;
        sh.last_thr = -1;
    }
    __syncthreads();
    const uint32_t tile = sh.tile;
    const int64_t g0 = (int64_t)tile * TILE;
    const uint64_t len = a.len;
    uint32_t w[17];
    const uint32_t total = tile_prologue(a.data, len, g0, buf, sh, w, a.err);
    const uint64_t lnl_tile = sh.lastpos >= 0 ? a.abs_offset + (uint64_t)(g0 + sh.lastpos + 1) : 0;

    if (wid == 0) {
        uint64_t lbase, lnlb;
        if (LOOKBACK) {
            if (tile == 0) {
                lbase = a.pos->lines;
                lnlb = a.abs_offset;
                if (lane == 0) {
                    lb_store(a.lb_cnt, LB_INC | (lbase + total));
                    lb_store(a.lb_lnl, LB_INC | (lnl_tile > lnlb ? lnl_tile : lnlb));
                }
            } else {
                if (lane == 0) {
                    lb_store(a.lb_cnt + tile, LB_AGG | total);
                    lb_store(a.lb_lnl + tile, LB_AGG | lnl_tile);
                }
                lbase = look_back<true>(a.lb_cnt, tile, a.err);
                lnlb = look_back<false>(a.lb_lnl, tile, a.err);
                if (lane == 0) {
                    lb_store(a.lb_cnt + tile, LB_INC | (lbase + total));
                    lb_store(a.lb_lnl + tile, LB_INC | (lnl_tile > lnlb ? lnl_tile : lnlb));
                }
            }
            if (tile == a.n_tiles - 1 && lane == 0) {
                // advance the running stream position for the next chunk
                a.pos->lines = lbase + total;
                a.pos->ends_open = (len > 0 && a.data[len - 1] != '\n') ? 1 : 0;
            }
        } else {
            lbase = a.tp_cnt[tile];
            lnlb = a.tp_lnl[tile];
        }
        if (lane == 0) {
            sh.line_base = lbase;
            sh.lnl_before = lnlb;
        }
    }
    __syncthreads();
    const uint64_t lbase = sh.line_base;
#pragma unroll 1
    for (int i = 0; i < 64; ++i) {
        const int q = 64 * tid + i;
        if ((uint64_t)(g0 + q) >= len) break;
        if (buf[FH + q - 1] != '\n') continue;
        const uint32_t c = sh.tpre[tid] + nl_before_in_thread(buf, tid, q);
        const uint64_t li = lbase + c;
        if ((li & 3) != 1) continue;
        // find the end of the line
        int64_t e = g0 + q;
        while ((uint64_t)e < len && (e - g0 < TILE + BH ? buf[FH + (e - g0)] : a.data[e]) != '\n') ++e;
        const uint64_t L = (uint64_t)e - (uint64_t)(g0 + q);
        if (L > 1 && L >= a.k) {
            const unsigned long long n = atomicAdd(a.line_count, 1ull);
            if (n < a.line_cap) {
                a.lines_out[n].start = (uint64_t)(g0 + q);
                a.lines_out[n].len = L;
                a.lines_out[n].line_index = li;
            } else {
                atomicOr(a.err, ERR_LINE_OVERFLOW);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Fast path, step 1: streaming tile scan (no inter-tile dependency).
// Per tile: '\n' aggregate for the line scan, SWAR prefix scan at every byte
// on both strands, exact verification, and one 24-byte hit record per
// verified window with its tile-local line context.  Line index / order are
// resolved by hit_kernel after a scan over the per-tile aggregates.
// ---------------------------------------------------------------------------
constexpr int QCAP = 256;

struct alignas(16) ScanShared {
    uint16_t cpre[NCH_MAIN];     // exclusive '\n' count per 16-byte chunk inside the tile
    uint32_t nlmap[NCH_MAIN / 32];   // bit c: chunk c holds a real '\n' 
    uint32_t wsum[TPB / 64][4];  // per-wave totals of the four packed chunk columns
    int32_t last_chunk;          // highest chunk holding a real '\n' (-1 = none)
    int32_t lastpos;             // tile-relative position of the tile's last real '\n'
    uint32_t nh;                 // hit records written by this tile
    uint32_t nx;                 // ... of which on lines that cross a tile edge
    uint32_t tcnt;               // real '\n' count of the tile
    uint32_t qn;                 // verified-hit queue fill
    alignas(8) uint32_t q[QCAP]; // candidate words (byte kernel) / QCAP/2 {entry, mask} pairs (plane kernel)
};

// last '\n' (tile-relative) inside 16-byte chunk c at a position < limit, -1 if none
__device__ __forceinline__ int last_newline_in_chunk(const uint8_t *buf, int c, int limit = 1 << 30) {
    const uint4 x = *(const uint4 *)(buf + FH + 16 * c);
    const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
    int last = -1;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int pos = 16 * c + 4 * j;
        const int rem = limit - pos;
        uint32_t z = nl_flags(xs[j]);
        z = rem <= 0 ? 0u : rem < 4 ? (z & ((1u << (8 * rem)) - 1u)) : z;
        last = z ? pos + ((31 - __clz(z)) >> 3) : last;
    }
    return last;
}

// One verified prefix hit (queue entry (q << 1) | strand): window analysis,
// tile-local line context, hit record.
// THREAD_MAP: sh.nlmap holds one bit per 64-byte thread region (plane
// kernel; chunks inside a region are resolved through cpre), else one bit per
// 16-byte chunk (byte kernel).
// bytes [from, to) of a 32-bit word (clamped to 0..4)
__device__ __forceinline__ uint32_t byte_range_mask(int from, int to) {
    from = from < 0 ? 0 : from > 4 ? 4 : from;
    to = to < 0 ? 0 : to > 4 ? 4 : to;
    const uint32_t a = to >= 4 ? ~0u : (1u << (8 * to)) - 1u, b = from >= 4 ? ~0u : (1u << (8 * from)) - 1u;
    return a & ~b;
}

// WIDE: k > 32 (the window's first k - 32 bases go to hits_hi / ovf_hi).
// !THREAD_MAP (the byte kernel, which also serves non-ACGT prefixes): only the
// suffix bytes decide `exotic` -- the key is P + the suffix's 2-bit code, so a
// prefix may hold any bytes
template <bool THREAD_MAP, bool WIDE>
__device__ __forceinline__ void emit_hit(const ScanArgs &a, const uint8_t *buf, ScanShared &sh, uint32_t tile,
                                      uint32_t e) {
    const uint32_t k = a.k, plen = a.plen;
    const uint32_t strand = e & 1u;
    const int q = (int)(e >> 1);
    const int s0 = strand ? q + (int)plen - (int)k : q;   // window start, tile-relative
    // window bytes: ACGT check (v_perm against "ACGT"), '\n' check, 2-bit codes
    uint32_t exo_bits = 0, nl_bits = 0;          // (OR-accumulated; tested once)
    uint64_t code = 0;
    const int sfx0 = strand ? 0 : (int)plen, sfx1 = strand ? (int)(k - plen) : (int)k;   // suffix bytes
#pragma unroll 4
    for (uint32_t b = 0; b < k; b += 4) {
        const uint32_t x = lds_word(buf, s0 + (int)b);
        const uint32_t nb = k - b >= 4 ? 4u : k - b;
        const uint32_t mk = nb == 4 ? 0xFFFFFFFFu : ((1u << (8 * nb)) - 1u);
        const uint32_t c = ((x >> 1) ^ (x >> 2)) & 0x03030303u;
        const uint32_t expect = __builtin_amdgcn_perm(0u, 0x54474341u, c);   // "ACGT"[c] per byte
        const uint32_t mx = THREAD_MAP ? mk : mk & byte_range_mask(sfx0 - (int)b, sfx1 - (int)b);
        exo_bits |= (expect ^ x) & mx;
        nl_bits |= nl_flags(x) & mk;
        // the four 2-bit codes, first byte most significant: c0 * 64 + c1 * 16 + c2 * 4 + c3
        const uint32_t pk = __builtin_amdgcn_udot4(c, 0x01041040u, 0u, false);
        code = (code << (2 * nb)) | (pk >> (2 * (4 - nb)));
    }
    const bool exotic = exo_bits != 0, hasnl = nl_bits != 0;
    // k > 32: code keeps the last 32 bases; the first k - 32 (the window's
    // bytes are ACGT-checked above)
    uint64_t chi = 0;
    if (WIDE) {
        for (uint32_t b = 0; b < k - 32; b += 4) {
            const uint32_t x = lds_word(buf, s0 + (int)b);
            const uint32_t nb = k - 32 - b >= 4 ? 4u : k - 32 - b;
            const uint32_t c = ((x >> 1) ^ (x >> 2)) & 0x03030303u;
            const uint32_t pk = __builtin_amdgcn_udot4(c, 0x01041040u, 0u, false);
            chi = (chi << (2 * nb)) | (pk >> (2 * (4 - nb)));
        }
    }
    // crosses a line end (or the end of input); k == 1: line.length > 1
    const bool valid = !hasnl && !(k == 1 && buf[FH + s0 - 1] == '\n' && buf[FH + s0 + 1] == '\n');
    // tile-local line context of the window start: '\n' count before s0 and
    // the start of its line if that lies inside this tile.  The reads that
    // only depend on s0 (chunk, cpre of its region, region bitmap word) go
    // out together; at most two more dependent rounds follow.
    uint32_t c_local = 0;
    int lstart = -1;
    if (valid && s0 > 0) {
        const int cs = (s0 - 1) >> 4;               // chunk holding byte s0-1
        const uint4 x4 = *(const uint4 *)(buf + FH + 16 * cs);
        uint32_t cp[4] = {0, 0, 0, 0};              // THREAD_MAP: cpre of cs's 64-byte region
        uint32_t mw = 0;
        const int rb = cs & ~3;
        if (THREAD_MAP) {
            const uint2 c2 = *(const uint2 *)(sh.cpre + rb);
            cp[0] = c2.x & 0xFFFFu;
            cp[1] = c2.x >> 16;
            cp[2] = c2.y & 0xFFFFu;
            cp[3] = c2.y >> 16;
            if (rb > 0) mw = sh.nlmap[((rb >> 2) - 1) >> 5];
        }
        const uint32_t xs[4] = {x4.x, x4.y, x4.z, x4.w};
        uint32_t cnt = 0;
        int last = -1;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int pos = 16 * cs + 4 * j;
            const int rem = s0 - pos;
            uint32_t z = nl_flags(xs[j]);
            z = rem <= 0 ? 0u : rem < 4 ? (z & ((1u << (8 * rem)) - 1u)) : z;
            cnt += __popc(z);
            last = z ? pos + ((31 - __clz(z)) >> 3) : last;
        }
        const uint32_t ccs = THREAD_MAP ? cp[cs - rb] : (uint32_t)sh.cpre[cs];
        c_local = ccs + cnt;
        if (last >= 0) {
            lstart = last + 1;
        } else if (c_local > 0) {
            // the line started in the last earlier chunk that holds a '\n'
            int c = -1;
            if (THREAD_MAP) {
                // inside cs's region first: chunk rb + j holds a '\n' iff cpre rises after it
                if (ccs > cp[0]) {
#pragma unroll
                    for (int j = 2; j >= 0; --j)
                        if (c < 0 && rb + j < cs && cp[j] < ccs) c = rb + j;
                } else {
                    const int rr = (rb >> 2) - 1;        // earlier regions: region bitmap
                    int wi = rr >> 5;
                    uint32_t m = mw & (0xFFFFFFFFu >> (31 - (rr & 31)));
                    while (m == 0) m = sh.nlmap[--wi];
                    const int rg = 4 * (32 * wi + 31 - __clz(m));
                    const uint2 d2 = *(const uint2 *)(sh.cpre + rg);
                    const uint32_t nxt = sh.cpre[rg + 4];      // (rg + 4 <= rb <= cs)
                    const uint32_t d[4] = {d2.x & 0xFFFFu, d2.x >> 16, d2.y & 0xFFFFu, d2.y >> 16};
                    c = d[3] < nxt ? rg + 3 : d[2] < d[3] ? rg + 2 : d[1] < d[2] ? rg + 1 : rg;
                }
            } else {
                const int cc = cs - 1;               // chunk bitmap
                int wi = cc >> 5;
                uint32_t m = sh.nlmap[wi] & (0xFFFFFFFFu >> (31 - (cc & 31)));
                while (m == 0) m = sh.nlmap[--wi];
                c = 32 * wi + 31 - __clz(m);
            }
            lstart = last_newline_in_chunk(buf, c) + 1;
        }
    }
    // slots and the cross count: one LDS atomic per wave, not per hit.  The
    // hit kernel ranks hits of lines inside the tile; lines that cross a tile
    // edge are placed at finish (same predicate there).
    const bool cross = valid && (lstart < 0 || c_local == sh.tcnt);
    const unsigned long long vm = __ballot(valid), xm = __ballot(cross), act = __ballot(1);
    const int lane = threadIdx.x & 63, leader = __ffsll((long long)act) - 1;
    uint32_t base = 0;
    if (lane == leader) {
        if (vm) base = atomicAdd(&sh.nh, (uint32_t)__popcll(vm));
        if (xm) atomicAdd(&sh.nx, (uint32_t)__popcll(xm));
    }
    base = (uint32_t)__shfl((int)base, leader);
    if (!valid) return;
    const uint32_t slot = base + (uint32_t)__popcll(vm & ((1ull << lane) - 1ull));   // < 2 * TILE: fits qm[31:17]
    HitRec r;
    r.code = code;
    r.tile = tile;
    r.qm = (uint32_t)q | (strand << 14) | ((exotic ? 1u : 0u) << 15) | ((lstart >= 0 ? 1u : 0u) << 16) | (slot << 17);
    r.c_local = c_local;
    r.lstart = lstart >= 0 ? (uint32_t)lstart : 0u;
    // (round 5: the ablations "record computed, not stored" and "every record
    // to the same 64 slots" are gone -- they leave the hit kernel reading
    // unwritten records, which faulted in the finish)
    if (slot < HMAX) {
        a.hits[(uint64_t)tile * HMAX + slot] = r;
        if (WIDE) a.hits_hi[(uint64_t)tile * HMAX + slot] = chi;
    } else {
        const unsigned long long o = atomicAdd(a.ovf_count, 1ull);
        if (o < a.ovf_cap) {
            a.ovf[o] = r;
            if (WIDE) a.ovf_hi[o] = chi;
        } else {
            atomicOr(a.err, ERR_OVF_OVERFLOW);
        }
    }
}

// One candidate word (4 window starts at tile position q0 with a 4-byte
// match on some strand): exact prefix test of its 8 (position, strand)
// windows, then one hit record per verified window.
template <bool WIDE>
__device__ __forceinline__ void scan_word(const ScanArgs &a, const uint8_t *buf, ScanShared &sh, uint32_t tile,
                                          const uint32_t *pw, uint32_t q0) {
    const uint32_t plen = a.plen, P4 = a.p4, R4 = a.r4, PM = a.pmask;
    const uint32_t lo = *(const uint32_t *)(buf + FH + q0);
    const uint32_t hi = *(const uint32_t *)(buf + FH + q0 + 4);
    uint32_t bits = 0;
#pragma unroll
    for (uint32_t jj = 0; jj < 4; ++jj) {
        const uint32_t win = align4(hi, lo, jj);
        bits |= (((win ^ P4) & PM) == 0 ? 1u : 0u) << (2 * jj);
        bits |= (((win ^ R4) & PM) == 0 ? 1u : 0u) << (2 * jj + 1);
    }
    while (bits) {
        const uint32_t bit = __ffs(bits) - 1;
        bits &= bits - 1;
        const uint32_t strand = bit & 1u;
        const int q = (int)q0 + (int)(bit >> 1);
        bool ok = true;
#pragma unroll 1
        for (uint32_t b = 4; b < plen && ok; b += 4) {
            const uint32_t n = plen - b;
            const uint32_t mk = n >= 4 ? 0xFFFFFFFFu : ((1u << (8 * n)) - 1u);
            ok = ((lds_word(buf, q + (int)b) ^ pw[(strand ? KMAX_TILE / 4 : 0) + b / 4]) & mk) == 0;
        }
        if (ok) emit_hit<false, WIDE>(a, buf, sh, tile, ((uint32_t)q << 1) | strand);
    }
}

// Fast path, step 1 — streaming tile scan, coalesced layout.  Lane t of the
// workgroup owns the 16-byte chunks c = t + 256*i (i < 4) of the tile, exactly
// as it loaded them (one 1 KiB coalesced load per wave-instruction); the three
// look-ahead bytes of a chunk come from the next lane (shfl) or, at wave
// edges, from the LDS copy.  Per chunk: '\n' count (SWAR), and the 4-byte
// window at each of its 16 positions compared to P[0:4] and rc(P)[0:4] with
// v_cmp (the compiler ORs the lane masks on the scalar unit).  A packed
// 4 x 16-bit block scan gives the exclusive '\n' count of every chunk.
template <bool FULL4, bool WIDE>
__global__ __launch_bounds__(TPB) void scan_tile_kernel(ScanArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[BUFSZ];
    __shared__ ScanShared sh;
    __shared__ __attribute__((aligned(16))) uint8_t s_pr[2 * KMAX_TILE];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint64_t len = a.len;
    const bool halo = tid < NCH_FRONT + NCH_BACK;
    const int hc = tid < NCH_FRONT ? tid : NCH_FRONT + NCH_MAIN + (tid - NCH_FRONT);
    const uint32_t tile = blockIdx.x;
    const int64_t g0 = (int64_t)tile * TILE;
    {
        // every tile but the first / last has its halos inside [0, len): plain
        // 16-B loads with no per-chunk bounds logic, all issued back to back
        uint4 v[4];
        uint4 vh = make_uint4(0, 0, 0, 0);
        if (g0 - FH >= 0 && (uint64_t)(g0 + TILE + BH) <= len) {
            const uint8_t *src = a.data + g0 + 16 * tid;
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = *(const uint4 *)(src + 16 * TPB * i);
            // every lane loads (lanes >= 9 repeat chunk 0): no divergent load, so no early wait
            vh = *(const uint4 *)(a.data + g0 - FH + 16 * (halo ? hc : 0));
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = load_chunk(a.data, g0 + (int64_t)(tid + TPB * i) * 16, len);
            if (halo) vh = load_chunk(a.data, g0 - FH + (int64_t)hc * 16, len);
        }
        if (tid == 0) {
            sh.last_chunk = -1;
            sh.nh = 0;
            sh.nx = 0;
            sh.qn = 0;
        }
        uint32_t orall = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            orall |= v[i].x | v[i].y | v[i].z | v[i].w;
            *(uint4 *)(buf + FH + (tid + TPB * i) * 16) = v[i];
        }
        if (halo) *(uint4 *)(buf + hc * 16) = vh;
        if (tid < 2 * KMAX_TILE) s_pr[tid] = a.PR[tid];     // (behind the tile loads)
        if (orall & 0x80808080u) atomicOr(a.err, ERR_NONASCII);
    }
    __syncthreads();

    // ---- per chunk (from LDS, conflict-free 16-B rows): '\n' count and SWAR candidates ----
    const uint32_t P4 = a.p4, R4 = a.r4, PM = a.pmask;
    uint32_t cand = 0;           // bit 4*i + j: word j of chunk i has a 4-byte match
    uint64_t packed = 0;         // 16-bit '\n' count of chunk i in bits [16i, 16i+16)
    // only the last tile has bytes past len (sentinels): keep the masking out of the hot loop
    const bool tail_tile = (uint64_t)(g0 + TILE) > len;
    const bool do_swar = !(KH_ABLATE(a) & 2u);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int c = tid + TPB * i;
        const uint4 xv = *(const uint4 *)(buf + FH + 16 * c);
        const uint32_t x[5] = {xv.x, xv.y, xv.z, xv.w, *(const uint32_t *)(buf + FH + 16 * c + 16)};
        uint32_t cnt = 0;
        if (!tail_tile) {
#pragma unroll
            for (int j = 0; j < 4; ++j) cnt += __popc(nl_flags(x[j]));
        } else {
            const int64_t gc = g0 + (int64_t)c * 16;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int64_t n = (int64_t)len - (gc + 4 * j);
                uint32_t z = nl_flags(x[j]);
                z = n <= 0 ? 0u : n < 4 ? (z & ((1u << (8 * n)) - 1u)) : z;
                cnt += __popc(z);
            }
        }
        if (do_swar) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                // 4-byte windows at the word's 4 positions vs P[0:4] / rc(P)[0:4]:
                // xor + min on the vector unit (the compare-and-OR form would
                // load the scalar unit, which this kernel is short of)
                const uint32_t x0 = x[j];
                const uint32_t x1 = align4(x[j + 1], x[j], 1);
                const uint32_t x2 = align4(x[j + 1], x[j], 2);
                const uint32_t x3 = align4(x[j + 1], x[j], 3);
                uint32_t m;
                if (FULL4) {
                    m = min(min(min(x0 ^ P4, x1 ^ P4), min(x2 ^ P4, x3 ^ P4)),
                            min(min(x0 ^ R4, x1 ^ R4), min(x2 ^ R4, x3 ^ R4)));
                } else {
                    m = min(min(min((x0 ^ P4) & PM, (x1 ^ P4) & PM), min((x2 ^ P4) & PM, (x3 ^ P4) & PM)),
                            min(min((x0 ^ R4) & PM, (x1 ^ R4) & PM), min((x2 ^ R4) & PM, (x3 ^ R4) & PM)));
                }
                cand |= m == 0 ? (1u << (4 * i + j)) : 0u;
            }
        }
        packed |= (uint64_t)cnt << (16 * i);
        // chunk bitmap + highest chunk with a '\n', from one ballot (no per-lane atomics)
        const unsigned long long m = __ballot(cnt != 0);
        if (lane == 0) {
            const int c0 = c;                               // wave's first chunk of this column
            sh.nlmap[c0 >> 5] = (uint32_t)m;
            sh.nlmap[(c0 >> 5) + 1] = (uint32_t)(m >> 32);
            if (m) atomicMax(&sh.last_chunk, c0 + 63 - (int)__clzll((long long)m));
        }
    }

    // ---- block scan of the 4 packed chunk columns (16-bit fields never carry) ----
    const uint64_t incl = (uint64_t)wave_incl_sum((uint32_t)packed) |
                          ((uint64_t)wave_incl_sum((uint32_t)(packed >> 32)) << 32);
    if (lane == 63) {
#pragma unroll
        for (int i = 0; i < 4; ++i) sh.wsum[wid][i] = (uint32_t)(incl >> (16 * i)) & 0xFFFFu;
    }
    __syncthreads();
    {
        uint32_t col_total[4], col_off[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            col_total[i] = 0;
            col_off[i] = 0;
#pragma unroll
            for (int ww = 0; ww < TPB / 64; ++ww) {
                col_total[i] += sh.wsum[ww][i];
                col_off[i] += ww < wid ? sh.wsum[ww][i] : 0;
            }
        }
        const uint64_t excl = incl - packed;
        uint32_t base = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            sh.cpre[tid + TPB * i] = (uint16_t)(base + col_off[i] + ((excl >> (16 * i)) & 0xFFFFu));
            base += col_total[i];
        }
        if (tid == 0) {
            a.tsum[tile].cnt = base;
            sh.tcnt = base;
        }
    }
    if (tid == 0) {
        const int lc = sh.last_chunk;
        // (the last tile's sentinel bytes past len are not lines)
        const int64_t lim = (int64_t)len - g0;
        const int lp = lc >= 0 ? last_newline_in_chunk(buf, lc, lim < TILE ? (int)lim : TILE) : -1;
        sh.lastpos = lp;
        a.tsum[tile].lnl = lp >= 0 ? a.abs_offset + (uint64_t)(g0 + lp + 1) : 0;
    }
    const uint32_t k = a.k, plen = a.plen;
    if (plen > k || (KH_ABLATE(a) & 1u)) cand = 0;
    const uint32_t *pw = (const uint32_t *)s_pr;             // P words, then rc(P) words

    // ---- candidate words -> LDS queue (one LDS atomic per wave) -> verified
    //      hits -> hit records, one queued word per lane: the rare, branchy
    //      work runs once per tile in as few waves as possible ----
    __syncthreads();             // cpre / nlmap visible
    {
        const uint32_t nc = __popc(cand);
        const uint32_t incl_c = wave_incl_sum(nc);
        const uint32_t wtotal = (uint32_t)__builtin_amdgcn_readlane((int)incl_c, 63);
        uint32_t pos = 0;
        if (wtotal) {
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(&sh.qn, wtotal);
            pos = (uint32_t)__builtin_amdgcn_readfirstlane((int)__shfl((int)base, 0)) + incl_c - nc;
        }
        while (cand) {
            const int bitc = __ffs(cand) - 1;
            cand &= cand - 1;
            const uint32_t q0 = 16u * (uint32_t)(tid + TPB * (bitc >> 2)) + 4u * (uint32_t)(bitc & 3);
            if (pos < QCAP) sh.q[pos] = q0;
            else scan_word<WIDE>(a, buf, sh, tile, pw, q0);   // queue full (short prefixes): process in place
            ++pos;
        }
    }
    __syncthreads();
    const uint32_t nq = min(sh.qn, (uint32_t)QCAP);
    for (uint32_t h = tid; h < nq; h += TPB) scan_word<WIDE>(a, buf, sh, tile, pw, sh.q[h]);
    if (nq > 64 || sh.qn > QCAP) {
        __syncthreads();         // uniform: every wave may have written records
        if (tid == 0) {
            a.tsum[tile].nh = sh.nh;
            a.tsum[tile].nx = sh.nh > (uint32_t)HMAX ? sh.nh : sh.nx;   // overflowed: all hits cross
            if (sh.nh > (uint32_t)HMAX || (sh.nh && sh.tcnt == 0)) set_info(a.err, INFO_LONGSEG);
        }
    } else if (tid == 0) {                       // wave 0 wrote them all (a word can hold 8 hits)
        a.tsum[tile].nh = sh.nh;
        a.tsum[tile].nx = sh.nh > (uint32_t)HMAX ? sh.nh : sh.nx;
        if (sh.nh > (uint32_t)HMAX || (sh.nh && sh.tcnt == 0)) set_info(a.err, INFO_LONGSEG);
    }
}


// Plane-kernel candidate (q << 1) | strand: byte-exact prefix check (the
// planes alias non-ACGT bytes), then the hit record.
template <bool WIDE>
__device__ __forceinline__ void verify_emit(const ScanArgs &a, const uint8_t *buf, ScanShared &sh, uint32_t tile,
                                            const uint32_t *pw, uint32_t e) {
    const uint32_t strand = e & 1u, plen = a.plen;
    const int q = (int)(e >> 1);
    bool ok = true;
#pragma unroll 1
    for (uint32_t b = 0; b < plen && ok; b += 4) {
        const uint32_t n = plen - b;
        const uint32_t mk = n >= 4 ? 0xFFFFFFFFu : ((1u << (8 * n)) - 1u);
        ok = ((lds_word(buf, q + (int)b) ^ pw[(strand ? KMAX_TILE / 4 : 0) + b / 4]) & mk) == 0;
    }
    if (KH_ABLATE(a) & 4u) {                         // experiments: verified, no record
        if (ok) atomicAdd(&sh.nx, 0u);
        return;
    }
    if (ok) emit_hit<true, WIDE>(a, buf, sh, tile, e);
}

// ---------------------------------------------------------------------------
// Plane kernel (ACGT prefixes).  Same tile staging as scan_tile_kernel, but
// after the coalesced load each thread works on its own 64 contiguous bytes
// (+4 look-ahead): the bytes become two bit-planes, bits 1 and 2 of each
// byte, which already tell A (00) C (10) G (11) T (01) apart -- 32 positions
// per 32-bit word, packed with v_dot4_u32_u8, no per-byte recoding.  The prefix (up to 5 bases) is
// then tested at 32 positions per bit-op on both strands:
//   match = AND_i (L>>i == P_i.lo) & (H>>i == P_i.hi)     (funnel shifts)
// Non-ACGT bytes alias to some code, so a candidate is re-checked byte for
// byte before its hit record is written.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t plane_match(uint32_t L0, uint32_t H0, uint32_t L1, uint32_t H1,
                                                const uint32_t *kl, const uint32_t *kh, uint32_t pb,
                                                const uint32_t *SL, const uint32_t *SH) {
    uint32_t acc = (L0 ^ kl[0]) & (H0 ^ kh[0]);
#pragma unroll
    for (uint32_t i = 1; i < 5; ++i) {
        if (i < pb) acc = acc & (SL[i] ^ kl[i]) & (SH[i] ^ kh[i]);
    }
    return acc;
}

// The reference's default prefix, ATGAC (lib/kmers.js:67, BASELINE C2 / C4),
// compiled in: its plane masks are constants, so the compiler folds the XORs
// into the AND chains (v_bitop3 with the complements absorbed) -- about 40 VALU
// fewer per thread.  Bit 4i .. 4i+3 of the word: kl, kh, rl, rh of base i
// (1 = the mask is ~0, i.e. the base's plane bit is 0).
__host__ __device__ constexpr uint32_t plane_masks_const(const char *p, const char *r) {
    uint32_t m = 0;
    for (int i = 0; i < 5; ++i) {
        const uint32_t cp = (((uint32_t)p[i] >> 1) & 1u) | ((((uint32_t)p[i] >> 2) & 1u) << 1);
        const uint32_t cr = (((uint32_t)r[i] >> 1) & 1u) | ((((uint32_t)r[i] >> 2) & 1u) << 1);
        m |= ((cp & 1u) ? 0u : 1u) << (4 * i);
        m |= ((cp & 2u) ? 0u : 1u) << (4 * i + 1);
        m |= ((cr & 1u) ? 0u : 1u) << (4 * i + 2);
        m |= ((cr & 2u) ? 0u : 1u) << (4 * i + 3);
    }
    return m;
}
constexpr uint32_t PM_ATGAC = plane_masks_const("ATGAC", "GTCAT");

template <bool FULL5, bool WIDE, uint32_t PM = 0>
__global__ __launch_bounds__(TPB) void scan_planes_kernel(ScanArgs a, PlaneArgs pa) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[BUFSZ];
    __shared__ ScanShared sh;
    __shared__ __attribute__((aligned(16))) uint8_t s_pr[2 * KMAX_TILE];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint64_t len = a.len;
    const bool halo = tid < NCH_FRONT + NCH_BACK;
    const int hc = tid < NCH_FRONT ? tid : NCH_FRONT + NCH_MAIN + (tid - NCH_FRONT);
    const uint32_t tile = blockIdx.x;
    const int64_t g0 = (int64_t)tile * TILE;
    {
        uint4 v[4];
        uint4 vh = make_uint4(0, 0, 0, 0);
        if (g0 - FH >= 0 && (uint64_t)(g0 + TILE + BH) <= len) {
            const uint8_t *src = a.data + g0 + 16 * tid;
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = *(const uint4 *)(src + 16 * TPB * i);
            vh = *(const uint4 *)(a.data + g0 - FH + 16 * (halo ? hc : 0));
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = load_chunk(a.data, g0 + (int64_t)(tid + TPB * i) * 16, len);
            if (halo) vh = load_chunk(a.data, g0 - FH + (int64_t)hc * 16, len);
        }
        if (tid == 0) {
            sh.last_chunk = -1;
            sh.nh = 0;
            sh.nx = 0;
            sh.qn = 0;
        }
        uint32_t orall = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            orall |= v[i].x | v[i].y | v[i].z | v[i].w;
            *(uint4 *)(buf + FH + (tid + TPB * i) * 16) = v[i];
        }
        if (halo) *(uint4 *)(buf + hc * 16) = vh;
        if (tid < 2 * KMAX_TILE) s_pr[tid] = a.PR[tid];
        if (orall & 0x80808080u) atomicOr(a.err, ERR_NONASCII);
    }
    __syncthreads();

    // ---- this thread's 64 bytes (4 chunks) + 4 look-ahead bytes ----
    uint32_t w[17];
    {
        const uint4 *src = (const uint4 *)(buf + FH + 64 * tid);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint4 x = src[j];
            w[4 * j] = x.x;
            w[4 * j + 1] = x.y;
            w[4 * j + 2] = x.z;
            w[4 * j + 3] = x.w;
        }
        w[16] = *(const uint32_t *)(buf + FH + 64 * tid + 64);
    }
    const bool tail_tile = (uint64_t)(g0 + TILE) > len;
    const uint32_t k0a = 0x0A0A0A0Au, k7f = 0x7F7F7F7Fu;
    uint32_t ccnt[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        uint32_t cnt = 0;
        if (!tail_tile) {
#pragma unroll
            for (int i = 0; i < 4; ++i) cnt += __popc(not_nl_bits_xad(w[4 * j + i], k0a, k7f));
            cnt = 16u - cnt;
        } else {
            const int64_t gc = g0 + 64 * tid + 16 * j;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t n = (int64_t)len - (gc + 4 * i);
                uint32_t z = nl_flags(w[4 * j + i]);
                z = n <= 0 ? 0u : n < 4 ? (z & ((1u << (8 * n)) - 1u)) : z;
                cnt += __popc(z);
            }
        }
        ccnt[j] = cnt;
    }
    const uint32_t ttot = ccnt[0] + ccnt[1] + ccnt[2] + ccnt[3];
    {
        const unsigned long long m = __ballot(ttot != 0);
        if (lane == 0) {
            sh.nlmap[2 * wid] = (uint32_t)m;
            sh.nlmap[2 * wid + 1] = (uint32_t)(m >> 32);
            if (m) atomicMax(&sh.last_chunk, 64 * wid + 63 - (int)__clzll((long long)m));   // (a thread index here)
        }
    }
    const uint32_t incl = wave_incl_sum(ttot);
    if (lane == 63) sh.wsum[wid][0] = incl;

    // ---- bit-planes of the 68 bytes: gL/gH groups of 8 bases (2 words) ----
    // y = low nibbles of x0, x1's low nibbles above them (v_bfi): byte i holds
    // base i's bits 1 / 2 at bits 1 / 2 (x0) and 5 / 6 (x1), so ONE v_dot4
    // with weights 2^i per plane puts the 8 bases at consecutive bits
    const uint32_t W0 = 0x08040201u;
    uint32_t L[3], H[3];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        uint32_t gl[4], gh[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const uint32_t x0 = w[8 * h + 2 * p], x1 = w[8 * h + 2 * p + 1];
            uint32_t y;                          // (inline: the compiler splits it into two ands and a bitop3)
            asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(y) : "s"(0x0F0F0F0Fu), "v"(x0), "v"(x1 << 4));
            gl[p] = __builtin_amdgcn_udot4(y & 0x22222222u, W0, 0u, false);
            gh[p] = __builtin_amdgcn_udot4(y & 0x44444444u, W0, 0u, false);
        }
        // gl: bits 1..8, gh: bits 2..9 for 8 bases
        L[h] = (gl[0] >> 1) | (gl[1] << 7) | (gl[2] << 15) | (gl[3] << 23);
        H[h] = (gh[0] >> 2) | (gh[1] << 6) | (gh[2] << 14) | (gh[3] << 22);
    }
    {
        const uint32_t x = w[16];
        L[2] = __builtin_amdgcn_udot4(x & 0x02020202u, W0, 0u, false) >> 1;
        H[2] = __builtin_amdgcn_udot4(x & 0x04040404u, W0, 0u, false) >> 2;
    }
    uint32_t mf[2], mr[2];
    const uint32_t pb = FULL5 ? 5u : pa.pb;
    uint32_t kl[5], kh[5], rl[5], rh[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        if constexpr (PM != 0) {
            kl[i] = ((PM >> (4 * i)) & 1u) ? ~0u : 0u;
            kh[i] = ((PM >> (4 * i + 1)) & 1u) ? ~0u : 0u;
            rl[i] = ((PM >> (4 * i + 2)) & 1u) ? ~0u : 0u;
            rh[i] = ((PM >> (4 * i + 3)) & 1u) ? ~0u : 0u;
        } else {
            kl[i] = pa.kl[i];
            kh[i] = pa.kh[i];
            rl[i] = pa.rl[i];
            rh[i] = pa.rh[i];
        }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        uint32_t SL[5], SH[5];
        SL[0] = L[h];
        SH[0] = H[h];
#pragma unroll
        for (uint32_t i = 1; i < 5; ++i) {
            SL[i] = __builtin_amdgcn_alignbit(L[h + 1], L[h], i);
            SH[i] = __builtin_amdgcn_alignbit(H[h + 1], H[h], i);
        }
        mf[h] = plane_match(L[h], H[h], L[h + 1], H[h + 1], kl, kh, pb, SL, SH);
        mr[h] = plane_match(L[h], H[h], L[h + 1], H[h + 1], rl, rh, pb, SL, SH);
    }
    if (a.k < a.plen || (KH_ABLATE(a) & 1u)) mf[0] = mf[1] = mr[0] = mr[1] = 0;

    // ---- block scan of the per-thread '\\n' counts -> cpre per chunk ----
    __syncthreads();
    {
        uint32_t pre = incl - ttot, tot = 0;
#pragma unroll
        for (int ww = 0; ww < TPB / 64; ++ww) {
            pre += ww < wid ? sh.wsum[ww][0] : 0u;
            tot += sh.wsum[ww][0];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            sh.cpre[4 * tid + j] = (uint16_t)pre;
            pre += ccnt[j];
        }
        if (tid == 0) {
            a.tsum[tile].cnt = tot;
            sh.tcnt = tot;
        }
    }
    __syncthreads();             // cpre visible
    if (tid == 0) {
        const int lt = sh.last_chunk;            // highest thread region with a '\\n'
        int lp = -1;
        if (lt >= 0) {
            int c = 4 * lt + 3;
            while ((c == NCH_MAIN - 1 ? sh.tcnt : (uint32_t)sh.cpre[c + 1]) == sh.cpre[c]) --c;
            const int64_t lim = (int64_t)len - g0;
            lp = last_newline_in_chunk(buf, c, lim < TILE ? (int)lim : TILE);
        }
        sh.lastpos = lp;
        a.tsum[tile].lnl = lp >= 0 ? a.abs_offset + (uint64_t)(g0 + lp + 1) : 0;
    }

    // ---- candidates -> LDS queue: one {first window, mask} entry per nonzero
    //      32-position mask (ballot + mbcnt, one LDS atomic per wave); the
    //      rare, branchy verification runs once per tile in as few waves as
    //      possible ----
    const uint32_t *pw = (const uint32_t *)s_pr;
    uint2 *qe = (uint2 *)sh.q;
    constexpr uint32_t QE = QCAP / 2;
    {
        const uint32_t mm[4] = {mf[0], mf[1], mr[0], mr[1]};
        unsigned long long bl[4];
        uint32_t tot = 0;
#pragma unroll
        for (int hs = 0; hs < 4; ++hs) {
            bl[hs] = __ballot(mm[hs] != 0);
            tot += (uint32_t)__popcll(bl[hs]);
        }
        if (tot) {
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(&sh.qn, tot);
            base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
#pragma unroll
            for (int hs = 0; hs < 4; ++hs) {
                if (bl[hs]) {
                    if (mm[hs]) {
                        const uint32_t pos = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(bl[hs] >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)bl[hs], 0u));
                        const uint32_t e0 = ((64u * (uint32_t)tid + 32u * (uint32_t)(hs & 1)) << 1) | (uint32_t)(hs >> 1);
                        if (pos < QE) {
                            qe[pos] = make_uint2(e0, mm[hs]);
                        } else {                 // queue full: process in place
                            uint32_t m = mm[hs];
                            while (m) {
                                const uint32_t bit = __ffs(m) - 1;
                                m &= m - 1;
                                verify_emit<WIDE>(a, buf, sh, tile, pw, e0 + (bit << 1));
                            }
                        }
                    }
                    base += (uint32_t)__popcll(bl[hs]);
                }
            }
        }
    }
    __syncthreads();
    const uint32_t nq = min(sh.qn, QE);
    for (uint32_t h = tid; h < nq; h += TPB) {
        const uint2 en = qe[h];
        uint32_t m = en.y;
        while (m) {
            const uint32_t bit = __ffs(m) - 1;
            m &= m - 1;
            verify_emit<WIDE>(a, buf, sh, tile, pw, en.x + (bit << 1));
        }
    }
    if (nq > 64 || sh.qn > QE) {
        __syncthreads();
        if (tid == 0) {
            a.tsum[tile].nh = sh.nh;
            a.tsum[tile].nx = sh.nh > (uint32_t)HMAX ? sh.nh : sh.nx;
            if (sh.nh > (uint32_t)HMAX || (sh.nh && sh.tcnt == 0)) set_info(a.err, INFO_LONGSEG);
        }
    } else if (tid == 0) {
        a.tsum[tile].nh = sh.nh;
        a.tsum[tile].nx = sh.nh > (uint32_t)HMAX ? sh.nh : sh.nx;
        if (sh.nh > (uint32_t)HMAX || (sh.nh && sh.tcnt == 0)) set_info(a.err, INFO_LONGSEG);
    }
}

// Resolve one hit: global line index / line start from the tile scans, the
// reference's sequence-line rule (lib/kmers.js:151-155), first-occurrence
// order key (line << (pbits + 1) | strand << pbits | strand ? maxrel - rel : rel).
// Returns the packed key (invalid_key when the hit does not count as a packed
// key: non-sequence line, or a record) and writes records for exotic windows
// / record mode.  *lk = order of the hit among its tile's hits (local).
__device__ __forceinline__ uint64_t resolve_hit(const HitArgs &a, uint64_t pos_lines, const HitRec &r,
                                                uint64_t code_hi, const TileSum &tb, uint64_t *order_out,
                                                uint32_t *lk, bool *lvalid_out, uint64_t *key_hi) {
    const uint32_t t = r.tile;
    const uint32_t strand = (r.qm >> 14) & 1u;
    const bool exotic = (r.qm >> 15) & 1u;
    const bool lvalid = (r.qm >> 16) & 1u;
    const int q = (int)(r.qm & 0x3FFFu);
    const int s0 = strand ? q + (int)a.plen - (int)a.k : q;     // >= -63
    const uint64_t tile_abs = a.abs_offset + (uint64_t)t * TILE;
    const uint64_t li = pos_lines + tb.cnt + r.c_local;
    const uint64_t lstart = lvalid ? tile_abs + r.lstart : tb.lnl;
    const uint64_t sabs = tile_abs + (uint64_t)(int64_t)s0;
    uint64_t rel = sabs - lstart;
    const bool seq = (li & 3) == 1;
    const uint64_t maxrel = (1ull << a.pbits) - 1ull;
    if (rel > maxrel) {
        if (seq && !KH_ABLATE(a)) atomicOr(a.err, ERR_LINE_TOO_LONG);
        rel = maxrel;                            // (non-sequence lines only need a consistent order)
    }
    if ((li >> (63 - a.pbits)) && !KH_ABLATE(a)) atomicOr(a.err, ERR_LINE_TOO_LONG);   // (line field full: long-line mode)
    const uint64_t order = (li << (a.pbits + 1)) | ((uint64_t)strand << a.pbits) | (strand ? maxrel - rel : rel);
    *order_out = order;
    const uint32_t sp = (uint32_t)(s0 + 64);     // < 2^15
    *lk = (r.c_local << 17) | (strand << 16) | (strand ? 0xFFFFu - sp : sp);
    *lvalid_out = lvalid;
    uint64_t key = a.invalid_key;
    *key_hi = a.wide ? a.invalid_key : 0;        // (wide: the invalid marker is in the high word)
    if (a.wide) key = 0;
    if (seq) {
        if (a.packed && !exotic) {
            if (a.k > 32) {
                uint64_t h = code_hi, l = r.code;
                if (strand) revcomp_code128(code_hi, r.code, a.k, &h, &l);
                key = l & a.smask;
                *key_hi = h & a.smask_hi;
            } else {
                key = (strand ? revcomp_code(r.code, a.k) : r.code) & a.smask;
            }
        } else {
            const unsigned long long n = atomicAdd(a.rec_count, 1ull);
            if (n < a.rec_cap) {
                Record rec;
                rec.order = order;
                rec.pos = (uint64_t)t * TILE + (uint64_t)(int64_t)s0;
                rec.len = a.k;
                rec.strand = strand;
                a.recs[n] = rec;
            } else {
                atomicOr(a.err, ERR_REC_OVERFLOW);
            }
        }
    }
    return key;
}

// Write one resolved packed hit at its rank slot, or to the cross list.
__device__ __forceinline__ void place_hit(const HitArgs &a, uint64_t slot, bool cross, uint64_t xi, uint64_t key,
                                          uint64_t key_hi, uint64_t order) {
    // (no rank payload: the finish sorts (key, iota))
    if (!cross) {
        if (slot >= a.rcap) {                    // only when hits overflowed the lists: redone
            atomicOr(a.err, ERR_OVF_OVERFLOW);
            return;
        }
        if (a.rkey32) a.rkey32[slot] = (uint32_t)key;
        else a.rkey[slot] = key;
        if (a.wide) a.rkeyh[slot] = key_hi;
        a.rord[slot] = order;
    } else if (xi < a.xcap) {
        a.xord[xi] = order;
        a.xslot[xi] = (uint32_t)slot;
        if (a.wide) {                            // (the cross kernels move the index; cross_wide_fix the key)
            a.xkey[xi] = xi;
            a.xkeyl[xi] = key;
            a.xkeyh[xi] = key_hi;
        } else {
            a.xkey[xi] = key;
        }
    } else {
        atomicOr(a.err, ERR_CROSS_OVERFLOW);
    }
}

// Hits of HTPW consecutive tiles per wave, flattened onto the lanes (a tile
// has ~14 hits at 150 bp reads: one tile per wave would leave most lanes
// idle).  Phase 1: lane = one hit: resolve it, stage (local order, cross
// flag, key, order) in LDS.  Phase 2: rank each hit among its tile's hits by
// (line, strand, +-offset) and place it at out_base + hits-before-tile +
// rank, or on the cross list (line crosses a tile edge / tile overflowed).
constexpr uint32_t HTPW = 4;
constexpr uint32_t HENT = HTPW * HMAX;       // staged hits per wave
template <bool WIDE>
__global__ __launch_bounds__(256) void hit_kernel(HitArgs a) {
    __shared__ uint32_t s_lk[4][HENT];
    __shared__ uint8_t s_x[4][HENT];
    __shared__ uint64_t s_key[4][HENT];
    __shared__ uint64_t s_ord[4][HENT];
    __shared__ uint64_t s_keyh[WIDE ? 4 : 1][WIDE ? HENT : 1];
    const uint32_t wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t t0 = __builtin_amdgcn_readfirstlane((blockIdx.x * 4 + wid) * HTPW);
    if (t0 >= a.n_tiles) return;
    // (the overflow count, the stream position and the tiles' sums issued
    // together: one memory round trip before the hits, not three)
    const unsigned long long ovf = *a.ovf_count;
    const uint64_t pos_lines = a.pos->lines;
    TileSum ts[HTPW], tb[HTPW];
#pragma unroll
    for (uint32_t u = 0; u < HTPW; ++u) {
        const uint32_t t = min(t0 + u, a.n_tiles - 1);
        ts[u] = a.tsum[t];
        tb[u] = a.tscan[t];
    }
    if (ovf > a.ovf_cap) return;                 // overflowed scan: the host redoes the chunk
    uint32_t off[HTPW + 1];
    off[0] = 0;
#pragma unroll
    for (uint32_t u = 0; u < HTPW; ++u) off[u + 1] = off[u] + (t0 + u < a.n_tiles ? min(ts[u].nh, (uint32_t)HMAX) : 0u);
    const uint32_t total = off[HTPW];
    // phase 1
    for (uint32_t e0 = 0; e0 < total; e0 += 64) {
        const uint32_t e = e0 + lane;
        if (e < total) {
            uint32_t u = 0;
#pragma unroll
            for (uint32_t v = 1; v < HTPW; ++v) u += e >= off[v] ? 1u : 0u;
            const uint32_t i = e - off[u];
            TileSum tsu = ts[0], tbu = tb[0];
#pragma unroll
            for (uint32_t v = 1; v < HTPW; ++v)
                if (u == v) {
                    tsu = ts[v];
                    tbu = tb[v];
                }
            const uint64_t hslot = (uint64_t)(t0 + u) * HMAX + i;
            const HitRec r = a.hits[hslot];
            uint64_t order, kh;
            uint32_t lk;
            bool lvalid;
            const uint64_t key = resolve_hit(a, pos_lines, r, a.k > 32 ? a.hits_hi[hslot] : 0, tbu, &order, &lk, &lvalid,
                                             &kh);
            s_lk[wid][e] = lk;
            s_x[wid][e] = (tsu.nh > (uint32_t)HMAX || !lvalid || r.c_local == (uint32_t)tsu.cnt) ? 1 : 0;
            s_key[wid][e] = key;
            if (WIDE) s_keyh[WIDE ? wid : 0][WIDE ? e : 0] = kh;
            s_ord[wid][e] = order;
        }
    }
    if (!a.packed) return;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    // phase 2
    for (uint32_t e0 = 0; e0 < total; e0 += 64) {
        const uint32_t e = e0 + lane;
        if (e >= total) continue;
        uint32_t u = 0;
#pragma unroll
        for (uint32_t v = 1; v < HTPW; ++v) u += e >= off[v] ? 1u : 0u;
        uint32_t lo = off[0], hi = off[1], nh = ts[0].nh;
        uint64_t hb = tb[0].nh, xb = tb[0].nx;
#pragma unroll
        for (uint32_t v = 1; v < HTPW; ++v)
            if (u == v) {
                lo = off[v];
                hi = off[v + 1];
                nh = ts[v].nh;
                hb = tb[v].nh;
                xb = tb[v].nx;
            }
        const uint32_t i = e - lo;
        const bool cross = s_x[wid][e] != 0;
        uint32_t rank = i, xr = i;            // overflowed tile: the in-tile ordinal
        if (nh <= (uint32_t)HMAX) {
            const uint32_t lk = s_lk[wid][e];
            rank = 0;
            xr = 0;
            for (uint32_t j = lo; j < hi; ++j) {
                const uint32_t less = s_lk[wid][j] < lk ? 1u : 0u;
                rank += less;
                xr += less & (uint32_t)s_x[wid][j];
            }
        }
        place_hit(a, a.out_base + hb + rank, cross, a.xbase + xb + xr, s_key[wid][e],
                  WIDE ? s_keyh[WIDE ? wid : 0][WIDE ? e : 0] : 0, s_ord[wid][e]);
    }
}

// hits that did not fit their tile's slots (their tile is all cross)
__global__ __launch_bounds__(256) void hit_overflow_kernel(HitArgs a) {
    const uint64_t n = *a.ovf_count <= a.ovf_cap ? *a.ovf_count : 0;   // overflowed: the host redoes the chunk
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const HitRec r = a.ovf[i];
        const TileSum tb = a.tscan[r.tile];
        uint64_t order, kh;
        uint32_t lk;
        bool lvalid;
        const uint64_t key = resolve_hit(a, a.pos->lines, r, a.k > 32 ? a.ovf_hi[i] : 0, tb, &order, &lk, &lvalid, &kh);
        if (!a.packed) continue;
        const uint32_t ord = r.qm >> 17;
        place_hit(a, a.out_base + tb.nh + ord, true, a.xbase + tb.nx + ord, key, kh, order);
    }
    // chunk tail, by the last block to finish (every hit of the chunk has read
    // pos by then): advance the stream position past the chunk, publish the
    // chunk's hit / cross counts and copy the counters to host memory
    __shared__ bool last;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        last = atomicAdd(a.ticket, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last || threadIdx.x != 0) return;
    __threadfence();
    const uint32_t nt = a.n_tiles;
    StreamPos *pos = (StreamPos *)a.pos;
    pos->lines += a.tscan[nt - 1].cnt + a.tsum[nt - 1].cnt;
    pos->ends_open = (a.len > 0 && a.data[a.len - 1] != '\n') ? 1 : 0;
    *a.ends_open = pos->ends_open;
    *a.chunk_hits = a.tscan[nt - 1].nh + a.tsum[nt - 1].nh;
    *a.chunk_cross = a.tscan[nt - 1].nx + a.tsum[nt - 1].nx;
    *a.ticket = 0;
    __threadfence();
    if (a.host_out) {
        for (int i = 0; i < 8; ++i)
            a.host_out[i] = __hip_atomic_load(a.scal + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __threadfence_system();
        __hip_atomic_store(a.host_out + 9, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---------------------------------------------------------------------------
// exclusive scan of the per-tile sums: block reduce, then per-block scan with
// the prefix of the preceding blocks (in-kernel for up to TSCAN_INLINE_MAX
// blocks, else from a scanned block-sum array)
// ---------------------------------------------------------------------------
__device__ __forceinline__ TileSum ts_shfl_up(const TileSum &v, int d) {
    TileSum r;
    r.cnt = (uint64_t)__shfl_up((unsigned long long)v.cnt, d);
    r.nh = (uint32_t)__shfl_up((int)v.nh, d);
    r.nx = (uint32_t)__shfl_up((int)v.nx, d);
    r.lnl = (uint64_t)__shfl_up((unsigned long long)v.lnl, d);
    return r;
}
__device__ __forceinline__ TileSum ts_zero() {
    TileSum z;
    z.cnt = 0;
    z.nh = 0;
    z.nx = 0;
    z.lnl = 0;
    return z;
}
// inclusive wave scan
__device__ __forceinline__ TileSum ts_wave_scan(TileSum v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const TileSum o = ts_shfl_up(v, d);
        if (lane >= d) v = tile_sum_op(o, v);
    }
    return v;
}
// block (256 threads) exclusive scan of one value per thread; returns the exclusive prefix, *total the sum
__device__ __forceinline__ TileSum ts_block_scan(TileSum v, TileSum *total) {
    __shared__ TileSum wsum[4];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const TileSum incl = ts_wave_scan(v);
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    TileSum pre = ts_zero(), tot = ts_zero();
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        if (w < wid) pre = tile_sum_op(pre, wsum[w]);
        tot = tile_sum_op(tot, wsum[w]);
    }
    __syncthreads();
    *total = tot;
    const TileSum ex = ts_shfl_up(incl, 1);
    return lane == 0 ? pre : tile_sum_op(pre, ex);
}

__global__ __launch_bounds__(256) void tile_reduce_kernel(const TileSum *in, uint32_t n, TileSum *bsum) {
    const uint32_t base = blockIdx.x * TSCAN_BLOCK;
    TileSum v = ts_zero();
#pragma unroll
    for (uint32_t i = 0; i < TSCAN_BLOCK / 256; ++i) {
        const uint32_t t = base + i * 256 + threadIdx.x;
        if (t < n) v = tile_sum_op(v, in[t]);
    }
    TileSum tot;
    (void)ts_block_scan(v, &tot);
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(256) void tile_scan_kernel(const TileSum *in, uint32_t n, const TileSum *bsum,
                                                        uint32_t bsum_scanned, TileSum init, TileSum *out) {
    const uint32_t b = blockIdx.x;
    TileSum pre;
    if (bsum_scanned) {
        pre = tile_sum_op(init, bsum[b]);
    } else {
        TileSum v = ts_zero();
        for (uint32_t j = threadIdx.x; j < b; j += 256) v = tile_sum_op(v, bsum[j]);
        TileSum tot;
        (void)ts_block_scan(v, &tot);
        pre = tile_sum_op(init, tot);
    }
    // 4 consecutive tiles per thread
    const uint32_t t0 = b * TSCAN_BLOCK + threadIdx.x * 4;
    TileSum x[4];
    TileSum acc = ts_zero();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        x[i] = t0 + i < n ? in[t0 + i] : ts_zero();
        acc = tile_sum_op(acc, x[i]);
    }
    TileSum tot;
    TileSum ex = tile_sum_op(pre, ts_block_scan(acc, &tot));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (t0 + i < n) out[t0 + i] = ex;
        ex = tile_sum_op(ex, x[i]);
    }
}

// set the running stream position (kernel argument: no host staging, no sync)
// Feed prologue: the lazy reset / set_position of the host API, the position
// snapshot for an overflow redo, the chunk's counters -- one launch.
__global__ void prep_kernel(StreamPos *pos, StreamPos *saved, unsigned int *err, uint64_t *scal, uint32_t flags,
                            uint64_t lines) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    StreamPos p = *pos;
    if (flags & PREP_RESET) {
        p.lines = p.unused = p.ends_open = p.pad = 0;
        *err = 0;
    }
    if (flags & PREP_SETPOS) {
        p.lines = lines;
        p.unused = p.ends_open = p.pad = 0;
    }
    if (flags & (PREP_RESET | PREP_SETPOS)) *pos = p;
    if (flags & PREP_SAVE) *saved = p;
    if (flags & PREP_ZERO) scal[0] = scal[1] = scal[2] = 0;   // records, overflow hits, cross hits of the chunk
}

// Two-pass mode, pass 1: per-tile '\n' count and last '\n' position.
__global__ __launch_bounds__(TPB) void tile_aggregate_kernel(const uint8_t *data, uint64_t len,
                                                             uint64_t *agg_cnt, uint64_t *agg_last,
                                                             unsigned int *err) {
    __shared__ uint32_t s_cnt[TPB / 64];
    __shared__ int32_t s_last;
    const int tid = threadIdx.x;
    const int64_t g0 = (int64_t)blockIdx.x * TILE;
    if (tid == 0) s_last = -1;
    __syncthreads();
    uint32_t cnt = 0, orall = 0;
    int last = -1;
    for (int i = 0; i < 4; ++i) {
        const int off = (tid + TPB * i) * 16;
        uint4 v = load_chunk(data, g0 + off, len);
        orall |= v.x | v.y | v.z | v.w;
        uint32_t ws[4] = {v.x, v.y, v.z, v.w};
        for (int j = 0; j < 4; ++j) {
            uint32_t z = nl_flags(ws[j]);
            for (int b = 0; b < 4; ++b) {
                int64_t p = g0 + off + 4 * j + b;
                if (((z >> (8 * b + 7)) & 1u) && p < (int64_t)len) {
                    ++cnt;
                    last = max(last, off + 4 * j + b);
                }
            }
        }
    }
    if (orall & 0x80808080u) atomicOr(err, ERR_NONASCII);
    for (int d = 32; d >= 1; d >>= 1) cnt += __shfl_xor(cnt, d);
    if ((tid & 63) == 0) s_cnt[tid >> 6] = cnt;
    if (last >= 0) atomicMax(&s_last, last);
    __syncthreads();
    if (tid == 0) {
        agg_cnt[blockIdx.x] = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
        agg_last[blockIdx.x] = s_last < 0 ? 0 : (uint64_t)(g0 + s_last + 1);   // chunk-relative line start + 0 = none
    }
}

// ---------------------------------------------------------------------------
// general windows kernel (any k, any step, any prefix incl. empty)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void windows_kernel(WindowArgs a) {
    const uint64_t nl = *a.n_lines;
    const uint32_t k = a.k, step = a.step, plen = a.plen;
    for (uint64_t li = blockIdx.x; li < nl; li += gridDim.x) {
        const SeqLine sl = a.lines[li];
        const uint8_t *line = a.data + sl.start;
        const uint64_t L = sl.len;
        const uint64_t nwin = L - k + 1;       // sl.len >= k guaranteed
        if (nwin - 1 > (1ull << a.pbits) - 1ull || (sl.line_index >> (63 - a.pbits))) {
            if (threadIdx.x == 0) atomicOr(a.err, ERR_LINE_TOO_LONG);
            continue;
        }
        for (int strand = 0; strand < 2; ++strand) {
            for (uint64_t j = threadIdx.x; j < nwin; j += blockDim.x) {
                const uint64_t ini = j * step;
                const uint64_t lo = ini < L ? ini : L;
                const uint64_t hi = ini + k < L ? ini + k : L;
                const uint64_t klen = hi - lo;
                if (klen < plen) continue;
                bool ok = true;
                for (uint32_t b = 0; b < plen && ok; ++b) {
                    const uint8_t c = strand ? comp_byte(line[L - 1 - lo - b]) : line[lo + b];
                    ok = c == a.P[b];
                }
                if (!ok) continue;
                unsigned long long n = atomicAdd(a.rec_count, 1ull);
                if (n < a.rec_cap) {
                    Record r;
                    r.order = (sl.line_index << (a.pbits + 1)) | ((uint64_t)strand << a.pbits) | j;
                    r.pos = strand ? sl.start + (L - hi) : sl.start + lo;
                    r.len = (uint32_t)klen;
                    r.strand = strand;
                    a.recs[n] = r;
                } else {
                    atomicOr(a.err, ERR_REC_OVERFLOW);
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// General path, device merge (step 1: every record is a key of exactly k
// bytes; any k, any prefix bytes).  A chunk's records become session entries
// (key bytes, count 1, first-occurrence key); a merge groups equal keys by a
// 128-bit hash of their bytes (radix sorts on the device), checks the bytes of
// every pair of neighbours with equal hashes (a collision is reported, never
// merged), and reduces each group to (key, count sum, min first).
// ---------------------------------------------------------------------------
// (GEN_G lanes per record, 64 / GEN_G records per wave step: several rows'
// loads in flight per wave -- one wave per row was latency-bound)
constexpr uint32_t GEN_G = 8;
__global__ __launch_bounds__(256) void gen_append_kernel(const Record *__restrict__ recs, uint64_t n,
                                                         const uint8_t *__restrict__ data, uint32_t k,
                                                         uint8_t *__restrict__ keys, uint64_t *__restrict__ cnt,
                                                         uint64_t *__restrict__ first) {
    const uint32_t lane = threadIdx.x & 63, sub = lane % GEN_G;
    const uint64_t nw = (uint64_t)gridDim.x * 4 * (64 / GEN_G);
    for (uint64_t i = ((uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * (64 / GEN_G) + lane / GEN_G; i < n; i += nw) {
        const Record r = recs[i];
        uint8_t *o = keys + i * k;
        const uint8_t *src = data + r.pos;
        if (r.strand) {
            for (uint32_t b = sub; b < k; b += GEN_G) o[b] = comp_byte(src[k - 1 - b]);
        } else {
            for (uint32_t b = sub; b < k; b += GEN_G) o[b] = src[b];
        }
        if (sub == 0) {
            cnt[i] = 1;
            first[i] = r.order;
        }
    }
}

// Windows of the general path (step 1, any k, any prefix bytes), one lane per
// window position of the flattened window space: each wave takes an equal
// contiguous range of positions (Σ W over the chunk's sequence lines), finds
// its first line by a binary search of wbase, then loads the descriptors of
// 64 lines at a time (lane j: line li + j) and walks every position those
// lines cover, 64 per step: each lane finds its own line among the 64 by a
// 6-step shuffle search (lines without windows take no positions).  A lane
// tests its position s on both strands: forward iff the line's bytes at s are
// P, reverse iff the bytes at s + k - |P| are rc(P) (the reverse strand's
// window L - k - s, lib/kmers.js:88-100, 153).  The first 8 bytes of both
// tests are loaded at once (no chain of dependent byte loads) and compared
// with P / rc(P) held in registers.  Accepted windows are queued per wave in
// LDS and written as records with one atomic per flush.
__device__ __forceinline__ uint64_t gen_load8(const uint8_t *p, uint32_t n) {
    uint64_t w = 0;
#pragma unroll
    for (uint32_t t = 0; t < 8; ++t)
        if (t < n) w |= (uint64_t)p[t] << (8 * t);
    return w;
}

__device__ __forceinline__ bool gen_match(const uint8_t *p, const uint8_t *P, uint32_t plen, uint64_t P8) {
    const uint32_t n0 = plen < 8 ? plen : 8;
    if (gen_load8(p, n0) != P8) return false;
    bool ok = true;
    for (uint32_t b = 8; b < plen && ok; b += 8) {
        const uint32_t n = plen - b < 8 ? plen - b : 8;
        ok = gen_load8(p + b, n) == gen_load8(P + b, n);
    }
    return ok;
}

constexpr uint32_t GW_Q = 128;                   // records queued per wave (>= the 128 of one step; 12 KB of LDS per workgroup)

__global__ __launch_bounds__(256) void gen_windows_kernel(GenWinArgs a) {
    __shared__ Record q[4][GW_Q];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    Record *wq = q[wv];
    const uint64_t npos = a.total / 2;
    const uint64_t nw = (uint64_t)gridDim.x * 4, gw = (uint64_t)blockIdx.x * 4 + wv;
    uint64_t f = npos * gw / nw;
    const uint64_t fend = npos * (gw + 1) / nw;
    const uint32_t k = a.k, plen = a.plen;
    // (no prefix: every window is a record, at slots 2g / 2g + 1 of its
    // flattened position g -- the host sized the list to the total)
    if (plen == 0 && gw == 0 && lane == 0) *a.rec_count = a.total;
    if (f >= fend) return;
    const uint64_t P8 = gen_load8(a.P, plen < 8 ? plen : 8), R8 = gen_load8(a.RP, plen < 8 ? plen : 8);
    // first line: the last li with wbase[li] / 2 <= f
    uint64_t lo = 0, hi = a.n_lines;                 // invariant: wbase[lo] / 2 <= f < wbase[hi] / 2 (hi: +inf)
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) / 2;
        if (a.wbase[mid] / 2 <= f) lo = mid; else hi = mid;
    }
    uint64_t li = lo;
    uint32_t cnt = 0;
    auto flush = [&]() {
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(a.rec_count, (unsigned long long)cnt);
        base = __shfl(base, 0);
        for (uint32_t i = lane; i < cnt; i += 64) {
            if (base + i < a.rec_cap) a.recs[base + i] = wq[i];
            else atomicOr(a.err, ERR_REC_OVERFLOW);
        }
        cnt = 0;
    };
    while (f < fend) {
        // lines li .. li + 63: starts (flat positions), descriptors, covered end E
        const uint64_t lj = li + lane;
        const bool lin = lj < a.n_lines;
        const uint64_t B = lin ? a.wbase[lj] / 2 : ~0ull;
        SeqLine sl = {0, 0, 0};
        if (lin) sl = a.lines[lj];
        const uint64_t Wl = sl.len >= k ? sl.len - k + 1 : 0;
        const uint64_t E = __shfl(lin ? B + Wl : ~0ull, 63);
        const uint64_t fe = E < fend ? E : fend;
        uint32_t j = 0;
        constexpr int U = 1;                     // steps per iteration (4: slower, 8.4 vs 6.8 ms at k = 70)
        const uint32_t n0 = plen < 8 ? plen : 8;
        while (f < fe) {
            uint64_t st[U], s[U], L[U], lidx[U], wf[U], wr[U], gg[U];
            bool act[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t g = f + 64 * u + lane;
                gg[u] = g;
                act[u] = g < fe;
                // lane's line: the last j with B_j <= g, 6 shuffle steps
                j = 0;
#pragma unroll
                for (uint32_t sp = 32; sp >= 1; sp >>= 1) {
                    const uint64_t bj = __shfl(B, (int)(j + sp));
                    if (j + sp < 64 && bj <= g) j += sp;
                }
                st[u] = __shfl(sl.start, (int)j);
                L[u] = __shfl(sl.len, (int)j);
                lidx[u] = __shfl(sl.line_index, (int)j);
                s[u] = g - __shfl(B, (int)j);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                wf[u] = wr[u] = ~0ull;
                if (act[u]) {
                    const uint8_t *line = a.data + st[u];
                    wf[u] = gen_load8(line + s[u], n0);
                    wr[u] = gen_load8(line + s[u] + k - plen, n0);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (plen == 0) {                     // every window: position g's records at 2g, 2g + 1 (no queue)
                    if (act[u]) {
                        const uint64_t lo_key = lidx[u] << (a.pbits + 1);
                        Record r;
                        r.order = lo_key | s[u];
                        r.pos = st[u] + s[u];
                        r.len = k;
                        r.strand = 0;
                        a.recs[2 * gg[u]] = r;
                        r.order = lo_key | (1ull << a.pbits) | (L[u] - k - s[u]);
                        r.strand = 1;
                        a.recs[2 * gg[u] + 1] = r;
                    }
                    continue;
                }
                bool fw = act[u] && wf[u] == P8, rv = act[u] && wr[u] == R8;
                if (plen > 8) {                      // (long prefixes: the rest byte for byte)
                    const uint8_t *line = a.data + st[u];
                    fw = fw && gen_match(line + s[u], a.P, plen, P8);
                    rv = rv && gen_match(line + s[u] + k - plen, a.RP, plen, R8);
                }
                const unsigned long long mf = __ballot(fw), mr = __ballot(rv);
                const uint32_t n = (uint32_t)(__popcll(mf) + __popcll(mr));
                if (n) {
                    if (cnt + n > GW_Q) flush();
                    const unsigned long long below = (1ull << lane) - 1ull;
                    const uint64_t lo_key = lidx[u] << (a.pbits + 1);
                    if (fw) {
                        Record r;
                        r.order = lo_key | s[u];
                        r.pos = st[u] + s[u];
                        r.len = k;
                        r.strand = 0;
                        wq[cnt + __popcll(mf & below)] = r;
                    }
                    if (rv) {
                        Record r;
                        r.order = lo_key | (1ull << a.pbits) | (L[u] - k - s[u]);
                        r.pos = st[u] + s[u];
                        r.len = k;
                        r.strand = 1;
                        wq[cnt + __popcll(mf) + __popcll(mr & below)] = r;
                    }
                    cnt += n;
                }
            }
            f += 64 * U;
        }
        // next 64 lines: from the line holding position f (f >= E: line li + 64 on)
        if (f >= E) {
            f = E;
            li += 64;
        } else {
            li += (uint32_t)__shfl((int)j, 63);    // (f >= fend: the loop ends)
        }
    }
    if (cnt) flush();
}

// Windows of the general path for an A/C/G/T prefix (the common case: k > 64
// with a prefix such as ATGAC), from the raw chunk instead of the flattened
// window space: a workgroup takes 16 KiB of the chunk, each thread its own 64
// bytes, turned into the two bit planes of scan_planes_kernel, and the first
// min(|P|, 5) bases of P and of rc(P) are tested at 32 positions per bit-op.
// A candidate x (rare) is checked byte for byte against P / rc(P) (the planes
// alias other bytes); its line is r = the newlines before x -- the tile's
// count from chunk_lines (tbase) plus the newlines of the tile before x (a
// block scan of the threads' newline masks) -- so no search: x is in a
// sequence line iff r = first + 4m (the mod-4 record rule, as chunk_lines).
// Candidates (x, m, strand) go out; gen_fix_kernel keeps those whose window
// lies inside line m: forward window [x, x + k), reverse window
// [x + |P| - k, x + |P|) (lib/kmers.js:88-100, 153: the reverse strand's
// window at L - k - s).
// Candidates are queued in LDS and written with one atomic per workgroup.
constexpr uint32_t GC_Q = 512;                   // records queued per workgroup
constexpr uint32_t GC_TPB = 32;                  // tiles per workgroup (one queue flush per ~32 tiles)

__device__ __forceinline__ bool gen_bytes_eq(const uint8_t *d, uint64_t len, uint64_t x, const uint8_t *P,
                                             uint32_t plen) {
    if (x + plen > len) return false;
    for (uint32_t b = 0; b < plen; ++b)
        if (d[x + b] != P[b]) return false;
    return true;
}

__global__ __launch_bounds__(256) void gen_cand_kernel(GenWinArgs a, PlaneArgs pa) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[TILE + 16];
    __shared__ Record q[GC_Q];
    __shared__ uint32_t qn, wsum[4];
    __shared__ unsigned long long qbase;
    __shared__ uint8_t sp[2 * 16];                   // P, rc(P) (|P| <= 16: verified in LDS)
    const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t plen = a.plen, k = a.k;
    const bool lds_verify = plen <= 16;
    if (lds_verify && tid < 2 * plen) sp[tid < plen ? tid : 16 + tid - plen] = tid < plen ? a.P[tid] : a.RP[tid - plen];
    if (tid == 0) qn = 0;
    const uint64_t ntiles = (a.len + TILE - 1) / TILE;
    const uint64_t t0 = (uint64_t)blockIdx.x * GC_TPB, t1 = t0 + GC_TPB < ntiles ? t0 + GC_TPB : ntiles;
    // the queue goes out with one atomic when it is half full (and at the end):
    // one device-scope atomic on one address costs ~12 ns, serialised -- one
    // per 16 KiB tile was 2 ms at C2 size
    auto flush = [&]() {
        const uint32_t nq = min(qn, GC_Q);
        if (tid == 0 && nq) qbase = atomicAdd(a.rec_count, (unsigned long long)nq);
        __syncthreads();
        for (uint32_t i = tid; i < nq; i += 256) {
            if (qbase + i < a.rec_cap) a.recs[qbase + i] = q[i];
            else atomicOr(a.err, ERR_REC_OVERFLOW);
        }
        __syncthreads();
        if (tid == 0) qn = 0;
    };
    for (uint64_t tile = t0; tile < t1; ++tile) {
        const int64_t g0 = (int64_t)tile * TILE;
        {
            uint4 v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = load_chunk(a.data, g0 + 16 * (int64_t)(tid + TPB * i), a.len);
#pragma unroll
            for (int i = 0; i < 4; ++i) *(uint4 *)(buf + 16 * (tid + TPB * i)) = v[i];
            if (tid == 0) *(uint4 *)(buf + TILE) = load_chunk(a.data, g0 + TILE, a.len);
        }
        __syncthreads();
        uint32_t w[17];
        {
            const uint4 *src = (const uint4 *)(buf + 64 * tid);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint4 x = src[j];
                w[4 * j] = x.x;
                w[4 * j + 1] = x.y;
                w[4 * j + 2] = x.z;
                w[4 * j + 3] = x.w;
            }
            w[16] = *(const uint32_t *)(buf + 64 * tid + 64);
        }
        // planes of the 68 bytes (as scan_planes_kernel: one v_dot4 per 8 bases and plane)
        const uint32_t W0 = 0x08040201u;
        uint32_t L[3], H[3];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            uint32_t gl[4], gh[4];
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const uint32_t x0 = w[8 * h + 2 * p], x1 = w[8 * h + 2 * p + 1];
                const uint32_t y = (x0 & 0x0F0F0F0Fu) | ((x1 << 4) & 0xF0F0F0F0u);
                gl[p] = __builtin_amdgcn_udot4(y & 0x22222222u, W0, 0u, false);
                gh[p] = __builtin_amdgcn_udot4(y & 0x44444444u, W0, 0u, false);
            }
            L[h] = (gl[0] >> 1) | (gl[1] << 7) | (gl[2] << 15) | (gl[3] << 23);
            H[h] = (gh[0] >> 2) | (gh[1] << 6) | (gh[2] << 14) | (gh[3] << 22);
        }
        L[2] = __builtin_amdgcn_udot4(w[16] & 0x02020202u, W0, 0u, false) >> 1;
        H[2] = __builtin_amdgcn_udot4(w[16] & 0x04040404u, W0, 0u, false) >> 2;
        uint32_t m4[4];                              // forward h = 0, 1; reverse h = 0, 1
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            uint32_t SL[5], SH[5];
            SL[0] = L[h];
            SH[0] = H[h];
#pragma unroll
            for (uint32_t i = 1; i < 5; ++i) {
                SL[i] = __builtin_amdgcn_alignbit(L[h + 1], L[h], i);
                SH[i] = __builtin_amdgcn_alignbit(H[h + 1], H[h], i);
            }
            m4[h] = plane_match(L[h], H[h], L[h + 1], H[h + 1], pa.kl, pa.kh, pa.pb, SL, SH);
            m4[2 + h] = plane_match(L[h], H[h], L[h + 1], H[h + 1], pa.rl, pa.rh, pa.pb, SL, SH);
        }
        // newlines of this thread's 64 bytes (bit b: byte b is '\n'), and the
        // tile's newlines before them (bytes past the chunk read as '\n': they
        // only follow every position that is tested)
        uint64_t nlm = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t z = w[j] ^ 0x0A0A0A0Au;
            const uint32_t ne = (((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z) & 0x80808080u;   // 0x80: not '\n'
            nlm |= (uint64_t)__builtin_amdgcn_udot4((~ne & 0x80808080u) >> 7, W0, 0u, false) << (4 * j);
        }
        const uint32_t nc = (uint32_t)__popcll(nlm);
        const uint32_t incl = wave_incl_sum(nc);
        if (lane == 63) wsum[wid] = incl;
        __syncthreads();
        uint64_t r0 = a.tbase[tile] + incl - nc;                  // newlines before this thread's bytes
        for (uint32_t v = 0; v < wid; ++v) r0 += wsum[v];
#pragma unroll
        for (int hs = 0; hs < 4; ++hs) {
            uint32_t m = m4[hs];
            const uint32_t strand = (uint32_t)hs >> 1;
            while (m) {
                const uint32_t bit = __ffs(m) - 1;
                m &= m - 1;
                const int64_t xs = g0 + 64 * (int64_t)tid + 32 * (hs & 1) + bit;
                const uint64_t x = (uint64_t)xs;
                if (x >= a.len) continue;
                if (lds_verify) {                      // the tile's bytes (+ 16 of halo) are in LDS
                    const uint32_t o = (uint32_t)(xs - g0);
                    const uint8_t *pp = sp + (strand ? 16 : 0);
                    uint32_t dif = 0;
                    for (uint32_t bb = 0; bb < plen; ++bb) dif |= (uint32_t)(buf[o + bb] ^ pp[bb]);
                    if (dif || x + plen > a.len) continue;
                } else if (!gen_bytes_eq(a.data, a.len, x, strand ? a.RP : a.P, plen)) {
                    continue;
                }
                // the line holding x: r = newlines before x; a sequence line iff r = first + 4m
                const uint32_t b = 32 * (hs & 1) + bit;
                const uint64_t rl = r0 + (uint64_t)__popcll(nlm & ((1ull << b) - 1ull));
                if (rl < a.first || ((rl - a.first) & 3u) != 0) continue;
                const uint64_t m_ = (rl - a.first) >> 2;
                if (m_ >= a.n_lines) continue;
                // a candidate (position, sequence ordinal, strand): gen_fix_kernel
                // reads its line and keeps it iff the window fits
                Record r;
                r.pos = x;
                r.order = m_;
                r.len = k;
                r.strand = strand;
                const uint32_t qi = atomicAdd(&qn, 1u);
                if (qi < GC_Q) {
                    q[qi] = r;
                } else {                                   // (a crowded tile: straight to the list)
                    const unsigned long long gi = atomicAdd(a.rec_count, 1ull);
                    if (gi < a.rec_cap) a.recs[gi] = r;
                    else atomicOr(a.err, ERR_REC_OVERFLOW);
                }
            }
        }
        __syncthreads();                               // (buf and wsum are reused by the next tile)
        if (qn >= GC_Q / 2 || tile + 1 == t1) flush();
    }
}

// gen_cand_kernel's candidates -> records: the candidate's sequence line (one
// load per candidate, all in flight together -- inside the tile kernel this
// load held every wave with a candidate), the window inside it or dropped;
// the kept records compacted with one atomic per wave
__global__ __launch_bounds__(256) void gen_fix_kernel(const Record *__restrict__ cand, uint64_t n,
                                                      const SeqLine *__restrict__ lines, uint32_t k, uint32_t plen,
                                                      uint32_t pbits, Record *__restrict__ recs,
                                                      unsigned long long *rec_count, uint64_t rec_cap,
                                                      unsigned int *err) {
    // a workgroup takes a contiguous range of candidates in rounds of 256,
    // kept records queued in LDS, one atomic per GF_Q of them
    constexpr uint32_t GF_Q = 2048;
    __shared__ Record q[GF_Q];
    __shared__ uint32_t qn;
    __shared__ unsigned long long qbase;
    const uint32_t tid = threadIdx.x;
    const uint64_t per = ((n + gridDim.x - 1) / gridDim.x + 255) / 256 * 256;
    const uint64_t i0 = (uint64_t)blockIdx.x * per, i1 = i0 + per < n ? i0 + per : n;
    if (tid == 0) qn = 0;
    __syncthreads();
    auto flush = [&]() {
        const uint32_t nq = min(qn, GF_Q);
        if (tid == 0 && nq) qbase = atomicAdd(rec_count, (unsigned long long)nq);
        __syncthreads();
        for (uint32_t i = tid; i < nq; i += 256) {
            if (qbase + i < rec_cap) recs[qbase + i] = q[i];
            else atomicOr(err, ERR_REC_OVERFLOW);
        }
        __syncthreads();
        if (tid == 0) qn = 0;
        __syncthreads();
    };
    for (uint64_t b = i0; b < i1; b += 256) {
        const uint64_t i = b + tid;
        if (i < i1) {
            const Record c = cand[i];
            const SeqLine sl = lines[c.order];
            const uint64_t x = c.pos, end = sl.start + sl.len;
            Record r;
            r.len = k;
            r.strand = c.strand;
            bool keep = false;
            if (sl.len && x >= sl.start) {
                if (!c.strand) {
                    keep = x + k <= end;
                    r.order = (sl.line_index << (pbits + 1)) | (x - sl.start);
                    r.pos = x;
                } else {
                    keep = x + plen <= end && x + plen >= sl.start + k;
                    const uint64_t sp = x + plen - k - sl.start;           // window start in the line
                    r.order = (sl.line_index << (pbits + 1)) | (1ull << pbits) | (sl.len - k - sp);
                    r.pos = sl.start + sp;
                }
            }
            if (keep) q[atomicAdd(&qn, 1u)] = r;        // (<= 256 per round, flushed below)
        }
        __syncthreads();
        // one decision for the whole workgroup: read qn, then a barrier before
        // any wave can add to it in the next round (else the waves could take
        // different branches and meet different barriers)
        const uint32_t nq = qn;
        __syncthreads();
        if (nq > GF_Q - 256 || b + 256 >= i1) flush();
    }
}

__device__ __forceinline__ uint64_t gen_mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// two independent 64-bit hashes of each k-byte key, GEN_G lanes per key: lane
// l takes the key's 8-byte words l, l + GEN_G, ...; each word is mixed with its
// position (so the sums over the lanes are position-sensitive), the mixed
// words are summed over the lanes, and the sums finalised
__global__ __launch_bounds__(256) void gen_hash_kernel(const uint8_t *__restrict__ keys, uint64_t n, uint32_t k,
                                                       uint64_t seed, uint64_t *__restrict__ h1,
                                                       uint64_t *__restrict__ h2, uint32_t *__restrict__ idx) {
    const uint32_t lane = threadIdx.x & 63, sub = lane % GEN_G;
    const uint64_t nw = (uint64_t)gridDim.x * 4 * (64 / GEN_G);
    const uint64_t i0 = ((uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * (64 / GEN_G) + lane / GEN_G;
    const uint64_t nstep = (n + nw - 1) / nw;                 // (uniform trip count: the shuffles below)
    for (uint64_t t = 0; t < nstep; ++t) {
        const uint64_t i = i0 + t * nw;
        const bool live = i < n;
        const uint8_t *p = keys + (live ? i : 0) * k;
        uint64_t a = 0, b = 0;
        for (uint32_t j = 8 * sub; live && j < k; j += 8 * GEN_G) {
            uint64_t w = 0;
            const uint32_t m = k - j < 8 ? k - j : 8;
            for (uint32_t q = 0; q < m; ++q) w |= (uint64_t)p[j + q] << (8 * q);
            a += gen_mix(w ^ (seed + (uint64_t)j * 0x9E3779B97F4A7C15ull));
            b += gen_mix((w + 0x632BE59BD9B4E019ull) ^ (~seed + (uint64_t)j * 0xD6E8FEB86659FD93ull));
        }
#pragma unroll
        for (uint32_t d = GEN_G / 2; d >= 1; d >>= 1) {
            a += __shfl_xor(a, (int)d);
            b += __shfl_xor(b, (int)d);
        }
        if (live && sub == 0) {
            h1[i] = gen_mix(a ^ k);
            h2[i] = gen_mix(b + k);
            idx[i] = (uint32_t)i;
        }
    }
}

// after the sort by (h1, h2): a group starts where the hash changes; equal
// hashes with different bytes are a collision (flagged, the caller redoes the
// merge with another seed).  Heads record their sorted position by group.
__global__ __launch_bounds__(256) void gen_heads_kernel(const uint64_t *h1, const uint64_t *h2, const uint32_t *idx,
                                                        uint64_t n, const uint8_t *keys, uint32_t k, uint32_t *head,
                                                        unsigned int *collide) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        bool same = i > 0 && h1[i] == h1[i - 1] && h2[i] == h2[i - 1];
        if (same) {
            const uint8_t *x = keys + (uint64_t)idx[i] * k, *y = keys + (uint64_t)idx[i - 1] * k;
            bool eq = true;
            for (uint32_t b = 0; b < k && eq; ++b) eq = x[b] == y[b];
            if (!eq) atomicOr(collide, 1u);
        }
        head[i] = same ? 0u : 1u;
    }
}

// groups: gid (inclusive scan of the heads, 1-based) -> start of each group
__global__ __launch_bounds__(256) void gen_starts_kernel(const uint32_t *head, const uint32_t *gid, uint64_t n,
                                                         uint32_t *start) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        if (head[i]) start[gid[i] - 1] = (uint32_t)i;
        if (i == n - 1) start[gid[i]] = (uint32_t)n;
    }
}

// GEN_G lanes per group: its key (the head's bytes, copied by the lanes), the
// count sum and the min first (lanes stride over the group's members)
__global__ __launch_bounds__(256) void gen_reduce_kernel(const uint32_t *__restrict__ start, uint64_t ng,
                                                         const uint32_t *__restrict__ idx,
                                                         const uint8_t *__restrict__ keys,
                                                         const uint64_t *__restrict__ cnt,
                                                         const uint64_t *__restrict__ first, uint32_t k,
                                                         uint8_t *__restrict__ okeys, uint64_t *__restrict__ ocnt,
                                                         uint64_t *__restrict__ ofirst) {
    const uint32_t lane = threadIdx.x & 63, sub = lane % GEN_G;
    const uint64_t nw = (uint64_t)gridDim.x * 4 * (64 / GEN_G);
    const uint64_t g0 = ((uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * (64 / GEN_G) + lane / GEN_G;
    const uint64_t nstep = (ng + nw - 1) / nw;                // (uniform trip count: the shuffles below)
    for (uint64_t t = 0; t < nstep; ++t) {
        const uint64_t g = g0 + t * nw;
        const bool live = g < ng;
        const uint32_t s0 = live ? start[g] : 0u, s1 = live ? start[g + 1] : 0u;
        uint64_t c = 0, f = ~0ull;
        for (uint32_t i = s0 + sub; i < s1; i += GEN_G) {
            const uint32_t j = idx[i];
            c += cnt[j];
            f = min(f, first[j]);
        }
#pragma unroll
        for (uint32_t d = GEN_G / 2; d >= 1; d >>= 1) {
            c += __shfl_xor(c, (int)d);
            f = min(f, (uint64_t)__shfl_xor(f, (int)d));
        }
        if (!live) continue;
        const uint8_t *src = keys + (uint64_t)idx[s0] * k;
        uint8_t *o = okeys + g * k;
        for (uint32_t b = sub; b < k; b += GEN_G) o[b] = src[b];
        if (sub == 0) {
            ocnt[g] = c;
            ofirst[g] = f;
        }
    }
}

// ---------------------------------------------------------------------------
// dense-hit path: windows of sequence lines straight into rank slots
// ---------------------------------------------------------------------------
// 2-bit code of the k bytes at p (first base most significant); *exotic if a
// byte is not A/C/G/T.  `safe`: p + k + 4 stays inside the buffer (word loads).
__device__ __forceinline__ uint64_t window_code(const uint8_t *p, uint32_t k, bool safe, bool *exotic) {
    uint64_t code = 0;
    bool ex = false;
    if (safe && k <= (uint32_t)KMAX_DENSE) {
        // every word of the window loaded before any is used (one memory
        // round trip per window, not one per word: the dense-hit path's
        // windows kernel was bound by that chain)
        const uintptr_t ad = (uintptr_t)p;
        const uint32_t *wp = (const uint32_t *)(ad & ~(uintptr_t)3);
        const uint32_t sh = (uint32_t)(ad & 3);
        constexpr uint32_t NWMAX = KMAX_DENSE / 4 + 1;
        const uint32_t nwk = (k + 3) / 4;
        uint32_t wv[NWMAX];
#pragma unroll
        for (uint32_t i = 0; i < NWMAX; ++i) wv[i] = i <= nwk ? wp[i] : 0u;
#pragma unroll
        for (uint32_t i = 0; i < NWMAX - 1; ++i) {
            const uint32_t b = 4 * i;
            if (b >= k) break;
            const uint32_t x = align4(wv[i + 1], wv[i], sh);
            const uint32_t nb = k - b >= 4 ? 4u : k - b;
            const uint32_t mk = nb == 4 ? 0xFFFFFFFFu : ((1u << (8 * nb)) - 1u);
            const uint32_t c = ((x >> 1) ^ (x >> 2)) & 0x03030303u;
            ex |= ((__builtin_amdgcn_perm(0u, 0x54474341u, c) ^ x) & mk) != 0;
            const uint32_t pk = ((c & 3u) << 6) | (((c >> 8) & 3u) << 4) | (((c >> 16) & 3u) << 2) | ((c >> 24) & 3u);
            code = (code << (2 * nb)) | (pk >> (2 * (4 - nb)));
        }
    } else if (safe) {
        const uintptr_t ad = (uintptr_t)p;
        const uint32_t *wp = (const uint32_t *)(ad & ~(uintptr_t)3);
        const uint32_t sh = (uint32_t)(ad & 3);
        uint32_t cur = wp[0];
#pragma unroll 1
        for (uint32_t b = 0, i = 0; b < k; b += 4, ++i) {
            const uint32_t nxt = wp[i + 1];
            const uint32_t x = align4(nxt, cur, sh);
            cur = nxt;
            const uint32_t nb = k - b >= 4 ? 4u : k - b;
            const uint32_t mk = nb == 4 ? 0xFFFFFFFFu : ((1u << (8 * nb)) - 1u);
            const uint32_t c = ((x >> 1) ^ (x >> 2)) & 0x03030303u;
            ex |= ((__builtin_amdgcn_perm(0u, 0x54474341u, c) ^ x) & mk) != 0;
            const uint32_t pk = ((c & 3u) << 6) | (((c >> 8) & 3u) << 4) | (((c >> 16) & 3u) << 2) | ((c >> 24) & 3u);
            code = (code << (2 * nb)) | (pk >> (2 * (4 - nb)));
        }
    } else {
#pragma unroll 1
        for (uint32_t b = 0; b < k; ++b) {
            const uint32_t x = p[b];
            const uint32_t c = ((x >> 1) ^ (x >> 2)) & 3u;
            ex |= x != ((0x54474341u >> (8 * c)) & 0xFFu);
            code = (code << 2) | c;
        }
    }
    *exotic = ex;
    return code;
}

__device__ __forceinline__ void win_record(const WinArgs &a, uint64_t order, uint64_t pos, uint32_t strand,
                                           uint32_t len) {
    const unsigned long long n = atomicAdd(a.rec_count, 1ull);
    if (n < a.rec_cap) {
        Record rec;
        rec.order = order;
        rec.pos = pos;
        rec.len = len;
        rec.strand = strand;
        a.recs[n] = rec;
    } else {
        atomicOr(a.err, ERR_REC_OVERFLOW);
    }
}

// (an invalid key's order is never read -- compaction, exchange and the heads
// read orders at valid ranks only -- so it is not written: at C2 size with a
// 2-base prefix that skips 20 GB of stores)
__device__ __forceinline__ void win_place(const WinArgs &a, uint64_t rank, uint64_t key, uint64_t order) {
    if (a.rkey32) a.rkey32[rank] = (uint32_t)key;
    else a.rkey[rank] = key;
    if (key != a.invalid_key) a.rord[rank] = order;
}

// ---- sequence lines of a chunk without look-back (dense-hit path) ----
// pass 1: '\n' count per 16 KiB tile; pass 2 (after a scan): the chunk-relative
// position of every '\n', in order; then sequence line m is read off the
// newline array directly (line li runs from NL[li-li0-1]+1 to NL[li-li0]).
__device__ __forceinline__ uint32_t thread_nl_flags(const uint8_t *data, uint64_t len, int64_t g, uint32_t (&z)[16],
                                                    uint32_t *orall) {
    uint32_t cnt = 0, o = 0;
    if ((uint64_t)g + 64 <= len) {
        const uint4 *src = (const uint4 *)(data + g);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint4 x = src[j];
            o |= x.x | x.y | x.z | x.w;
            z[4 * j] = nl_flags(x.x);
            z[4 * j + 1] = nl_flags(x.y);
            z[4 * j + 2] = nl_flags(x.z);
            z[4 * j + 3] = nl_flags(x.w);
        }
    } else {
#pragma unroll 1
        for (int j = 0; j < 16; ++j) {
            uint32_t x = 0;
            for (int b = 0; b < 4; ++b) {
                const uint64_t p = (uint64_t)g + 4 * j + b;
                x |= (uint32_t)(p < len ? data[p] : 0u) << (8 * b);
            }
            o |= x;
            z[j] = nl_flags(x);
        }
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) cnt += __popc(z[j]);
    *orall = o;
    return cnt;
}

__global__ __launch_bounds__(256) void nl_count_kernel(const uint8_t *data, uint64_t len, uint32_t *tcount,
                                                       unsigned int *err) {
    __shared__ uint32_t ws[4];
    uint32_t z[16], o = 0;
    const int64_t g = (int64_t)blockIdx.x * TILE + 64 * threadIdx.x;
    const uint32_t cnt = (uint64_t)g < len ? thread_nl_flags(data, len, g, z, &o) : 0u;
    if (o & 0x80808080u) atomicOr(err, ERR_NONASCII);
    const uint32_t incl = wave_incl_sum(cnt);
    if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = incl;
    __syncthreads();
    if (threadIdx.x == 0) tcount[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ __launch_bounds__(256) void nl_write_kernel(const uint8_t *data, uint64_t len, const uint64_t *tbase,
                                                       uint64_t *nl) {
    __shared__ uint32_t ws[4];
    uint32_t z[16], orall;
    const int64_t g = (int64_t)blockIdx.x * TILE + 64 * threadIdx.x;
    const uint32_t cnt = (uint64_t)g < len ? thread_nl_flags(data, len, g, z, &orall) : 0u;
    const uint32_t incl = wave_incl_sum(cnt);
    const int wid = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 63) ws[wid] = incl;
    __syncthreads();
    uint64_t o = tbase[blockIdx.x] + incl - cnt;
    for (int w = 0; w < wid; ++w) o += ws[w];
    if (!cnt) return;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        uint32_t m = z[j];
        while (m) {
            const int b = __ffs(m) - 1;          // bit 7 of a byte
            m &= m - 1;
            nl[o++] = (uint64_t)g + 4 * j + (b >> 3);
        }
    }
}

// '\n' count per tile AND its tile-relative positions (u16) in the tile's
// fixed slot array of `cap` entries, in one pass: the sequence lines are then
// found from the slots after a scan of the counts, without a second pass over
// the input.  A tile with more than `cap` newlines (lines shorter than
// TILE / cap bytes on average) sets ERR_LINE_OVERFLOW: the host then writes
// the global position array the two-pass way (nl_write_kernel).
__global__ __launch_bounds__(256) void nl_slots_kernel(const uint8_t *data, uint64_t len, uint32_t cap,
                                                       uint16_t *slots, uint32_t *tcount, unsigned int *err) {
    __shared__ uint32_t ws[4];
    uint32_t z[16], o = 0;
    const int64_t g = (int64_t)blockIdx.x * TILE + 64 * threadIdx.x;
    const uint32_t cnt = (uint64_t)g < len ? thread_nl_flags(data, len, g, z, &o) : 0u;
    if (o & 0x80808080u) atomicOr(err, ERR_NONASCII);
    const uint32_t incl = wave_incl_sum(cnt);
    const int wid = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 63) ws[wid] = incl;
    __syncthreads();
    const uint32_t total = ws[0] + ws[1] + ws[2] + ws[3];
    if (threadIdx.x == 0) {
        tcount[blockIdx.x] = total;
        if (total > cap) atomicOr(err, ERR_LINE_OVERFLOW);
    }
    if (!cnt || total > cap) return;
    uint32_t o2 = incl - cnt;
    for (int w = 0; w < wid; ++w) o2 += ws[w];
    uint16_t *dst = slots + (uint64_t)blockIdx.x * cap;
    const uint32_t t0 = 64 * threadIdx.x;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        uint32_t m = z[j];
        while (m) {
            const int b = __ffs(m) - 1;          // bit 7 of a byte
            m &= m - 1;
            dst[o2++] = (uint16_t)(t0 + 4 * j + (b >> 3));
        }
    }
}

// Sequence lines from the tile slots, one wave per tile: newline r
// (chunk-relative, r = tbase[tile] + i) ends line r, which is sequence
// ordinal (r - first) / 4 when r - first is a multiple of 4; its start is the
// previous newline + 1 -- slot i - 1, or the last newline of the nearest
// earlier tile that has one (0: the chunk's first line).  The open trailing
// segment (line n_nl, no newline after it) ends at len.
__device__ __forceinline__ uint64_t nl_before_tile(const uint16_t *slots, const uint32_t *tcount, uint32_t cap,
                                                   int64_t tile) {
    for (int64_t u = tile - 1; u >= 0; --u) {
        const uint32_t n = tcount[u];
        if (n) return (uint64_t)u * TILE + slots[(uint64_t)u * cap + n - 1] + 1;
    }
    return 0;
}

__device__ __forceinline__ void put_seq_line(uint64_t st, uint64_t en, uint64_t li, uint32_t k, uint32_t step,
                                             uint32_t lsh, uint64_t maxrel, SeqLine *line, uint64_t *wc,
                                             unsigned int *err) {
    SeqLine sl;
    sl.line_index = li;
    sl.start = st;                 // (also without windows: the starts stay ascending -- gen_cand_kernel searches them)
    sl.len = 0;
    uint64_t w2 = 0;
    const uint64_t L = en > st ? en - st : 0;
    if (L > 1 && L >= k) {
        sl.len = L;
        const uint64_t W = L - k + 1;
        // (err null: no order key, no limit)
        if (err && (W - 1 > maxrel || (li >> (lsh - 1)))) atomicOr(err, ERR_LINE_TOO_LONG);
        w2 = 2 * ((W + step - 1) / step);
    }
    *line = sl;
    *wc = w2;
}

__global__ __launch_bounds__(256) void seq_lines_slots_kernel(const uint16_t *slots, const uint32_t *tcount,
                                                              const uint64_t *tbase, uint32_t n_tiles, uint32_t cap,
                                                              uint64_t len, uint64_t li0, uint64_t first,
                                                              uint64_t n_nl, uint64_t n_seq, uint32_t k,
                                                              uint32_t step, SeqLine *lines, uint64_t *wcount,
                                                              unsigned int *err, uint64_t maxrel) {
    const uint32_t lsh = 64 - __popcll(maxrel);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t tile = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tile >= n_tiles) return;
    const uint32_t n = tcount[tile];
    const uint64_t rb = tbase[tile];
    const uint16_t *src = slots + (uint64_t)tile * cap;
    const uint64_t t0 = (uint64_t)tile * TILE;
    for (uint32_t i = lane; i < n; i += 64) {
        const uint64_t r = rb + i;
        if (r < first || ((r - first) & 3) != 0) continue;
        const uint64_t en = t0 + src[i];
        const uint64_t st = i ? t0 + src[i - 1] + 1 : nl_before_tile(slots, tcount, cap, tile);
        const uint64_t m = (r - first) >> 2;
        put_seq_line(st, en, li0 + r, k, step, lsh, maxrel, lines + m, wcount + m, err);
    }
    if (tile == n_tiles - 1 && lane == 0 && n_seq && first + 4 * (n_seq - 1) == n_nl) {
        const uint64_t st = n ? t0 + src[n - 1] + 1 : nl_before_tile(slots, tcount, cap, tile);
        put_seq_line(st, len, li0 + n_nl, k, step, lsh, maxrel, lines + n_seq - 1, wcount + n_seq - 1, err);
    }
}

// sequence ordinal m -> SeqLine (len 0: no windows) and its window count 2W
__global__ __launch_bounds__(256) void seq_lines_kernel(const uint64_t *nl, uint64_t n_nl, uint64_t len,
                                                        uint64_t li0, uint64_t n_seq, uint32_t k, uint32_t step,
                                                        SeqLine *lines,
                                                        uint64_t *wcount, unsigned int *err, uint64_t maxrel) {
    const uint32_t lsh = 64 - __popcll(maxrel);            // line index bits: 63 - pbits
    const uint64_t first = (1u - (uint32_t)li0) & 3u;      // first sequence line, relative to li0
    for (uint64_t m = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; m < n_seq; m += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = first + 4 * m;                  // line index - li0
        SeqLine sl;
        sl.line_index = li0 + r;
        sl.start = 0;
        sl.len = 0;
        uint64_t w2 = 0;
        if (r <= n_nl) {
            const uint64_t st = r == 0 ? 0 : nl[r - 1] + 1;
            const uint64_t en = r < n_nl ? nl[r] : len;    // (r == n_nl: the open trailing segment)
            const uint64_t L = en > st ? en - st : 0;
            sl.start = st;                                 // (ascending starts, as put_seq_line)
            if (L > 1 && L >= k) {
                sl.len = L;
                const uint64_t W = L - k + 1;
                // (err null: no order key, no limit)
                if (err && (W - 1 > maxrel || (sl.line_index >> (lsh - 1)))) atomicOr(err, ERR_LINE_TOO_LONG);
                w2 = 2 * ((W + step - 1) / step);
            }
        }
        lines[m] = sl;
        wcount[m] = w2;
    }
}

__global__ void pos_after_kernel(StreamPos *pos, uint64_t lines, const uint8_t *data, uint64_t len,
                                 unsigned long long *ends_open) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        pos->lines = lines;
        pos->ends_open = (len > 0 && data[len - 1] != '\n') ? 1 : 0;
        *ends_open = pos->ends_open;
    }
}

// one workgroup per sequence line (grid-stride), one thread per forward
// position s: the forward window at s when s % step == 0 and the reverse
// strand's window at p = W - 1 - s when p % step == 0.  lib/kmers.js:88-100
// steps through the line and through its complement from their own starts,
// W times (index j, ini = j * step): past L - k the substring is cut short,
// past L it is "" -- the short keys become records, the empty ones a count.
// Order keys: step 1, line | strand | (strand ? maxrel - s : s) as on the
// tile path; step > 1, line | strand | j (the loop index) on both strands.
// One WAVE per sequence line for reads (4 lines in flight per workgroup, the
// next line's descriptor loaded while the current one is written: a
// workgroup per line left half its lanes idle on 150-byte reads and walked
// its lines one dependent chain at a time, 21.8 ms at C2 size, prefix AT);
// one WORKGROUP per line when the lines are long (contigs: a few thousand
// lines would leave most of the chip idle with a wave each)
__global__ __launch_bounds__(256) void windows_packed_kernel(WinArgs a) {
    const uint32_t k = a.k, plen = a.plen;
    const uint32_t tailbits = 2 * (k - plen);
    const bool bl = a.block_lines != 0;
    const uint32_t lane = bl ? threadIdx.x : (threadIdx.x & 63), LW = bl ? 256u : 64u;
    const uint64_t nwv = bl ? (uint64_t)gridDim.x : (uint64_t)gridDim.x * 4;
    uint64_t li = bl ? (uint64_t)blockIdx.x : (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    SeqLine nxt = {0, 0, 0};
    if (li < a.n_lines) nxt = a.lines[li];
    for (; li < a.n_lines; li += nwv) {
        const SeqLine sl = nxt;                  // dense by sequence ordinal
        if (li + nwv < a.n_lines) nxt = a.lines[li + nwv];
        if (sl.len == 0) continue;
        const uint64_t W = sl.len - k + 1;
        const uint64_t maxrel = (1ull << a.pbits) - 1ull;
        if (W - 1 > maxrel) continue;            // reported by seq_lines_kernel
        const uint64_t base = a.out_base + a.wbase[li];
        const uint64_t lo = sl.line_index << (a.pbits + 1);
        const uint32_t step = a.step;
        const uint64_t Ws = (W + step - 1) / step;   // windows per strand
        for (uint64_t s = lane; s < W; s += LW) {
            const bool fw = step == 1 || s % step == 0, rv = step == 1 || (W - 1 - s) % step == 0;
            if (!fw && !rv) continue;
            const uint64_t pos = sl.start + s;
            bool exotic;
            const uint64_t code = window_code(a.data + pos, k, pos + k + 4 <= a.len, &exotic);
            const uint64_t rc = revcomp_code(code, k);
            const uint64_t of = lo | (step == 1 ? s : s / step);
            const uint64_t orr = lo | (1ull << a.pbits) | (step == 1 ? maxrel - s : (W - 1 - s) / step);
            // prefix tests on the codes: a non-ACGT byte in the prefix bases never
            // matches (its code aliases, so exotic windows re-check the bytes)
            bool mf = plen == 0 || (code >> tailbits) == a.pcode;
            bool mr = plen == 0 || (rc >> tailbits) == a.pcode;
            if (exotic && plen) {
                for (uint32_t b = 0; b < plen; ++b) {
                    const uint32_t cf = (uint32_t)(a.pcode >> (2 * (plen - 1 - b))) & 3u;
                    const uint8_t xf = a.data[pos + b];
                    mf = mf && xf == (uint8_t)((0x54474341u >> (8 * cf)) & 0xFFu);
                    const uint32_t cr = (uint32_t)(a.rcode >> (2 * (plen - 1 - b))) & 3u;
                    const uint8_t xr = a.data[pos + k - plen + b];
                    mr = mr && xr == (uint8_t)((0x54474341u >> (8 * cr)) & 0xFFu);
                }
            }
            const uint64_t rf = base + s / step, rr = base + Ws + (W - 1 - s) / step;
            if (fw) win_place(a, rf, (mf && !exotic) ? (code & a.smask) : a.invalid_key, of);
            if (rv) win_place(a, rr, (mr && !exotic) ? (rc & a.smask) : a.invalid_key, orr);
            if (exotic) {
                if (mf && fw) win_record(a, of, pos, 0, k);
                if (mr && rv) win_record(a, orr, pos, 1, k);
            }
        }
        if (step == 1 || Ws >= W) continue;
        // indices j in [Ws, W) of each strand: p = j * step > L - k
        const uint64_t L = sl.len, ntail = W - Ws;
        for (uint64_t t = lane; t < 2 * ntail; t += LW) {
            const uint32_t strand = t >= ntail ? 1u : 0u;
            const uint64_t j = Ws + (strand ? t - ntail : t), p = j * step;
            if (p >= L) continue;                    // "": counted below
            const uint64_t len = L - p;              // (< k)
            if (len < plen) continue;
            bool ok = true;
            for (uint32_t b = 0; b < plen && ok; ++b) {
                const uint8_t c = strand ? comp_byte(a.data[sl.start + L - 1 - p - b]) : a.data[sl.start + p + b];
                ok = c == a.P[b];
            }
            // the reverse strand's S[p, L) is rc of the line's first L - p bytes
            if (ok) win_record(a, lo | ((uint64_t)strand << a.pbits) | j, sl.start + (strand ? 0 : p), strand,
                               (uint32_t)len);
        }
        if (plen == 0 && lane == 0) {
            const uint64_t j0 = (L + step - 1) / step;   // first index whose substring is ""
            if (j0 < W) {
                atomicAdd(&a.empty[0], (unsigned long long)(2 * (W - j0)));
                atomicMin(&a.empty[1], (unsigned long long)(lo | j0));
            }
        }
    }
}

// ---------------------------------------------------------------------------
// result materialisation
// ---------------------------------------------------------------------------
// Cross entries (in natural-slot order) sorted by order key: the i-th
// smallest order takes the i-th natural slot.  Large lists: radix-sorted on
// the host side of the pipeline, then cross_scatter_kernel.
__device__ __forceinline__ void put_key(uint64_t *rkey, uint32_t *rkey32, uint64_t slot, uint64_t key) {
    if (rkey32) rkey32[slot] = (uint32_t)key;
    else rkey[slot] = key;
}

__global__ __launch_bounds__(256) void cross_scatter_kernel(const uint32_t *slot, const uint64_t *ord,
                                                            const uint64_t *key, uint64_t n, uint64_t *rkey,
                                                            uint32_t *rkey32, uint64_t *rord) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t sl = slot[i];
        put_key(rkey, rkey32, sl, key[i]);
        rord[sl] = ord[i];
    }
}

// Small lists (n <= XSMALL): one workgroup, bitonic sort of (order, index) in
// LDS, then the scatter.
constexpr uint32_t XSMALL = 16384;
__global__ __launch_bounds__(1024) void cross_sort_small_kernel(const uint32_t *slot, const uint64_t *ord,
                                                                const uint64_t *key, uint32_t n, uint64_t *rkey,
                                                                uint32_t *rkey32, uint64_t *rord) {
    __shared__ uint64_t so[XSMALL];
    __shared__ uint16_t si[XSMALL];
    uint32_t N = 2;
    while (N < n) N <<= 1;
    for (uint32_t i = threadIdx.x; i < N; i += blockDim.x) {
        so[i] = i < n ? ord[i] : ~0ull;
        si[i] = (uint16_t)i;
    }
    __syncthreads();
    for (uint32_t k = 2; k <= N; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = threadIdx.x; i < N; i += blockDim.x) {
                const uint32_t p = i ^ j;
                if (p > i) {
                    const uint64_t x = so[i], y = so[p];
                    const bool asc = (i & k) == 0;
                    if ((x > y) == asc) {
                        so[i] = y;
                        so[p] = x;
                        const uint16_t t = si[i];
                        si[i] = si[p];
                        si[p] = t;
                    }
                }
            }
            __syncthreads();
        }
    }
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t sl = slot[i];
        put_key(rkey, rkey32, sl, key[si[i]]);
        rord[sl] = so[i];
    }
}

// Common case (no long lines, no overflowed tile): the cross list is already
// ordered by line, and one line's entries come from at most two tiles
// (<= 2 * HMAX).  One thread per line segment: insertion sort by order key,
// then the scatter to the natural slots.
__global__ __launch_bounds__(256) void cross_segsort_kernel(uint64_t *ord, uint64_t *key, const uint32_t *slot,
                                                            uint64_t n, uint64_t *rkey, uint32_t *rkey32,
                                                            uint64_t *rord, uint32_t lsh) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t line = ord[i] >> lsh;     // (the line bits of a segment never change while it is sorted)
        if (i > 0 && (ord[i - 1] >> lsh) == line) continue;
        uint64_t e = i + 1;
        while (e < n && (ord[e] >> lsh) == line) ++e;
        for (uint64_t j = i + 1; j < e; ++j) {
            const uint64_t v = ord[j], kv = key[j];
            uint64_t p = j;
            while (p > i && ord[p - 1] > v) {
                ord[p] = ord[p - 1];
                key[p] = key[p - 1];
                --p;
            }
            ord[p] = v;
            key[p] = kv;
        }
        for (uint64_t j = i; j < e; ++j) {
            const uint32_t sl = slot[j];
            put_key(rkey, rkey32, sl, key[j]);
            rord[sl] = ord[j];
        }
    }
}

// End of the key group starting at sorted index i: galloping then binary search.
template <typename K>
__device__ __forceinline__ uint64_t group_end(const K *skey, uint64_t i, uint64_t n, K key) {
    uint64_t lo = i, step = 1, hi = n;
    for (;;) {
        const uint64_t p = lo + step;
        if (p >= n || skey[p] != key) {
            hi = p < n ? p : n;
            break;
        }
        lo = p;
        step <<= 1;
    }
    while (hi - lo > 1) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (skey[mid] == key) lo = mid;
        else hi = mid;
    }
    return hi;
}

// After the stable key sort (payload = rank): the first element of each key
// group has the smallest rank = the key's first occurrence.  Every rank gets
// its record written (srank is a permutation), so no clearing pass is needed.
template <typename K>
__global__ __launch_bounds__(256) void heads_kernel(const K *skey, const uint32_t *srank, uint64_t n, K invalid_key,
                                                    const uint64_t *rcnt, HeadRec *hrec, uint32_t *hcnt) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const K k = skey[i];
        HeadRec v;
        v.key = 0;
        v.count = 0;
        if (k != invalid_key && (i == 0 || skey[i - 1] != k)) {
            const uint64_t e = group_end(skey, i, n, k);
            uint64_t cnt = e - i;
            if (rcnt) {
                cnt = 0;
                for (uint64_t j = i; j < e; ++j) cnt += rcnt[srank[j]];
            }
            v.key = k;
            v.count = cnt;
        }
        const uint32_t r = srank[i];
        hrec[r] = v;
        hcnt[r] = v.count ? 1u : 0u;
    }
}

// Sort finish without per-entry counts: hcnt is prefilled with 1 (every rank
// a singleton head), so only members of key groups of >= 2 and invalid keys
// are scattered: the head (smallest rank, stable sort) gets the group size,
// the others 0.  Where keys are mostly unique (k=31, no prefix) almost
// nothing is written at random.
template <typename K>
__global__ __launch_bounds__(256) void heads_sparse_kernel(const K *skey, const uint32_t *srank, uint64_t n,
                                                           K invalid_key, uint32_t *hcnt) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const K k = skey[i];
        const bool dp = i > 0 && skey[i - 1] == k;
        const bool dn = i + 1 < n && skey[i + 1] == k;
        if (k != invalid_key && !dp && !dn) continue;
        uint32_t v = 0;
        if (k != invalid_key && !dp) v = (uint32_t)(group_end(skey, i, n, k) - i);
        hcnt[srank[i]] = v;
    }
}

// ---------------------------------------------------------------------------
// Wide keys (2(k - |P|) >= 64 bits, k <= 64): two words per key, hi in a
// parallel array.  The rank finish sorts (lo, rank) and then, stably,
// (hi, rank) -- LSD order: by (hi, lo), ranks ascending within a key.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void gather_u64_kernel(const uint64_t *src, const uint32_t *idx, uint64_t n,
                                                         uint64_t *dst) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        dst[i] = src[idx[i]];
}

__global__ __launch_bounds__(256) void gather_u32_kernel(const uint32_t *src, const uint32_t *idx, uint64_t n,
                                                         uint32_t *dst) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        dst[i] = src[idx[i]];
}

// after apply_cross the cross slots hold their entry's index: put the key there
__global__ __launch_bounds__(256) void cross_wide_fix_kernel(const uint32_t *xslot, uint64_t n, const uint64_t *xkeyl,
                                                             const uint64_t *xkeyh, uint64_t *rkey, uint64_t *rkeyh) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t sl = xslot[i];
        const uint64_t x = rkey[sl];
        rkey[sl] = xkeyl[x];
        rkeyh[sl] = xkeyh[x];
    }
}

// heads_sparse_kernel over (hi, lo) pairs: hcnt prefilled with 1; members of
// groups of >= 2 and invalid keys (hi == invalid_hi) are written
__global__ __launch_bounds__(256) void heads_wide_kernel(const uint64_t *shi, const uint64_t *slo,
                                                         const uint32_t *srank, uint64_t n, uint64_t invalid_hi,
                                                         uint32_t *hcnt) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t h = shi[i], l = slo[i];
        const bool dp = i > 0 && shi[i - 1] == h && slo[i - 1] == l;
        const bool dn = i + 1 < n && shi[i + 1] == h && slo[i + 1] == l;
        const bool inv = h == invalid_hi;
        if (!inv && !dp && !dn) continue;
        uint32_t v = 0;
        if (!inv && !dp) {
            uint64_t e = i + 1;                  // (groups are short: hits of one k-mer)
            while (e < n && shi[e] == h && slo[e] == l) ++e;
            v = (uint32_t)(e - i);
        }
        hcnt[srank[i]] = v;
    }
}

// ---------------------------------------------------------------------------
// Bucket finish (u32 keys of <= 24 bits): instead of sorting, partition the
// ranked hits by key >> BKT_LOW into <= 2048 buckets (LDS-privatised
// histogram, scan, scatter), then one workgroup per bucket keeps an LDS table
// of 2^BKT_LOW keys: min rank (= first occurrence) and count, and writes the
// head record of every key present at its first-occurrence rank.
// ---------------------------------------------------------------------------
constexpr uint32_t BKT_EPB = 4096;           // elements per partition block

__global__ __launch_bounds__(256) void bucket_hist_kernel(const uint32_t *key, uint64_t n, uint32_t invalid,
                                                          uint32_t shift, uint32_t nb, uint32_t nblk,
                                                          uint32_t *H, uint32_t *hcnt) {
    __shared__ uint32_t hist[BKT_MAX];
    for (uint32_t b = threadIdx.x; b < nb; b += 256) hist[b] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * BKT_EPB;
    // clear the head counts of this block's ranks (bucket_heads sets the heads')
    for (uint32_t j = 4 * threadIdx.x; j < BKT_EPB; j += 4 * 256) {
        const uint64_t i = base + j;
        if (i + 4 <= n) *(uint4 *)(hcnt + i) = make_uint4(0, 0, 0, 0);
        else for (uint64_t t = i; t < n; ++t) hcnt[t] = 0;
    }
#pragma unroll 4
    for (uint32_t j = threadIdx.x; j < BKT_EPB; j += 256) {
        const uint64_t i = base + j;
        if (i < n) {
            const uint32_t k = key[i];
            if (k != invalid) atomicAdd(&hist[k >> shift], 1u);
        }
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += 256) H[(uint64_t)b * nblk + blockIdx.x] = hist[b];
}

// Offsets of the partition (one launch, no library scan): workgroup b scans
// bucket b's row of block counts (H[b * nblk + blk] -> Hs, bucket-relative)
// and publishes the bucket's total; the last workgroup to finish turns the
// totals into the buckets' starts (bbase[nb] = all keys).  The ticket add is
// acquire-release at agent scope (HIP memory model); the totals are read
// back by atomics.
__global__ __launch_bounds__(256) void bucket_offsets_kernel(const uint32_t *H, uint32_t nb, uint32_t nblk,
                                                             uint32_t *Hs, uint32_t *btot, uint32_t *bbase,
                                                             unsigned int *ticket) {
    __shared__ uint32_t ws[4];
    __shared__ bool last;
    const uint32_t b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t per = (nblk + 255) / 256, j0 = tid * per, j1 = min(j0 + per, nblk);
    const uint32_t *row = H + (uint64_t)b * nblk;
    uint32_t sum = 0;
    for (uint32_t j = j0; j < j1; ++j) sum += row[j];
    const uint32_t incl = wave_incl_sum(sum);
    if (lane == 63) ws[wid] = incl;
    __syncthreads();
    uint32_t pre = incl - sum;
    for (uint32_t w = 0; w < wid; ++w) pre += ws[w];
    uint32_t *out = Hs + (uint64_t)b * nblk;
    for (uint32_t j = j0; j < j1; ++j) {
        const uint32_t v = row[j];
        out[j] = pre;
        pre += v;
    }
    if (tid == 0) {
        // release (the total reaches memory before the ticket announces it) and
        // acquire (the last workgroup sees every earlier total) at agent scope:
        // the compiler emits the L2 writeback / invalidate the XCDs need
        __hip_atomic_store(btot + b, ws[0] + ws[1] + ws[2] + ws[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == nb - 1;
    }
    __syncthreads();
    if (!last) return;
    // bucket starts: nb <= BKT_MAX totals, 8 per thread
    uint32_t v[BKT_MAX / 256], s = 0;
#pragma unroll
    for (uint32_t u = 0; u < BKT_MAX / 256; ++u) {
        const uint32_t q = tid * (BKT_MAX / 256) + u;
        // (read by an atomic, at the memory side: an agent-scope load may be
        // served by this XCD's L2, which can hold the line from an earlier call)
        v[u] = q < nb ? __hip_atomic_fetch_add(btot + q, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        s += v[u];
    }
    const uint32_t inc2 = wave_incl_sum(s);
    __syncthreads();
    if (lane == 63) ws[wid] = inc2;
    __syncthreads();
    uint32_t p = inc2 - s;
    for (uint32_t w = 0; w < wid; ++w) p += ws[w];
#pragma unroll
    for (uint32_t u = 0; u < BKT_MAX / 256; ++u) {
        const uint32_t q = tid * (BKT_MAX / 256) + u;
        if (q < nb) bbase[q] = p;
        p += v[u];
    }
    if (tid == 255) bbase[nb] = p;
    if (tid == 0) *ticket = 0;
}

// (race probes for bucket_scatter_kernel, in experiment builds only: see the
// Makefile's probes target and tools/bkt_race_probe.py)
#if defined(KMERHIP_EXPERIMENTS) && defined(KMERHIP_PROBE_BKT_DELAY)
#define BKT_PROBE_DELAY 1
#else
#define BKT_PROBE_DELAY 0
#endif
#if defined(KMERHIP_EXPERIMENTS) && defined(KMERHIP_PROBE_BKT_NOFIX)
#define BKT_PROBE_NOFIX 1
#else
#define BKT_PROBE_NOFIX 0
#endif

// Scatter with the block's elements first grouped by bucket in LDS, so that
// each bucket's run goes out as one contiguous (coalesced) piece.
__global__ __launch_bounds__(256) void bucket_scatter_kernel(const uint32_t *key, uint64_t n, uint32_t invalid,
                                                             uint32_t shift, uint32_t nb, uint32_t nblk,
                                                             const uint32_t *Hs, const uint32_t *bbase, uint16_t *pkey,
                                                             uint32_t *prank) {
    __shared__ uint32_t cnt[BKT_MAX];          // per bucket: count, then local start
    __shared__ uint32_t skey[BKT_EPB];
    __shared__ uint32_t srank[BKT_EPB];
    __shared__ uint32_t wtot[4];
    for (uint32_t b = threadIdx.x; b < nb; b += 256) cnt[b] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * BKT_EPB;
    uint32_t kk[BKT_EPB / 256], li[BKT_EPB / 256];
#pragma unroll
    for (uint32_t u = 0; u < BKT_EPB / 256; ++u) {
        const uint64_t i = base + u * 256 + threadIdx.x;
        kk[u] = i < n ? key[i] : invalid;
        li[u] = kk[u] != invalid ? atomicAdd(&cnt[kk[u] >> shift], 1u) : 0u;
    }
    __syncthreads();
    // exclusive scan of the bucket counts (nb <= BKT_MAX, <= 8 per thread)
    uint32_t loc[BKT_MAX / 256], sum = 0;
#pragma unroll
    for (uint32_t u = 0; u < BKT_MAX / 256; ++u) {
        const uint32_t b = threadIdx.x * (BKT_MAX / 256) + u;
        loc[u] = b < nb ? cnt[b] : 0u;
        sum += loc[u];
    }
    // the global position of this block's first key of each owned bucket,
    // loaded now so that the loads are in flight during the scan and the
    // placement (one round trip, not one per bucket after them)
    uint32_t gpos[BKT_MAX / 256];
#pragma unroll
    for (uint32_t u = 0; u < BKT_MAX / 256; ++u) {
        const uint32_t b = threadIdx.x * (BKT_MAX / 256) + u;
        gpos[u] = b < nb && loc[u] ? bbase[b] + Hs[(uint64_t)b * nblk + blockIdx.x] : 0u;
    }
    const uint32_t incl = wave_incl_sum(sum);
    if ((threadIdx.x & 63) == 63) wtot[threadIdx.x >> 6] = incl;
    __syncthreads();
    uint32_t pre = incl - sum;
    for (uint32_t w = 0; w < (threadIdx.x >> 6); ++w) pre += wtot[w];
    uint32_t lst[BKT_MAX / 256];
#pragma unroll
    for (uint32_t u = 0; u < BKT_MAX / 256; ++u) {
        const uint32_t b = threadIdx.x * (BKT_MAX / 256) + u;
        lst[u] = pre;                            // local start of bucket b in skey / srank
        if (b < nb) cnt[b] = pre;
        pre += loc[u];
    }
    const uint32_t valid = wtot[0] + wtot[1] + wtot[2] + wtot[3];
    __syncthreads();
#if BKT_PROBE_DELAY
    // race probe (experiment build only): waves 1..3 start placing late, so
    // wave 0 reaches the rewrite of cnt[] below first
    if (threadIdx.x >= 64)
        for (int z = 0; z < 64; ++z) __builtin_amdgcn_s_sleep(127);
#endif
#pragma unroll
    for (uint32_t u = 0; u < BKT_EPB / 256; ++u) {
        if (kk[u] != invalid) {
            const uint32_t p = cnt[kk[u] >> shift] + li[u];
#if BKT_PROBE_DELAY
            if (p >= BKT_EPB) continue;             // (the probe keeps a raced store in range)
#endif
            skey[p] = kk[u];
            srank[p] = (uint32_t)(base + u * 256 + threadIdx.x);
        }
    }
    // every wave has read its local starts before cnt[] is rewritten (without
    // this barrier a wave that got here first overwrote a bucket's local start
    // while a slower wave still placed keys by it: keys landed in wrong skey
    // slots, and stale slots went out -- the intermittent lost counts / keys)
#if !BKT_PROBE_NOFIX
    __syncthreads();
#endif
    // cnt[b] := global position of local element 0 of bucket b (mod 2^32:
    // element e of bucket b goes to cnt[b] + e)
#pragma unroll
    for (uint32_t u = 0; u < BKT_MAX / 256; ++u) {
        const uint32_t b = threadIdx.x * (BKT_MAX / 256) + u;
        if (b < nb && loc[u]) cnt[b] = gpos[u] - lst[u];
    }
    __syncthreads();
    const uint32_t lo_mask = (1u << shift) - 1u;
    for (uint32_t e = threadIdx.x; e < valid; e += 256) {
        const uint32_t k = skey[e], b = k >> shift;
        const uint32_t pos = cnt[b] + e;
#if BKT_PROBE_DELAY
        // (the probe keeps a raced store, and the ranks later kernels index by, in range)
        if (b >= nb || pos >= n || srank[e] >= n) continue;
#endif
        pkey[pos] = (uint16_t)(k & lo_mask);
        prank[pos] = srank[e];
    }
}

__global__ __launch_bounds__(1024) void bucket_heads_kernel(const uint16_t *pkey, const uint32_t *prank,
                                                            const uint32_t *bbase, uint32_t shift, uint32_t *hcnt) {
    __shared__ uint32_t minr[1u << BKT_LOW];
    __shared__ uint32_t cnt[1u << BKT_LOW];
    const uint32_t b = blockIdx.x, nk = 1u << shift;
    for (uint32_t j = threadIdx.x; j < nk; j += blockDim.x) {
        minr[j] = 0xFFFFFFFFu;
        cnt[j] = 0;
    }
    __syncthreads();
    const uint32_t lo = bbase[b], hi = bbase[b + 1];
    // 16 keys per thread loaded before any is used: one memory round trip per
    // 16 K keys, not one per 1 K (the loop waited on every load, ~10 per bucket)
    constexpr uint32_t U = 16;
    for (uint32_t e0 = lo; e0 < hi; e0 += U * 1024) {
        uint32_t j[U], r[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t e = e0 + u * 1024 + threadIdx.x;
            j[u] = e < hi ? pkey[e] : 0u;
            r[u] = e < hi ? prank[e] : 0u;
        }
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            if (e0 + u * 1024 + threadIdx.x < hi) {
                atomicMin(&minr[j[u]], r[u]);
                atomicAdd(&cnt[j[u]], 1u);
            }
        }
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < nk; j += blockDim.x) {
        const uint32_t c = cnt[j];
        if (c) hcnt[minr[j]] = c;       // (the key is rkey32 at that rank)
    }
}

// Heads (hcnt != 0) per EMIT_RPB ranks: the emit workgroups' prefixes.
constexpr uint32_t EMIT_RPB = 1024;
__global__ __launch_bounds__(256) void head_count_kernel(const uint32_t *hcnt, uint64_t n, uint32_t *ecnt) {
    __shared__ uint32_t ws[4];
    const uint64_t r0 = (uint64_t)blockIdx.x * EMIT_RPB + 4 * threadIdx.x;
    uint32_t c = 0;
    if (r0 + 4 <= n) {
        const uint4 v = *(const uint4 *)(hcnt + r0);
        c = (v.x != 0) + (v.y != 0) + (v.z != 0) + (v.w != 0);
    } else {
        for (uint64_t r = r0; r < n; ++r) c += hcnt[r] != 0;
    }
    c = wave_incl_sum(c);
    if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) ecnt[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// Ordered output, EMIT_RPB ranks per workgroup in rounds of 256 (thread t:
// rank base + 256 i + t).  A flagged rank (its key's first occurrence) emits
// output entry o = heads before it: the workgroup's prefix (the sum of the
// earlier workgroups' head counts, or their scan when there are many), then
// ballot / mbcnt inside the workgroup.  Entry: decoded key (P + suffix,
// 'ACGT' from the 2-bit code, first base most significant), count,
// first-occurrence order -- or the packed (code, {first, count}) pair for a
// partial result.
__global__ __launch_bounds__(256) void emit_kernel(EmitArgs a) {
    // decoded keys of a round's heads, staged so that the round's output
    // range [o0 * k, oend * k) is written with coalesced dword stores
    __shared__ __attribute__((aligned(16))) uint8_t kbuf[256 * KMAX_TILE];
    __shared__ uint32_t s_w[EMIT_RPB / 256][4];  // heads per (round, wave)
    __shared__ uint64_t s_pre;
    __shared__ uint32_t s_wp[4];
    const uint64_t n = a.n;
    const uint32_t k = a.k, plen = a.plen;
    const bool staged = !a.partial && (k & 3);     // else: aligned direct stores
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint64_t rb = (uint64_t)blockIdx.x * EMIT_RPB;
    constexpr int NR = EMIT_RPB / 256;
    uint32_t hcr[NR];
    unsigned long long hm[NR];
#pragma unroll
    for (int i = 0; i < NR; ++i) {
        const uint64_t r = rb + 256 * i + tid;
        hcr[i] = r < n ? a.hcnt[r] : 0u;
        hm[i] = __ballot(hcr[i] != 0);
        if (lane == 0) s_w[i][wid] = (uint32_t)__popcll(hm[i]);
    }
    // every head's key, count and first occurrence loaded now, all rounds'
    // loads in flight together (the rounds' stores would otherwise order them)
    uint64_t ekey[NR], ecnt[NR], efirst[NR], ekeyh[NR];
#pragma unroll
    for (int i = 0; i < NR; ++i) {
        const uint64_t r = rb + 256 * i + tid;
        ekey[i] = ecnt[i] = efirst[i] = ekeyh[i] = 0;
        if (hcr[i]) {
            if (a.hrec) {
                const HeadRec v = a.hrec[r];
                ekey[i] = v.key;
                ecnt[i] = v.count;
            } else {
                ekey[i] = a.rkey32 ? (uint64_t)a.rkey32[r] : a.rkey64[r];
                if (a.rkeyh) ekeyh[i] = a.rkeyh[r];
                ecnt[i] = hcr[i];
            }
            efirst[i] = a.rord[r];
        }
    }
    if (a.epre) {                                // scanned workgroup prefixes
        if (tid == 0) s_pre = a.epre[blockIdx.x];
    } else {                                     // few workgroups: sum the earlier ones' counts
        uint32_t p = 0;                          // (<= EMIT_DIRECT_MAX workgroups: fits 32 bits)
        for (uint32_t j = tid; j < blockIdx.x; j += 256) p += a.ecnt[j];
        p = wave_incl_sum(p);
        if (lane == 63) s_wp[wid] = p;
    }
    __syncthreads();
    if (!a.epre && tid == 0) s_pre = (uint64_t)s_wp[0] + s_wp[1] + s_wp[2] + s_wp[3];
    __syncthreads();
    uint64_t o0 = s_pre;                         // first output entry of the round
#pragma unroll
    for (int i = 0; i < NR; ++i) {
        const uint64_t r = rb + 256 * i + tid;
        if (rb + 256 * i >= n) break;            // (uniform)
        uint32_t before = 0, rt = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            before += w < wid ? s_w[i][w] : 0u;
            rt += s_w[i][w];
        }
        const uint32_t hc = hcr[i];
        const uint32_t f = hc ? 1u : 0u;
        const uint64_t o64 = o0 + before +
                             __builtin_amdgcn_mbcnt_hi((uint32_t)(hm[i] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)hm[i], 0u));
        const uint64_t oend = o0 + rt;
        if (r == n - 1) {
            *a.nuniq = o64 + f;
            if (a.nuniq_host) {
                *a.nuniq_host = o64 + f;
                __threadfence_system();
            }
        }
        const uint64_t o = o64;
        if (f) {
            const uint64_t key = ekey[i], cnt = ecnt[i], keyh = ekeyh[i], first = efirst[i];
            if (a.partial) {
                a.ukey[o] = key;
                Agg v;
                v.first = first;
                v.count = cnt;
                a.uval[o] = v;
            } else {
                a.cnt_out[o] = cnt;
                a.first_out[o] = first;
                uint8_t *out = staged ? kbuf + (o - o0) * k : a.keys_out + o * k;
                // word w = bases 4w .. 4w + 3, stored as soon as it is formed
                // (static indices only: no private-memory array)
                const uint32_t nw = (k + 3) / 4;
                uint32_t w0 = 0, w1 = 0, w2 = 0;
                for (int w = 0; w < KMAX_TILE / 4; ++w) {
                    if ((uint32_t)w >= nw) break;
                    uint32_t v = 0;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const uint32_t pos = 4 * w + j;
                        uint32_t ch = 0;
                        if (pos < plen) {
                            ch = a.P[pos];
                        } else if (pos < k) {
                            const uint32_t sh = 2 * (k - 1 - pos);      // (< 128)
                            const uint32_t b = (uint32_t)(sh < 64 ? key >> sh : keyh >> (sh - 64)) & 3u;
                            ch = (0x54474341u >> (8 * b)) & 0xFFu;
                        }
                        v |= ch << (8 * j);
                    }
                    if (k == 16) {                     // one 16-byte store
                        if (w == 0) w0 = v;
                        else if (w == 1) w1 = v;
                        else if (w == 2) w2 = v;
                        else *(uint4 *)out = make_uint4(w0, w1, w2, v);
                    } else if ((k & 3) == 0) {
                        *(uint32_t *)(out + 4 * w) = v;
                    } else {
                        for (uint32_t b = 4 * w; b < k && b < 4 * (uint32_t)w + 4; ++b)
                            out[b] = (uint8_t)(v >> (8 * (b & 3)));
                    }
                }
            }
        }
        if (staged) {                            // (uniform: no barrier skipped by part of the block)
            __syncthreads();
            const uint64_t g0 = (uint64_t)o0 * k, g1 = (uint64_t)oend * k;
            const uint64_t a0 = (g0 + 3) & ~3ull, a1 = g1 & ~3ull;
            if (a0 >= a1) {
                for (uint64_t g = g0 + threadIdx.x; g < g1; g += 256) a.keys_out[g] = kbuf[g - g0];
            } else {
                if (threadIdx.x < a0 - g0) a.keys_out[g0 + threadIdx.x] = kbuf[threadIdx.x];
                if (threadIdx.x < g1 - a1) a.keys_out[a1 + threadIdx.x] = kbuf[a1 - g0 + threadIdx.x];
                const uint32_t sh = (uint32_t)(a0 - g0);
                for (uint64_t g = a0 + 4 * threadIdx.x; g < a1; g += 4 * 256) {
                    const uint32_t l = (uint32_t)(g - g0);
                    const uint32_t v = sh == 0 ? *(const uint32_t *)(kbuf + l)
                                               : (uint32_t)kbuf[l] | ((uint32_t)kbuf[l + 1] << 8) |
                                                     ((uint32_t)kbuf[l + 2] << 16) | ((uint32_t)kbuf[l + 3] << 24);
                    *(uint32_t *)(a.keys_out + g) = v;
                }
            }
            __syncthreads();                     // kbuf is reused by the next round
        }
        o0 = oend;
    }
}

// merged partials (in shard order = first-occurrence order) -> rank arrays
__global__ __launch_bounds__(256) void merge_prep_kernel(const uint64_t *keys, const Agg *vals, uint64_t n,
                                                         uint64_t *rkey, uint32_t *rkey32, uint64_t *rord,
                                                         uint64_t *rcnt, uint32_t *ridx) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const Agg v = vals[i];
        put_key(rkey, rkey32, i, keys[i]);
        rord[i] = v.first;
        rcnt[i] = v.count;
        ridx[i] = (uint32_t)i;
    }
}

// ---------------------------------------------------------------------------
// Multi-GPU hit exchange: the session's ranked hits, partitioned by owning
// rank (equal slices of the packed-key space, multi.key_owner), stable within
// each owner so that every destination's run stays in rank (= first
// occurrence) order.  Non-counting slots (invalid key) are dropped.
// ---------------------------------------------------------------------------
constexpr uint32_t XP_EPB = 4096;            // rank slots per partition block

__device__ __forceinline__ uint32_t xkey_owner(uint64_t key, uint32_t kbits, uint32_t world) {
    const uint32_t s = kbits > 40 ? kbits - 40 : 0;
    const uint64_t o = ((key >> s) * (uint64_t)world) >> (kbits - s);
    return o < world ? (uint32_t)o : world - 1u;
}

__device__ __forceinline__ uint64_t xget_key(const uint64_t *rkey, const uint32_t *rkey32, uint64_t i) {
    return rkey32 ? (uint64_t)rkey32[i] : rkey[i];
}

__global__ __launch_bounds__(256) void xpart_hist_kernel(const uint64_t *rkey, const uint32_t *rkey32, uint64_t n,
                                                         uint64_t invalid, uint32_t kbits, uint32_t world,
                                                         uint32_t nblk, uint32_t *H) {
    __shared__ uint32_t hist[XP_MAXW];
    for (uint32_t o = threadIdx.x; o < world; o += 256) hist[o] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * XP_EPB;
    for (uint32_t j = threadIdx.x; j < XP_EPB; j += 256) {
        const uint64_t i = base + j;
        if (i < n) {
            const uint64_t k = xget_key(rkey, rkey32, i);
            if (k != invalid) atomicAdd(&hist[xkey_owner(k, kbits, world)], 1u);
        }
    }
    __syncthreads();
    for (uint32_t o = threadIdx.x; o < world; o += 256) H[(uint64_t)o * nblk + blockIdx.x] = hist[o];
}

// Stable scatter: slots are taken in rank order, 256 per round; inside a wave
// the lanes of one owner are ranked with a ballot, across waves and rounds
// with per-owner LDS counters.
__global__ __launch_bounds__(256) void xpart_scatter_kernel(const uint64_t *rkey, const uint32_t *rkey32,
                                                            const uint64_t *rord, uint64_t n, uint64_t invalid,
                                                            uint32_t kbits, uint32_t world, uint32_t nblk,
                                                            const uint32_t *Hs, XHit *out) {
    __shared__ uint32_t run[XP_MAXW];          // owner's slots taken by earlier rounds (+ block start)
    __shared__ uint32_t wcnt[4][XP_MAXW];      // this round: per wave, per owner
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t o = threadIdx.x; o < world; o += 256) {
        run[o] = Hs[(uint64_t)o * nblk + blockIdx.x];
        wcnt[0][o] = wcnt[1][o] = wcnt[2][o] = wcnt[3][o] = 0;
    }
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * XP_EPB;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (uint32_t u = 0; u < XP_EPB / 256; ++u) {
        const uint64_t i = base + u * 256 + threadIdx.x;
        uint64_t key = invalid;
        if (i < n) key = xget_key(rkey, rkey32, i);
        const bool valid = key != invalid;
        const uint32_t o = valid ? xkey_owner(key, kbits, world) : 0u;
        uint32_t pre = 0;
        uint64_t pending = __ballot(valid);
        while (pending) {
            const int leader = __ffsll((long long)pending) - 1;
            const uint32_t lo = __shfl(o, leader);
            const uint64_t m = __ballot(valid && o == lo);
            if (valid && o == lo) pre = __popcll(m & lt);
            if ((int)lane == leader) wcnt[wave][lo] = __popcll(m);
            pending &= ~m;
        }
        __syncthreads();
        if (valid) {
            uint32_t p = run[o] + pre;
            for (uint32_t w = 0; w < wave; ++w) p += wcnt[w][o];
            XHit h;
            h.ord = rord[i];
            h.key = key;
            out[p] = h;
        }
        __syncthreads();
        for (uint32_t t = threadIdx.x; t < world; t += 256) {
            run[t] += wcnt[0][t] + wcnt[1][t] + wcnt[2][t] + wcnt[3][t];
            wcnt[0][t] = wcnt[1][t] = wcnt[2][t] = wcnt[3][t] = 0;
        }
        __syncthreads();
    }
}

// per-owner totals of the partition (exclusive scan Hs of H, owner-major)
__global__ void xpart_counts_kernel(const uint32_t *H, const uint32_t *Hs, uint32_t world, uint32_t nblk,
                                    uint64_t *counts) {
    const uint64_t last = (uint64_t)world * nblk - 1;
    for (uint32_t o = threadIdx.x; o < world; o += blockDim.x) {
        const uint64_t lo = Hs[(uint64_t)o * nblk];
        const uint64_t hi = o + 1 < world ? (uint64_t)Hs[(uint64_t)(o + 1) * nblk] : (uint64_t)Hs[last] + H[last];
        counts[o] = hi - lo;
    }
}

// received hits (concatenated by source rank = rank order) -> rank arrays
__global__ __launch_bounds__(256) void xprep_kernel(const XHit *x, uint64_t n, uint64_t *rkey, uint32_t *rkey32,
                                                    uint64_t *rord, uint32_t *ridx) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const XHit h = x[i];
        put_key(rkey, rkey32, i, h.key);
        rord[i] = h.ord;
        ridx[i] = (uint32_t)i;
    }
}

// (key i at i * stride: the host map reads them back at that fixed stride)
__global__ __launch_bounds__(256) void gather_records_kernel(const Record *recs, uint64_t stride,
                                                             uint64_t n, const uint8_t *data, uint8_t *out) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const Record r = recs[i];
        uint8_t *o = out + i * stride;
        const uint8_t *src = data + r.pos;
        if (r.strand) {
            for (uint32_t b = 0; b < r.len; ++b) o[b] = comp_byte(src[r.len - 1 - b]);
        } else {
            for (uint32_t b = 0; b < r.len; ++b) o[b] = src[b];
        }
    }
}

// Ordered merge of per-rank result lists: row i of the output is source row
// idx[i] (k-byte key, count, first-occurrence key).  One thread per row; keys
// copied 4 bytes at a time when k allows.
// out row i = in row idx[i] (k-byte keys with their count and first): G lanes
// per row (G = k for k <= 8, else GEN_G), 64 / G rows per wave step, lanes
// striding over the row's bytes -- several rows' loads in flight per wave
__global__ __launch_bounds__(256) void permute_rows_kernel(const uint8_t *__restrict__ keys,
                                                           const uint64_t *__restrict__ cnt,
                                                           const uint64_t *__restrict__ first,
                                                           const uint32_t *__restrict__ idx, uint64_t n, uint32_t k,
                                                           uint8_t *__restrict__ okeys, uint64_t *__restrict__ ocnt,
                                                           uint64_t *__restrict__ ofirst) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t G = k <= GEN_G ? k : GEN_G, rpw = 64 / G;   // rows per wave step
    const uint32_t r = lane / G, b0 = lane % G;
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    for (uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); w * rpw < n; w += nw) {
        const uint64_t i = w * rpw + r;
        if (r >= rpw || i >= n) continue;
        const uint64_t j = idx[i];
        const uint8_t *src = keys + j * k;
        uint8_t *dst = okeys + i * k;
        for (uint32_t b = b0; b < k; b += G) dst[b] = src[b];
        if (b0 == 0) {
            ocnt[i] = cnt[j];
            ofirst[i] = first[j];
        }
    }
}

hipError_t launch_permute_rows(const uint8_t *keys, const uint64_t *cnt, const uint64_t *first, const uint32_t *idx,
                               uint64_t n, uint32_t k, uint8_t *okeys, uint64_t *ocnt, uint64_t *ofirst,
                               hipStream_t s) {
    if (n == 0 || k == 0) return hipSuccess;
    const uint64_t rpw = 64 / (k <= GEN_G ? k : GEN_G);
    uint64_t blocks = ((n + rpw - 1) / rpw + 3) / 4;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(permute_rows_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, keys, cnt, first, idx, n, k,
                       okeys, ocnt, ofirst);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// synthetic FASTQ: record i = "@r%010d\n" + 150 bases + "\n+\n"
// + 150 x 'I' + "\n" (317 B), base b = "ACGT"[(mix(seed*G + i*8 + b/32) >> 2(b%32)) & 3]
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix_mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void synth_kernel(uint8_t *out, uint64_t seed, uint64_t first_read,
                                                    uint64_t n_reads) {
    const uint64_t total = n_reads * 317;
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c * 16 < total;
         c += (uint64_t)gridDim.x * blockDim.x) {
        uint8_t bytes[16];
        for (int b = 0; b < 16; ++b) {
            const uint64_t o = c * 16 + b;
            uint8_t ch = 0;
            if (o < total) {
                const uint64_t r = o / 317, p = o % 317, i = first_read + r;
                if (p == 0) ch = '@';
                else if (p == 1) ch = 'r';
                else if (p < 12) {
                    uint64_t v = i;
                    for (int d = 11 - (int)p; d > 0; --d) v /= 10;
                    ch = (uint8_t)('0' + v % 10);
                } else if (p == 12 || p == 163 || p == 165 || p == 316) ch = '\n';
                else if (p < 163) {
                    const uint64_t bidx = p - 13;
                    const uint64_t wv = splitmix_mix(seed * 0x9E3779B97F4A7C15ull + i * 8 + bidx / 32);
                    ch = (uint8_t)"ACGT"[(wv >> (2 * (bidx % 32))) & 3];
                } else if (p == 164) ch = '+';
                else ch = 'I';
            }
            bytes[b] = ch;
        }
        const uint64_t o = c * 16;
        if (o + 16 <= total) {
            uint4 v;
            uint32_t *vw = (uint32_t *)&v;
            for (int j = 0; j < 4; ++j)
                vw[j] = bytes[4 * j] | (bytes[4 * j + 1] << 8) | (bytes[4 * j + 2] << 16) |
                        ((uint32_t)bytes[4 * j + 3] << 24);
            *(uint4 *)(out + o) = v;
        } else {
            for (int b = 0; o + b < total; ++b) out[o + b] = bytes[b];
        }
    }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
hipError_t launch_lines(const TileArgs &a, bool lookback, hipStream_t s) {
    if (lookback) hipLaunchKernelGGL((lines_kernel<true>), dim3(a.n_tiles), dim3(TPB), 0, s, a);
    else hipLaunchKernelGGL((lines_kernel<false>), dim3(a.n_tiles), dim3(TPB), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_scan_planes(const ScanArgs &a, const PlaneArgs &pa, hipStream_t s) {
    const dim3 g(a.n_tiles);
    uint32_t pm = 0;                         // the planes' masks as plane_masks_const encodes them
    for (int i = 0; i < 5; ++i)
        pm |= (pa.kl[i] ? 1u : 0u) << (4 * i) | (pa.kh[i] ? 1u : 0u) << (4 * i + 1) |
              (pa.rl[i] ? 1u : 0u) << (4 * i + 2) | (pa.rh[i] ? 1u : 0u) << (4 * i + 3);
    if (pa.pb >= 5 && pm == PM_ATGAC) {     // the default prefix, compiled in
        if (a.k > 32) hipLaunchKernelGGL((scan_planes_kernel<true, true, PM_ATGAC>), g, dim3(TPB), 0, s, a, pa);
        else hipLaunchKernelGGL((scan_planes_kernel<true, false, PM_ATGAC>), g, dim3(TPB), 0, s, a, pa);
        return hipGetLastError();
    }
    if (a.k > 32) {
        if (pa.pb >= 5) hipLaunchKernelGGL((scan_planes_kernel<true, true>), g, dim3(TPB), 0, s, a, pa);
        else hipLaunchKernelGGL((scan_planes_kernel<false, true>), g, dim3(TPB), 0, s, a, pa);
    } else {
        if (pa.pb >= 5) hipLaunchKernelGGL((scan_planes_kernel<true, false>), g, dim3(TPB), 0, s, a, pa);
        else hipLaunchKernelGGL((scan_planes_kernel<false, false>), g, dim3(TPB), 0, s, a, pa);
    }
    return hipGetLastError();
}
hipError_t launch_scan_tiles(const ScanArgs &a, hipStream_t s) {
    const dim3 g(a.n_tiles);
    if (a.k > 32) {
        if (a.plen >= 4) hipLaunchKernelGGL((scan_tile_kernel<true, true>), g, dim3(TPB), 0, s, a);
        else hipLaunchKernelGGL((scan_tile_kernel<false, true>), g, dim3(TPB), 0, s, a);
    } else {
        if (a.plen >= 4) hipLaunchKernelGGL((scan_tile_kernel<true, false>), g, dim3(TPB), 0, s, a);
        else hipLaunchKernelGGL((scan_tile_kernel<false, false>), g, dim3(TPB), 0, s, a);
    }
    return hipGetLastError();
}

hipError_t launch_hits(const HitArgs &a, hipStream_t s) {
    const dim3 grid((a.n_tiles + 4 * HTPW - 1) / (4 * HTPW));
    if (a.wide) hipLaunchKernelGGL(hit_kernel<true>, grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL(hit_kernel<false>, grid, dim3(256), 0, s, a);
    hipLaunchKernelGGL(hit_overflow_kernel, dim3(64), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_tile_reduce(const TileSum *in, uint32_t n, TileSum *bsum, hipStream_t s) {
    hipLaunchKernelGGL(tile_reduce_kernel, dim3((n + TSCAN_BLOCK - 1) / TSCAN_BLOCK), dim3(256), 0, s, in, n, bsum);
    return hipGetLastError();
}
hipError_t launch_tile_scan(const TileSum *in, uint32_t n, const TileSum *bsum, bool bsum_scanned, TileSum init,
                            TileSum *out, hipStream_t s) {
    hipLaunchKernelGGL(tile_scan_kernel, dim3((n + TSCAN_BLOCK - 1) / TSCAN_BLOCK), dim3(256), 0, s, in, n, bsum,
                       bsum_scanned ? 1u : 0u, init, out);
    return hipGetLastError();
}
hipError_t launch_prep(StreamPos *pos, StreamPos *saved, unsigned int *err, uint64_t *scal, uint32_t flags,
                       uint64_t lines, hipStream_t s) {
    hipLaunchKernelGGL(prep_kernel, dim3(1), dim3(64), 0, s, pos, saved, err, scal, flags, lines);
    return hipGetLastError();
}
hipError_t launch_tile_aggregate(const uint8_t *data, uint64_t len, uint32_t n_tiles, uint64_t *agg_cnt,
                                 uint64_t *agg_lnl, unsigned int *err, hipStream_t s) {
    hipLaunchKernelGGL(tile_aggregate_kernel, dim3(n_tiles), dim3(TPB), 0, s, data, len, agg_cnt, agg_lnl, err);
    return hipGetLastError();
}

hipError_t launch_windows(const WindowArgs &a, uint32_t grid, hipStream_t s) {
    hipLaunchKernelGGL(windows_kernel, dim3(grid), dim3(256), 0, s, a);
    return hipGetLastError();
}

static uint32_t grid_for(uint64_t n) {
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    return (uint32_t)(blocks ? blocks : 1);
}

hipError_t launch_gen_cand(const GenWinArgs &a, const PlaneArgs &pa, hipStream_t s) {
    if (a.len == 0 || a.n_lines == 0) return hipSuccess;
    const uint64_t tiles = (a.len + TILE - 1) / TILE;
    hipLaunchKernelGGL(gen_cand_kernel, dim3((uint32_t)((tiles + GC_TPB - 1) / GC_TPB)), dim3(256), 0, s, a, pa);
    return hipGetLastError();
}

hipError_t launch_gen_fix(const Record *cand, uint64_t n, const SeqLine *lines, uint32_t k, uint32_t plen,
                          uint32_t pbits, Record *recs, unsigned long long *rec_count, uint64_t rec_cap,
                          unsigned int *err, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint64_t blocks = std::min<uint64_t>(2048, (n + 4095) / 4096);   // >= 4 K candidates per workgroup
    hipLaunchKernelGGL(gen_fix_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, cand, n, lines, k, plen, pbits, recs,
                       rec_count, rec_cap, err);
    return hipGetLastError();
}

hipError_t launch_gen_windows(const GenWinArgs &a, hipStream_t s) {
    if (a.total == 0) return hipSuccess;
    const uint64_t waves = std::min<uint64_t>(65536, (a.total / 2 + 255) / 256);   // >= 256 positions per wave
    hipLaunchKernelGGL(gen_windows_kernel, dim3((uint32_t)((waves + 3) / 4)), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_gen_append(const Record *recs, uint64_t n, const uint8_t *data, uint32_t k, uint8_t *keys,
                             uint64_t *cnt, uint64_t *first, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(gen_append_kernel, dim3(grid_for(GEN_G * n)), dim3(256), 0, s, recs, n, data, k, keys, cnt, first);
    return hipGetLastError();
}

hipError_t launch_gen_hash(const uint8_t *keys, uint64_t n, uint32_t k, uint64_t seed, uint64_t *h1, uint64_t *h2,
                           uint32_t *idx, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(gen_hash_kernel, dim3(grid_for(GEN_G * n)), dim3(256), 0, s, keys, n, k, seed, h1, h2, idx);
    return hipGetLastError();
}

hipError_t launch_gen_heads(const uint64_t *h1, const uint64_t *h2, const uint32_t *idx, uint64_t n, const uint8_t *keys,
                            uint32_t k, uint32_t *head, unsigned int *collide, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(gen_heads_kernel, dim3(grid_for(n)), dim3(256), 0, s, h1, h2, idx, n, keys, k, head, collide);
    return hipGetLastError();
}

hipError_t launch_gen_starts(const uint32_t *head, const uint32_t *gid, uint64_t n, uint32_t *start, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(gen_starts_kernel, dim3(grid_for(n)), dim3(256), 0, s, head, gid, n, start);
    return hipGetLastError();
}

hipError_t launch_gen_reduce(const uint32_t *start, uint64_t ng, const uint32_t *idx, const uint8_t *keys,
                             const uint64_t *cnt, const uint64_t *first, uint32_t k, uint8_t *okeys, uint64_t *ocnt,
                             uint64_t *ofirst, hipStream_t s) {
    if (ng == 0) return hipSuccess;
    hipLaunchKernelGGL(gen_reduce_kernel, dim3(grid_for(GEN_G * ng)), dim3(256), 0, s, start, ng, idx, keys, cnt, first, k,
                       okeys, ocnt, ofirst);
    return hipGetLastError();
}

hipError_t launch_cross_scatter(const uint32_t *slot, const uint64_t *ord, const uint64_t *key, uint64_t n,
                                uint64_t *rkey, uint32_t *rkey32, uint64_t *rord, hipStream_t s) {
    if (n) hipLaunchKernelGGL(cross_scatter_kernel, dim3(grid_for(n)), dim3(256), 0, s, slot, ord, key, n, rkey, rkey32,
                              rord);
    return hipGetLastError();
}
hipError_t launch_cross_sort_small(const uint32_t *slot, const uint64_t *ord, const uint64_t *key, uint64_t n,
                                   uint64_t *rkey, uint32_t *rkey32, uint64_t *rord, hipStream_t s) {
    if (n > XSMALL) return hipErrorInvalidValue;
    if (n) hipLaunchKernelGGL(cross_sort_small_kernel, dim3(1), dim3(1024), 0, s, slot, ord, key, (uint32_t)n, rkey,
                              rkey32, rord);
    return hipGetLastError();
}
hipError_t launch_cross_segsort(uint64_t *ord, uint64_t *key, const uint32_t *slot, uint64_t n, uint64_t *rkey,
                                uint32_t *rkey32, uint64_t *rord, uint32_t pbits, hipStream_t s) {
    if (n) hipLaunchKernelGGL(cross_segsort_kernel, dim3(grid_for(n)), dim3(256), 0, s, ord, key, slot, n, rkey, rkey32,
                              rord, pbits + 1);
    return hipGetLastError();
}
// ---------------------------------------------------------------------------
// compaction of the dense-hit rank arrays (keys != invalid, in rank order):
// count per 4,096 ranks, scan, then each workgroup writes its valid (key,
// order) pairs at its offset + rank among them (row-major ballots) -- the
// keys read twice, the orders only where valid; a library select over an
// index iterator and two gathers took 39 ms for 2.7 G windows (C2, prefix AT)
// ---------------------------------------------------------------------------
constexpr uint32_t CP_ROWS = 16;                 // rows of 256 ranks per workgroup

template <typename K>
__global__ __launch_bounds__(256) void compact_count_kernel(const K *__restrict__ key, uint64_t n, K invalid,
                                                            uint32_t *__restrict__ bcnt) {
    __shared__ uint32_t ws[4];
    const uint64_t base = (uint64_t)blockIdx.x * (256 * CP_ROWS);
    uint32_t c = 0;
#pragma unroll
    for (uint32_t j = 0; j < CP_ROWS; ++j) {
        const uint64_t i = base + 256 * j + threadIdx.x;
        c += (i < n && key[i] != invalid) ? 1u : 0u;
    }
    c = wave_incl_sum(c);
    if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) bcnt[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

template <typename K>
__global__ __launch_bounds__(256) void compact_write_kernel(const K *__restrict__ key, const uint64_t *__restrict__ ord,
                                                            uint64_t n, K invalid, const uint64_t *__restrict__ boff,
                                                            K *__restrict__ okey, uint64_t *__restrict__ oord) {
    __shared__ uint32_t wc[CP_ROWS * 4];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t base = (uint64_t)blockIdx.x * (256 * CP_ROWS);
    K kv[CP_ROWS];
    uint32_t below[CP_ROWS];
    bool v[CP_ROWS];
#pragma unroll
    for (uint32_t j = 0; j < CP_ROWS; ++j) {
        const uint64_t i = base + 256 * j + threadIdx.x;
        kv[j] = i < n ? key[i] : invalid;
        v[j] = kv[j] != invalid;
        const unsigned long long m = __ballot(v[j]);
        below[j] = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) wc[4 * j + w] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (threadIdx.x < 64) {                            // exclusive scan of the 64 (row, wave) counts
        const uint32_t x = wc[threadIdx.x];
        const uint32_t inc = wave_incl_sum(x);
        wc[threadIdx.x] = inc - x;
    }
    __syncthreads();
    const uint64_t o0 = boff[blockIdx.x];
#pragma unroll
    for (uint32_t j = 0; j < CP_ROWS; ++j) {
        if (!v[j]) continue;
        const uint64_t i = base + 256 * j + threadIdx.x;
        const uint64_t o = o0 + wc[4 * j + w] + below[j];
        okey[o] = kv[j];
        oord[o] = ord[i];
    }
}

hipError_t launch_compact_count(const uint32_t *k32, const uint64_t *k64, uint64_t n, uint64_t invalid, uint32_t *bcnt,
                                hipStream_t s) {
    const uint64_t nb = (n + 256 * CP_ROWS - 1) / (256 * CP_ROWS);
    if (k32) hipLaunchKernelGGL(compact_count_kernel<uint32_t>, dim3((uint32_t)nb), dim3(256), 0, s, k32, n,
                                (uint32_t)invalid, bcnt);
    else hipLaunchKernelGGL(compact_count_kernel<uint64_t>, dim3((uint32_t)nb), dim3(256), 0, s, k64, n, invalid, bcnt);
    return hipGetLastError();
}

hipError_t launch_compact_write(const uint32_t *k32, const uint64_t *k64, const uint64_t *ord, uint64_t n,
                                uint64_t invalid, const uint64_t *boff, uint32_t *o32, uint64_t *o64, uint64_t *oord,
                                hipStream_t s) {
    const uint64_t nb = (n + 256 * CP_ROWS - 1) / (256 * CP_ROWS);
    if (k32) hipLaunchKernelGGL(compact_write_kernel<uint32_t>, dim3((uint32_t)nb), dim3(256), 0, s, k32, ord, n,
                                (uint32_t)invalid, boff, o32, oord);
    else hipLaunchKernelGGL(compact_write_kernel<uint64_t>, dim3((uint32_t)nb), dim3(256), 0, s, k64, ord, n, invalid,
                            boff, o64, oord);
    return hipGetLastError();
}

hipError_t launch_gather_u32(const uint32_t *src, const uint32_t *idx, uint64_t n, uint32_t *dst, hipStream_t s) {
    if (n) hipLaunchKernelGGL(gather_u32_kernel, dim3(grid_for(n)), dim3(256), 0, s, src, idx, n, dst);
    return hipGetLastError();
}
hipError_t launch_gather_u64(const uint64_t *src, const uint32_t *idx, uint64_t n, uint64_t *dst, hipStream_t s) {
    if (n) hipLaunchKernelGGL(gather_u64_kernel, dim3(grid_for(n)), dim3(256), 0, s, src, idx, n, dst);
    return hipGetLastError();
}
hipError_t launch_cross_wide_fix(const uint32_t *xslot, uint64_t n, const uint64_t *xkeyl, const uint64_t *xkeyh,
                                 uint64_t *rkey, uint64_t *rkeyh, hipStream_t s) {
    if (n) hipLaunchKernelGGL(cross_wide_fix_kernel, dim3(grid_for(n)), dim3(256), 0, s, xslot, n, xkeyl, xkeyh, rkey,
                              rkeyh);
    return hipGetLastError();
}
hipError_t launch_heads_wide(const uint64_t *shi, const uint64_t *slo, const uint32_t *srank, uint64_t n,
                             uint64_t invalid_hi, uint32_t *hcnt, hipStream_t s) {
    if (n) hipLaunchKernelGGL(heads_wide_kernel, dim3(grid_for(n)), dim3(256), 0, s, shi, slo, srank, n, invalid_hi,
                              hcnt);
    return hipGetLastError();
}
hipError_t launch_heads(const uint64_t *skey, const uint32_t *srank, uint64_t n, uint64_t invalid_key,
                        const uint64_t *rcnt, HeadRec *hrec, uint32_t *hcnt, hipStream_t s) {
    if (n)
        hipLaunchKernelGGL(heads_kernel<uint64_t>, dim3(grid_for(n)), dim3(256), 0, s, skey, srank, n, invalid_key, rcnt,
                           hrec, hcnt);
    return hipGetLastError();
}
hipError_t launch_heads_sparse(const uint64_t *skey64, const uint32_t *skey32, const uint32_t *srank, uint64_t n,
                               uint64_t invalid_key, uint32_t *hcnt, hipStream_t s) {
    if (!n) return hipSuccess;
    if (skey32)
        hipLaunchKernelGGL(heads_sparse_kernel<uint32_t>, dim3(grid_for(n)), dim3(256), 0, s, skey32, srank, n,
                           (uint32_t)invalid_key, hcnt);
    else
        hipLaunchKernelGGL(heads_sparse_kernel<uint64_t>, dim3(grid_for(n)), dim3(256), 0, s, skey64, srank, n,
                           invalid_key, hcnt);
    return hipGetLastError();
}
hipError_t launch_heads32(const uint32_t *skey, const uint32_t *srank, uint64_t n, uint32_t invalid_key,
                          const uint64_t *rcnt, HeadRec *hrec, uint32_t *hcnt, hipStream_t s) {
    if (n)
        hipLaunchKernelGGL(heads_kernel<uint32_t>, dim3(grid_for(n)), dim3(256), 0, s, skey, srank, n, invalid_key, rcnt,
                           hrec, hcnt);
    return hipGetLastError();
}
hipError_t launch_bucket_hist(const uint32_t *key, uint64_t n, uint32_t invalid, uint32_t shift, uint32_t nb,
                              uint32_t nblk, uint32_t *H, uint32_t *hcnt, hipStream_t s) {
    hipLaunchKernelGGL(bucket_hist_kernel, dim3(nblk), dim3(256), 0, s, key, n, invalid, shift, nb, nblk, H, hcnt);
    return hipGetLastError();
}
hipError_t launch_bucket_offsets(const uint32_t *H, uint32_t nb, uint32_t nblk, uint32_t *Hs, uint32_t *btot,
                                 uint32_t *bbase, unsigned int *ticket, hipStream_t s) {
    hipLaunchKernelGGL(bucket_offsets_kernel, dim3(nb), dim3(256), 0, s, H, nb, nblk, Hs, btot, bbase, ticket);
    return hipGetLastError();
}
hipError_t launch_bucket_scatter(const uint32_t *key, uint64_t n, uint32_t invalid, uint32_t shift, uint32_t nb,
                                 uint32_t nblk, const uint32_t *Hs, const uint32_t *bbase, uint16_t *pkey,
                                 uint32_t *prank, hipStream_t s) {
    hipLaunchKernelGGL(bucket_scatter_kernel, dim3(nblk), dim3(256), 0, s, key, n, invalid, shift, nb, nblk, Hs, bbase,
                       pkey, prank);
    return hipGetLastError();
}
hipError_t launch_bucket_heads(const uint16_t *pkey, const uint32_t *prank, const uint32_t *bbase, uint32_t nb,
                               uint32_t shift, uint32_t *hcnt, hipStream_t s) {
    hipLaunchKernelGGL(bucket_heads_kernel, dim3(nb), dim3(1024), 0, s, pkey, prank, bbase, shift, hcnt);
    return hipGetLastError();
}
uint64_t emit_blocks(uint64_t n) { return (n + EMIT_RPB - 1) / EMIT_RPB; }
hipError_t launch_head_count(const uint32_t *hcnt, uint64_t n, uint32_t *ecnt, hipStream_t s) {
    if (n) hipLaunchKernelGGL(head_count_kernel, dim3((uint32_t)emit_blocks(n)), dim3(256), 0, s, hcnt, n, ecnt);
    return hipGetLastError();
}
hipError_t launch_emit(const EmitArgs &a, hipStream_t s) {
    if (a.n) hipLaunchKernelGGL(emit_kernel, dim3((uint32_t)emit_blocks(a.n)), dim3(256), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_merge_prep(const uint64_t *keys, const Agg *vals, uint64_t n, uint64_t *rkey, uint32_t *rkey32,
                             uint64_t *rord, uint64_t *rcnt, uint32_t *ridx, hipStream_t s) {
    if (n)
        hipLaunchKernelGGL(merge_prep_kernel, dim3(grid_for(n)), dim3(256), 0, s, keys, vals, n, rkey, rkey32, rord, rcnt,
                           ridx);
    return hipGetLastError();
}
hipError_t launch_xpart_hist(const uint64_t *rkey, const uint32_t *rkey32, uint64_t n, uint64_t invalid,
                             uint32_t kbits, uint32_t world, uint32_t nblk, uint32_t *H, hipStream_t s) {
    if (world == 0 || world > XP_MAXW || nblk == 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(xpart_hist_kernel, dim3(nblk), dim3(256), 0, s, rkey, rkey32, n, invalid, kbits, world, nblk, H);
    return hipGetLastError();
}
hipError_t launch_xpart_scatter(const uint64_t *rkey, const uint32_t *rkey32, const uint64_t *rord, uint64_t n,
                                uint64_t invalid, uint32_t kbits, uint32_t world, uint32_t nblk, const uint32_t *H,
                                const uint32_t *Hs, XHit *out, uint64_t *counts, hipStream_t s) {
    if (world == 0 || world > XP_MAXW || nblk == 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(xpart_scatter_kernel, dim3(nblk), dim3(256), 0, s, rkey, rkey32, rord, n, invalid, kbits, world,
                       nblk, Hs, out);
    hipLaunchKernelGGL(xpart_counts_kernel, dim3(1), dim3(256), 0, s, H, Hs, world, nblk, counts);
    return hipGetLastError();
}
hipError_t launch_xprep(const XHit *x, uint64_t n, uint64_t *rkey, uint32_t *rkey32, uint64_t *rord, uint32_t *ridx,
                        hipStream_t s) {
    if (n) hipLaunchKernelGGL(xprep_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, n, rkey, rkey32, rord, ridx);
    return hipGetLastError();
}
hipError_t launch_gather_records(const Record *recs, uint64_t stride, uint64_t n, const uint8_t *data,
                                 uint8_t *out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(gather_records_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, recs, stride, n, data, out);
    return hipGetLastError();
}

hipError_t launch_nl_count(const uint8_t *data, uint64_t len, uint32_t n_tiles, uint32_t *tcount, unsigned int *err,
                           hipStream_t s) {
    hipLaunchKernelGGL(nl_count_kernel, dim3(n_tiles), dim3(256), 0, s, data, len, tcount, err);
    return hipGetLastError();
}
hipError_t launch_nl_write(const uint8_t *data, uint64_t len, uint32_t n_tiles, const uint64_t *tbase, uint64_t *nl,
                           hipStream_t s) {
    hipLaunchKernelGGL(nl_write_kernel, dim3(n_tiles), dim3(256), 0, s, data, len, tbase, nl);
    return hipGetLastError();
}
hipError_t launch_nl_slots(const uint8_t *data, uint64_t len, uint32_t n_tiles, uint32_t cap, uint16_t *slots,
                          uint32_t *tcount, unsigned int *err, hipStream_t s) {
    hipLaunchKernelGGL(nl_slots_kernel, dim3(n_tiles), dim3(256), 0, s, data, len, cap, slots, tcount, err);
    return hipGetLastError();
}
hipError_t launch_seq_lines_slots(const uint16_t *slots, const uint32_t *tcount, const uint64_t *tbase,
                                  uint32_t n_tiles, uint32_t cap, uint64_t len, uint64_t li0, uint64_t first,
                                  uint64_t n_nl, uint64_t n_seq, uint32_t k, uint32_t step, SeqLine *lines,
                                  uint64_t *wcount, unsigned int *err, uint64_t maxrel, hipStream_t s) {
    if (!n_seq) return hipSuccess;
    hipLaunchKernelGGL(seq_lines_slots_kernel, dim3((n_tiles + 3) / 4), dim3(256), 0, s, slots, tcount, tbase,
                       n_tiles, cap, len, li0, first, n_nl, n_seq, k, step, lines, wcount, err, maxrel);
    return hipGetLastError();
}
hipError_t launch_seq_lines(const uint64_t *nl, uint64_t n_nl, uint64_t len, uint64_t li0, uint64_t n_seq, uint32_t k,
                            uint32_t step, SeqLine *lines, uint64_t *wcount, unsigned int *err, uint64_t maxrel,
                            hipStream_t s) {
    if (n_seq)
        hipLaunchKernelGGL(seq_lines_kernel, dim3(grid_for(n_seq)), dim3(256), 0, s, nl, n_nl, len, li0, n_seq, k, step,
                           lines, wcount, err, maxrel);
    return hipGetLastError();
}
hipError_t launch_pos_after(StreamPos *pos, uint64_t lines, const uint8_t *data, uint64_t len,
                            unsigned long long *ends_open, hipStream_t s) {
    hipLaunchKernelGGL(pos_after_kernel, dim3(1), dim3(64), 0, s, pos, lines, data, len, ends_open);
    return hipGetLastError();
}
hipError_t launch_windows_packed(const WinArgs &a, hipStream_t s) {
    if (a.n_lines) {
        const uint64_t cap = a.block_lines ? 65536 : 262144;          // workgroups / waves, one line each at a time
        const uint64_t w = a.n_lines < cap ? a.n_lines : cap;
        hipLaunchKernelGGL(windows_packed_kernel, dim3((uint32_t)(a.block_lines ? w : (w + 3) / 4)), dim3(256), 0, s, a);
    }
    return hipGetLastError();
}
hipError_t launch_synth_fastq(uint8_t *out, uint64_t seed, uint64_t first_read, uint64_t n_reads, hipStream_t s) {
    const uint64_t chunks = (n_reads * 317 + 15) / 16;
    uint64_t blocks = (chunks + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(synth_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, out, seed, first_read, n_reads);
    return hipGetLastError();
}

}  // namespace kmerhip
