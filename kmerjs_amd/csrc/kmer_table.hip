// kmer_table.hip — table mode: unordered canonical k-mer counts for
// configurations whose result is too large for an ordered Map (BASELINE C3:
// 100 M reads, k = 31, no prefix -> ~12 G distinct canonical keys; the
// reference Map stops at 2^24 keys, lib/kmers.js:95).
//
// Same counting rule as the ordered paths (lib/kmers.js:88-100 on every
// sequence line and on its complement, :151-155), stored canonically (SURVEY.md
// App. A.6): a forward window w counts toward c = min(w, rc w) when w or rc(w)
// starts with the prefix; the Map is recovered as {c: C, rc c: C} (filtered
// by the prefix; palindromes 2 C).
//
// Pipeline (hash-partitioned, every write pass coalesced; no global atomics
// on the data path):
//   pass 1  per sequence line, a run of 16 consecutive windows per lane: bit
//           planes of the run's bytes (v_dot4 of aligned dwords), each window
//           a shift of them, canonical code, h = tab_mix(code).  hist1 counts keys per
//           (workgroup, top-10-bit partition) in LDS; scatter1 re-reads the
//           input (1.3 B/window, cheaper than a key buffer), ranks each key in
//           its partition with an LDS atomic, sorts a round of 8 K keys in LDS
//           and writes each partition's run contiguously (two 512-thread
//           workgroups per CU: one's stores overlap the other's formation).
//   pass 2  per run of a partition: the next 10 bits, LDS sort in rounds of
//           8 K keys -> B2 in 2^20 buckets, contiguous per bucket; each round
//           writes a bucket's keys only up to its last 64-B boundary and
//           carries the rest into the next round (whole blocks, no partial
//           lines left behind).
//   final   one persistent workgroup per CU, unit by unit (a bucket, or a
//           group of small buckets): a counting sort of the unit's keys into
//           4,096 LDS bins and a per-thread dedupe of adjacent bins; crowded
//           units use an LDS open-addressing table (8 K slots, CAS claim,
//           atomic count) with ranges split and redone when they do not fit.
//           Entries (remainder, count) are written back to the bucket's range;
//           Map statistics on the fly.
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "kmer_internal.hpp"

namespace kmerhip {

namespace {

constexpr int TAB_RPL = 16;                  // segments (keys) per lane per round
constexpr int TAB_WG1 = 1024;                // scatter workgroup (16 waves)
constexpr int TAB_ROUND = TAB_RPL * TAB_WG1; // keys sorted in LDS per round
constexpr uint64_t TAB_EMPTY = 1ull << 63;   // empty slot (remainders are < 2^44)
constexpr uint64_t TAB_RMASK = (1ull << TAB_RBITS) - 1;

__device__ __forceinline__ uint32_t tab_incl_sum(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}

// Exclusive scan of one value per thread over a 1024-thread workgroup;
// `ws` = 16 words of LDS scratch.  Returns the exclusive prefix, *total the sum.
__device__ __forceinline__ uint32_t block_excl_1024(uint32_t v, uint32_t *ws, uint32_t *total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t inc = tab_incl_sum(v);
    if (lane == 63) ws[wid] = inc;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < 16; ++w) {
        const uint32_t x = ws[w];
        before += w < wid ? x : 0u;
        all += x;
    }
    *total = all;
    return before + inc - v;
}

// exclusive scan of one value per thread over a 512-thread workgroup (ws: 8 words)
__device__ __forceinline__ uint32_t block_excl_512(uint32_t v, uint32_t *ws, uint32_t *total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t inc = tab_incl_sum(v);
    if (lane == 63) ws[wid] = inc;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        const uint32_t x = ws[w];
        before += w < wid ? x : 0u;
        all += x;
    }
    *total = all;
    return before + inc - v;
}
__device__ __forceinline__ uint32_t readlane32(uint32_t v, uint32_t i) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)i);
}



// A wave's position in its workgroup's share of sequence lines.
struct TabCur {
    uint64_t m, end;               // next sequence ordinal of this wave, end of the workgroup's share
    uint64_t seg;                  // first window of the next segment in line m
    uint32_t stride;               // waves per workgroup
    uint64_t dstart, dlen;         // lane i < 16: line m + stride * i (prefetched a round ahead)
};

// the descriptors of the wave's next 16 lines (lane i < 16: line c.m + stride * i)
__device__ __forceinline__ void tab_fetch(const TabArgs &a, TabCur &c) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t mi = c.m + (uint64_t)c.stride * (lane & 15);
    c.dstart = 0;
    c.dlen = 0;
    if (lane < 16 && mi < c.end) {
        c.dstart = a.lines[mi].start;
        c.dlen = a.lines[mi].len;
    }
}

__device__ __forceinline__ void tab_record(const TabArgs &a, uint64_t pos, uint32_t strand) {
    const unsigned long long i = atomicAdd(a.rec_count, 1ull);
    if (i < a.rec_cap) {
        Record r;
        r.order = 0;
        r.pos = pos;
        r.len = a.k;
        r.strand = strand;
        a.recs[i] = r;
    } else {
        atomicOr(a.err, ERR_REC_OVERFLOW);
    }
}

// One round of a wave: a lane takes NS CONSECUTIVE windows of one line.  Lanes are dealt out over the wave's next 16 lines
// (ceil(windows left / NS) lanes per line); a lane loads the line bytes its
// windows span as aligned dwords, turns them into three bit planes (lo / hi
// base bits, non-ACGT) of up to 52 positions with v_dot4, and every window is
// then a shift of the planes (a window-per-lane formation with six ballots and
// funnels per window issued 2.5x the instructions: hist1 41.6 -> 23.1 ms,
// scatter1 84.4 -> 64.2 ms at C3).  key[OFF + m] = h of the lane's window m,
// bit m of the result set iff it is counted; non-ACGT windows become records
// (rec).
__device__ __forceinline__ uint64_t tab_brev64(uint64_t x) {
    return ((uint64_t)__brev((uint32_t)x) << 32) | __brev((uint32_t)(x >> 32));
}

__device__ __forceinline__ uint64_t tab_key(const TabArgs &a, uint64_t cf, uint64_t cr) {
#ifdef KMERHIP_EXPERIMENTS
    if (a.narrow == 2) {                             // (A/B only, results WRONG: the cost of the mix)
        const uint64_t c = tab_canon_n(cf, cr, a.k);
        return (c << 54) | ((c >> 10) << TAB_NSH);
    }
#endif
    return a.narrow ? tab_mix_n(tab_canon_n(cf, cr, a.k)) : tab_mix(cf < cr ? cf : cr);
}

// pass-1 key stores: narrow keys as 32 bits below the partition (h >> 23)
__device__ __forceinline__ void b1_store(const TabArgs &a, uint64_t i, uint64_t h) {
    if (a.narrow) ((uint32_t *)a.B1)[i] = (uint32_t)(h >> TAB_NSH) & 0x7FFFFFFFu;
    else a.B1[i] = h;
}
__device__ __forceinline__ void b1_fill(const TabArgs &a, uint64_t i) {
    if (a.narrow) ((uint32_t *)a.B1)[i] = TAB_SENT32;
    else a.B1[i] = TAB_SENT;
}

template <int NS, int OFF, bool PFX>
__device__ __forceinline__ uint32_t tab_round(const TabArgs &a, TabCur &c, bool rec, uint64_t (&key)[TAB_RPL]) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t k = a.k;
    // the next 16 lines of this wave (fetched by the previous round)
    const uint64_t W = c.dlen >= k ? c.dlen - k + 1 : 0;          // windows of the line
    const uint64_t rem = lane == 0 ? (W > c.seg ? W - c.seg : 0) : W;
    const uint32_t need = lane < 16 ? (uint32_t)((rem + NS - 1) / NS) : 0u;   // (<= 2^32 lanes: pieces are short)
    const uint32_t cum = tab_incl_sum(need);                      // inclusive over lanes 0..15
    const uint32_t tot = readlane32(cum, 15);
    // this lane's line: the first i with cum_i > lane
    uint32_t li = 0;
#pragma unroll
    for (uint32_t i = 0; i < 16; ++i) li += readlane32(cum, i) <= lane ? 1u : 0u;
    const bool act = lane < tot && li < 16;
    const uint32_t lsrc = li < 16 ? li : 15u;
    const uint32_t before = (uint32_t)__shfl((int)(cum - need), (int)lsrc);
    const uint64_t st = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)c.dstart, (int)lsrc)) |
                        ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(c.dstart >> 32), (int)lsrc) << 32);
    const uint64_t Wl = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)W, (int)lsrc)) |
                        ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(W >> 32), (int)lsrc) << 32);
    const uint64_t w0 = (li == 0 ? c.seg : 0) + (uint64_t)(lane - before) * NS;
    // advance the cursor past what this round takes
    if (tot <= 64) {
        c.m += (uint64_t)c.stride * 16;
        c.seg = 0;
    } else {
        // line i* holds lane 63; it is done iff its last lane is lane 63
        const uint32_t is = readlane32(li, 63);
        const uint32_t ci = readlane32(cum, is), bi = ci - readlane32(need, is);
        if (ci == 64) {
            c.m += (uint64_t)c.stride * (is + 1);
            c.seg = 0;
        } else {
            c.seg = (is == 0 ? c.seg : 0) + (uint64_t)(64 - bi) * NS;
            c.m += (uint64_t)c.stride * is;
        }
    }
    // the next round's descriptors load while this round's bytes do
    tab_fetch(a, c);
    // planes of the bytes [st + w0, st + w0 + NS + k - 1), from aligned dwords
    uint64_t LO = 0, HI = 0, EX = 0;
    const uint8_t *p = a.data + st + w0;
    const uint32_t off = (uint32_t)((uintptr_t)p & 3u);
    const uint32_t *pw = (const uint32_t *)(p - off);
    const uint8_t *end = a.data + a.len;
    constexpr int NDW = (NS + 31 + 3 + 3) / 4;
#pragma unroll
    for (int i = 0; i < NDW; ++i) {
        uint32_t x = 0x41414141u;                                  // ('A': outside the line, never counted)
        const uint8_t *q = (const uint8_t *)(pw + i);
        if (act && q < end && (uint32_t)(4 * i) < off + NS + k - 1) {
            if (q + 4 <= end) {
                x = pw[i];
            } else {                                               // the input's last dword: no read past its end
                for (int j = 0; j < 4; ++j)
                    if (q + j < end) x = (x & ~(0xFFu << (8 * j))) | ((uint32_t)q[j] << (8 * j));
            }
        }
        const uint32_t lo4 = __builtin_amdgcn_udot4((x ^ (x >> 1)) & 0x02020202u, 0x08040201u, 0u, false) >> 1;
        const uint32_t hi4 = __builtin_amdgcn_udot4(x & 0x04040404u, 0x08040201u, 0u, false) >> 2;
        const uint32_t cc = ((x >> 1) ^ (x >> 2)) & 0x03030303u;
        const uint32_t ne = __builtin_amdgcn_perm(0u, 0x54474341u, cc) ^ x;      // 0 where the byte is A/C/G/T
        const uint32_t nz = (((ne & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | ne) & 0x80808080u;
        const uint32_t ex4 = __builtin_amdgcn_udot4(nz >> 7, 0x08040201u, 0u, false);
        LO |= (uint64_t)lo4 << (4 * i);
        HI |= (uint64_t)hi4 << (4 * i);
        EX |= (uint64_t)ex4 << (4 * i);
    }
    LO >>= off;
    HI >>= off;
    EX >>= off;
    const uint32_t kmask = k >= 32 ? ~0u : ((1u << k) - 1u);
    if (!PFX) {
        // no prefix, and every byte the lane's windows span is A/C/G/T (the
        // common case): every window counts, no per-window tests; rc(w) from
        // the complemented planes reversed once per round
        const uint32_t nv = act ? (uint32_t)(Wl - w0 < (uint64_t)NS ? Wl - w0 : (uint64_t)NS) : 0u;
        const uint32_t nb = nv + k - 1;                            // bytes spanned (<= 47)
        if (nv > 0 && (EX & ((1ull << nb) - 1)) == 0) {
            const uint64_t RLO = tab_brev64(~LO), RHI = tab_brev64(~HI);
#pragma unroll
            for (int m = 0; m < NS; ++m) {
                const uint32_t flo = (uint32_t)(LO >> m) & kmask, fhi = (uint32_t)(HI >> m) & kmask;
                const uint32_t rlo = (uint32_t)(RLO >> (64 - m - k)) & kmask;
                const uint32_t rhi = (uint32_t)(RHI >> (64 - m - k)) & kmask;
                const uint64_t cf = ((uint64_t)fhi << k) | flo, cr = ((uint64_t)rhi << k) | rlo;
                key[OFF + m] = tab_key(a, cf, cr);
            }
            return ((nv >= 32 ? ~0u : (1u << nv) - 1u)) << OFF;
        }
    }
    const uint32_t sh = 32 - k;
    uint32_t valid = 0;
#pragma unroll
    for (int m = 0; m < NS; ++m) {
        if (!act || w0 + m >= Wl) continue;
        const uint32_t flo = (uint32_t)(LO >> m) & kmask, fhi = (uint32_t)(HI >> m) & kmask;
        const uint32_t fx = (uint32_t)(EX >> m) & kmask;
        const uint32_t rlo = __brev(~flo & kmask) >> sh, rhi = __brev(~fhi & kmask) >> sh, rx = __brev(fx) >> sh;
        const bool fm = (((flo ^ a.plo) | (fhi ^ a.phi) | fx) & a.pmask) == 0;   // w starts with P
        const bool rm = (((rlo ^ a.plo) | (rhi ^ a.phi) | rx) & a.pmask) == 0;   // rc(w) starts with P
        if (fx == 0) {
            if (fm || rm) {
                const uint64_t cf = ((uint64_t)fhi << k) | flo, cr = ((uint64_t)rhi << k) | rlo;
                key[OFF + m] = tab_key(a, cf, cr);
                valid |= 1u << m;
            }
        } else if (rec) {
            const uint64_t pos = st + w0 + m;
            if (a.canonical) {
                tab_record(a, pos, 0);
            } else {
                if (fm) tab_record(a, pos, 0);
                if (rm) tab_record(a, pos, 1);
            }
        }
    }
    return valid << OFF;
}

__device__ __forceinline__ TabCur tab_cursor(const TabArgs &a, uint32_t waves) {
    TabCur c;
    const uint64_t m0 = (uint64_t)blockIdx.x * a.lpw;
    c.end = m0 + a.lpw < a.n_lines ? m0 + a.lpw : a.n_lines;
    c.m = m0 + (threadIdx.x >> 6);
    c.seg = 0;
    c.stride = waves;
    tab_fetch(a, c);
    return c;
}

}  // namespace

// pass 1, histogram: keys per (workgroup, partition)
template <bool PFX>
__global__ __launch_bounds__(256) void tab_hist1_kernel(TabArgs a) {
    __shared__ uint32_t hist[TAB_NB];
    for (uint32_t i = threadIdx.x; i < TAB_NB; i += 256) hist[i] = 0;
    __syncthreads();
    TabCur c = tab_cursor(a, 4);
    while (c.m < c.end) {
        uint64_t key[TAB_RPL];
        uint32_t v = tab_round<TAB_RPL, 0, PFX>(a, c, false, key);
#pragma unroll
        for (int j = 0; j < TAB_RPL; ++j)
            if (v & (1u << j)) atomicAdd(&hist[key[j] >> (64 - TAB_L1)], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < TAB_NB; i += 256) a.H1[(uint64_t)i * a.nwg + blockIdx.x] = hist[i];
}

// pass 1, scatter in half-size workgroups: 512 threads, rounds of 8 K keys,
// 80 KB of LDS -- two workgroups per CU, so that one's write-out overlaps the
// other's window formation (one 1,024-thread workgroup per CU runs its
// formation, LDS sort and stores strictly one after another).  Thread t keeps
// bins 2t and 2t + 1.
constexpr int TAB_WGH = 512;
template <bool PFX>
__global__ __launch_bounds__(TAB_WGH) void tab_scatter1h_kernel(TabArgs a) {
    __shared__ uint64_t srt[TAB_RPL * TAB_WGH];
    __shared__ uint64_t cur[TAB_NB];
    __shared__ uint32_t bcnt[TAB_NB];
    __shared__ uint16_t bst[TAB_NB];                 // (round starts < 8 K)
    uint32_t *const ws = (uint32_t *)srt;            // (scan scratch: srt is free between rounds)
    const uint32_t t = threadIdx.x, b0 = 2 * t, b1 = 2 * t + 1;
    cur[b0] = a.base + a.H1s[(uint64_t)b0 * a.nwg + blockIdx.x];
    cur[b1] = a.base + a.H1s[(uint64_t)b1 * a.nwg + blockIdx.x];
    bcnt[b0] = 0;
    bcnt[b1] = 0;
    __syncthreads();
    TabCur c = tab_cursor(a, TAB_WGH / 64);
    while (true) {
        uint64_t key[TAB_RPL];
        uint32_t rank[TAB_RPL];
        uint32_t v = 0;
        if (c.m < c.end) v = tab_round<TAB_RPL, 0, PFX>(a, c, true, key);
#pragma unroll
        for (int j = 0; j < TAB_RPL; ++j)
            rank[j] = (v & (1u << j)) ? atomicAdd(&bcnt[key[j] >> (64 - TAB_L1)], 1u) : 0u;
        __syncthreads();
        uint32_t total;
        const uint32_t c0 = bcnt[b0], c1 = bcnt[b1];
        const uint32_t st0 = block_excl_512(c0 + c1, ws, &total), st1 = st0 + c0;
        bst[b0] = (uint16_t)st0;
        bst[b1] = (uint16_t)st1;
        cur[b0] -= st0;                           // (write-out: B1[cur[p] + i], one LDS read per key)
        cur[b1] -= st1;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < TAB_RPL; ++j)
            if (v & (1u << j)) srt[bst[key[j] >> (64 - TAB_L1)] + rank[j]] = key[j];
        __syncthreads();
        for (uint32_t i = t; i < total; i += TAB_WGH) {
            const uint64_t h = srt[i];
            b1_store(a, cur[(uint32_t)(h >> (64 - TAB_L1))] + i, h);
        }
        __syncthreads();
        cur[b0] += st0 + c0;
        cur[b1] += st1 + c1;
        bcnt[b0] = 0;
        bcnt[b1] = 0;
        if (!__syncthreads_or(c.m < c.end)) break;
    }
}

// pass 1 without the counting pass (no prefix, k <= 31: every window of a
// line is a key, so a workgroup's share of keys is known from its lines):
// partition p's keys of workgroup w go to a run of fixed capacity at base +
// p * R + pcw[w] (the workgroup's mean share mu + 2 sqrt(mu) + 4, rounded up
// to 8 keys: table_pass1_fixed in kmer_tabhost.hip), in the same LDS-sorted rounds as
// tab_scatter1h; the run's unused tail is filled with TAB_SENT, which pass 2
// skips.  A key past its run's capacity goes to its partition's spill area,
// right after the partition's runs (one LDS-free global atomic per spilled
// key: ~2 % of the runs spill a few keys), so a partition stays ONE
// contiguous range for pass 2; a full spill area (a repeated k-mer crowding
// one partition) sends the chunk to the counting pass.  Saves tab_hist1's
// second formation of every window.
template <bool PFX>
__global__ __launch_bounds__(TAB_WGH) void tab_scatter1f_kernel(TabArgs a) {
    __shared__ uint64_t srt[TAB_RPL * TAB_WGH];
    __shared__ uint32_t fill[TAB_NB];
    __shared__ uint32_t bcnt[TAB_NB];
    __shared__ uint16_t bst[TAB_NB];                 // (round starts < 8 K)
    uint32_t *const ws = (uint32_t *)srt;            // (scan scratch: srt is free between rounds)
    const uint32_t t = threadIdx.x, b0 = 2 * t, b1 = 2 * t + 1;
    const uint64_t r0 = a.base + a.pcw[blockIdx.x];
    const uint32_t cap = (uint32_t)(a.pcw[blockIdx.x + 1] - a.pcw[blockIdx.x]);
    const uint64_t R = a.PS;                         // (partition stride: runs + spill area)
    fill[b0] = 0;
    fill[b1] = 0;
    bcnt[b0] = 0;
    bcnt[b1] = 0;
    __syncthreads();
    TabCur c = tab_cursor(a, TAB_WGH / 64);
    while (true) {
        uint64_t key[TAB_RPL];
        uint32_t rank[TAB_RPL];
        uint32_t v = 0;
        if (c.m < c.end) v = tab_round<TAB_RPL, 0, PFX>(a, c, true, key);
#pragma unroll
        for (int j = 0; j < TAB_RPL; ++j)
            rank[j] = (v & (1u << j)) ? atomicAdd(&bcnt[key[j] >> (64 - TAB_L1)], 1u) : 0u;
        __syncthreads();
        uint32_t total;
        const uint32_t c0 = bcnt[b0], c1 = bcnt[b1];
        const uint32_t st0 = block_excl_512(c0 + c1, ws, &total), st1 = st0 + c0;
        bst[b0] = (uint16_t)st0;
        bst[b1] = (uint16_t)st1;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < TAB_RPL; ++j)
            if (v & (1u << j)) srt[bst[key[j] >> (64 - TAB_L1)] + rank[j]] = key[j];
        __syncthreads();
        for (uint32_t i = t; i < total; i += TAB_WGH) {
            const uint64_t h = srt[i];
            const uint32_t p = (uint32_t)(h >> (64 - TAB_L1));
            const uint32_t j = fill[p] + (i - bst[p]);
            if (j < cap) {
                b1_store(a, r0 + p * R + j, h);
            } else {                                 // past the run: the partition's spill area
                const unsigned long long o = atomicAdd(&a.pcur[p], 1ull);
                if (o < a.S) b1_store(a, a.base + p * R + a.R + o, h);
                else atomicAdd(&a.pcur[TAB_NB], 1ull);
            }
        }
        __syncthreads();
        fill[b0] += c0;
        fill[b1] += c1;
        bcnt[b0] = 0;
        bcnt[b1] = 0;
        if (!__syncthreads_or(c.m < c.end)) break;
    }
    // the runs' unused tails (a wave per partition)
    for (uint32_t p = t >> 6; p < TAB_NB; p += TAB_WGH / 64) {
        const uint32_t f = min(fill[p], cap);
        for (uint32_t j = f + (t & 63); j < cap; j += 64) b1_fill(a, r0 + p * R + j);
    }
}

// the unused slots of the spill areas (tab_scatter1f): TAB_SENT, skipped by pass 2
__global__ __launch_bounds__(256) void tab_spill_fill_kernel(bool narrow, uint64_t *B1, uint64_t base, uint64_t R,
                                                             uint64_t S, uint64_t PS, const unsigned long long *pcur) {
    const uint32_t p = blockIdx.x;
    const uint64_t used = pcur[p] < S ? pcur[p] : S;
    for (uint64_t i = used + threadIdx.x; i < S; i += 256) {
        if (narrow) ((uint32_t *)B1)[base + p * PS + R + i] = TAB_SENT32;
        else B1[base + p * PS + R + i] = TAB_SENT;
    }
}

// keys (windows) of each pass-1 workgroup's share of lines: the fixed runs of
// tab_scatter1f are sized from them
__global__ __launch_bounds__(256) void tab_wg_windows_kernel(const SeqLine *lines, uint64_t n, uint64_t lpw,
                                                             uint32_t k, uint64_t *W) {
    __shared__ uint64_t ws[4];
    const uint64_t m0 = (uint64_t)blockIdx.x * lpw, m1 = m0 + lpw < n ? m0 + lpw : n;
    uint64_t x = 0;
    for (uint64_t m = m0 + threadIdx.x; m < m1; m += 256) {
        const uint64_t len = lines[m].len;
        x += len >= k ? len - k + 1 : 0;
    }
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = x;
    __syncthreads();
    if (threadIdx.x == 0) W[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// pass 1, scatter: the same keys, LDS-sorted by partition in rounds of 16 K,
// written as one contiguous run per partition and round
template <bool PFX>
__global__ __launch_bounds__(TAB_WG1) void tab_scatter1_kernel(TabArgs a) {
    __shared__ uint64_t srt[TAB_ROUND];
    __shared__ uint64_t cur[TAB_NB];
    __shared__ uint32_t bcnt[TAB_NB], bst[TAB_NB];
    __shared__ uint32_t ws[16];
    const uint32_t t = threadIdx.x;
    cur[t] = a.base + a.H1s[(uint64_t)t * a.nwg + blockIdx.x];
    bcnt[t] = 0;
    __syncthreads();
    TabCur c = tab_cursor(a, TAB_WG1 / 64);
    while (true) {
        uint64_t key[TAB_RPL];
        uint32_t rank[TAB_RPL];
        uint32_t v = 0;
        if (c.m < c.end) v = tab_round<TAB_RPL, 0, PFX>(a, c, true, key);
#pragma unroll
        for (int j = 0; j < TAB_RPL; ++j)
            rank[j] = (v & (1u << j)) ? atomicAdd(&bcnt[key[j] >> (64 - TAB_L1)], 1u) : 0u;
        __syncthreads();
        uint32_t total;
        const uint32_t cnt = bcnt[t];
        const uint32_t my_st = block_excl_1024(cnt, ws, &total);
        bst[t] = my_st;
        cur[t] -= my_st;                          // (write-out: B1[cur[p] + i], one LDS read per key)
        __syncthreads();
#pragma unroll
        for (int j = 0; j < TAB_RPL; ++j)
            if (v & (1u << j)) srt[bst[key[j] >> (64 - TAB_L1)] + rank[j]] = key[j];
        __syncthreads();
#ifndef TAB_EXP_S1_NOSTORE                         // (experiment builds only)
        for (uint32_t i = t; i < total; i += TAB_WG1) {
            const uint64_t h = srt[i];
            b1_store(a, cur[(uint32_t)(h >> (64 - TAB_L1))] + i, h);
        }
#endif
        __syncthreads();
        cur[t] += my_st + cnt;
        bcnt[t] = 0;
        if (!__syncthreads_or(c.m < c.end)) break;
    }
}

// Long lines (contigs) are cut into pieces of <= TAB_PIECE windows, so that
// pass 1's per-workgroup shares of lines carry similar work: table mode has no
// order, so a piece is just a shorter line (its k-1 byte overlap with the next
// piece holds no window start of its own).  wcount = 2 W per line.
// *split is set when a line does not map to exactly one piece (long or empty)
__global__ __launch_bounds__(256) void tab_piece_count_kernel(const uint64_t *wcount, uint64_t n, uint32_t *pc,
                                                              uint32_t *split) {
    bool any = false;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t w = wcount[i] / 2;
        const uint32_t np = (uint32_t)((w + TAB_PIECE - 1) / TAB_PIECE);
        pc[i] = np;
        any |= np != 1u;
    }
    if (__any(any) && (threadIdx.x & 63) == 0) atomicOr(split, 1u);
}

__global__ __launch_bounds__(256) void tab_piece_write_kernel(const SeqLine *lines, const uint64_t *wcount,
                                                              const uint64_t *pbase, uint64_t n, uint32_t k,
                                                              SeqLine *out) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t w = wcount[i] / 2;
        const SeqLine sl = lines[i];
        uint64_t o = pbase[i];
        for (uint64_t s0 = 0; s0 < w; s0 += TAB_PIECE) {
            const uint64_t pw = w - s0 < TAB_PIECE ? w - s0 : TAB_PIECE;
            SeqLine p;
            p.start = sl.start + s0;
            p.len = pw + k - 1;
            p.line_index = sl.line_index;
            out[o++] = p;
        }
    }
}

// chunk-relative start of every pass-1 partition (+ the chunk's key total)
__global__ void tab_p1_offsets_kernel(const uint64_t *H1s, uint32_t nwg, uint64_t *out) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < TAB_NB) out[p] = H1s[(uint64_t)p * nwg];
}

// pass 2, histogram: keys per (unit, bucket bin)
__global__ __launch_bounds__(256) void tab_hist2_kernel(const uint64_t *B1, const TabUnit *units, uint32_t *H2) {
    __shared__ uint32_t hist[TAB_NB];
    for (uint32_t i = threadIdx.x; i < TAB_NB; i += 256) hist[i] = 0;
    __syncthreads();
    const TabUnit un = units[blockIdx.x];
    const uint64_t *src = B1 + un.start;
    uint32_t len = un.len;
    // 16-B loads, 4 in flight per thread (the unit's first key alone when it
    // is not 16-B aligned, and its last when an odd count remains)
    // (TAB_SENT: an unused pass-1 slot, not a key)
    if (((uintptr_t)src & 8u) && len) {
        if (threadIdx.x == 0 && src[0] != TAB_SENT) atomicAdd(&hist[(uint32_t)(src[0] >> TAB_RBITS) & (TAB_NB - 1)], 1u);
        ++src;
        --len;
    }
    const ulonglong2 *s2 = (const ulonglong2 *)src;
    const uint32_t np = len / 2;
    uint32_t i = threadIdx.x;
    for (; i + 3 * 256 < np; i += 4 * 256) {
        ulonglong2 x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) x[u] = s2[i + u * 256];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (x[u].x != TAB_SENT) atomicAdd(&hist[(uint32_t)(x[u].x >> TAB_RBITS) & (TAB_NB - 1)], 1u);
            if (x[u].y != TAB_SENT) atomicAdd(&hist[(uint32_t)(x[u].y >> TAB_RBITS) & (TAB_NB - 1)], 1u);
        }
    }
    for (; i < np; i += 256) {
        const ulonglong2 x = s2[i];
        if (x.x != TAB_SENT) atomicAdd(&hist[(uint32_t)(x.x >> TAB_RBITS) & (TAB_NB - 1)], 1u);
        if (x.y != TAB_SENT) atomicAdd(&hist[(uint32_t)(x.y >> TAB_RBITS) & (TAB_NB - 1)], 1u);
    }
    if ((len & 1u) && threadIdx.x == 0 && src[len - 1] != TAB_SENT)
        atomicAdd(&hist[(uint32_t)(src[len - 1] >> TAB_RBITS) & (TAB_NB - 1)], 1u);
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < TAB_NB; b += 256) H2[un.hbase + (uint64_t)b * un.nunits + un.u] = hist[b];
}

// pass 2, scatter: a unit's keys into their buckets (LDS sort per round)
__global__ __launch_bounds__(TAB_WG1) void tab_scatter2_kernel(const uint64_t *B1, const TabUnit *units,
                                                               const uint64_t *H2s, uint64_t *B2) {
    __shared__ uint64_t srt[TAB_ROUND];
    __shared__ uint64_t cur[TAB_NB];
    __shared__ uint32_t bcnt[TAB_NB], bst[TAB_NB];
    __shared__ uint32_t ws[16];
    const uint32_t t = threadIdx.x;
    const TabUnit un = units[blockIdx.x];
    const uint64_t *src = B1 + un.start;
#ifdef TAB_EXP_S2_COPY                            // (experiment builds only: a plain streaming copy)
    for (uint32_t i = t; i < un.len; i += TAB_WG1) B2[un.start + i] = src[i];
    return;
#endif
    cur[t] = H2s[un.hbase + (uint64_t)t * un.nunits + un.u];
    bcnt[t] = 0;
    __syncthreads();
    // the next round's keys are loaded as soon as this round's sit in LDS, in
    // flight while the round is written out
    uint64_t key[TAB_RPL];
#pragma unroll
    for (int j = 0; j < TAB_RPL; ++j) {
        const uint32_t i = j * TAB_WG1 + t;
        key[j] = i < un.len ? src[i] : 0;
    }
    for (uint32_t r0 = 0; r0 < un.len; r0 += TAB_ROUND) {
        uint32_t rank[TAB_RPL];
#pragma unroll
        for (int j = 0; j < TAB_RPL; ++j) {
            const uint32_t i = r0 + j * TAB_WG1 + t;
            rank[j] = i < un.len && key[j] != TAB_SENT
                          ? atomicAdd(&bcnt[(uint32_t)(key[j] >> TAB_RBITS) & (TAB_NB - 1)], 1u) : 0u;
        }
        __syncthreads();
        uint32_t total;
        const uint32_t cnt = bcnt[t];
        const uint32_t my_st = block_excl_1024(cnt, ws, &total);
        bst[t] = my_st;
        cur[t] -= my_st;                          // (write-out: B2[cur[b] + i], one LDS read per key)
        __syncthreads();
#pragma unroll
        for (int j = 0; j < TAB_RPL; ++j) {
            const uint32_t i = r0 + j * TAB_WG1 + t;
            if (i < un.len && key[j] != TAB_SENT) srt[bst[(uint32_t)(key[j] >> TAB_RBITS) & (TAB_NB - 1)] + rank[j]] = key[j];
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < TAB_RPL; ++j) {
            const uint32_t i = r0 + TAB_ROUND + j * TAB_WG1 + t;
            key[j] = i < un.len ? src[i] : 0;
        }
#ifndef TAB_EXP_S2_NOSTORE                         // (experiment builds only: -DTAB_EXP_S2_NOSTORE)
        for (uint32_t i = t; i < total; i += TAB_WG1) {
            const uint64_t h = srt[i];
#ifdef TAB_EXP_NT
            __builtin_nontemporal_store(h, &B2[cur[(uint32_t)(h >> TAB_RBITS) & (TAB_NB - 1)] + i]);
#else
            B2[cur[(uint32_t)(h >> TAB_RBITS) & (TAB_NB - 1)] + i] = h;
#endif
        }
#endif
        __syncthreads();
        cur[t] += my_st + cnt;
        bcnt[t] = 0;
        __syncthreads();
    }
}

// pass 2, scatter with aligned write-out: rounds of 8 K keys; each bucket's
// keys of a round go out only up to the last 64-B boundary of its B2 range
// (8 keys), the rest (<= 7 keys) is carried in the bucket owner's registers
// into the next round's LDS sort.  A round then writes whole 64-B blocks
// (besides the first, partial block of each (unit, bucket) range) instead of
// ~16-key runs that straddle lines, which left partial L2 lines to be evicted
// before the next round completed them.  Thread t owns bucket t; bucket
// order inside a range is free (table mode has no order).
constexpr int TS2_RPL = 10;                           // (A/B: 8 / 9 / 10 -> C3 scatter2 56.8 / 56.2 / 56.2 ms)
constexpr int TS2_ROUND = TS2_RPL * TAB_WG1;           // new keys per round
constexpr int TS2_CARRY = 7;                           // carried keys per bucket (< one 64-B block)
__global__ __launch_bounds__(TAB_WG1) void tab_scatter2c_kernel(const uint64_t *B1, const TabUnit *units,
                                                                const uint64_t *H2s, uint64_t *B2) {
    __shared__ uint64_t srt[TS2_ROUND + TS2_CARRY * TAB_WG1];
    __shared__ uint64_t cur[TAB_NB];
    __shared__ uint32_t bcnt[TAB_NB], bst[TAB_NB];
    __shared__ uint32_t ws[16];
    const uint32_t t = threadIdx.x;
    const TabUnit un = units[blockIdx.x];
    const uint64_t *src = B1 + un.start;
    uint64_t dest = H2s[un.hbase + (uint64_t)t * un.nunits + un.u];   // next B2 slot of bucket t
    cur[t] = dest;
    bcnt[t] = 0;
    uint32_t cc = 0;                               // carried keys of bucket t
    uint64_t ck[TS2_CARRY];
#pragma unroll
    for (int i = 0; i < TS2_CARRY; ++i) ck[i] = 0;
    __syncthreads();
    uint64_t key[TS2_RPL];
#pragma unroll
    for (int j = 0; j < TS2_RPL; ++j) {
        const uint32_t i = j * TAB_WG1 + t;
        key[j] = i < un.len ? src[i] : 0;
    }
    for (uint32_t r0 = 0; r0 < un.len; r0 += TS2_ROUND) {
        const bool last = r0 + TS2_ROUND >= un.len;
        uint32_t rank[TS2_RPL];
#pragma unroll
        for (int j = 0; j < TS2_RPL; ++j) {
            const uint32_t i = r0 + j * TAB_WG1 + t;
            rank[j] = i < un.len && key[j] != TAB_SENT
                          ? atomicAdd(&bcnt[(uint32_t)(key[j] >> TAB_RBITS) & (TAB_NB - 1)], 1u) : 0u;
        }
        __syncthreads();
        const uint32_t n_new = bcnt[t], tot = n_new + cc;
        uint32_t total;
        const uint32_t my_st = block_excl_1024(tot, ws, &total);
        // keys of bucket t written this round: up to the last 64-B boundary
        const uint64_t aend = last ? dest + tot : ((dest + tot) & ~7ull);
        const uint32_t full = aend > dest ? (uint32_t)(aend - dest) : 0u;
        bst[t] = my_st;
        cur[t] = dest - my_st;                    // (write-out: B2[cur[b] + i] for i < bst[b] + full)
        __syncthreads();
        // this round's keys first, then the carried ones
#pragma unroll
        for (int j = 0; j < TS2_RPL; ++j) {
            const uint32_t i = r0 + j * TAB_WG1 + t;
            if (i < un.len && key[j] != TAB_SENT) srt[bst[(uint32_t)(key[j] >> TAB_RBITS) & (TAB_NB - 1)] + rank[j]] = key[j];
        }
#pragma unroll
        for (int i = 0; i < TS2_CARRY; ++i)
            if ((uint32_t)i < cc) srt[my_st + n_new + i] = ck[i];
        bcnt[t] = my_st + full;                   // (write-out limit of bucket t)
        __syncthreads();
#pragma unroll
        for (int j = 0; j < TS2_RPL; ++j) {
            const uint32_t i = r0 + TS2_ROUND + j * TAB_WG1 + t;
            key[j] = i < un.len ? src[i] : 0;
        }
        for (uint32_t i = t; i < total; i += TAB_WG1) {
            const uint64_t h = srt[i];
            const uint32_t b = (uint32_t)(h >> TAB_RBITS) & (TAB_NB - 1);
            if (i < bcnt[b]) B2[cur[b] + i] = h;
        }
        // the rest of bucket t is carried
        cc = tot - full;
#pragma unroll
        for (int i = 0; i < TS2_CARRY; ++i)
            if ((uint32_t)i < cc) ck[i] = srt[my_st + full + i];
        dest += full;
        __syncthreads();
        bcnt[t] = 0;
        __syncthreads();
    }
}

// pass 2 without the histogram pass (tab_hist2): when a bucket holds many
// keys (C3: ~11.4 K) its count is close to its mean, so bucket q gets a FIXED
// capacity region B2[q cap, (q + 1) cap) (mean + 6 sigma + 16, rounded to 8:
// one bucket in ~10^9 overflows, and then ERR_TAB_CAP sends the finish back
// to the counted route).  One workgroup per pass-1 partition walks the
// partition's units in order with scatter2c's rounds (LDS sort, aligned
// write-out, the carry in the bucket owner's registers across rounds AND
// units); the regions start on 64-B boundaries, so every block but the
// bucket's last is written whole.  blen[q] = the bucket's keys.  The unused
// tail of a region is never written nor read: the final takes (q cap,
// blen[q]) and writes its entries compactly (start = the scan of blen).
// Small buckets (C5: ~480 keys) share a REGION: qg consecutive buckets of the
// partition (rpp = ceil(1,024 / qg) regions per partition, region of bucket
// offset b = b gmag >> 20), whose summed count is again near its mean (C5: 11
// buckets, ~5.3 K keys, 8 % slack); the final sorts a region's keys by bucket
// anyway.  Fewer, larger regions also give longer write-out runs.
// NAR (narrow keys, k <= 21: h's low 22 bits are 0): B2 holds the 32-bit key
// (uint32_t)(h >> 22) = bucket offset << 22 | the remainder's top 22 bits (the
// partition is the region's), half the bytes; the LDS sort runs on those
// 32-bit keys and the write-out aligns to 16 keys (64 B).
// B1N: pass-1 keys of 32 bits (narrow, from this session's pass 1)
template <bool NAR, bool B1N>
__global__ __launch_bounds__(TAB_WG1) void tab_scatter2f_kernel(const uint64_t *B1, const TabUnit *units,
                                                                const uint32_t *ufirst, uint32_t p0, uint64_t cap,
                                                                uint32_t rpp, uint32_t gmag, void *B2v,
                                                                uint32_t *blen, unsigned int *err) {
    using KT = typename std::conditional<NAR, uint32_t, uint64_t>::type;
    constexpr int CARRY = NAR ? 15 : TS2_CARRY;    // (< one 64-B block of keys)
    constexpr uint64_t AL = NAR ? 16 : 8;
    __shared__ uint64_t srt_raw[TS2_ROUND + TS2_CARRY * TAB_WG1];
    static_assert(sizeof(KT) * (TS2_ROUND + CARRY * TAB_WG1) <= sizeof(srt_raw), "scatter2f LDS");
    KT *const srt = (KT *)srt_raw;
    KT *const B2 = (KT *)B2v;
    __shared__ uint64_t cur[TAB_NB];
    __shared__ uint32_t bcnt[TAB_NB], bst[TAB_NB];
    __shared__ uint32_t ws[16];
    __shared__ uint32_t sovf;
    const uint32_t t = threadIdx.x, p = p0 + blockIdx.x;
    // region (p, b) of a key (threads t < rpp own regions)
    auto reg = [&](uint64_t h) { return (((uint32_t)(h >> TAB_RBITS) & (TAB_NB - 1)) * gmag) >> 20; };
    auto regk = [&](KT x) {
        return NAR ? (((uint32_t)x >> (TAB_RBITS - TAB_NSH)) * gmag) >> 20 : reg((uint64_t)x);
    };
    auto kt = [&](uint64_t h) { return NAR ? (KT)((h >> TAB_NSH) & 0x7FFFFFFFu) : (KT)h; };
    // a pass-1 slot as loaded (B1N: 32 bits), and as h (B1N: without the
    // partition bits, which no step here reads) -- converted at use, so the
    // next round's loads stay in flight through the write-out
    using LT = typename std::conditional<B1N, uint32_t, uint64_t>::type;
    auto hk = [&](LT v) -> uint64_t {
        if (!B1N) return (uint64_t)v;
        return (uint32_t)v == TAB_SENT32 ? TAB_SENT : (uint64_t)v << TAB_NSH;
    };
    const uint64_t q = (uint64_t)p * rpp + t;
    const uint64_t pbase = (uint64_t)p * rpp * cap;   // (region (p, b): pbase + b cap)
    uint64_t dest = q * cap;                       // next B2 slot of region t
    const uint64_t cend = dest + cap;
    bcnt[t] = 0;
    if (t == 0) sovf = 0;
    uint32_t cc = 0;                               // carried keys of region t
    KT ck[CARRY];
#pragma unroll
    for (int i = 0; i < CARRY; ++i) ck[i] = 0;
    __syncthreads();
    const uint32_t u0 = ufirst[p], nun = units[u0].nunits;
    for (uint32_t ui = 0; ui < nun; ++ui) {
        const TabUnit un = units[u0 + ui];
        const LT *src = (const LT *)B1 + un.start;
        LT key[TS2_RPL];
#pragma unroll
        for (int j = 0; j < TS2_RPL; ++j) {
            const uint32_t i = j * TAB_WG1 + t;
            key[j] = i < un.len ? src[i] : 0;
        }
        for (uint32_t r0 = 0; r0 < un.len; r0 += TS2_ROUND) {
            const bool last = ui + 1 == nun && r0 + TS2_ROUND >= un.len;
            uint32_t rank[TS2_RPL];
#pragma unroll
            for (int j = 0; j < TS2_RPL; ++j) {
                const uint32_t i = r0 + j * TAB_WG1 + t;
                rank[j] = i < un.len && hk(key[j]) != TAB_SENT
                              ? atomicAdd(&bcnt[reg(hk(key[j]))], 1u) : 0u;
            }
            __syncthreads();
            const uint32_t n_new = bcnt[t], tot = n_new + cc;
            uint32_t total;
            const uint32_t my_st = block_excl_1024(tot, ws, &total);
            const uint64_t aend = last ? dest + tot : ((dest + tot) & ~(AL - 1));
            const uint32_t full = aend > dest ? (uint32_t)(aend - dest) : 0u;
            bst[t] = my_st;
            cur[t] = dest - my_st;
            __syncthreads();
#pragma unroll
            for (int j = 0; j < TS2_RPL; ++j) {
                const uint32_t i = r0 + j * TAB_WG1 + t;
                if (i < un.len && hk(key[j]) != TAB_SENT)
                    srt[bst[reg(hk(key[j]))] + rank[j]] = kt(hk(key[j]));
            }
#pragma unroll
            for (int i = 0; i < CARRY; ++i)
                if ((uint32_t)i < cc) srt[my_st + n_new + i] = ck[i];
            bcnt[t] = my_st + full;
            __syncthreads();
#pragma unroll
            for (int j = 0; j < TS2_RPL; ++j) {
                const uint32_t i = r0 + TS2_ROUND + j * TAB_WG1 + t;
                key[j] = i < un.len ? src[i] : 0;
            }
            for (uint32_t i = t; i < total; i += TAB_WG1) {
                const KT h = srt[i];
                const uint32_t b = regk(h);
                if (i < bcnt[b]) {
                    const uint64_t pos = cur[b] + i;
                    if (pos < pbase + (uint64_t)(b + 1) * cap) B2[pos] = h;
                    else sovf = 1;                   // (benign race: any writer sets it)
                }
            }
            cc = tot - full;
#pragma unroll
            for (int i = 0; i < CARRY; ++i)
                if ((uint32_t)i < cc) ck[i] = srt[my_st + full + i];
            dest += full;
            __syncthreads();
            bcnt[t] = 0;
            __syncthreads();
        }
    }
    if (t < rpp) blen[q] = (uint32_t)((dest < cend ? dest : cend) - q * cap);
    if (t == 0 && sovf) atomicOr(err, ERR_TAB_CAP);
}

hipError_t launch_tab_scatter2f(const uint64_t *B1, const TabUnit *units, const uint32_t *ufirst, uint32_t p0,
                                uint32_t np, uint64_t cap, uint32_t rpp, uint32_t gmag, bool narrow, bool b1n,
                                void *B2, uint32_t *blen, unsigned int *err, hipStream_t s) {
    if (rpp == 0 || rpp > TAB_NB || (cap & (narrow ? 15 : 7)) || (b1n && !narrow)) return hipErrorInvalidValue;
    if (!np) return hipSuccess;
    if (b1n)
        hipLaunchKernelGGL((tab_scatter2f_kernel<true, true>), dim3(np), dim3(TAB_WG1), 0, s, B1, units, ufirst, p0,
                           cap, rpp, gmag, B2, blen, err);
    else if (narrow)
        hipLaunchKernelGGL((tab_scatter2f_kernel<true, false>), dim3(np), dim3(TAB_WG1), 0, s, B1, units, ufirst, p0,
                           cap, rpp, gmag, B2, blen, err);
    else
        hipLaunchKernelGGL((tab_scatter2f_kernel<false, false>), dim3(np), dim3(TAB_WG1), 0, s, B1, units, ufirst, p0,
                           cap, rpp, gmag, B2, blen, err);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void tab_region_starts_kernel(const uint64_t *rstart, uint32_t rpp, uint32_t gmag,
                                                                uint64_t *start) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < TAB_NQ) start[q] = rstart[tab_region(q, rpp, gmag)];
    if (q == 0) start[TAB_NQ] = rstart[(uint64_t)TAB_NB * rpp];
}

hipError_t launch_tab_region_starts(const uint64_t *rstart, uint32_t rpp, uint32_t gmag, uint64_t *start,
                                    hipStream_t s) {
    hipLaunchKernelGGL(tab_region_starts_kernel, dim3(TAB_NQ / 256), dim3(256), 0, s, rstart, rpp, gmag, start);
    return hipGetLastError();
}

// bucket q = (p, b) starts at the scanned H2 entry of (p, b, unit 0)
// (the end: the keys counted by pass 2 -- B1 may hold TAB_SENT slots)
__global__ __launch_bounds__(256) void tab_starts_kernel(const uint64_t *H2s, const uint32_t *H2, uint64_t nh,
                                                         const TabUnit *pfirst, uint64_t *start) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < TAB_NQ) {
        const TabUnit u = pfirst[q >> TAB_L2];
        start[q] = H2s[u.hbase + (uint64_t)(q & (TAB_NB - 1)) * u.nunits];
    }
    if (q == 0) start[TAB_NQ] = nh ? H2s[nh - 1] + H2[nh - 1] : 0;
}

namespace {

// A final workgroup's Map statistics -> 3 device atomics per WORKGROUP (wave
// sums through LDS): device-scope atomics on one line serialise (~12 ns each),
// and every wave of the grid reaches this point at about the same time
__device__ __forceinline__ void tab_stats_out(unsigned long long *stats, uint64_t c, uint64_t kk, uint64_t sm,
                                              uint32_t waves, unsigned long long (*red)[3]) {
    for (int d = 32; d >= 1; d >>= 1) {
        c += __shfl_xor(c, d);
        kk += __shfl_xor(kk, d);
        sm += __shfl_xor(sm, d);
    }
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) {
        red[w][0] = c;
        red[w][1] = kk;
        red[w][2] = sm;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t0 = 0, t1 = 0, t2 = 0;
        for (uint32_t v = 0; v < waves; ++v) {
            t0 += red[v][0];
            t1 += red[v][1];
            t2 += red[v][2];
        }
        if (t0) {
            atomicAdd(&stats[0], t0);
            atomicAdd(&stats[1], t1);
            atomicAdd(&stats[2], t2);
        }
    }
}

// LDS slot of a remainder: its low bits are weak (a product's low bits see
// only the code's low bits), so the slot comes from a second multiply's top bits
__device__ __forceinline__ uint32_t tab_slot(uint64_t rem) {
    return (uint32_t)((rem * TAB_MUL) >> 51) & (TAB_SLOTS - 1);
}

__device__ __forceinline__ bool lds_flag(uint32_t *f) {
    return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0;
}

constexpr uint32_t TAB_PROBE_MAX = 256;      // a longer probe marks the range as overflowing

// Insert N of a lane's held keys (key[OFF + j] takes part iff bit OFF + j of
// `pend` is set) together:
// every step issues one CAS per pending key (independent, so their LDS round
// trips overlap) instead of walking each key's probe sequence in turn, which
// serialises the wave on its longest probe for every key.  CAS(EMPTY -> rem)
// returning EMPTY claims the slot, returning rem finds it; the count add needs
// no return.  Returns the slots this lane claimed.
template <int N, int M>
__device__ __forceinline__ uint32_t tab_insert_grp(uint64_t *tkey, uint32_t *tcnt, const uint64_t (&key)[M], int g,
                                                   uint32_t pend, uint32_t *ovf) {
    // (g is a constant once the caller's loop is unrolled: key[g + j] stays in registers)
    pend = (pend >> g) & ((1u << N) - 1u);
    uint64_t rem[N];
    uint32_t slot[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        rem[j] = key[g + j];
        slot[j] = tab_slot(rem[j]);
    }
    uint32_t claimed = 0;
    for (uint32_t step = 0; __any(pend != 0); ++step) {
        if (step == TAB_PROBE_MAX) {
            if (pend) __hip_atomic_store(ovf, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            break;
        }
#pragma unroll
        for (int j = 0; j < N; ++j) {
            if (!(pend & (1u << j))) continue;
            const uint64_t old = atomicCAS((unsigned long long *)&tkey[slot[j]], (unsigned long long)TAB_EMPTY,
                                           (unsigned long long)rem[j]);
            if (old == TAB_EMPTY || old == rem[j]) {
                __hip_atomic_fetch_add(&tcnt[slot[j]], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                claimed += old == TAB_EMPTY ? 1u : 0u;
                pend &= ~(1u << j);
            } else {
                slot[j] = (slot[j] + 1) & (TAB_SLOTS - 1);
            }
        }
    }
    return claimed;
}


}  // namespace

constexpr int TAB_KPT = 12;                   // bucket keys held per thread (register path)
constexpr uint32_t TAB_REG_MAX = TAB_KPT * TAB_FWG;
constexpr uint32_t TAB_SC = 1024;             // bucket starts cached in LDS per refill

// final: each workgroup merges a contiguous range of buckets in an LDS hash
// table, one UNIT at a time: a run of consecutive small buckets whose keys
// together fit one LDS range (<= range_keys), or one large bucket split into
// 2^sb remainder ranges.  A key enters the table as h - (first bucket of the
// unit << 44) = (bucket offset << 44) | remainder (offset < 64, so never the
// empty marker).  Entries (remainder, count) go to `out` at their bucket's
// start, the distinct count to nd[q], the Map statistics on the fly.
// Latency: bucket starts come from an LDS cache refilled every 1024 buckets;
// a unit of <= 12 K keys is held in registers (12 per thread), and the next
// unit's keys are loaded as soon as the current one's last range is merged,
// in flight while it is emitted.  Larger buckets (repeated keys, inputs
// beyond ~130 M reads) stream from HBM once per range.  The table is clean
// between ranges: emission clears the slots it reads.  Grouping small buckets
// divides the per-range fixed cost (barriers, key latency, the slot scan) by
// the group size (canonical C5: ~1 K keys per bucket).
constexpr uint32_t TAB_GMAX = 64;             // buckets per unit

constexpr uint32_t TAB_SB = 4096;             // sort path: bins (top 12 remainder bits)
constexpr uint32_t TAB_SORT_RUN = 128;        // sort path: largest 4-bin run a thread dedupes

__device__ __forceinline__ bool tab_cap_failed(const TabFinal &a);

__global__ __launch_bounds__(TAB_FWG) void tab_final_kernel(TabFinal a) {
    if (tab_cap_failed(a)) return;
    // hash table (8,192 slots of u64 key + u32 count) = the sort path's key array (12,288 u64)
    __shared__ uint64_t lbuf[TAB_SLOTS + TAB_SLOTS / 2];
    uint64_t *const tkey = lbuf;
    uint32_t *const tcnt = (uint32_t *)(lbuf + TAB_SLOTS);
    __shared__ uint32_t scnt[TAB_SB], sst[TAB_SB];
    __shared__ uint32_t sws[16], smax;
    __shared__ uint64_t stk[2 * 64];          // range stack [lo, hi) of unit keys
    __shared__ uint64_t sc[TAB_SC + 2];       // start[cbase .. cbase + TAB_SC + 1]
    __shared__ uint32_t nout[TAB_GMAX];       // entries emitted per bucket of the unit
    __shared__ uint32_t occ, sp, ovf;
    const uint32_t t = threadIdx.x, lane = t & 63;
    const uint32_t k = a.k;
    const uint32_t kmask = k >= 32 ? ~0u : ((1u << k) - 1u), sh = 32 - k;
    // [q0, q1): this workgroup's share of [qlo, qhi), or (list mode) an entry
    // of the sort kernel's leftover list
    uint32_t q0 = 0, q1 = 0;
    const uint64_t rk = a.range_keys;
    uint64_t st_canon = 0, st_keys = 0, st_sum = 0;
    uint64_t kn[TAB_KPT];
    // (experiments: phase clocks of wave 0, 100 MHz, in a -DTAB_PROF build only)
#ifdef TAB_PROF
    const bool prof = a.prof != nullptr && t == 0;
#else
    constexpr bool prof = false;
#endif
    uint64_t pt[6] = {0, 0, 0, 0, 0, 0}, tm = prof ? wall_clock64() : 0;
    auto mark = [&](int p) {
        if (prof) {
            const uint64_t x = wall_clock64();
            pt[p] += x - tm;
            tm = x;
        }
    };
    // a unit's keys (lanes past its end re-read its first key and are masked
    // at use): unconditional loads, all in flight together
    // (narrow B2, b2n: 32-bit keys h >> 22 without the partition bits, which
    // come from the unit's bucket ux)
    auto load_keys = [&](uint32_t ux, uint64_t s0x, uint64_t nx) {
        if (nx - 1 < (uint64_t)TAB_REG_MAX) {
            // (lane tests as t < nx - 1024 j: immediates, no per-j index registers)
            const int left = (int)nx - (int)t;
            if (a.b2n) {
                const uint32_t *src = (const uint32_t *)a.B2 + s0x;
                const uint64_t pb = (uint64_t)(ux >> TAB_L2) << (64 - TAB_L1);
#pragma unroll
                for (int j = 0; j < TAB_KPT; ++j)
                    kn[j] = pb | (uint64_t)src[left > j * (int)TAB_FWG ? j * TAB_FWG + t : 0u] << TAB_NSH;
            } else {
                const uint64_t *src = a.B2 + s0x;
#pragma unroll
                for (int j = 0; j < TAB_KPT; ++j) kn[j] = src[left > j * (int)TAB_FWG ? j * TAB_FWG + t : 0u];
            }
        }
    };
    auto refill = [&](uint32_t cb) {
        __syncthreads();
        for (uint32_t i = t; i < TAB_SC + 2; i += TAB_FWG) sc[i] = a.start[cb + i < TAB_NQ ? cb + i : TAB_NQ];
        __syncthreads();
    };
    // Map statistics of one canonical entry h (App. A.6)
    auto account = [&](uint64_t h, uint64_t cnt) {
        const uint64_t code = tab_code(h, k, a.narrow, a.inv);
        const uint32_t lo = (uint32_t)code & kmask, hi = (uint32_t)(code >> k) & kmask;
        const uint32_t rlo2 = __brev(~lo & kmask) >> sh, rhi2 = __brev(~hi & kmask) >> sh;
        const bool pal = lo == rlo2 && hi == rhi2;
        st_canon += 1;
        if (a.canonical) {
            // one key per class: the lexicographically smaller of w, rc w
            // (first differing base decides), counted C times
            const uint32_t dif = (lo ^ rlo2) | (hi ^ rhi2);
            const uint32_t j = dif ? __ffs(dif) - 1 : 0;
            const uint32_t bw = (((hi >> j) & 1u) << 1) | ((lo >> j) & 1u);
            const uint32_t br = (((rhi2 >> j) & 1u) << 1) | ((rlo2 >> j) & 1u);
            const bool wmin = dif == 0 || bw < br;
            const uint32_t clo = wmin ? lo : rlo2, chi = wmin ? hi : rhi2;
            const bool cs = (((clo ^ a.plo) | (chi ^ a.phi)) & a.pmask) == 0;
            st_keys += cs ? 1u : 0u;
            st_sum += cs ? cnt : 0;
        } else {
            const bool fs = (((lo ^ a.plo) | (hi ^ a.phi)) & a.pmask) == 0;
            const bool rs = !pal && (((rlo2 ^ a.plo) | (rhi2 ^ a.phi)) & a.pmask) == 0;
            st_keys += (fs ? 1u : 0u) + (rs ? 1u : 0u);
            st_sum += (fs ? (pal ? 2 * cnt : cnt) : 0) + (rs ? cnt : 0);
        }
    };
    uint32_t cbase = 0;
    // the unit starting at bucket u: its end (uniform over the workgroup; the
    // start cache must hold u's start, i.e. u <= cbase + TAB_SC)
    // (groups for the sort path fill the registers; the hash path's ranges
    // split a group whose distinct keys overflow the table)
    const uint64_t gk = !(KH_ABLATE(a) & 4) ? (uint64_t)TAB_REG_MAX : rk;
    // (fixed-capacity buckets, capq: one bucket per unit, keys at B2[q capq ..
    // q capq + inlen[q]), entries out at start[q])
    // (regions of qg buckets: u is a region's first bucket; the general kernel
    // sees them only in list mode, whole regions)
    auto unit_n = [&](uint32_t u, uint32_t e) -> uint64_t {
        return a.capq ? (uint64_t)a.inlen[tab_region(u, a.rpp, a.gmag)] : sc[e - cbase] - sc[u - cbase];
    };
    auto unit_in = [&](uint32_t u) -> uint64_t {
        return a.capq ? (uint64_t)tab_region(u, a.rpp, a.gmag) * a.capq : sc[u - cbase];
    };
    auto unit_end = [&](uint32_t u) -> uint32_t {
        uint32_t e = u + 1;
        if (a.capq) return min(u + a.qg, ((u >> TAB_L2) + 1) << TAB_L2);
        uint64_t tot = sc[u + 1 - cbase] - sc[u - cbase];
        if (tot > gk) return e;
        while (e < q1 && e - cbase < TAB_SC && e - u < TAB_GMAX) {
            const uint64_t ne = sc[e + 1 - cbase] - sc[e - cbase];
            if (tot + ne > gk) break;
            tot += ne;
            ++e;
        }
        return e;
    };
    for (uint32_t i = t; i < TAB_SLOTS; i += TAB_FWG) {
        tkey[i] = TAB_EMPTY;
        tcnt[i] = 0;
    }
    bool dirty = false;
    const uint32_t n_items = a.left ? *a.left_n : 1u;
    for (uint32_t item = a.left ? blockIdx.x : 0u; item < n_items; item += a.left ? gridDim.x : 1u) {
    if (a.left) {
        q0 = a.left[2 * item];
        q1 = a.left[2 * item + 1];
    } else {
        const uint32_t per = (a.qhi - a.qlo + gridDim.x - 1) / gridDim.x;
        q0 = min(a.qlo + blockIdx.x * per, a.qhi);
        q1 = q0 + per < a.qhi ? q0 + per : a.qhi;
    }
    cbase = q0;
    refill(cbase);
    uint32_t q = q0, qe = q0 < q1 ? unit_end(q0) : q0;
    if (q0 < q1) load_keys(q0, unit_in(q0), unit_n(q0, qe));
    while (q < q1) {
        if (q - cbase >= TAB_SC) {
            cbase = q;
            refill(cbase);
        }
        const uint32_t g = qe - q;                        // buckets in the unit
        const uint64_t s0 = sc[q - cbase], n = unit_n(q, qe), s0in = unit_in(q);   // (s0: output start)
        const uint64_t qbase = (uint64_t)q << TAB_RBITS;
        // the next unit (its keys are loaded while this one is emitted)
        const uint32_t qn = qe, qne = qn < q1 ? unit_end(qn) : qn;
        const bool more = qn < q1;
        const uint64_t s0n = more ? unit_in(qn) : 0, nn = more ? unit_n(qn, qne) : 0;
        const bool inreg = n <= TAB_REG_MAX;
        if (n == 0) {
            for (uint32_t i = t; i < g; i += TAB_FWG) a.nd[q + i] = 0;
            if (more) load_keys(qn, s0n, nn);
            mark(5);
            q = qn;
            qe = qne;
            continue;
        }
        if (n >= (1ull << 32) && t == 0) atomicOr(a.err, ERR_COUNT_OVERFLOW);   // (u32 counts)
        __syncthreads();                         // the previous unit is done with the LDS state
        if (t == 0) {
            // a group: one range over its keys; a large bucket: 2^sb remainder ranges
            // (<= 16 initial ranges: the stack holds 64, and a range with more
            // distinct keys than the table takes is split on demand)
            uint32_t sb = 0;
            while (g == 1 && sb < 4 && (n >> sb) > rk) ++sb;
            const uint32_t nsub = 1u << sb;
            const uint64_t w = ((uint64_t)g << TAB_RBITS) >> sb;
            for (uint32_t i = 0; i < nsub; ++i) {      // popped in ascending order
                stk[2 * i] = (uint64_t)(nsub - 1 - i) * w;
                stk[2 * i + 1] = (uint64_t)(nsub - i) * w;
            }
            sp = nsub;
        }
        for (uint32_t i = t; i < g; i += TAB_FWG) nout[i] = 0;
#pragma unroll
        for (int j = 0; j < TAB_KPT; ++j) kn[j] -= qbase;
        if (prof)
            for (int j = 0; j < TAB_KPT; ++j) asm volatile("" ::"v"(kn[j]));   // (clock after the key loads)
        mark(0);
        // Sort path (any unit held in registers: one bucket at C3, a group of
        // up to 64 small buckets at C5).  A counting sort of the unit's keys
        // into 4,096 LDS bins by their top 12 bits, then every thread dedupes
        // its 4 adjacent bins (~11 keys at C3) by comparison: one returning
        // LDS atomic per key and plain LDS stores, instead of a CAS + a count
        // add per key (plus probes) and a slot scan per range.  A unit with a
        // crowded run of bins (many copies of one key) takes the hash path below.
        if (inreg && !(KH_ABLATE(a) & 4)) {
            // bins: the top 12 bits of (bucket offset << 44 | remainder), so a
            // group's buckets occupy consecutive bin ranges
            const uint32_t bsh = TAB_RBITS + (g > 1 ? 32 - __clz(g - 1) : 0) - 12;
            for (uint32_t i = t; i < TAB_SB; i += TAB_FWG) scnt[i] = 0;
            if (t == 0) smax = 0;
            __syncthreads();
            uint32_t rank[TAB_KPT];
            {
                const int left = (int)n - (int)t;
#pragma unroll
                for (int j = 0; j < TAB_KPT; ++j)
                    rank[j] = left > j * (int)TAB_FWG
                                  ? atomicAdd(&scnt[(uint32_t)(kn[j] >> bsh) & (TAB_SB - 1)], 1u)
                                  : 0u;
            }
            __syncthreads();
            uint32_t c4[4], st4[4], s4 = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                c4[i] = scnt[4 * t + i];
                s4 += c4[i];
            }
            uint32_t tot = 0;
            uint32_t run = block_excl_1024(s4, sws, &tot);
            {
                uint32_t mx = s4;
                for (int d = 32; d >= 1; d >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, d));
                if (lane == 0) atomicMax(&smax, mx);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                st4[i] = run;
                sst[4 * t + i] = run;
                run += c4[i];
            }
            __syncthreads();
            if (smax <= TAB_SORT_RUN) {                 // (uniform)
                {
                    const int left = (int)n - (int)t;
#pragma unroll
                    for (int j = 0; j < TAB_KPT; ++j)
                        if (left > j * (int)TAB_FWG)
                            lbuf[sst[(uint32_t)(kn[j] >> bsh) & (TAB_SB - 1)] + rank[j]] = kn[j];
                }
                // the registers are free: the next unit's keys load during the dedupe
                if (more) load_keys(qn, s0n, nn);
                __syncthreads();
                // each distinct key once, with the count of its copies (a
                // key's copies share its bin); output slots from one LDS
                // counter bump per wave and key round (order inside a bucket
                // is free)
#pragma unroll 1
                for (int b = 0; b < 4; ++b)
                    for (uint32_t i = st4[b]; i < st4[b] + c4[b]; ++i) {
                        const uint64_t x = lbuf[i];
                        bool first = true;
                        for (uint32_t j = st4[b]; j < i; ++j) first &= lbuf[j] != x;
                        uint32_t cnt = 1;
                        if (first)
                            for (uint32_t j = i + 1; j < st4[b] + c4[b]; ++j) cnt += lbuf[j] == x ? 1u : 0u;
                        // one counter bump per wave, key round and bucket present
                        const uint32_t ql = (uint32_t)(x >> TAB_RBITS);
                        unsigned long long fm = __ballot(first);
                        uint32_t pos = 0;
                        if (g == 1 && fm) {              // (uniform) one bucket: one bump
                            const int ld = __ffsll((long long)fm) - 1;
                            uint32_t base = 0;
                            if (lane == (uint32_t)ld) base = atomicAdd(&nout[0], (uint32_t)__popcll(fm));
                            base = (uint32_t)__shfl((int)base, ld);
                            pos = base + (uint32_t)__popcll(fm & ((1ull << lane) - 1ull));
                            fm = 0;
                        }
                        while (fm) {
                            const int ld = __ffsll((long long)fm) - 1;
                            const uint32_t qx = (uint32_t)__shfl((int)ql, ld);
                            const unsigned long long mq = __ballot(first && ql == qx);
                            uint32_t base = 0;
                            if (lane == (uint32_t)ld) base = atomicAdd(&nout[qx], (uint32_t)__popcll(mq));
                            base = (uint32_t)__shfl((int)base, ld);
                            if (first && ql == qx) pos = base + (uint32_t)__popcll(mq & ((1ull << lane) - 1ull));
                            fm &= ~mq;
                        }
                        if (first) {
                            a.out[(g == 1 ? s0 : sc[q + ql - cbase]) + pos] = ((x & TAB_RMASK) << 20) | cnt;
                            account(qbase + x, cnt);
                        }
                    }
                __syncthreads();
                for (uint32_t i = t; i < g; i += TAB_FWG) a.nd[q + i] = nout[i];
                dirty = true;                    // the hash path clears the table before use
                if (prof) pt[4] += 1;
                q = qn;
                qe = qne;
                continue;
            }
        }
        if (dirty) {                             // (uniform) lbuf held sort-path keys
            for (uint32_t i = t; i < TAB_SLOTS; i += TAB_FWG) {
                tkey[i] = TAB_EMPTY;
                tcnt[i] = 0;
            }
            dirty = false;                       // (the range loop's barrier publishes it)
        }
        while (true) {
            __syncthreads();
            const uint32_t top = sp;
            if (top == 0) break;
            const uint64_t rlo = stk[2 * (top - 1)], rhi = stk[2 * (top - 1) + 1];
            __syncthreads();
            if (t == 0) {
                sp = top - 1;
                occ = 0;
                ovf = 0;
            }
            __syncthreads();
            mark(1);
            if (prof) pt[4] += 1ull << 32;       // ranges
            if (inreg) {
                uint32_t pend = 0;
                const int left = (int)n - (int)t;
#pragma unroll
                for (int j = 0; j < TAB_KPT; ++j)
                    if (left > j * (int)TAB_FWG && kn[j] >= rlo && kn[j] < rhi && !(KH_ABLATE(a) & 1)) pend |= 1u << j;
                // (groups of four keys: enough CAS round trips in flight
                // without spilling the held keys)
                uint32_t cl = 0;
#pragma unroll
                for (int gi = 0; gi < TAB_KPT; gi += 4) cl += tab_insert_grp<4>(tkey, tcnt, kn, gi, pend, &ovf);
                for (int d = 32; d >= 1; d >>= 1) cl += __shfl_xor(cl, d);
                if (lane == 0 && cl) atomicAdd(&occ, cl);
            } else {
                const uint64_t *src = a.B2 + s0in;
                const uint32_t *src32 = (const uint32_t *)a.B2 + s0in;
                const uint64_t pb = (uint64_t)(q >> TAB_L2) << (64 - TAB_L1);
                for (uint64_t i = t; i < n; i += TAB_FWG) {
                    if (lds_flag(&ovf)) break;
                    uint64_t r1[1] = {(a.b2n ? pb | (uint64_t)src32[i] << TAB_NSH : src[i]) - qbase};
                    if (r1[0] >= rlo && r1[0] < rhi) {
                        uint32_t cl = tab_insert_grp<1>(tkey, tcnt, r1, 0, 1u, &ovf);
                        if (cl) atomicAdd(&occ, cl);
                    }
                }
            }
            __syncthreads();
            if (t == 0 && occ > a.cap) ovf = 1u;     // more distinct keys than the range may hold
            __syncthreads();
            mark(2);
            if (ovf) {
                for (uint32_t i = t; i < TAB_SLOTS; i += TAB_FWG) {
                    tkey[i] = TAB_EMPTY;
                    tcnt[i] = 0;
                }
                if (t == 0) {
                    if (rhi - rlo < 2 || sp + 2 > 64) {
                        atomicOr(a.err, ERR_TAB_SPLIT);
                    } else {
                        const uint64_t mid = rlo + (rhi - rlo) / 2;
                        stk[2 * sp] = mid;
                        stk[2 * sp + 1] = rhi;
                        stk[2 * sp + 2] = rlo;
                        stk[2 * sp + 3] = mid;
                        sp += 2;
                    }
                }
                continue;
            }
            // the unit's last range is merged: load the next unit's keys now,
            // in flight while this one is emitted
            if (top == 1 && more) load_keys(qn, s0n, nn);
            // emit (and clear) the occupied slots: per wave, one LDS counter
            // bump per bucket present among the wave's entries
#pragma unroll 1
            for (uint32_t i = t; i < TAB_SLOTS && !(KH_ABLATE(a) & 2); i += TAB_FWG) {
                const uint64_t key = tkey[i];
                const bool v = key != TAB_EMPTY;
                uint64_t m = __ballot(v);
                if (!m) continue;
                const uint32_t ql = v ? (uint32_t)(key >> TAB_RBITS) : 0u;
                uint32_t pos = 0;
                uint64_t obase = s0;
                if (g == 1) {                            // (uniform) one bucket: one counter bump per wave
                    const int ld = __ffsll((long long)m) - 1;
                    uint32_t base = 0;
                    if (lane == (uint32_t)ld) base = atomicAdd(&nout[0], (uint32_t)__popcll(m));
                    base = (uint32_t)__shfl((int)base, ld);
                    pos = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                } else {
                    while (m) {                          // one pass per distinct bucket in the wave
                        const int ld = __ffsll((long long)m) - 1;
                        const uint32_t qx = (uint32_t)__shfl((int)ql, ld);
                        const uint64_t mq = __ballot(v && ql == qx);
                        uint32_t base = 0;
                        if (lane == (uint32_t)ld) base = atomicAdd(&nout[qx], (uint32_t)__popcll(mq));
                        base = (uint32_t)__shfl((int)base, ld);
                        if (v && ql == qx) pos = base + (uint32_t)__popcll(mq & ((1ull << lane) - 1ull));
                        m &= ~mq;
                    }
                    if (v) obase = sc[q + ql - cbase];
                }
                if (!v) continue;
                const uint64_t rem = key & TAB_RMASK;
                const uint64_t cnt = tcnt[i];
                tkey[i] = TAB_EMPTY;
                tcnt[i] = 0;
                const uint32_t qq = q + ql;
                a.out[obase + pos] = (rem << 20) | (cnt < TAB_CMAX ? cnt : TAB_CMAX);
                const uint64_t h = ((uint64_t)qq << TAB_RBITS) | rem;
                if (cnt >= TAB_CMAX) {
                    const unsigned long long bi = atomicAdd(a.big_count, 1ull);
                    if (bi < a.big_cap) {
                        a.big[bi].h = h;
                        a.big[bi].count = cnt;
                    } else {
                        atomicOr(a.err, ERR_BIG_OVERFLOW);
                    }
                }
                account(h, cnt);
            }
            mark(3);
        }
        // (the range loop left after a barrier: every emission bump is in nout)
        for (uint32_t i = t; i < g; i += TAB_FWG) a.nd[q + i] = nout[i];
        if (prof) pt[4] += g;                        // buckets
        q = qn;
        qe = qne;
    }
    __syncthreads();                                 // (the next item refills the start cache)
    }
    if (prof)
        for (int i = 0; i < 6; ++i) a.prof[blockIdx.x * 8 + i] = pt[i];
    {
        __shared__ unsigned long long red[16][3];
        tab_stats_out(a.stats, st_canon, st_keys, st_sum, TAB_FWG / 64, red);
    }
}

// ---------------------------------------------------------------------------
// Sort final: the common case of the final merge, two 512-thread workgroups
// per CU (their phases overlap each other's barriers and key loads).  A unit
// -- one bucket of up to 12,288 keys (C3: ~11.4 K), or a group of consecutive
// small buckets of up to 6,144 keys together (C5) -- is held in registers
// (24 keys per thread), counting-sorted into 8,192 LDS bins by the top 13 bits
// of (bucket offset << 44 | remainder) -- 16-bit counts, two per LDS word --
// and every held key then scans its own bin (~1.4 keys at C3): the first copy
// of a key emits it with the number of copies.  One bucket's bin fixes the
// remainder's top 13 bits, so its LDS entries keep only the low 32 (48 KiB for
// 12,288 keys); a group's keep all 64 bits (6,144 keys, the same 48 KiB).  Units that do not fit -- larger
// buckets, or a bin with more than TS_BINMAX keys (many copies of a key) --
// go to the leftover list for the general kernel (hash path, range splits).
// ---------------------------------------------------------------------------
namespace {
constexpr int TS_KPT = 24;                            // keys held per thread
constexpr uint32_t TS_CAP1 = TS_KPT * TAB_SWG;        // one bucket: 12,288 keys, 32-bit LDS entries
constexpr uint32_t TS_CAPG = TS_CAP1 / 2;             // a group: 6,144 keys, 64-bit LDS entries
static_assert(TS_CAPG == TAB_SORT_GROUP_KEYS && TS_CAP1 == TAB_SORT_KEYS, "the host sizes regions by TS_CAPG / TS_CAP1");
constexpr uint32_t TS_BINMAX = 64;                    // fuller bins: leftover (general kernel)
constexpr uint32_t TS_GMAX = 64;                      // buckets per group
constexpr uint32_t TS_SC = 512;                       // bucket starts cached per refill

}  // namespace

// a fixed-capacity pass 2 that overflowed (ERR_TAB_CAP): the finals leave B1
// (the pass-1 keys, under the table) intact for the counted route's redo
__device__ __forceinline__ bool tab_cap_failed(const TabFinal &a) {
    return a.capq && (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ERR_TAB_CAP);
}

// NBB_: log2 of the bins.  14 (fixed regions of one wide bucket or of narrow
// keys, the common case at size): 16,384 bins, half the keys per bin for the
// copy scan, in the LDS the group path's bucket-start cache (and 128 keys of
// the unit) gave up: units of <= 12,160 keys, no groups of 64-bit keys.  13:
// everything else.
template <uint32_t NBB_>
__global__ __launch_bounds__(TAB_SWG, 4) void tab_sort_final_kernel(TabFinal a) {
    constexpr uint32_t NB = 1u << NBB_;
    constexpr uint32_t CAP1 = NBB_ == 14 ? (uint32_t)TAB_SORT_KEYS_BIG : TS_CAP1;
    constexpr uint32_t WPT = NB / 2 / TAB_SWG;          // bin-count words per thread (scan)
    if (tab_cap_failed(a)) return;
    __shared__ __attribute__((aligned(16))) uint32_t lkey[CAP1];   // sorted unit: u32 (one bucket) or u64 (a group)
    __shared__ uint32_t bst[NB / 2];                  // bin counts, then starts: bin b in half b & 1 of word b >> 1
    __shared__ uint64_t sc[NBB_ == 13 ? TS_SC + 2 : 1];   // start[cbase .. cbase + TS_SC + 1]
    __shared__ uint32_t nout[TS_GMAX];
    __shared__ uint32_t ws[8], smax;
    uint64_t *const lkey64 = (uint64_t *)lkey;
    const uint32_t t = threadIdx.x, lane = t & 63;
    const uint32_t k = a.k;
    const uint32_t kmask = k >= 32 ? ~0u : ((1u << k) - 1u), sh = 32 - k;
    uint32_t q0, q1;
    if (a.capq) {
        // fixed regions (one bucket or qg of them): shares of whole regions
        // (qlo, qhi: partition boundaries)
        const uint32_t rlo = (a.qlo >> TAB_L2) * a.rpp, nr = ((a.qhi - a.qlo) >> TAB_L2) * a.rpp;
        const uint32_t per = (nr + gridDim.x - 1) / gridDim.x;
        const uint32_t r0 = rlo + min(blockIdx.x * per, nr), r1 = min(r0 + per, rlo + nr);
        auto first_bucket = [&](uint32_t r) { return (r / a.rpp) << TAB_L2 | (r % a.rpp) * a.qg; };
        q0 = first_bucket(r0);
        q1 = first_bucket(r1);
    } else {
        const uint32_t per = (a.qhi - a.qlo + gridDim.x - 1) / gridDim.x;
        q0 = min(a.qlo + blockIdx.x * per, a.qhi);
        q1 = q0 + per < a.qhi ? q0 + per : a.qhi;
    }
    uint64_t st_canon = 0, st_keys = 0, st_sum = 0;
    // no prefix, odd k, Map view (C3): every entry is two Map keys, never a
    // palindrome; no prefix, canonical view (C5): every entry is one key with
    // its count -- no decoding needed in either
    const bool plain_odd = a.pmask == 0 && !a.canonical && (k & 1u);
    const bool plain_canon = a.pmask == 0 && a.canonical;
    // Map statistics of one canonical entry h (App. A.6; as in tab_final_kernel)
    auto account = [&](uint64_t h, uint64_t cnt) {
        if (plain_odd) {
            st_canon += 1;
            st_keys += 2;
            st_sum += 2 * cnt;
            return;
        }
        if (plain_canon) {
            st_canon += 1;
            st_keys += 1;
            st_sum += cnt;
            return;
        }
        const uint64_t code = tab_code(h, k, a.narrow, a.inv);
        const uint32_t lo = (uint32_t)code & kmask, hi = (uint32_t)(code >> k) & kmask;
        const uint32_t rlo2 = __brev(~lo & kmask) >> sh, rhi2 = __brev(~hi & kmask) >> sh;
        const bool pal = lo == rlo2 && hi == rhi2;
        st_canon += 1;
        if (a.canonical) {
            const uint32_t dif = (lo ^ rlo2) | (hi ^ rhi2);
            const uint32_t j = dif ? __ffs(dif) - 1 : 0;
            const uint32_t bw = (((hi >> j) & 1u) << 1) | ((lo >> j) & 1u);
            const uint32_t br = (((rhi2 >> j) & 1u) << 1) | ((rlo2 >> j) & 1u);
            const bool wmin = dif == 0 || bw < br;
            const uint32_t clo = wmin ? lo : rlo2, chi = wmin ? hi : rhi2;
            const bool cs = (((clo ^ a.plo) | (chi ^ a.phi)) & a.pmask) == 0;
            st_keys += cs ? 1u : 0u;
            st_sum += cs ? cnt : 0;
        } else {
            const bool fs = (((lo ^ a.plo) | (hi ^ a.phi)) & a.pmask) == 0;
            const bool rs = !pal && (((rlo2 ^ a.plo) | (rhi2 ^ a.phi)) & a.pmask) == 0;
            st_keys += (fs ? 1u : 0u) + (rs ? 1u : 0u);
            st_sum += (fs ? (pal ? 2 * cnt : cnt) : 0) + (rs ? cnt : 0);
        }
    };
    uint32_t cbase = q0;
    auto refill = [&](uint32_t cb) {
        __syncthreads();
        for (uint32_t i = t; i < TS_SC + 2; i += TAB_SWG) sc[i] = a.start[cb + i < TAB_NQ ? cb + i : TAB_NQ];
        __syncthreads();
    };
    auto leftover = [&](uint32_t qa, uint32_t qb) {
        if (t == 0) {
            const unsigned int i = atomicAdd(a.left_n, 1u);
            a.left[2 * i] = qa;
            a.left[2 * i + 1] = qb;
        }
    };
    if (!a.capq) refill(cbase);
    uint32_t q = q0;
    while (q < q1) {
        if (!a.capq && q - cbase >= TS_SC) {
            cbase = q;
            refill(cbase);
        }
        // the unit at q (uniform: every thread reads the same cached starts):
        // a fixed region, or consecutive contiguous buckets up to TS_CAPG keys
        uint32_t qe = q + 1;
        uint64_t n, s0, s0in;                          // keys, output start, input start
        if (a.capq) {
            const uint32_t r = tab_region(q, a.rpp, a.gmag);
            qe = min(q + a.qg, ((q >> TAB_L2) + 1) << TAB_L2);
            n = a.inlen[r];
            s0 = a.rstart[r];
            s0in = (uint64_t)r * a.capq;
        } else {
            n = sc[q + 1 - cbase] - sc[q - cbase];
            if (n <= TS_CAPG) {
                while (qe < q1 && qe - cbase < TS_SC && qe - q < TS_GMAX) {
                    const uint64_t ne = sc[qe + 1 - cbase] - sc[qe - cbase];
                    if (n + ne > TS_CAPG) break;
                    n += ne;
                    ++qe;
                }
            }
            s0 = s0in = sc[q - cbase];
        }
        const uint32_t g = qe - q;
        if (n == 0) {
            for (uint32_t i = t; i < g; i += TAB_SWG) a.nd[q + i] = 0;
            q = qe;
            continue;
        }
        if (n > CAP1) {                             // (g == 1) a crowded bucket
            leftover(q, qe);
            q = qe;
            continue;
        }
        const uint64_t qbase = (uint64_t)q << TAB_RBITS;
        const int left = (int)n - (int)t;
        // Three instantiations, so that each keeps only its own registers
        // live: ONE bucket of 64-bit keys (its bin fixes the remainder's top
        // bits: 32-bit LDS entries), a GRoup of buckets of 64-bit keys (64-bit
        // entries, half the keys), and NARrow keys (a fixed region of 32-bit
        // keys, bucket offset << 22 | the remainder's top 22 bits: one bucket
        // or a group, 32-bit entries, all the keys).  Held keys: lo = low 32
        // bits (narrow: the key), hi = the rest (a group's), pk = bin, later
        // bin << 14 | sorted position.  Returns false when a bin is crowded.
        auto sort_unit = [&](auto mode_tag) -> bool {
            constexpr int MODE = decltype(mode_tag)::value;
            constexpr bool ONE = MODE == 0, GRP = MODE == 1, NAR = MODE == 2;
            constexpr int KPT = GRP ? TS_KPT / 2 : TS_KPT;
            const uint32_t obits = g > 1 ? 32 - __clz(g - 1) : 0;
            const uint32_t bsh = (NAR ? TAB_RBITS - TAB_NSH : TAB_RBITS) + obits - NBB_;
            const bool single = g == 1;                  // (ONE: always)
            uint32_t lo[KPT], hi[GRP ? KPT : 1], pk[KPT];
            if (NAR) {
                const uint32_t *src = (const uint32_t *)a.B2 + s0in;
                const uint32_t qoff = (q & (TAB_NB - 1)) << (TAB_RBITS - TAB_NSH);
#pragma unroll
                for (int j = 0; j < KPT; ++j) {
                    lo[j] = src[left > j * (int)TAB_SWG ? j * TAB_SWG + t : 0u] - qoff;
                    pk[j] = (lo[j] >> bsh) & (NB - 1);
                }
            } else {
                const uint64_t *src = a.B2 + s0in;
#pragma unroll
                for (int j = 0; j < KPT; ++j) {
                    const uint64_t x = src[left > j * (int)TAB_SWG ? j * TAB_SWG + t : 0u] - qbase;
                    lo[j] = (uint32_t)x;
                    if (GRP) hi[GRP ? j : 0] = (uint32_t)(x >> 32);
                    pk[j] = (uint32_t)(x >> bsh) & (NB - 1);
                }
            }
            __syncthreads();                           // the previous unit is done with the LDS state
            for (uint32_t i = t; i < NB / 2; i += TAB_SWG) bst[i] = 0;
            if (t == 0) smax = 0;
            for (uint32_t i = t; i < g; i += TAB_SWG) nout[i] = 0;
            __syncthreads();
            // bin counts; the returned value is the key's rank in its bin (< 2^14)
#pragma unroll
            for (int j = 0; j < KPT; ++j)
                if (left > j * (int)TAB_SWG)
                    pk[j] = pk[j] << 14 |
                            ((__hip_atomic_fetch_add(&bst[pk[j] >> 1], 1u << (16 * (pk[j] & 1u)), __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP) >> (16 * (pk[j] & 1u))) & 0xFFFFu);
            __syncthreads();
            {
                // bin starts: thread t scans words WPT t .. WPT t + WPT - 1
                // (16 words: read again after the block scan rather than held)
                constexpr int HOLD = WPT <= 8 ? (int)WPT : 1;
                uint32_t c8[HOLD], sum = 0, mx = 0;
#pragma unroll
                for (int i = 0; i < (int)WPT; ++i) {
                    const uint32_t c = bst[WPT * t + i];
                    if (WPT <= 8) c8[i < HOLD ? i : 0] = c;
                    const uint32_t lo16 = c & 0xFFFFu, hi16 = c >> 16;
                    sum += lo16 + hi16;
                    mx = max(mx, max(lo16, hi16));
                }
                uint32_t tot;
                uint32_t run = block_excl_512(sum, ws, &tot);
                for (int d = 32; d >= 1; d >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, d));
                if (lane == 0) atomicMax(&smax, mx);
#pragma unroll
                for (int i = 0; i < (int)WPT; ++i) {
                    const uint32_t c = WPT <= 8 ? c8[i < HOLD ? i : 0] : bst[WPT * t + i];
                    const uint32_t lo16 = c & 0xFFFFu, hi16 = c >> 16;
                    bst[WPT * t + i] = run | (run + lo16) << 16;   // (starts < 2^14)
                    run += lo16 + hi16;
                }
            }
            __syncthreads();
            // a region of several buckets: each bucket's exact output start
            // (its keys' bins are consecutive: bins j << sbb .. of offset j),
            // also for a region left to the general kernel
            const uint32_t sbb = NBB_ - obits;
            if (!single && a.capq && t < g) a.wstart[q + t] = s0 + (bst[(t << sbb) >> 1] & 0xFFFFu);
            if (smax > TS_BINMAX) return false;        // (uniform) many copies of a key
            // counting-sort scatter: bin start + rank in the bin (bst[b] stays the start of bin b)
#pragma unroll
            for (int j = 0; j < KPT; ++j)
                if (left > j * (int)TAB_SWG) {
                    const uint32_t b = pk[j] >> 14;
                    const uint32_t pos = ((bst[b >> 1] >> (16 * (b & 1u))) & 0xFFFFu) + (pk[j] & 0x3FFFu);
                    if (GRP)
                        lkey64[pos] = (uint64_t)hi[GRP ? j : 0] << 32 | lo[j];
                    else
                        lkey[pos] = lo[j];
                    pk[j] = b << 14 | pos;
                }
            __syncthreads();
            // a group: the held keys are taken again in SORTED order (key j of
            // thread t = sorted position 512 j + t), so a wave's keys are
            // consecutive bins -- mostly one bucket, and the first copies'
            // output slots take one counter bump per wave and bucket present
            // (in load order a wave held keys of every bucket of a fixed
            // region: C5 final 6.0 vs 3.4 ms)
            if (!single) {
#pragma unroll
                for (int j = 0; j < KPT; ++j)
                    if (left > j * (int)TAB_SWG) {
                        const uint32_t i = j * TAB_SWG + t;
                        if (GRP) {
                            const uint64_t x = lkey64[i];
                            lo[j] = (uint32_t)x;
                            hi[GRP ? j : 0] = (uint32_t)(x >> 32);
                            pk[j] = ((uint32_t)(x >> bsh) & (NB - 1)) << 14 | i;
                        } else {
                            lo[j] = lkey[i];
                            pk[j] = ((lo[j] >> bsh) & (NB - 1)) << 14 | i;
                        }
                    }
            }
            // every held key scans its bin [end of bin b - 1, end of bin b) for
            // copies of itself; the first copy emits (key, copies).  Keys go in
            // groups of G, element m of all G bins read together (G LDS reads
            // in flight per step, steps = the largest bin of the group: ~3 keys
            // per bin at C3) instead of one key's bin after another.
            constexpr int G = GRP ? 4 : 6;           // (A/B at C3 / C5: ONE 4 / 6 / 8 / 12 -> 60.9 / 58.3 / 59.7 / 82 ms; groups 3 / 4 / 6)
#pragma unroll
            for (int g0 = 0; g0 < KPT; g0 += G) {
                if (!__any(left > g0 * (int)TAB_SWG)) break;
                uint32_t bb[G], cf[G], cmax = 0;          // bb: b0 | c << 14; cf: copies | first << 8
#pragma unroll
                for (int u = 0; u < G; ++u) {
                    const int j = g0 + u;
                    const bool valid = left > j * (int)TAB_SWG;
                    const uint32_t b = pk[j] >> 14;
                    const uint32_t b0 = (bst[b >> 1] >> (16 * (b & 1u))) & 0xFFFFu;
                    const uint32_t b1 = (KH_ABLATE(a) & 8) ? b0 : b + 1 < NB ? (bst[(b + 1) >> 1] >> (16 * ((b + 1) & 1u))) & 0xFFFFu : (uint32_t)n;
                    const uint32_t c = valid ? b1 - b0 : 0u;
                    bb[u] = b0 | c << 14;
                    cf[u] = valid ? ((KH_ABLATE(a) & 8) ? 0x101u : 0x100u) : 0u;   // (experiments: no bin scan)
                    cmax = max(cmax, c);
                }
                for (uint32_t m = 0; m < cmax; ++m) {
#pragma unroll
                    for (int u = 0; u < G; ++u) {
                        const int j = g0 + u;
                        const uint32_t b0 = bb[u] & 0x3FFFu, c = bb[u] >> 14;
                        const bool in = m < c;
                        const uint32_t mm = in ? b0 + m : b0;
                        bool eq;
                        if (GRP) {
                            const uint64_t xk = ((uint64_t)hi[GRP ? j : 0] << 32) | lo[j];
                            eq = in && lkey64[mm] == xk;
                        } else {
                            eq = in && lkey[mm] == lo[j];
                        }
                        cf[u] += eq ? 1u : 0u;
                        if (eq && b0 + m < (pk[j] & 0x3FFFu)) cf[u] &= 0xFFu;    // an earlier copy
                    }
                }
                // one bucket: the group's output slots from ONE counter bump per wave
                uint32_t gbase = 0;
                if (single) {
                    uint32_t tot = 0;
#pragma unroll
                    for (int u = 0; u < G; ++u) tot += (uint32_t)__popcll(__ballot((cf[u] >> 8) != 0u));
                    if (tot) {
                        if (lane == 0) gbase = atomicAdd(&nout[0], tot);
                        gbase = (uint32_t)__builtin_amdgcn_readlane((int)gbase, 0);
                    }
                }
                const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
                for (int u = 0; u < G; ++u) {
                    const int j = g0 + u;
                    const uint32_t b = pk[j] >> 14;
                    // (one bucket: the bin is the remainder's top NBB_ bits, bits 31 .. 43)
                    const uint64_t xj = ONE ? (((uint64_t)b << (TAB_RBITS - NBB_)) | (lo[j] & ((1u << (TAB_RBITS - NBB_)) - 1u)))
                                        : GRP ? (((uint64_t)hi[GRP ? j : 0] << 32) | lo[j])
                                              : (uint64_t)lo[j] << TAB_NSH;
                    const bool first = (cf[u] >> 8) != 0u;
                    const uint32_t cnt = cf[u] & 0xFFu;
                    // output slots: one LDS counter bump per wave and bucket present
                    unsigned long long fm = __ballot(first);
                    uint32_t pos = 0, ql = 0;
                    if (single) {
                        pos = gbase + (uint32_t)__popcll(fm & below);
                        gbase += (uint32_t)__popcll(fm);
                    } else {
                        ql = (uint32_t)(xj >> TAB_RBITS);
                        while (fm) {
                            const int ld = __ffsll((long long)fm) - 1;
                            const uint32_t qx = (uint32_t)__shfl((int)ql, ld);
                            const unsigned long long mq = __ballot(first && ql == qx);
                            uint32_t base = 0;
                            if (lane == (uint32_t)ld) base = atomicAdd(&nout[qx], (uint32_t)__popcll(mq));
                            base = (uint32_t)__shfl((int)base, ld);
                            if (first && ql == qx) pos = base + (uint32_t)__popcll(mq & ((1ull << lane) - 1ull));
                            fm &= ~mq;
                        }
                    }
                    if (first) {
                        if (!(KH_ABLATE(a) & 32))
                            a.out[(single ? s0 : a.capq ? s0 + (bst[(ql << sbb) >> 1] & 0xFFFFu) : sc[q + ql - cbase]) + pos] =
                                ((xj & TAB_RMASK) << 20) | cnt;
                        if (!(KH_ABLATE(a) & 16)) account(qbase + xj, cnt);
                    }
                }
            }
            return true;
        };
        bool ok = false;
        if (a.b2n)
            ok = sort_unit(std::integral_constant<int, 2>{});
        else if (g == 1 || NBB_ == 14)           // (NBB_ 14: one wide bucket per region, g == 1)
            ok = sort_unit(std::integral_constant<int, 0>{});
        else if constexpr (NBB_ == 13)
            ok = sort_unit(std::integral_constant<int, 1>{});
        if (!ok) {
            leftover(q, qe);
            q = qe;
            continue;
        }
        __syncthreads();
        for (uint32_t i = t; i < g; i += TAB_SWG) a.nd[q + i] = nout[i];
        q = qe;
    }
    __syncthreads();                                 // (the key array is free: the reduction's scratch)
    tab_stats_out(a.stats, st_canon, st_keys, st_sum, TAB_SWG / 64, (unsigned long long (*)[3])lkey);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
hipError_t launch_tab_hist1(const TabArgs &a, hipStream_t s) {
    // (no prefix: the windows' fast path, kmer_table.hip tab_round)
    if (a.pmask == 0)
        hipLaunchKernelGGL(tab_hist1_kernel<false>, dim3(a.nwg), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(tab_hist1_kernel<true>, dim3(a.nwg), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_tab_scatter1(const TabArgs &a, hipStream_t s) {
    // KMERHIP_TAB_S1=full: one 1,024-thread workgroup per CU (A/B experiments)
    static const bool half = [] {
        const char *e = exp_env("KMERHIP_TAB_S1");
        return !(e && strcmp(e, "full") == 0);
    }();
    if (half) {
        if (a.pmask == 0)
            hipLaunchKernelGGL(tab_scatter1h_kernel<false>, dim3(a.nwg), dim3(TAB_WGH), 0, s, a);
        else
            hipLaunchKernelGGL(tab_scatter1h_kernel<true>, dim3(a.nwg), dim3(TAB_WGH), 0, s, a);
        return hipGetLastError();
    }
    if (a.pmask == 0)
        hipLaunchKernelGGL(tab_scatter1_kernel<false>, dim3(a.nwg), dim3(TAB_WG1), 0, s, a);
    else
        hipLaunchKernelGGL(tab_scatter1_kernel<true>, dim3(a.nwg), dim3(TAB_WG1), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_tab_p1_offsets(const uint64_t *H1s, uint32_t nwg, uint64_t *out, hipStream_t s) {
    hipLaunchKernelGGL(tab_p1_offsets_kernel, dim3(TAB_NB / 256), dim3(256), 0, s, H1s, nwg, out);
    return hipGetLastError();
}

hipError_t launch_tab_piece_count(const uint64_t *wcount, uint64_t n, uint32_t *pc, uint32_t *split, hipStream_t s) {
    uint64_t blocks = (n + 255) / 256;
    blocks = blocks < 1 ? 1 : blocks > 16384 ? 16384 : blocks;
    hipLaunchKernelGGL(tab_piece_count_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, wcount, n, pc, split);
    return hipGetLastError();
}

hipError_t launch_tab_piece_write(const SeqLine *lines, const uint64_t *wcount, const uint64_t *pbase, uint64_t n,
                                  uint32_t k, SeqLine *out, hipStream_t s) {
    uint64_t blocks = (n + 255) / 256;
    blocks = blocks < 1 ? 1 : blocks > 16384 ? 16384 : blocks;
    hipLaunchKernelGGL(tab_piece_write_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, lines, wcount, pbase, n, k,
                       out);
    return hipGetLastError();
}

hipError_t launch_tab_hist2(const uint64_t *B1, const TabUnit *units, uint32_t n_units, uint32_t *H2, hipStream_t s) {
    hipLaunchKernelGGL(tab_hist2_kernel, dim3(n_units), dim3(256), 0, s, B1, units, H2);
    return hipGetLastError();
}

hipError_t launch_tab_scatter2(const uint64_t *B1, const TabUnit *units, uint32_t n_units, const uint64_t *H2s,
                               uint64_t *B2, hipStream_t s) {
    // KMERHIP_TAB_S2=plain: the 16 K-round kernel without aligned write-out (A/B experiments)
    static const bool plain = [] {
        const char *e = exp_env("KMERHIP_TAB_S2");
        return e && strcmp(e, "plain") == 0;
    }();
    if (plain)
        hipLaunchKernelGGL(tab_scatter2_kernel, dim3(n_units), dim3(TAB_WG1), 0, s, B1, units, H2s, B2);
    else
        hipLaunchKernelGGL(tab_scatter2c_kernel, dim3(n_units), dim3(TAB_WG1), 0, s, B1, units, H2s, B2);
    return hipGetLastError();
}

hipError_t launch_tab_starts(const uint64_t *H2s, const uint32_t *H2, uint64_t nh, const TabUnit *pfirst,
                             uint64_t *start, hipStream_t s) {
    hipLaunchKernelGGL(tab_starts_kernel, dim3(TAB_NQ / 256), dim3(256), 0, s, H2s, H2, nh, pfirst, start);
    return hipGetLastError();
}

hipError_t launch_tab_scatter1f(const TabArgs &a, hipStream_t s) {
    if (a.pmask == 0)
        hipLaunchKernelGGL(tab_scatter1f_kernel<false>, dim3(a.nwg), dim3(TAB_WGH), 0, s, a);
    else
        hipLaunchKernelGGL(tab_scatter1f_kernel<true>, dim3(a.nwg), dim3(TAB_WGH), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_tab_spill_fill(bool narrow, uint64_t *B1, uint64_t base, uint64_t R, uint64_t S, uint64_t PS,
                                 const unsigned long long *pcur, hipStream_t s) {
    hipLaunchKernelGGL(tab_spill_fill_kernel, dim3(TAB_NB), dim3(256), 0, s, narrow, B1, base, R, S, PS, pcur);
    return hipGetLastError();
}

hipError_t launch_tab_wg_windows(const SeqLine *lines, uint64_t n, uint64_t lpw, uint32_t k, uint32_t nwg,
                                 uint64_t *W, hipStream_t s) {
    hipLaunchKernelGGL(tab_wg_windows_kernel, dim3(nwg), dim3(256), 0, s, lines, n, lpw, k, W);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void tab_segcopy_kernel(const uint64_t *src, const TabSeg *segs, uint64_t *dst) {
    const TabSeg g = segs[blockIdx.x];
    for (uint64_t i = threadIdx.x; i < g.len; i += 256) dst[g.dst + i] = src[g.src + i];
}

hipError_t launch_tab_segcopy(const uint64_t *src, const TabSeg *segs, uint32_t n, uint64_t *dst, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(tab_segcopy_kernel, dim3(n), dim3(256), 0, s, src, segs, dst);
    return hipGetLastError();
}

// narrow pass-1 keys (32 bits below the partition) -> h
__global__ __launch_bounds__(256) void tab_widen_kernel(const uint32_t *src, const TabSeg *segs, uint64_t *dst) {
    const TabSeg g = segs[blockIdx.x];
    const uint64_t pb = g.part << (64 - TAB_L1);
    for (uint64_t i = threadIdx.x; i < g.len; i += 256) {
        const uint32_t x = src[g.src + i];
        dst[g.dst + i] = x == TAB_SENT32 ? TAB_SENT : pb | (uint64_t)x << TAB_NSH;
    }
}

hipError_t launch_tab_widen(const uint32_t *src, const TabSeg *segs, uint32_t n, uint64_t *dst, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(tab_widen_kernel, dim3(n), dim3(256), 0, s, src, segs, dst);
    return hipGetLastError();
}

// Linear digest of a table: sum over entries of count x tab_digest_mix(h)
// (mod 2^64; counts >= TAB_CMAX are corrected on the host from the big list).
// One wave per bucket; one atomic per wave.
__global__ __launch_bounds__(256) void tab_digest_kernel(const uint64_t *ent, const uint64_t *start,
                                                         const uint32_t *nd, uint32_t k, uint32_t narrow,
                                                         unsigned long long *out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
    uint64_t acc = 0;
    for (uint32_t q = wv; q < TAB_NQ; q += nw) {
        const uint64_t s0 = start[q];
        const uint32_t n = nd[q];
        for (uint32_t i = lane; i < n; i += 64) {
            const uint64_t w = ent[s0 + i];
            const uint64_t h = ((uint64_t)q << TAB_RBITS) | (w >> 20);
            // (the weight of the code's tab_mix hash, for narrow keys too)
            acc += (w & TAB_CMAX) * tab_digest_mix(tab_digest_key(h, k, narrow));
        }
    }
    for (int d = 32; d >= 1; d >>= 1) acc += (uint64_t)__shfl_xor((long long)acc, d);
    if (lane == 0 && acc) atomicAdd(out, (unsigned long long)acc);
}

hipError_t launch_tab_digest(const uint64_t *ent, const uint64_t *start, const uint32_t *nd, uint32_t k,
                            uint32_t narrow, unsigned long long *out, hipStream_t s) {
    hipLaunchKernelGGL(tab_digest_kernel, dim3(4096), dim3(256), 0, s, ent, start, nd, k, narrow, out);
    return hipGetLastError();
}

hipError_t launch_tab_sort_final(const TabFinal &a, uint32_t grid, hipStream_t s) {
    // (16,384 bins for fixed regions of one wide bucket or of narrow keys;
    // KMERHIP_TAB_BINS=8192: always 8,192, A/B experiments)
    static const bool big_ok = [] {
        const char *e = exp_env("KMERHIP_TAB_BINS");
        return !(e && strcmp(e, "8192") == 0);
    }();
    if (a.capq && a.capq <= TAB_SORT_KEYS_BIG && (a.qg == 1 || a.b2n) && big_ok)
        hipLaunchKernelGGL(tab_sort_final_kernel<14>, dim3(grid), dim3(TAB_SWG), 0, s, a);
    else
        hipLaunchKernelGGL(tab_sort_final_kernel<13>, dim3(grid), dim3(TAB_SWG), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_tab_final(const TabFinal &a, uint32_t grid, hipStream_t s) {
    hipLaunchKernelGGL(tab_final_kernel, dim3(grid), dim3(TAB_FWG), 0, s, a);
    return hipGetLastError();
}

}  // namespace kmerhip
