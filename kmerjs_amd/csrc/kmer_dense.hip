// kmer_dense.hip — the dense-hit ordered path (a prefix of 0-3 bases, or none;
// step 1, k <= 32): only the ACCEPTED windows are written, in rank order.
//
// lib/kmers.js:88-100 on a sequence line and on its complement (:151-155):
// the Map's insertion order is line by line, the line's forward windows by
// position s, then its complement's windows by position j, i.e. the reverse
// strand's windows by DESCENDING s (j = W - 1 - s).  The round-5 windows
// kernel gave every window of every line a rank slot (2.7 G slots at C2 size
// with prefix AT, 168.8 M of them accepted), wrote all of them and compacted
// before the finish; here two passes over the lines find each accepted
// window's rank directly:
//   count  per line, the accepted forward and reverse windows;
//   (scan) per line, its first rank slot;
//   write  per accepted window, slot = line base + its rank among the line's
//          accepted windows of its strand (forward: those at smaller s;
//          reverse: the line's forward count + those at LARGER s).
// Window formation (both passes): a lane takes 16 CONSECUTIVE windows of one
// line; the lanes of a wave are dealt out over its next 16 lines (ceil(windows
// left / 16) lanes per line, as table mode's pass 1).  The lane loads the <= 50
// bytes its windows span as 13 aligned dwords and packs their 2-bit codes
// (A/C/G/T = 0..3) with one v_dot4 per dword into two streams -- first base
// least significant (S) and most significant (R) -- so that window m is a
// constant shift of each: its code (first base most significant, the key
// layout of every ordered path) from R, its reverse complement ~S (the
// complement of the bases in reverse order is the LS stream's bitwise not).
// Non-ACGT bytes are flagged per byte (v_perm against "ACGT"); such windows
// are not ranked but become records when their prefix bytes match.
#include "kmer_internal.hpp"

namespace kmerhip {

namespace {

constexpr int DW_NS = 16;              // windows per lane per round

__device__ __forceinline__ uint32_t dw_incl_sum(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}

__device__ __forceinline__ uint32_t rl32(uint32_t v, uint32_t i) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)i);
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t src) {
    return (uint64_t)(uint32_t)__shfl((int)(uint32_t)v, (int)src) |
           ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(v >> 32), (int)src) << 32);
}

// the NW-word value w >>= n (runtime n < 64 NW)
template <int NW>
__device__ __forceinline__ void shrw(uint64_t (&w)[NW], uint32_t n) {
    const uint32_t q = n >> 6, r = n & 63u;
    uint64_t o[NW];
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        uint64_t lo = 0, hi = 0;
#pragma unroll
        for (int j = 0; j < NW; ++j) {               // (selects: no dynamic register indexing)
            lo = (uint32_t)j == i + q ? w[j] : lo;
            hi = (uint32_t)j == i + q + 1 ? w[j] : hi;
        }
        o[i] = r ? (lo >> r) | (hi << (64 - r)) : lo;
    }
#pragma unroll
    for (int i = 0; i < NW; ++i) w[i] = o[i];
}

// bits [n, n + 128) of w (n < 64, a constant once the window loops unroll):
// *lo = the first 64, *hi = the next 64 (0 past the stream)
template <int NW>
__device__ __forceinline__ void extract(const uint64_t (&w)[NW], uint32_t n, uint64_t *lo, uint64_t *hi) {
    *lo = n ? (w[0] >> n) | (w[1] << (64 - n)) : w[0];
    if (NW > 2) *hi = n ? (w[1] >> n) | (w[NW > 2 ? 2 : 1] << (64 - n)) : w[1];
    else *hi = n ? w[1] >> n : w[1];
}

// A wave's position in its share of sequence lines; lane i < 16 holds the
// descriptor (and, in the write pass, the counts and first slot) of line m + i.
struct DCur {
    uint64_t m, end, seg;              // next line, end of the share, first window of line m not yet taken
    uint64_t dstart, dlen, dli, dcnt, dbase;
    uint32_t cf, cr;                   // accepted windows of line m in earlier rounds (seg > 0)
};

template <bool WRITE>
__device__ __forceinline__ void dw_fetch(const DenseArgs &a, DCur &c) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t mi = c.m + lane;
    c.dstart = c.dlen = c.dli = c.dcnt = c.dbase = 0;
    if (lane < 16 && mi < c.end) {
        const SeqLine sl = a.lines[mi];
        c.dstart = sl.start;
        c.dlen = sl.len;
        c.dli = sl.line_index;
        if (WRITE) {
            c.dcnt = a.cnt[mi];
            c.dbase = a.hbase[mi];
        }
    }
}

// exotic window (a byte outside A/C/G/T): its strands whose prefix bytes match
// become records (their keys are gathered later), as the tile paths do
__device__ __forceinline__ void dw_record(const DenseArgs &a, uint64_t order, uint64_t pos, uint32_t strand) {
    const unsigned long long n = atomicAdd(a.rec_count, 1ull);
    if (n < a.rec_cap) {
        Record r;
        r.order = order;
        r.pos = pos;
        r.len = a.k;
        r.strand = strand;
        a.recs[n] = r;
    } else {
        atomicOr(a.err, ERR_REC_OVERFLOW);
    }
}

// a refused rank slot (count and write passes disagree): ERR_DENSE_RANK, and
// the first one's context for the host's error message
__device__ __forceinline__ void dw_refuse(const DenseArgs &a, uint64_t line, uint64_t s, uint32_t strand, uint64_t lcnt,
                                          uint64_t rank, uint64_t slot) {
    atomicOr(a.err, ERR_DENSE_RANK);
    if (a.dbg && atomicCAS(&a.dbg[0], 0ull, 1ull) == 0ull) {
        a.dbg[1] = line;
        a.dbg[2] = s;
        a.dbg[3] = strand;
        a.dbg[4] = lcnt;
        a.dbg[5] = rank;
        a.dbg[6] = slot;
        a.dbg[7] = a.out_end;
    }
}

}  // namespace

// One pass over a wave's share of lines (lpw consecutive sequence ordinals).
// COUNT (WRITE false): cnt[m] = accepted forward | accepted reverse << 32 and
// tot[m] = their sum, per line.  WRITE: keys and order keys of the accepted
// windows at their rank slots (out_base + hbase[m] + rank), records of the
// exotic ones.  WIDE (32 < k <= 64): 21 dwords per lane, 192-bit streams,
// 128-bit window codes (key = the low 64 bits, keyh = the bits above).
template <bool WRITE, bool WIDE>
__global__ __launch_bounds__(256) void dense_windows_kernel(DenseArgs a) {
    constexpr int NDW = WIDE ? 21 : 13;            // 16 + k - 1 bytes + 3 of alignment
    constexpr int NW = WIDE ? 3 : 2;               // stream words
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t k = a.k, plen = a.plen;
    const uint64_t maxrel = (1ull << a.pbits) - 1ull;
    // masks of a 2k-bit code (lo, hi) and of k per-byte flags
    const uint64_t cm_lo = k >= 32 ? ~0ull : ((1ull << (2 * k)) - 1ull);
    const uint64_t cm_hi = k <= 32 ? 0ull : k >= 64 ? ~0ull : ((1ull << (2 * k - 64)) - 1ull);
    const uint64_t kmask1 = k >= 64 ? ~0ull : ((1ull << k) - 1ull);
    const uint32_t tb = 2 * (k - plen);               // prefix bits sit above the suffix
    DCur c;
    c.m = wave * a.lpw;
    c.end = c.m + a.lpw < a.n_lines ? c.m + a.lpw : a.n_lines;
    c.seg = 0;
    c.cf = c.cr = 0;
    if (c.m >= c.end) return;
    dw_fetch<WRITE>(a, c);
    const uint8_t *const dend = a.data + a.len;
    // the top 2 |P| bits of a code (lo, hi)
    auto top = [&](uint64_t lo, uint64_t hi) -> uint64_t {
        if (!WIDE || tb < 64) return tb == 0 ? lo : (lo >> tb) | (WIDE && tb ? hi << (64 - tb) : 0ull);
        return hi >> (tb - 64);
    };
    while (c.m < c.end) {
        // ---- deal the lanes over lines m .. m + 15 ----
        const uint64_t Wraw = c.dlen >= k ? c.dlen - k + 1 : 0;
        const uint64_t Wi = Wraw && Wraw - 1 <= maxrel ? Wraw : 0;   // (longer lines: reported by the line pass)
        const uint64_t seg0 = c.seg;
        const uint64_t rem = lane == 0 ? (Wi > seg0 ? Wi - seg0 : 0) : Wi;
        const uint32_t need = lane < 16 ? (uint32_t)((rem + DW_NS - 1) / DW_NS) : 0u;
        const uint32_t cum = dw_incl_sum(need);
        const uint32_t tot = rl32(cum, 15);
        uint32_t li = 0;
#pragma unroll
        for (uint32_t i = 0; i < 16; ++i) li += rl32(cum, i) <= lane ? 1u : 0u;
        const bool act = lane < tot && li < 16;
        const uint32_t lsrc = li < 16 ? li : 15u;
        const uint32_t before = (uint32_t)__shfl((int)(cum - need), (int)lsrc);
        const uint64_t st = shfl64(c.dstart, lsrc);
        const uint64_t Wl = shfl64(Wi, lsrc);
        const uint64_t lix = shfl64(c.dli, lsrc);
        const uint64_t w0 = (li == 0 ? seg0 : 0) + (uint64_t)(lane - before) * DW_NS;
        uint64_t lcnt = 0, lbase = 0;
        if (WRITE) {
            lcnt = shfl64(c.dcnt, lsrc);
            lbase = shfl64(c.dbase, lsrc);
        }
        // the line lane 63 works on, and whether this round finishes it
        uint32_t is = 15, ci = 0;
        bool part = false;
        if (tot > 64) {
            is = rl32(li, 63);
            ci = rl32(cum, is);
            part = ci != 64;
        }
        // ---- the lane's 16 windows: codes of the bytes [st + w0, st + w0 + 16 + k - 1) ----
        uint32_t fmask = 0, rmask = 0;
        uint64_t S[NW], R[NW];                          // the code streams (kept for the write-out)
#pragma unroll
        for (int w = 0; w < NW; ++w) S[w] = R[w] = 0;
        const uint32_t nv = act ? (uint32_t)(Wl - w0 < (uint64_t)DW_NS ? Wl - w0 : (uint64_t)DW_NS) : 0u;
        if (nv && !WIDE) {
            // narrow keys: the 16 windows' prefix and exotic tests bit-parallel
            // over the lane's bytes (bit t = byte t of the span): base planes
            // LO / HI (A C G T = 00 01 10 11) and the non-ACGT flags EX, one
            // v_dot4 each per dword; the code streams only in the write pass
            const uint8_t *p = a.data + st + w0;
            const uint32_t off = (uint32_t)((uintptr_t)p & 3u);
            const uint32_t *pw = (const uint32_t *)(p - off);
            uint64_t LO = 0, HI = 0, EX = 0;
#pragma unroll
            for (int i = 0; i < NDW; ++i) {
                uint32_t x = 0x41414141u;                // ('A' past the input: never inside a window)
                const uint8_t *q = (const uint8_t *)(pw + i);
                if (q < dend && (uint32_t)(4 * i) < off + nv + k - 1) {
                    if (q + 4 <= dend) {
                        x = pw[i];
                    } else {
                        for (int j = 0; j < 4; ++j)
                            if (q + j < dend) x = (x & ~(0xFFu << (8 * j))) | ((uint32_t)q[j] << (8 * j));
                    }
                }
                const uint32_t cc = ((x >> 1) ^ (x >> 2)) & 0x03030303u;       // A C G T -> 0 1 2 3
                const uint32_t ne = __builtin_amdgcn_perm(0u, 0x54474341u, cc) ^ x;     // 0 where A/C/G/T
                const uint32_t nz = (((ne & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | ne) & 0x80808080u;
                EX |= (uint64_t)__builtin_amdgcn_udot4(nz >> 7, 0x08040201u, 0u, false) << (4 * i);
                LO |= (uint64_t)__builtin_amdgcn_udot4(cc & 0x01010101u, 0x08040201u, 0u, false) << (4 * i);
                HI |= (uint64_t)__builtin_amdgcn_udot4((cc >> 1) & 0x01010101u, 0x08040201u, 0u, false) << (4 * i);
                if (WRITE) {
                    const uint32_t ls = __builtin_amdgcn_udot4(cc, 0x40100401u, 0u, false);   // first byte lowest
                    const uint32_t ms = __builtin_amdgcn_udot4(cc, 0x01041040u, 0u, false);   // first byte highest
                    S[i / 8] |= (uint64_t)ls << (8 * (i % 8));
                    const int rb = 8 * (NDW - 1 - i);
                    R[rb / 64] |= (uint64_t)ms << (rb % 64);
                }
            }
            if (WRITE) {
                shrw<NW>(S, 2 * off);
                shrw<NW>(R, 2 * (4 * NDW - (DW_NS - 1) - off - k));
            }
            LO >>= off;
            HI >>= off;
            EX >>= off;
            const uint64_t vm = (1ull << nv) - 1ull;         // (nv <= 16)
            // window j starts with P: base j + i == P[i]; ends with rc(P): base j + k - |P| + i == rc(P)[i]
            uint64_t fw = vm, rv = vm;
            for (uint32_t i = 0; i < plen; ++i) {
                const uint32_t cp = (uint32_t)(a.pcode >> (2 * (plen - 1 - i))) & 3u;
                const uint32_t cr = 3u - ((uint32_t)(a.pcode >> (2 * i)) & 3u);   // rc(P)[i] = comp(P[|P| - 1 - i])
                const uint64_t ep = ((cp & 1u) ? LO : ~LO) & ((cp & 2u) ? HI : ~HI);
                const uint64_t er = ((cr & 1u) ? LO : ~LO) & ((cr & 2u) ? HI : ~HI);
                fw &= ep >> i;
                rv &= er >> (k - plen + i);
            }
            // windows holding a non-ACGT byte: an EX bit in [j, j + k)
            uint64_t E = EX;
            uint32_t span = 1;
            while (2 * span <= k) {
                E |= E >> span;
                span *= 2;
            }
            const uint64_t exw = (E | (E >> (k - span))) & vm;
            fmask = (uint32_t)(fw & ~exw);
            rmask = (uint32_t)(rv & ~exw);
            // (planes alias non-ACGT bytes: exotic candidates are checked byte for byte)
            uint32_t xc = WRITE ? (uint32_t)((fw | rv) & exw) : 0u;
            while (xc) {
                const uint32_t m = __ffs(xc) - 1;
                xc &= xc - 1;
                const uint64_t pos = st + w0 + m;
                bool bf = true, br = true;
                for (uint32_t b = 0; b < plen; ++b) {
                    bf = bf && a.data[pos + b] == a.P[b];
                    br = br && a.data[pos + k - plen + b] == a.RP[b];
                }
                const uint64_t s = w0 + m, lo = lix << (a.pbits + 1);
                if (bf) dw_record(a, lo | s, pos, 0);
                if (br) dw_record(a, lo | (1ull << a.pbits) | (maxrel - s), pos, 1);
            }
        } else if (nv) {
            const uint8_t *p = a.data + st + w0;
            const uint32_t off = (uint32_t)((uintptr_t)p & 3u);
            const uint32_t *pw = (const uint32_t *)(p - off);
            uint64_t EX0 = 0, EX1 = 0;
#pragma unroll
            for (int i = 0; i < NDW; ++i) {
                uint32_t x = 0x41414141u;                // ('A' past the input: never inside a window)
                const uint8_t *q = (const uint8_t *)(pw + i);
                if (q < dend && (uint32_t)(4 * i) < off + nv + k - 1) {
                    if (q + 4 <= dend) {
                        x = pw[i];
                    } else {
                        for (int j = 0; j < 4; ++j)
                            if (q + j < dend) x = (x & ~(0xFFu << (8 * j))) | ((uint32_t)q[j] << (8 * j));
                    }
                }
                const uint32_t cc = ((x >> 1) ^ (x >> 2)) & 0x03030303u;       // A C G T -> 0 1 2 3
                const uint32_t ls = __builtin_amdgcn_udot4(cc, 0x40100401u, 0u, false);   // first byte lowest
                const uint32_t ms = __builtin_amdgcn_udot4(cc, 0x01041040u, 0u, false);   // first byte highest
                const uint32_t ne = __builtin_amdgcn_perm(0u, 0x54474341u, cc) ^ x;     // 0 where A/C/G/T
                const uint32_t nz = (((ne & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | ne) & 0x80808080u;
                const uint64_t e4 = __builtin_amdgcn_udot4(nz >> 7, 0x08040201u, 0u, false);
                if (i < 16) EX0 |= e4 << (4 * i);
                else EX1 |= e4 << (4 * (i - 16));
                S[i / 8] |= (uint64_t)ls << (8 * (i % 8));
                const int rb = 8 * (NDW - 1 - i);        // R: dword i's byte at bits [rb, rb + 8)
                R[rb / 64] |= (uint64_t)ms << (rb % 64);
            }
            // S >> 2 off: window m's LS code at bits [2m, 2m + 2k); R >> 2 (4 NDW - 15 - off - k):
            // window m's MS code at bits [2 (15 - m), 2 (15 - m) + 2k)
            shrw<NW>(S, 2 * off);
            shrw<NW>(R, 2 * (4 * NDW - (DW_NS - 1) - off - k));
            EX0 = (EX0 >> off) | (off ? EX1 << (64 - off) : 0ull);
            EX1 >>= off;
#pragma unroll
            for (int m = 0; m < DW_NS; ++m) {
                if ((uint32_t)m >= nv) break;
                uint64_t fl, fh, sl, sh;
                extract<NW>(R, 2 * (DW_NS - 1 - m), &fl, &fh);   // the window's code
                extract<NW>(S, 2 * m, &sl, &sh);
                fl &= cm_lo;
                fh &= cm_hi;
                const uint64_t rl = ~sl & cm_lo, rh = ~sh & cm_hi;          // rc(window)'s code
                const uint64_t exm = (m ? (EX0 >> m) | (EX1 << (64 - m)) : EX0) & kmask1;
                bool mf = plen == 0 || top(fl, fh) == a.pcode;
                bool mr = plen == 0 || top(rl, rh) == a.pcode;
                if (exm) {
                    if (WRITE && (mf || mr)) {
                        // (non-ACGT bytes alias to a code: the prefix bytes themselves decide)
                        const uint64_t pos = st + w0 + m;
                        bool bf = true, br = true;
                        for (uint32_t b = 0; b < plen; ++b) {
                            bf = bf && a.data[pos + b] == a.P[b];
                            br = br && a.data[pos + k - plen + b] == a.RP[b];
                        }
                        const uint64_t s = w0 + m, lo = lix << (a.pbits + 1);
                        if (bf) dw_record(a, lo | s, pos, 0);
                        if (br) dw_record(a, lo | (1ull << a.pbits) | (maxrel - s), pos, 1);
                    }
                    continue;
                }
                fmask |= mf ? 1u << m : 0u;
                rmask |= mr ? 1u << m : 0u;
            }
        }
        // ---- ranks inside each line: segmented wave scans of the lane counts ----
        const uint32_t nf = __popc(fmask), nr = __popc(rmask);
        const uint32_t F = dw_incl_sum(nf), Rs = dw_incl_sum(nr);
        // carried counts of line m (seg0 > 0: earlier rounds took its first windows)
        const uint32_t carf = seg0 ? c.cf : 0u, carr = seg0 ? c.cr : 0u;
        // lane i < 16: line i's windows of this round = lanes [b_i, min(cum_i, 64))
        const uint32_t bi_ = cum - need, ei_ = cum < 64 ? cum : 64u;
        const uint32_t Fe = (uint32_t)__shfl((int)F, (int)(ei_ ? ei_ - 1 : 0));
        const uint32_t Re = (uint32_t)__shfl((int)Rs, (int)(ei_ ? ei_ - 1 : 0));
        const uint32_t Fb = (uint32_t)__shfl((int)F, (int)(bi_ ? bi_ - 1 : 0));
        const uint32_t Rb = (uint32_t)__shfl((int)Rs, (int)(bi_ ? bi_ - 1 : 0));
        const bool took = lane < 16 && need && bi_ < 64;
        const uint32_t sf = took ? Fe - (bi_ ? Fb : 0u) : 0u, sr = took ? Re - (bi_ ? Rb : 0u) : 0u;
        // this lane's line starts at lane `before`: the scans there, read by
        // every lane (a bpermute from a lane outside EXEC returns 0, so the
        // reads must not sit in a branch that disables the source lane)
        const uint32_t Fbl = (uint32_t)__shfl((int)F, (int)(before ? before - 1 : 0));
        const uint32_t Rbl = (uint32_t)__shfl((int)Rs, (int)(before ? before - 1 : 0));
        if (!WRITE) {
            // complete lines: their totals (carried + this round); a line still
            // open after the round carries its counts to the next
            const bool present = lane < 16 && c.m + lane < c.end;
            const bool complete = present && (tot <= 64 || lane < is || (lane == is && !part));
            if (complete) {
                const uint32_t f = sf + (lane == 0 ? carf : 0u), r = sr + (lane == 0 ? carr : 0u);
                a.cnt[c.m + lane] = (uint64_t)f | ((uint64_t)r << 32);
                a.tot[c.m + lane] = f + r;
            }
        } else if (nv) {
            // this lane's rank base among its line's accepted windows of this round and before
            const uint32_t Bf = before ? Fbl : 0u;
            const uint32_t Br = before ? Rbl : 0u;
            const uint32_t fb = F - nf - Bf + (li == 0 ? carf : 0u);
            const uint32_t rb = Rs - nr - Br + (li == 0 ? carr : 0u);
            const uint32_t LF = (uint32_t)lcnt, LR = (uint32_t)(lcnt >> 32);
            const uint64_t hb = a.out_base + lbase;
            const uint64_t lo = lix << (a.pbits + 1);
#pragma unroll
            for (int m = 0; m < DW_NS; ++m) {
                const uint32_t below = (1u << m) - 1u;
                const uint64_t s = w0 + m;
                // (the codes again from the streams: constant shifts, no per-window key registers)
                if (fmask & (1u << m)) {
                    uint64_t kl, kh;
                    extract<NW>(R, 2 * (DW_NS - 1 - m), &kl, &kh);
                    const uint64_t slot = hb + fb + __popc(fmask & below);
                    if (slot >= a.out_end) {             // (never: the count pass sized the arrays)
                        dw_refuse(a, c.m + lsrc, s, 0, lcnt, fb + __popc(fmask & below), slot);
                        continue;
                    }
                    if (a.rkey32) a.rkey32[slot] = (uint32_t)(kl & a.smask);
                    else a.rkey[slot] = kl & a.smask;
                    if (WIDE && a.rkeyh) a.rkeyh[slot] = kh & a.smask_hi;
                    a.rord[slot] = lo | s;
                }
                if (rmask & (1u << m)) {
                    uint64_t kl, kh;
                    extract<NW>(S, 2 * m, &kl, &kh);
                    const uint32_t rr = rb + __popc(rmask & below);
                    const uint64_t slot = hb + LF + (LR - 1u - rr);
                    if (rr >= LR || slot >= a.out_end) {
                        dw_refuse(a, c.m + lsrc, s, 1, lcnt, rr, slot);
                        continue;
                    }
                    if (a.rkey32) a.rkey32[slot] = (uint32_t)(~kl & a.smask);
                    else a.rkey[slot] = ~kl & a.smask;
                    if (WIDE && a.rkeyh) a.rkeyh[slot] = ~kh & a.smask_hi;
                    a.rord[slot] = lo | (1ull << a.pbits) | (maxrel - s);
                }
            }
        }
        // ---- advance: the next round starts at the first line not finished ----
        if (tot <= 64) {
            c.m += 16;
            c.seg = 0;
            c.cf = c.cr = 0;
        } else if (!part) {
            c.m += is + 1;
            c.seg = 0;
            c.cf = c.cr = 0;
        } else {
            const uint32_t bis = ci - rl32(need, is);
            const uint32_t cfi = rl32(sf, is), cri = rl32(sr, is);
            c.cf = (is == 0 ? carf : 0u) + cfi;
            c.cr = (is == 0 ? carr : 0u) + cri;
            c.seg = (is == 0 ? seg0 : 0) + (uint64_t)(64 - bis) * DW_NS;
            c.m += is;
        }
        if (c.m < c.end) dw_fetch<WRITE>(a, c);
    }
}

hipError_t launch_dense_windows(const DenseArgs &a, bool write, hipStream_t s) {
    if (!a.n_lines) return hipSuccess;
    const uint64_t waves = (a.n_lines + a.lpw - 1) / a.lpw;
    const uint32_t grid = (uint32_t)((waves + 3) / 4);
    const bool wide = a.k > 32;
    if (write && wide) hipLaunchKernelGGL((dense_windows_kernel<true, true>), dim3(grid), dim3(256), 0, s, a);
    else if (write) hipLaunchKernelGGL((dense_windows_kernel<true, false>), dim3(grid), dim3(256), 0, s, a);
    else if (wide) hipLaunchKernelGGL((dense_windows_kernel<false, true>), dim3(grid), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((dense_windows_kernel<false, false>), dim3(grid), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace kmerhip
