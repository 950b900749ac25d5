// kmer_fasta.hip — FASTA input (KMER_FLAG_FASTA; SURVEY §8(f) row 4, an
// extension: the reference has no FASTA parser -- test/kmers.js:53-61 "TODO:
// FASTA tests missing!", test/kmerFinderServer.js:158 "TODO: FIX FASTA
// parser" -- and applied to a .fsa file its readFile() counts only the lines
// with index % 4 == 1, lib/kmers.js:151).
//
// FASTA semantics (restated for the tests in oracle/kmer_oracle.c): a
// line starting with '>' opens a record (the header, not counted); the lines
// before the first header form a headerless record; a record's sequence is its
// other lines joined (one trailing '\r' of each line dropped, empty lines add
// nothing), so windows run across line breaks; each record's sequence s is
// counted as the reference counts a sequence line (length > 1, windows of s
// then of complement(s), prefix test, first-occurrence order by record).
//
// On the device a chunk of FASTA is rewritten, in one streaming pass plus a
// scan, into the FASTQ shape every counting path already reads: per record
// the four lines  header, joined sequence, "", ""  -- so the record's sequence
// is line 4r + 1 -- and the chunk is then counted like FASTQ (ordered, table,
// canonical; long records through long-line mode).  Chunks must be cut before
// a header line (kmer_count_buffer / kmer_count_file do; device feeds must).
//
// Byte rule (chunk byte i, c = B[i], h = the current line is a header):
//   at a line start:  h = (c == '>');  '>' at i > 0 -> "\n\n\n" first (closes
//                     the previous record: sequence line, line 3, line 4);
//                     i == 0 and c != '>' -> "\n" first (the headerless
//                     record's empty header line)
//   c == '\n'         -> "\n" in a header line, nothing in a sequence line
//   c == '\r' before '\n' or at the chunk end -> nothing; any other byte -> c
//   after the last byte: "\n\n\n" (+ "\n" when it ends an unterminated header)
// Whether a line is a header depends on its first byte, which may lie in an
// earlier tile: each tile (and each thread inside a tile) is a function of
// the incoming state h (FaFn), composed by an exclusive scan.
#include "kmer_internal.hpp"

namespace kmerhip {

namespace {

constexpr int FA_BPT = 64;                       // bytes per thread
constexpr int FA_TILE = TPB * FA_BPT;            // 16 KiB

// thread function packed in 64 bits: [47:24] c1, [23:0] c0, [49:48] kind
__device__ __forceinline__ uint64_t fa_pack(uint32_t kind, uint32_t c0, uint32_t c1) {
    return (uint64_t)c0 | ((uint64_t)c1 << 24) | ((uint64_t)kind << 48);
}
__device__ __forceinline__ uint32_t fa_kind(uint64_t f) { return (uint32_t)(f >> 48) & 3u; }
__device__ __forceinline__ uint32_t fa_c(uint64_t f, uint32_t s) { return (uint32_t)(f >> (s ? 24 : 0)) & 0xFFFFFFu; }
// a then b
__device__ __forceinline__ uint64_t fa_compose(uint64_t a, uint64_t b) {
    const uint32_t ka = fa_kind(a), kb = fa_kind(b);
    const uint32_t s0 = ka ? ka - 1 : 0u, s1 = ka ? ka - 1 : 1u;
    return fa_pack(kb ? kb : ka, fa_c(a, 0) + fa_c(b, s0), fa_c(a, 1) + fa_c(b, s1));
}

// One thread's walk over its 64 bytes [64 t, 64 t + 64) of the tile, held in
// registers (w[0..15]; the byte before: prev, the byte after: w[16] & 0xFF;
// out of the chunk: '\n').  The tile is read from LDS once, as four 16-byte
// words per thread: a byte-wise walk over LDS put 16 lanes on one bank
// (64-byte stride) and ran the rewrite at ~0.2 TB/s.
// WRITE: with the incoming state h, the output bytes go straight to global
// memory from offset o: whole 4-byte words, and single bytes only for the
// words this thread shares with its neighbours (its first and last).
template <bool WRITE>
__device__ __forceinline__ uint64_t fa_walk(const uint32_t (&w)[17], uint8_t prev, int64_t g, uint64_t len,
                                            uint32_t h_in, uint8_t *out, uint64_t o, uint32_t *nl_out) {
    uint32_t common = 0, dep = 0, nl = 0, h = h_in;
    bool saw = false;
    const int n = (int64_t)len - g <= 0 ? 0 : (int64_t)len - g >= FA_BPT ? FA_BPT : (int)((int64_t)len - g);
    const uint64_t a_start = (o + 3) & ~3ull;       // first word wholly this thread's
    uint32_t acc = 0;
    auto put = [&](uint32_t b) {
        if (o < a_start) {
            out[o] = (uint8_t)b;
        } else {
            acc |= b << (8 * (uint32_t)(o & 3));
            if ((o & 3) == 3) {
                *(uint32_t *)(out + (o & ~3ull)) = acc;
                acc = 0;
            }
        }
        ++o;
    };
#pragma unroll
    for (int j = 0; j < FA_BPT; ++j) {
        if (j < n) {
            const uint32_t c = (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            const uint32_t nx = (w[(j + 1) >> 2] >> (8 * ((j + 1) & 3))) & 0xFFu;
            const int64_t gi = g + j;
            if (prev == '\n') {                       // line start (the chunk start reads '\n' behind it)
                saw = true;
                h = c == '>';
                if (c == '>' && gi > 0) {
                    common += 3;
                    if (WRITE) { put('\n'); put('\n'); put('\n'); }
                }
                if (gi == 0 && c != '>') {
                    common += 1;
                    if (WRITE) put('\n');
                }
            }
            if (c == '\n') {
                ++nl;
                if (saw) common += h; else dep += 1;
                if (WRITE && h) put('\n');
            } else if (!(c == '\r' && ((uint64_t)gi + 1 == len || nx == '\n'))) {
                common += 1;
                if (WRITE) put(c);
            }
            if ((uint64_t)gi + 1 == len) {             // after the chunk's last byte
                common += 3;
                if (WRITE) { put('\n'); put('\n'); put('\n'); }
                if (c != '\n') {
                    if (saw) common += h; else dep += 1;
                    if (WRITE && h) put('\n');
                }
            }
            prev = (uint8_t)c;
        }
    }
    if (WRITE && (o & 3)) {                            // the last, partial word: bytes
        const uint64_t wa = o & ~3ull;
        for (uint32_t b = 0; b < (uint32_t)(o & 3); ++b)
            if (wa + b >= a_start) out[wa + b] = (uint8_t)(acc >> (8 * b));
    }
    *nl_out = nl;
    return fa_pack(saw ? 1u + h : 0u, common, common + dep);
}

// inclusive scan of thread functions over the workgroup; returns this
// thread's EXCLUSIVE prefix, *total = the whole tile's function
__device__ __forceinline__ uint64_t fa_block_scan(uint64_t f, uint64_t *wtot, uint64_t *total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t incl = f;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(incl, d);
        if (lane >= d) incl = fa_compose(y, incl);
    }
    uint64_t excl = __shfl_up(incl, 1);
    if (lane == 0) excl = fa_pack(0, 0, 0);
    if (lane == 63) wtot[wid] = incl;
    __syncthreads();
    uint64_t before = fa_pack(0, 0, 0), all = fa_pack(0, 0, 0);
#pragma unroll
    for (int w = 0; w < TPB / 64; ++w) {
        if (w < wid) before = fa_compose(before, wtot[w]);
        all = fa_compose(all, wtot[w]);
    }
    *total = all;
    return fa_compose(before, excl);
}

// tile bytes + one byte on each side into LDS (out of the chunk: '\n')
__device__ __forceinline__ void fa_stage(const uint8_t *data, uint64_t len, int64_t g0, uint8_t *buf) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int64_t g = g0 + 16 * (tid + TPB * i);
        uint4 v;
        if (g + 16 <= (int64_t)len) {
            v = *(const uint4 *)(data + g);
        } else {
            uint32_t w[4];
            for (int q = 0; q < 4; ++q) {
                uint32_t x = 0;
                for (int b = 0; b < 4; ++b) {
                    const int64_t p = g + 4 * q + b;
                    x |= (uint32_t)((uint64_t)p < len ? data[p] : (uint8_t)'\n') << (8 * b);
                }
                w[q] = x;
            }
            v = make_uint4(w[0], w[1], w[2], w[3]);
        }
        *(uint4 *)(buf + 16 * (tid + TPB * i)) = v;
    }
    if (tid == 0) buf[-1] = g0 > 0 ? data[g0 - 1] : (uint8_t)'\n';
    if (tid == 1) buf[FA_TILE] = (uint64_t)(g0 + FA_TILE) < len ? data[g0 + FA_TILE] : (uint8_t)'\n';
}

// per-byte 0x80 flags of bytes equal to c (ASCII bytes < 0x80)
__device__ __forceinline__ uint32_t fa_eq(uint32_t x, uint32_t c4) {
    const uint32_t t = x ^ c4;
    return ~(t + 0x7F7F7F7Fu) & 0x80808080u;
}
// the 0x80 flags of a word as 4 bits
__device__ __forceinline__ uint32_t fa_bits4(uint32_t f) {
    return ((f >> 7) & 1u) | ((f >> 14) & 2u) | ((f >> 21) & 4u) | ((f >> 28) & 8u);
}

// The common case, a block of sequence bytes: no '>' and no '\r' among the
// thread's 64 bytes, not the chunk's first or last block.  Every line start
// in it opens a sequence line (h = 0), so '\n' bytes are dropped, except the
// block's first '\n' when it ends a line that began earlier in state h = 1 (a
// header's end).  Counting: popcounts.  Writing: each input word compacted by
// one v_perm (selector from a 16-entry LDS table, by the word's drop mask)
// into a 64-bit accumulator; whole output words stored, the thread's first and
// last partial words as bytes.  Returns false when the block is not common.
__device__ __forceinline__ bool fa_fast_ok(const uint32_t (&w)[17], int64_t g, uint64_t len) {
    if (g <= 0 || (uint64_t)g + FA_BPT >= len) return false;
    uint32_t any = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) any |= fa_eq(w[i], 0x3E3E3E3Eu) | fa_eq(w[i], 0x0D0D0D0Du);
    return any == 0;
}

template <bool WRITE>
__device__ __forceinline__ uint64_t fa_fast(const uint32_t (&w)[17], uint8_t prev, uint32_t h_in, uint8_t *out,
                                            uint64_t o, const uint32_t *sel, uint32_t *nl_out) {
    uint32_t nlm[16], nl = 0, p0 = 64;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        nlm[i] = fa_bits4(fa_eq(w[i], 0x0A0A0A0Au));
        nl += __popc(nlm[i]);
        if (nlm[i] && p0 == 64) p0 = 4 * i + (__ffs(nlm[i]) - 1);
    }
    *nl_out = nl;
    const bool prev_nl = prev == '\n';
    const bool saw = prev_nl || p0 <= 62;
    const uint32_t common = 64 - nl, dep = (!prev_nl && nl) ? 1u : 0u;
    if (WRITE) {
        if (h_in && dep) nlm[p0 >> 2] &= ~(1u << (p0 & 3));   // a header's closing '\n' stays
        const uint64_t a_start = (o + 3) & ~3ull;
        uint64_t acc = 0;
        uint32_t accn = 0;
        auto emit_word = [&](uint32_t v) {            // output bytes [o, o + 4) -- whole words past a_start
            if (o >= a_start) {
                *(uint32_t *)(out + o) = v;
            } else {
                for (uint32_t b = 0; b < 4; ++b) out[o + b] = (uint8_t)(v >> (8 * b));
            }
            o += 4;
        };
        // (bytes before a_start are written singly, so the accumulator starts
        // aligned: the first (a_start - o) output bytes go out one by one)
        uint32_t lead = (uint32_t)(a_start - o);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t v = __builtin_amdgcn_perm(0u, w[i], sel[nlm[i]]);
            acc |= (uint64_t)v << (8 * accn);
            accn += 4 - __popc(nlm[i]);
            while (lead && accn) {                    // (at most 3 bytes, once per thread)
                out[o++] = (uint8_t)acc;
                acc >>= 8;
                --accn;
                --lead;
            }
            if (accn >= 4) {
                emit_word((uint32_t)acc);
                acc >>= 32;
                accn -= 4;
            }
        }
        for (uint32_t b = 0; b < accn; ++b) out[o + b] = (uint8_t)(acc >> (8 * b));
    }
    return fa_pack(saw ? 1u : 0u, common, common + dep);
}

// a thread's 64 bytes + the 4 after them, and the byte before
__device__ __forceinline__ uint8_t fa_regs(const uint8_t *buf, uint32_t (&w)[17]) {
    const uint4 *src = (const uint4 *)(buf + FA_BPT * threadIdx.x);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint4 x = src[j];
        w[4 * j] = x.x;
        w[4 * j + 1] = x.y;
        w[4 * j + 2] = x.z;
        w[4 * j + 3] = x.w;
    }
    w[16] = buf[FA_BPT * threadIdx.x + FA_BPT];      // (the next byte; buf[FA_TILE] is the neighbour tile's)
    return buf[FA_BPT * (int)threadIdx.x - 1];
}

struct FaShared {
    uint64_t wtot[TPB / 64];
    uint32_t nl[TPB / 64];
};

__global__ __launch_bounds__(TPB) void fa_tiles_kernel(const uint8_t *data, uint64_t len, FaTile *tiles) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[FA_TILE + 32];
    __shared__ FaShared sh;
    uint8_t *buf = stage + 16;
    const int64_t g0 = (int64_t)blockIdx.x * FA_TILE;
    fa_stage(data, len, g0, buf);
    __syncthreads();
    uint32_t nl = 0, w[17];
    const uint8_t prev = fa_regs(buf, w);
    const int64_t g = g0 + FA_BPT * threadIdx.x;
    const uint64_t f = fa_fast_ok(w, g, len) ? fa_fast<false>(w, prev, 0, nullptr, 0, nullptr, &nl)
                                             : fa_walk<false>(w, prev, g, len, 0, nullptr, 0, &nl);
    uint64_t total;
    uint32_t s = nl;
    for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d);
    if ((threadIdx.x & 63) == 0) sh.nl[threadIdx.x >> 6] = s;
    (void)fa_block_scan(f, sh.wtot, &total);
    if (threadIdx.x == 0) {
        FaTile t;
        t.kind = fa_kind(total);
        t.pad = 0;
        t.c0 = fa_c(total, 0);
        t.c1 = fa_c(total, 1);
        t.nl = (uint64_t)sh.nl[0] + sh.nl[1] + sh.nl[2] + sh.nl[3];
        tiles[blockIdx.x] = t;
    }
}

// tiles_x: exclusive scan of the tile functions (FaTileOp); the output of
// tile T starts at tiles_x[T] applied to state 0
__global__ __launch_bounds__(TPB) void fa_write_kernel(const uint8_t *data, uint64_t len, const FaTile *tiles_x,
                                                      uint8_t *out) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[FA_TILE + 32];
    __shared__ FaShared sh;
    __shared__ uint32_t sel[16];                 // v_perm selector keeping the bytes whose drop bit is clear
    uint8_t *buf = stage + 16;
    const int64_t g0 = (int64_t)blockIdx.x * FA_TILE;
    fa_stage(data, len, g0, buf);
    if (threadIdx.x < 16) {
        uint32_t v = 0x0C0C0C0Cu, n = 0;
        for (uint32_t b = 0; b < 4; ++b)
            if (!((threadIdx.x >> b) & 1u)) {
                v = (v & ~(0xFFu << (8 * n))) | (b << (8 * n));
                ++n;
            }
        sel[threadIdx.x] = v;
    }
    const FaTile px = tiles_x[blockIdx.x];
    const uint32_t h_tile = px.kind ? px.kind - 1 : 0u;  // (state at the chunk start: no line yet)
    const uint64_t off = px.c0;
    __syncthreads();
    uint32_t nl = 0, w[17];
    const uint8_t prev = fa_regs(buf, w);
    const int64_t g = g0 + FA_BPT * threadIdx.x;
    const bool fast = fa_fast_ok(w, g, len);
    const uint64_t f = fast ? fa_fast<false>(w, prev, 0, nullptr, 0, sel, &nl)
                            : fa_walk<false>(w, prev, g, len, 0, nullptr, 0, &nl);
    uint64_t total;
    const uint64_t ex = fa_block_scan(f, sh.wtot, &total);
    // this thread's incoming state and output offset
    const uint32_t kx = fa_kind(ex);
    const uint32_t h = kx ? kx - 1 : h_tile;
    if (fast)
        (void)fa_fast<true>(w, prev, h, out, off + fa_c(ex, h_tile), sel, &nl);
    else
        (void)fa_walk<true>(w, prev, g, len, h, out, off + fa_c(ex, h_tile), &nl);
}

}  // namespace

hipError_t launch_fa_tiles(const uint8_t *data, uint64_t len, uint32_t n_tiles, FaTile *tiles, hipStream_t s) {
    hipLaunchKernelGGL(fa_tiles_kernel, dim3(n_tiles), dim3(TPB), 0, s, data, len, tiles);
    return hipGetLastError();
}

hipError_t launch_fa_write(const uint8_t *data, uint64_t len, uint32_t n_tiles, const FaTile *tiles_x, uint8_t *out,
                           hipStream_t s) {
    hipLaunchKernelGGL(fa_write_kernel, dim3(n_tiles), dim3(TPB), 0, s, data, len, tiles_x, out);
    return hipGetLastError();
}

}  // namespace kmerhip
