// kmer_match.hip — k-mer -> template matching on the GPU (include/kmer_match.h).
//
// kmerFinder scores reference genomes ("templates") by the query k-mers they
// share (lib/kmerFinderServer.js:171-226, :736-849).  The reference does one
// Redis lrange per query k-mer and folds the lists into a JS Map, then loops
// winner-takes-all: the template with the most shared k-mers wins, its k-mers
// leave the query, everything is re-scored.  Here:
//
//   DB (once):  k-mers packed to 2-bit codes, (code, template) pairs radix
//               sorted (stable: a k-mer's templates stay in DB order), dedup,
//               CSR: U[m] sorted distinct codes, O[m + 1] list offsets, T[] templates.
//   round 1:    each query key packed and binary-searched in U; hits expanded to
//               (template, query) pairs in (query, list) order, radix sorted by
//               template (stable) -> per-template segments of query indices:
//               uScore = segment length, tScore = sum of counts (one wave per
//               template), first hit = the segment's first query.  Templates
//               ranked by (first query, template) = the Redis Map's insertion order.
//   winner:     one workgroup: max of uScore << 32 | ~rank.
//   remove:     the winner's segment: each query k-mer still present is
//               removed (atomic exchange) and its templates' scores drop.
//
// All integer work; the join is a few random reads per query key and the
// remove touches only the winner's k-mers.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/kmer_match.h"

namespace {

constexpr uint32_t NONE = 0xFFFFFFFFu;
thread_local std::string g_err;

kmer_status set_err(kmer_status s, const std::string &msg) {
    g_err = msg;
    return s;
}

#define MCHK(x)                                                                      \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) return set_err(KMER_E_DEVICE, std::string("HIP error: ") + hipGetErrorString(e_) + " at " #x); \
    } while (0)

template <typename T>
hipError_t dalloc(T **p, uint64_t n) {
    return hipMalloc((void **)p, std::max<uint64_t>(n, 1) * sizeof(T));
}

struct Temp {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipMalloc(&p, n);
        if (e == hipSuccess) cap = n;
        return e;
    }
    ~Temp() {
        if (p) (void)hipFree(p);
    }
};

// grow-only device array (buffers are reused by the next match on the DB)
template <typename T>
struct DArr {
    T *p = nullptr;
    uint64_t cap = 0;
    hipError_t ensure(uint64_t n) {
        n = std::max<uint64_t>(n, 1);
        if (n <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipMalloc((void **)&p, std::max(n, cap + cap / 2) * sizeof(T));
        if (e == hipSuccess) cap = std::max(n, cap + cap / 2);
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

#define MROC(tmp, CALL)                       \
    do {                                      \
        size_t b = 0;                         \
        void *t = nullptr;                    \
        MCHK(CALL);                           \
        MCHK((tmp).ensure(b + 16));           \
        t = (tmp).p;                          \
        MCHK(CALL);                           \
    } while (0)

int bit_width64(uint64_t x) {
    int b = 0;
    while (x) {
        ++b;
        x >>= 1;
    }
    return b;
}

__device__ __forceinline__ int base2(uint32_t c) {
    return c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : c == 'T' ? 3 : -1;
}

__device__ __forceinline__ bool pack_key(const uint8_t *p, uint32_t k, uint64_t *code) {
    uint64_t v = 0;
    bool ok = true;
    for (uint32_t i = 0; i < k; ++i) {
        const int b = base2(p[i]);
        ok &= b >= 0;
        v = (v << 2) | (uint64_t)(b & 3);
    }
    *code = v;
    return ok;
}

// ---------------------------------------------------------------------------
// DB kernels
// ---------------------------------------------------------------------------
__global__ void db_pack_kernel(const uint8_t *keys, uint64_t n, uint32_t k, uint64_t *codes, uint32_t *bad) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t c;
        if (!pack_key(keys + i * k, k, &c)) atomicOr(bad, 1u);
        codes[i] = c;
    }
}

// entry -> template (template t owns [ts[t], ts[t + 1]))
__global__ void db_tmpl_kernel(const uint64_t *ts, uint32_t nt, uint32_t *tmpl) {
    for (uint32_t t = blockIdx.x; t < nt; t += gridDim.x)
        for (uint64_t i = ts[t] + threadIdx.x; i < ts[t + 1]; i += blockDim.x) tmpl[i] = t;
}

// after the (code, template) sort: keep = not a repeated pair, head = first of its code
struct KeepHead {
    const uint64_t *c;
    const uint32_t *t;
    __device__ uint64_t operator()(uint64_t i) const {
        const bool head = i == 0 || c[i] != c[i - 1];
        const bool keep = head || t[i] != t[i - 1];
        return (keep ? 1ull : 0ull) | (head ? 1ull << 32 : 0ull);
    }
};

__global__ void db_csr_kernel(const uint64_t *c, const uint32_t *t, uint64_t n, const uint64_t *pos, uint64_t *U,
                              uint64_t *O, uint32_t *T) {
    KeepHead kh{c, t};
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t f = kh(i), p = pos[i];
        const uint64_t e = p & 0xFFFFFFFFull, u = p >> 32;
        if (f & 1) T[e] = t[i];
        if (f >> 32) {
            U[u] = c[i];
            O[u] = e;
        }
    }
}

// dir[p] = first U index whose code >> dsh is >= (dlo >> dsh) + p (p = 0 .. np)
__global__ void db_dir_kernel(const uint64_t *U, uint64_t m, uint64_t dlo, uint32_t dsh, uint64_t np, uint32_t *dir) {
    for (uint64_t p = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; p <= np; p += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t cell = (dlo >> dsh) + p;
        uint64_t lo = 0, hi = m;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if ((U[mid] >> dsh) < cell) lo = mid + 1;
            else hi = mid;
        }
        dir[p] = (uint32_t)lo;
    }
}

// ---------------------------------------------------------------------------
// query kernels
// ---------------------------------------------------------------------------
// pack + directory + binary search: qidx = DB k-mer index or NONE, hc = its
// list length.  The directory cell of a code (its bits above dsh, relative to
// the smallest DB code) bounds the search to a few entries.
__global__ void q_lookup_kernel(const uint8_t *keys, const uint64_t *offs, uint32_t klen, uint64_t n, uint32_t k,
                                const uint64_t *U, uint64_t m, const uint64_t *O, const uint32_t *dir, uint64_t dlo,
                                uint64_t dhi, uint32_t dsh, uint32_t *qidx, uint64_t *hc, uint32_t *present) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t b = offs ? offs[i] : i * klen;
        const uint64_t len = offs ? offs[i + 1] - b : klen;
        uint32_t idx = NONE;
        uint64_t code;
        if (len == k && m && pack_key(keys + b, k, &code) && code >= dlo && code <= dhi) {
            const uint64_t p = (code >> dsh) - (dlo >> dsh);
            uint64_t lo = dir[p], hi = dir[p + 1];      // first U[j] >= code, inside its directory cell
            while (lo < hi) {
                const uint64_t mid = (lo + hi) >> 1;
                if (U[mid] < code) lo = mid + 1;
                else hi = mid;
            }
            if (lo < m && U[lo] == code) idx = (uint32_t)lo;
        }
        qidx[i] = idx;
        hc[i] = idx == NONE ? 0 : O[idx + 1] - O[idx];
        present[i] = idx == NONE ? 0u : 1u;
    }
}

// hits in (query, list) order as (template, query) pairs, load-balanced: a
// wave takes 64 consecutive query keys and its lanes walk the wave's hits in
// order (lane-strided), each finding its owner key by a 6-step search over
// the lanes' hit offsets -- coalesced stores, no per-key loop imbalance.
__global__ __launch_bounds__(256) void q_emit_kernel(const uint32_t *qidx, const uint64_t *H, uint64_t n,
                                                     const uint64_t *O, const uint32_t *T, uint32_t *pt, uint32_t *pq) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint64_t w0 = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) & ~63ull; w0 < n;
         w0 += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = w0 + lane;
        const uint32_t idx = i < n ? qidx[i] : NONE;
        const uint64_t o = idx == NONE ? 0 : O[idx], c = idx == NONE ? 0 : O[idx + 1] - o;
        const uint64_t h = i < n ? H[i] : ~0ull;                // (past the end: never an owner)
        uint64_t end = i < n ? h + c : 0;
        for (int d = 32; d >= 1; d >>= 1) {
            const uint64_t x = __shfl_xor(end, d);
            end = x > end ? x : end;
        }
        const uint64_t start = __shfl(h, 0);
        // (wave-uniform trip count: every lane takes part in the shuffles)
        for (uint64_t r = start; r < end; r += 64) {
            const uint64_t e = r + lane;
            int lo = 0, hi = 63;                                // the last lane with h <= e owns e
#pragma unroll
            for (int it = 0; it < 6; ++it) {
                const int mid = (lo + hi + 1) >> 1;
                if (__shfl(h, mid) <= e) lo = mid;
                else hi = mid - 1;
            }
            const uint64_t hl = __shfl(h, lo), ol = __shfl(o, lo);
            if (e < end) {
                pt[e] = T[ol + (e - hl)];
                pq[e] = (uint32_t)(w0 + (uint64_t)lo);
            }
        }
    }
}

// seg[t] = first sorted hit of template >= t (t = 0 .. nt)
__global__ void q_seg_kernel(const uint32_t *st, uint64_t hits, uint32_t nt, uint64_t *seg) {
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t <= nt; t += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t lo = 0, hi = hits;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (st[mid] < t) lo = mid + 1;
            else hi = mid;
        }
        seg[t] = lo;
    }
}

// one wave per template: round-1 scores and its first-hit sort key
__global__ __launch_bounds__(256) void q_score_kernel(const uint64_t *seg, const uint32_t *sq, const uint64_t *cnt,
                                                      uint32_t nt, uint32_t *u0, uint64_t *t0, uint32_t *cu,
                                                      uint64_t *ct, uint64_t *fkey, uint32_t *nh) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint64_t t = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6; t < nt;
         t += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
        const uint64_t a = seg[t], b = seg[t + 1];
        uint64_t s = 0;
        for (uint64_t e = a + lane; e < b; e += 64) s += cnt[sq[e]];
        for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d);
        if (lane == 0) {
            const uint32_t u = (uint32_t)(b - a);
            u0[t] = u;
            cu[t] = u;
            t0[t] = s;
            ct[t] = s;
            fkey[t] = u ? ((uint64_t)sq[a] << 32) | t : ~0ull;
            if (u) atomicAdd(nh, 1u);
        }
    }
}

__global__ void q_order_kernel(const uint64_t *skey, uint32_t nh, uint32_t *order, uint32_t *rank) {
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < nh; r += gridDim.x * blockDim.x) {
        const uint32_t t = (uint32_t)skey[r];
        order[r] = t;
        rank[t] = r;
    }
}

// scal: [0] hits left; winner written to *w
__global__ __launch_bounds__(1024) void winner_kernel(const uint32_t *order, uint32_t nh, const uint32_t *cu,
                                                      const uint64_t *ct, const uint32_t *u0, const uint64_t *t0,
                                                      const uint64_t *scal, kmer_winner *w) {
    __shared__ uint64_t part[16];
    uint64_t best = 0;
    for (uint32_t r = threadIdx.x; r < nh; r += blockDim.x) {
        const uint32_t u = cu[order[r]];
        const uint64_t key = u ? ((uint64_t)u << 32) | (0xFFFFFFFFu - r) : 0;
        best = key > best ? key : best;
    }
    for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t o = __shfl_xor(best, d);
        best = o > best ? o : best;
    }
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (uint32_t i = 1; i < blockDim.x / 64; ++i) best = part[i] > best ? part[i] : best;
        kmer_winner o;
        memset(&o, 0, sizeof(o));
        o.tmpl = NONE;
        o.hits = scal[0];
        if (best) {
            const uint32_t t = order[0xFFFFFFFFu - (uint32_t)best];
            o.tmpl = t;
            o.uscore = cu[t];
            o.tscore = ct[t];
            o.first_uscore = u0[t];
            o.first_tscore = t0[t];
        }
        *w = o;
    }
}

// removeWinnerKmers: the winner's query k-mers still present leave the query
__global__ void remove_kernel(const uint64_t *seg, const uint32_t *sq, uint32_t w, uint32_t *present,
                              const uint32_t *qidx, const uint64_t *O, const uint32_t *T, const uint64_t *cnt,
                              uint32_t *cu, uint64_t *ct, uint64_t *scal) {
    const uint64_t a = seg[w], b = seg[w + 1];
    for (uint64_t e = a + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < b;
         e += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t q = sq[e];
        if (atomicExch(&present[q], 0u) == 0u) continue;
        const uint32_t idx = qidx[q];
        const uint64_t o = O[idx], len = O[idx + 1] - o, c = cnt[q];
        for (uint64_t j = 0; j < len; ++j) {
            const uint32_t t = T[o + j];
            atomicSub(&cu[t], 1u);
            atomicAdd((unsigned long long *)&ct[t], (unsigned long long)(0ull - c));
        }
        atomicAdd((unsigned long long *)&scal[0], (unsigned long long)(0ull - len));
    }
}

__global__ void removed_kernel(const uint32_t *qidx, const uint32_t *present, uint64_t n, uint8_t *flags) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        flags[i] = qidx[i] != NONE && present[i] == 0u ? 1 : 0;
}

uint32_t grid_for(uint64_t n, uint32_t block = 256, uint32_t cap = 65536) {
    const uint64_t g = (n + block - 1) / block;
    return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(g, cap));
}

}  // namespace

// Per-match arrays; a closed match hands them to its DB for the next one.
struct MatchBufs {
    DArr<uint64_t> cnt, H, seg, t0, ct, scal;
    DArr<uint32_t> qidx, present, sq, u0, cu, order, rank;
    DArr<kmer_winner> dw;
    kmer_winner *hw = nullptr;
    void release() {
        cnt.release(), H.release(), seg.release(), t0.release(), ct.release(), scal.release();
        qidx.release(), present.release(), sq.release(), u0.release(), cu.release(), order.release(), rank.release();
        dw.release();
        if (hw) (void)hipHostFree(hw);
        hw = nullptr;
    }
};

struct kmer_db {
    int device = 0;
    uint32_t k = 0, nt = 0;
    uint64_t m = 0, entries = 0;
    hipStream_t s = nullptr;
    uint64_t *U = nullptr, *O = nullptr;
    uint32_t *T = nullptr;
    uint32_t *dir = nullptr;                   // directory over the codes' high bits
    uint64_t dlo = ~0ull, dhi = 0;
    uint32_t dsh = 0;
    // scratch of a match build (matches of one DB are built one at a time)
    DArr<uint8_t> qkeys;
    DArr<uint64_t> qoffs, hc, fkey, fkey2;
    DArr<uint32_t> pt, pt2, pq2, nhd;
    Temp tmp;
    MatchBufs spare;                           // buffers of the last closed match
    bool has_spare = false;
    uint32_t live = 0;                         // open matches
    bool closing = false;                      // kmer_db_close called while matches were open
};

struct kmer_match {
    kmer_db *db = nullptr;
    uint64_t n = 0, hits0 = 0;
    uint32_t nh = 0;
    MatchBufs b;
    uint64_t *cnt = nullptr, *H = nullptr, *seg = nullptr, *t0 = nullptr, *ct = nullptr, *scal = nullptr;
    uint32_t *qidx = nullptr, *present = nullptr, *sq = nullptr, *u0 = nullptr, *cu = nullptr, *order = nullptr,
             *rank = nullptr;
    kmer_winner *dw = nullptr, *hw = nullptr;
    void release() {
        if (!db->has_spare) {                  // keep the buffers for the DB's next match
            db->spare = b;
            db->has_spare = true;
        } else {
            b.release();
        }
        b = MatchBufs();
    }
};

namespace {

void free_db(kmer_db *db) {
    if (!db) return;
    (void)hipSetDevice(db->device);
    if (db->U) (void)hipFree(db->U);
    if (db->O) (void)hipFree(db->O);
    if (db->T) (void)hipFree(db->T);
    if (db->dir) (void)hipFree(db->dir);
    db->qkeys.release(), db->qoffs.release(), db->hc.release(), db->fkey.release(), db->fkey2.release();
    db->pt.release(), db->pt2.release(), db->pq2.release(), db->nhd.release();
    if (db->has_spare) db->spare.release();
    if (db->s) (void)hipStreamDestroy(db->s);
    delete db;
}

kmer_status build_db(kmer_db *db, const char *keys, uint64_t n, const uint64_t *ts) {
    hipStream_t s = db->s;
    Temp tmp;
    uint8_t *dkeys = nullptr;
    uint64_t *c = nullptr, *c2 = nullptr, *dts = nullptr, *pos = nullptr;
    uint32_t *t = nullptr, *t2 = nullptr, *bad = nullptr;
    auto cleanup = [&]() {
        for (void *p : {(void *)dkeys, (void *)c, (void *)c2, (void *)dts, (void *)pos, (void *)t, (void *)t2,
                        (void *)bad})
            if (p) (void)hipFree(p);
    };
    struct Guard {
        decltype(cleanup) &f;
        ~Guard() { f(); }
    } guard{cleanup};
    MCHK(dalloc(&dkeys, n * db->k));
    MCHK(dalloc(&c, n));
    MCHK(dalloc(&c2, n));
    MCHK(dalloc(&t, n));
    MCHK(dalloc(&t2, n));
    MCHK(dalloc(&dts, (uint64_t)db->nt + 1));
    MCHK(dalloc(&pos, n));
    MCHK(dalloc(&bad, 1));
    MCHK(hipMemsetAsync(bad, 0, 4, s));
    // (the caller's arrays, read in place: waited for on every return path)
    struct SyncOnExit {
        hipStream_t s;
        ~SyncOnExit() { (void)hipStreamSynchronize(s); }
    } wait_uploads{s};
    MCHK(hipMemcpyAsync(dkeys, keys, n * db->k, hipMemcpyHostToDevice, s));
    MCHK(hipMemcpyAsync(dts, ts, ((uint64_t)db->nt + 1) * 8, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(db_pack_kernel, dim3(grid_for(n)), dim3(256), 0, s, dkeys, n, db->k, c, bad);
    hipLaunchKernelGGL(db_tmpl_kernel, dim3(std::min<uint32_t>(std::max<uint32_t>(db->nt, 1), 65536)), dim3(256), 0,
                       s, dts, db->nt, t);
    MCHK(hipGetLastError());
    uint32_t hbad = 0;
    MCHK(hipMemcpyAsync(&hbad, bad, 4, hipMemcpyDeviceToHost, s));
    MCHK(hipStreamSynchronize(s));
    if (hbad) return set_err(KMER_E_BAD_PARAM, "kmer_db_open: a template k-mer has a byte outside A/C/G/T");
    rocprim::double_buffer<uint64_t> kb(c, c2);
    rocprim::double_buffer<uint32_t> vb(t, t2);
    MROC(tmp, rocprim::radix_sort_pairs(t, b, kb, vb, (size_t)n, 0, 2 * db->k, s));
    const uint64_t *sc = kb.current();
    const uint32_t *stt = vb.current();
    rocprim::counting_iterator<uint64_t> iota(0);
    auto flags = rocprim::make_transform_iterator(iota, KeepHead{sc, stt});
    MROC(tmp, rocprim::exclusive_scan(t, b, flags, pos, (uint64_t)0, (size_t)n, rocprim::plus<uint64_t>(), s));
    uint64_t last[2] = {0, 0};
    MCHK(hipMemcpyAsync(&last[0], pos + n - 1, 8, hipMemcpyDeviceToHost, s));
    MCHK(hipStreamSynchronize(s));
    // (the last entry's own flags: recomputed on the host from the two sorted tails)
    uint64_t tail_c[2] = {0, 0};
    uint32_t tail_t[2] = {0, 0};
    MCHK(hipMemcpy(tail_c, sc + (n >= 2 ? n - 2 : 0), 8 * std::min<uint64_t>(n, 2), hipMemcpyDeviceToHost));
    MCHK(hipMemcpy(tail_t, stt + (n >= 2 ? n - 2 : 0), 4 * std::min<uint64_t>(n, 2), hipMemcpyDeviceToHost));
    bool head = n == 1 || tail_c[1] != tail_c[0];
    bool keep = head || tail_t[1] != tail_t[0];
    db->entries = (last[0] & 0xFFFFFFFFull) + (keep ? 1 : 0);
    db->m = (last[0] >> 32) + (head ? 1 : 0);
    if (db->entries >= NONE || db->m >= NONE)
        return set_err(KMER_E_BAD_PARAM, "kmer_db_open: more than 2^32 - 2 DB entries");
    MCHK(dalloc(&db->U, db->m));
    MCHK(dalloc(&db->O, db->m + 1));
    MCHK(dalloc(&db->T, db->entries));
    hipLaunchKernelGGL(db_csr_kernel, dim3(grid_for(n)), dim3(256), 0, s, sc, stt, n, pos, db->U, db->O, db->T);
    MCHK(hipGetLastError());
    MCHK(hipMemcpyAsync(db->O + db->m, &db->entries, 8, hipMemcpyHostToDevice, s));
    // directory: up to 2^20 cells over the bits below the codes' common prefix
    MCHK(hipMemcpyAsync(&db->dlo, db->U, 8, hipMemcpyDeviceToHost, s));
    MCHK(hipMemcpyAsync(&db->dhi, db->U + db->m - 1, 8, hipMemcpyDeviceToHost, s));
    MCHK(hipStreamSynchronize(s));
    const int span = bit_width64(db->dlo ^ db->dhi);
    db->dsh = (uint32_t)std::max(0, span - 20);
    const uint64_t np = (db->dhi >> db->dsh) - (db->dlo >> db->dsh) + 1;
    MCHK(dalloc(&db->dir, np + 1));
    hipLaunchKernelGGL(db_dir_kernel, dim3(grid_for(np + 1)), dim3(256), 0, s, db->U, db->m, db->dlo, db->dsh, np,
                       db->dir);
    MCHK(hipGetLastError());
    MCHK(hipStreamSynchronize(s));
    return KMER_OK;
}

kmer_status match_build(kmer_match *m, const uint8_t *dkeys, const uint64_t *doffs, uint32_t klen) {
    kmer_db *db = m->db;
    hipStream_t s = db->s;
    const uint64_t n = m->n;
    const uint32_t nt = db->nt;
    Temp &tmp = db->tmp;
    MatchBufs &b = m->b;
    MCHK(b.qidx.ensure(n));
    MCHK(b.present.ensure(n));
    MCHK(b.H.ensure(n));
    MCHK(b.seg.ensure((uint64_t)nt + 1));
    MCHK(b.u0.ensure(nt));
    MCHK(b.cu.ensure(nt));
    MCHK(b.t0.ensure(nt));
    MCHK(b.ct.ensure(nt));
    MCHK(b.order.ensure(nt));
    MCHK(b.rank.ensure(nt));
    MCHK(b.scal.ensure(2));
    MCHK(b.dw.ensure(1));
    if (!b.hw) MCHK(hipHostMalloc((void **)&b.hw, sizeof(kmer_winner), hipHostMallocDefault));
    MCHK(db->nhd.ensure(1));
    MCHK(db->fkey.ensure(nt));
    MCHK(db->fkey2.ensure(nt));
    MCHK(db->hc.ensure(n));
    m->qidx = b.qidx.p, m->present = b.present.p, m->H = b.H.p, m->seg = b.seg.p, m->u0 = b.u0.p;
    m->cu = b.cu.p, m->t0 = b.t0.p, m->ct = b.ct.p, m->order = b.order.p, m->rank = b.rank.p;
    m->scal = b.scal.p, m->dw = b.dw.p, m->hw = b.hw;
    uint32_t *nhd = db->nhd.p;
    uint64_t *fkey = db->fkey.p, *fkey2 = db->fkey2.p, *hc = db->hc.p;
    // hit counts per query key -> their exclusive scan
    hipLaunchKernelGGL(q_lookup_kernel, dim3(grid_for(n)), dim3(256), 0, s, dkeys, doffs, klen, n, db->k, db->U,
                       db->m, db->O, db->dir, db->dlo, db->dhi, db->dsh, m->qidx, hc, m->present);
    MCHK(hipGetLastError());
    if (n) MROC(tmp, rocprim::exclusive_scan(t, b, hc, m->H, (uint64_t)0, (size_t)n, rocprim::plus<uint64_t>(), s));
    uint64_t tail[2] = {0, 0};
    if (n) MCHK(hipMemcpyAsync(&tail[0], m->H + n - 1, 8, hipMemcpyDeviceToHost, s));
    if (n) MCHK(hipMemcpyAsync(&tail[1], hc + n - 1, 8, hipMemcpyDeviceToHost, s));
    MCHK(hipStreamSynchronize(s));
    const uint64_t hits = tail[0] + tail[1];
    m->hits0 = hits;
    MCHK(hipMemcpyAsync(m->scal, &m->hits0, 8, hipMemcpyHostToDevice, s));
    MCHK(hipMemsetAsync(nhd, 0, 4, s));
    if (hits >= NONE) return set_err(KMER_E_BAD_PARAM, "kmer_match_open: more than 2^32 - 2 hits");
    MCHK(db->pt.ensure(hits));
    MCHK(db->pt2.ensure(hits));
    MCHK(db->pq2.ensure(hits));
    MCHK(b.sq.ensure(hits));
    m->sq = b.sq.p;
    if (hits) {
        hipLaunchKernelGGL(q_emit_kernel, dim3(grid_for(n)), dim3(256), 0, s, m->qidx, m->H, n, db->O, db->T,
                           db->pt.p, db->pq2.p);
        MCHK(hipGetLastError());
        rocprim::double_buffer<uint32_t> kb(db->pt.p, db->pt2.p);
        rocprim::double_buffer<uint32_t> vb(db->pq2.p, m->sq);
        MROC(tmp, rocprim::radix_sort_pairs(t, b, kb, vb, (size_t)hits, 0, std::max(1, bit_width64(nt)), s));
        if (vb.current() != m->sq) MCHK(hipMemcpyAsync(m->sq, vb.current(), hits * 4, hipMemcpyDeviceToDevice, s));
        hipLaunchKernelGGL(q_seg_kernel, dim3(grid_for((uint64_t)nt + 1)), dim3(256), 0, s, kb.current(), hits, nt,
                           m->seg);
    } else {
        MCHK(hipMemsetAsync(m->seg, 0, ((uint64_t)nt + 1) * 8, s));
    }
    hipLaunchKernelGGL(q_score_kernel, dim3(grid_for((uint64_t)nt * 64)), dim3(256), 0, s, m->seg, m->sq, m->cnt, nt,
                       m->u0, m->t0, m->cu, m->ct, fkey, nhd);
    MCHK(hipGetLastError());
    MROC(tmp, rocprim::radix_sort_keys(t, b, fkey, fkey2, (size_t)std::max<uint32_t>(nt, 1), 0, 64, s));
    MCHK(hipMemcpyAsync(&m->nh, nhd, 4, hipMemcpyDeviceToHost, s));
    MCHK(hipStreamSynchronize(s));
    hipLaunchKernelGGL(q_order_kernel, dim3(grid_for(std::max<uint32_t>(m->nh, 1))), dim3(256), 0, s, fkey2, m->nh,
                       m->order, m->rank);
    MCHK(hipGetLastError());
    MCHK(hipStreamSynchronize(s));
    return KMER_OK;
}

kmer_status match_open_common(kmer_db *db, uint64_t n, kmer_match **out, kmer_match **mm) {
    if (!db || !out) return set_err(KMER_E_BAD_PARAM, "kmer_match_open: NULL argument");
    if (db->closing) return set_err(KMER_E_STATE, "kmer_match_open: the DB is closed");
    if (n >= NONE) return set_err(KMER_E_BAD_PARAM, "kmer_match_open: more than 2^32 - 2 query keys");
    *out = nullptr;
    MCHK(hipSetDevice(db->device));
    kmer_match *m = new kmer_match();
    m->db = db;
    m->n = n;
    ++db->live;
    if (db->has_spare) {                        // the last closed match's buffers
        m->b = db->spare;
        db->spare = MatchBufs();
        db->has_spare = false;
    }
    *mm = m;
    return KMER_OK;
}

}  // namespace

extern "C" {

kmer_status kmer_db_open(int32_t device, uint32_t k, const char *keys, uint64_t n_keys,
                         const uint64_t *template_start, uint32_t n_templates, kmer_db **out) {
    if (!out || (!keys && n_keys) || !template_start) return set_err(KMER_E_BAD_PARAM, "kmer_db_open: NULL argument");
    *out = nullptr;
    if (k == 0 || k > 32) return set_err(KMER_E_BAD_PARAM, "kmer_db_open: k must be 1..32");
    if (n_templates >= 0x7FFFFFFFu) return set_err(KMER_E_BAD_PARAM, "kmer_db_open: too many templates");
    if (template_start[0] != 0 || template_start[n_templates] != n_keys)
        return set_err(KMER_E_BAD_PARAM, "kmer_db_open: template_start must run from 0 to n_keys");
    for (uint32_t t = 0; t < n_templates; ++t)
        if (template_start[t + 1] < template_start[t])
            return set_err(KMER_E_BAD_PARAM, "kmer_db_open: template_start must not decrease");
    if (n_keys >= NONE) return set_err(KMER_E_BAD_PARAM, "kmer_db_open: more than 2^32 - 2 k-mers");
    MCHK(hipSetDevice(device));
    kmer_db *db = new kmer_db();
    db->device = device;
    db->k = k;
    db->nt = n_templates;
    hipError_t e = hipStreamCreateWithFlags(&db->s, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete db;
        MCHK(e);
    }
    kmer_status st = KMER_OK;
    if (n_keys) {
        st = build_db(db, keys, n_keys, template_start);
    } else {
        e = dalloc(&db->O, 1);
        if (e == hipSuccess) e = hipMemset(db->O, 0, 8);
        if (e != hipSuccess) st = set_err(KMER_E_DEVICE, "kmer_db_open: allocation failed");
    }
    if (st != KMER_OK) {
        free_db(db);
        return st;
    }
    *out = db;
    return KMER_OK;
}

kmer_status kmer_db_info(const kmer_db *db, uint32_t *k, uint32_t *n_templates, uint64_t *distinct,
                         uint64_t *entries) {
    if (!db) return set_err(KMER_E_BAD_PARAM, "kmer_db_info: NULL db");
    if (k) *k = db->k;
    if (n_templates) *n_templates = db->nt;
    if (distinct) *distinct = db->m;
    if (entries) *entries = db->entries;
    return KMER_OK;
}

kmer_status kmer_db_close(kmer_db *db) {
    if (db && db->live) {   // a match reads the DB's CSR and hands its buffers back at close:
        db->closing = true;  // the last kmer_match_close frees the DB
        return KMER_OK;
    }
    free_db(db);
    return KMER_OK;
}

kmer_status kmer_match_open(kmer_db *db, const char *keys, const uint64_t *offsets, const uint64_t *counts,
                            uint64_t n, kmer_match **out) {
    if (n && (!keys || !offsets || !counts)) return set_err(KMER_E_BAD_PARAM, "kmer_match_open: NULL argument");
    if (n && offsets[0] != 0) return set_err(KMER_E_BAD_PARAM, "kmer_match_open: offsets[0] must be 0");
    for (uint64_t i = 0; i < n; ++i)    // q_lookup_kernel packs keys + offsets[i] .. offsets[i + 1]
        if (offsets[i + 1] < offsets[i])
            return set_err(KMER_E_BAD_PARAM, "kmer_match_open: offsets must not decrease");
    kmer_match *m = nullptr;
    kmer_status st = match_open_common(db, n, out, &m);
    if (st != KMER_OK) return st;
    const uint64_t nbytes = n ? offsets[n] : 0;
    hipError_t e = db->qkeys.ensure(nbytes);
    if (e == hipSuccess) e = db->qoffs.ensure(n + 1);
    if (e == hipSuccess) e = m->b.cnt.ensure(n);
    m->cnt = m->b.cnt.p;
    if (e == hipSuccess && nbytes) e = hipMemcpyAsync(db->qkeys.p, keys, nbytes, hipMemcpyHostToDevice, db->s);
    if (e == hipSuccess && n) e = hipMemcpyAsync(db->qoffs.p, offsets, (n + 1) * 8, hipMemcpyHostToDevice, db->s);
    if (e == hipSuccess && n) e = hipMemcpyAsync(m->cnt, counts, n * 8, hipMemcpyHostToDevice, db->s);
    st = e == hipSuccess ? match_build(m, db->qkeys.p, db->qoffs.p, 0)
                         : set_err(KMER_E_DEVICE, std::string("HIP error: ") + hipGetErrorString(e));
    (void)hipStreamSynchronize(db->s);
    if (st != KMER_OK) {
        m->release();
        --m->db->live;
        delete m;
        return st;
    }
    *out = m;
    return KMER_OK;
}

kmer_status kmer_match_open_device(kmer_db *db, const void *d_keys, uint32_t klen, const void *d_counts, uint64_t n,
                                   void *stream, kmer_match **out) {
    if (n && (!d_keys || !d_counts || klen == 0))
        return set_err(KMER_E_BAD_PARAM, "kmer_match_open_device: NULL argument");
    kmer_match *m = nullptr;
    kmer_status st = match_open_common(db, n, out, &m);
    if (st != KMER_OK) return st;
    hipEvent_t ev = nullptr;
    hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(ev, (hipStream_t)stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(db->s, ev, 0);
    if (e == hipSuccess) e = m->b.cnt.ensure(n);
    m->cnt = m->b.cnt.p;
    if (e == hipSuccess && n) e = hipMemcpyAsync(m->cnt, d_counts, n * 8, hipMemcpyDeviceToDevice, db->s);
    st = e == hipSuccess ? match_build(m, (const uint8_t *)d_keys, nullptr, klen)
                         : set_err(KMER_E_DEVICE, std::string("HIP error: ") + hipGetErrorString(e));
    if (ev) (void)hipEventDestroy(ev);
    if (st != KMER_OK) {
        m->release();
        --m->db->live;
        delete m;
        return st;
    }
    *out = m;
    return KMER_OK;
}

kmer_status kmer_match_info(kmer_match *m, uint64_t *hits, uint32_t *n_templates) {
    if (!m) return set_err(KMER_E_BAD_PARAM, "kmer_match_info: NULL match");
    MCHK(hipSetDevice(m->db->device));
    kmer_winner w;
    kmer_status st = kmer_match_winner(m, &w);
    if (st != KMER_OK) return st;
    if (hits) *hits = w.hits;
    if (n_templates) {
        uint32_t n = 0;
        st = kmer_match_templates(m, KMER_ORDER_DB, 0, nullptr, nullptr, nullptr, &n);
        if (st != KMER_OK) return st;
        *n_templates = n;
    }
    return KMER_OK;
}

kmer_status kmer_match_templates(kmer_match *m, uint32_t order, uint32_t cap, uint32_t *tmpl, uint64_t *uscore,
                                 uint64_t *tscore, uint32_t *n) {
    if (!m || !n || (cap && (!tmpl || !uscore || !tscore)) || order > KMER_ORDER_DB)
        return set_err(KMER_E_BAD_PARAM, "kmer_match_templates: bad argument");
    MCHK(hipSetDevice(m->db->device));
    const uint32_t nt = m->db->nt, nh = m->nh;
    std::vector<uint32_t> ord(nh), cu(nt);
    std::vector<uint64_t> ct(nt);
    hipStream_t s = m->db->s;
    if (nh) MCHK(hipMemcpyAsync(ord.data(), m->order, nh * 4ull, hipMemcpyDeviceToHost, s));
    if (nt) MCHK(hipMemcpyAsync(cu.data(), m->cu, nt * 4ull, hipMemcpyDeviceToHost, s));
    if (nt) MCHK(hipMemcpyAsync(ct.data(), m->ct, nt * 8ull, hipMemcpyDeviceToHost, s));
    MCHK(hipStreamSynchronize(s));
    uint32_t c = 0;
    auto put = [&](uint32_t t) {
        if (!cu[t]) return;
        if (c < cap) {
            tmpl[c] = t;
            uscore[c] = cu[t];
            tscore[c] = ct[t];
        }
        ++c;
    };
    if (order == KMER_ORDER_FIRST_HIT) {
        for (uint32_t r = 0; r < nh; ++r) put(ord[r]);
    } else {
        for (uint32_t t = 0; t < nt; ++t) put(t);
    }
    *n = c;
    return KMER_OK;
}

kmer_status kmer_match_template_kmers(kmer_match *m, uint32_t tmpl, uint64_t cap, uint32_t *qidx, uint64_t *n) {
    if (!m || !n || tmpl >= m->db->nt || (cap && !qidx))
        return set_err(KMER_E_BAD_PARAM, "kmer_match_template_kmers: bad argument");
    MCHK(hipSetDevice(m->db->device));
    hipStream_t s = m->db->s;
    uint64_t ab[2];
    MCHK(hipMemcpyAsync(ab, m->seg + tmpl, 16, hipMemcpyDeviceToHost, s));
    MCHK(hipStreamSynchronize(s));
    const uint64_t len = ab[1] - ab[0];
    if (cap && len) {
        MCHK(hipMemcpyAsync(qidx, m->sq + ab[0], std::min(cap, len) * 4, hipMemcpyDeviceToHost, s));
        MCHK(hipStreamSynchronize(s));
    }
    *n = len;
    return KMER_OK;
}

kmer_status kmer_match_winner(kmer_match *m, kmer_winner *w) {
    if (!m || !w) return set_err(KMER_E_BAD_PARAM, "kmer_match_winner: NULL argument");
    MCHK(hipSetDevice(m->db->device));
    hipStream_t s = m->db->s;
    hipLaunchKernelGGL(winner_kernel, dim3(1), dim3(1024), 0, s, m->order, m->nh, m->cu, m->ct, m->u0, m->t0,
                       m->scal, m->dw);
    MCHK(hipGetLastError());
    MCHK(hipMemcpyAsync(m->hw, m->dw, sizeof(kmer_winner), hipMemcpyDeviceToHost, s));
    MCHK(hipStreamSynchronize(s));
    *w = *m->hw;
    return KMER_OK;
}

kmer_status kmer_match_remove(kmer_match *m, uint32_t tmpl, uint64_t *hits) {
    if (!m || tmpl >= m->db->nt) return set_err(KMER_E_BAD_PARAM, "kmer_match_remove: bad template");
    MCHK(hipSetDevice(m->db->device));
    hipStream_t s = m->db->s;
    uint64_t ab[2];
    MCHK(hipMemcpyAsync(ab, m->seg + tmpl, 16, hipMemcpyDeviceToHost, s));
    MCHK(hipStreamSynchronize(s));
    const uint64_t len = ab[1] - ab[0];
    if (len) {
        hipLaunchKernelGGL(remove_kernel, dim3(grid_for(len)), dim3(256), 0, s, m->seg, m->sq, tmpl, m->present,
                           m->qidx, m->db->O, m->db->T, m->cnt, m->cu, m->ct, m->scal);
        MCHK(hipGetLastError());
    }
    uint64_t h = 0;
    MCHK(hipMemcpyAsync(&h, m->scal, 8, hipMemcpyDeviceToHost, s));
    MCHK(hipStreamSynchronize(s));
    if (hits) *hits = h;
    return KMER_OK;
}

kmer_status kmer_match_removed(kmer_match *m, uint8_t *flags) {
    if (!m || (m->n && !flags)) return set_err(KMER_E_BAD_PARAM, "kmer_match_removed: NULL argument");
    if (!m->n) return KMER_OK;
    MCHK(hipSetDevice(m->db->device));
    hipStream_t s = m->db->s;
    uint8_t *d = nullptr;
    MCHK(dalloc(&d, m->n));
    hipLaunchKernelGGL(removed_kernel, dim3(grid_for(m->n)), dim3(256), 0, s, m->qidx, m->present, m->n, d);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(flags, d, m->n, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    (void)hipFree(d);
    MCHK(e);
    return KMER_OK;
}

kmer_status kmer_match_close(kmer_match *m) {
    if (!m) return KMER_OK;
    (void)hipSetDevice(m->db->device);
    (void)hipStreamSynchronize(m->db->s);
    kmer_db *db = m->db;
    m->release();
    delete m;
    if (--db->live == 0 && db->closing) free_db(db);
    return KMER_OK;
}

const char *kmer_match_last_error(void) { return g_err.c_str(); }

}  // extern "C"
