// kmer_group.hip — multi-device group counts (kmer_params.ndev > 1).
#include "kmer_host.hpp"

namespace kmerhip {

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
    const bool ordered = (mode == MODE_PACKED || mode == MODE_WINDOWS) && !c0->wide;
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


}  // namespace kmerhip
