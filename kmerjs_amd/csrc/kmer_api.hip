// kmer_api.hip — the C-ABI entry points (include/kmer_api.h): context
// lifecycle, device-resident feeds, multi-GPU exchange, results, table queries.
// The machinery behind them: kmer_host.hpp.
#include "kmer_host.hpp"

using namespace kmerhip;

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
        // peer access between every pair of distinct devices, so the group's
        // partial / key copies (hipMemcpyPeerAsync, kmer_group.hip) go device to
        // device over xGMI.  A pair the platform refuses (no P2P path) keeps
        // working: the runtime stages such peer copies through host memory;
        // g->peer_staged counts those pairs (KMERHIP_PEER_LOG prints them).
        for (kmer_ctx *a : g->group)
            for (kmer_ctx *b : g->group) {
                if (a->device == b->device) continue;
                int can = 0;
                if (hipDeviceCanAccessPeer(&can, a->device, b->device) != hipSuccess) can = 0;
                hipError_t e = hipErrorPeerAccessUnsupported;
                if (can && hipSetDevice(a->device) == hipSuccess) {
                    e = hipDeviceEnablePeerAccess(b->device, 0);
                    if (e == hipErrorPeerAccessAlreadyEnabled) {
                        (void)hipGetLastError();   // (enabled by an earlier group: fine)
                        e = hipSuccess;
                    }
                }
                if (e != hipSuccess) {
                    (void)hipGetLastError();
                    ++g->peer_staged;
                    if (getenv("KMERHIP_PEER_LOG"))
                        fprintf(stderr, "kmerhip: no peer access %d -> %d (%s): peer copies staged by the runtime\n",
                                a->device, b->device, hipGetErrorString(e));
                }
            }
        g->device = g->group[0]->device;
        g->mode = g->group[0]->mode;
        (void)hipSetDevice(g->device);
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
    else if (dense_ok && (plen == 0 ? k <= 31 : (acgt && plen <= 3 && k <= (uint32_t)KMAX_TILE)))
        c->mode = MODE_WINDOWS;                 // (a 1-3-base prefix hits densely: kmer_dense.hip, k <= 64)
    else if (win_step)
        c->mode = MODE_WINDOWS;                 // step > 1: every stepped window ranked (the tile scan has no line ends)
    else if (dense_ok && plen > 0 && k <= (uint32_t)KMAX_TILE)
        c->mode = MODE_PACKED;                  // (k > 32: 128-bit window codes; any prefix bytes: key = P + suffix code)
    else if (pp->step == 1 && plen > 0 && k <= (uint32_t)KMAX_TILE)
        c->mode = MODE_TILE_REC;
    else
        c->mode = MODE_GENERAL;
    // general path with step 1: every record is a k-byte key, merged on the
    // device (KMER_FLAG_NO_DENSE keeps the host record merge, for the tests)
    c->gm_on = c->mode == MODE_GENERAL && pp->step == 1 && !(pp->flags & KMER_FLAG_NO_DENSE);
    const bool packed_keys = c->mode == MODE_PACKED || c->mode == MODE_WINDOWS;
    c->kbits = packed_keys ? 2 * (k - plen) : 0;
    c->narrow = packed_keys && c->kbits <= 31;
    c->wide = packed_keys && c->kbits >= 64;
    c->planes = (c->mode == MODE_PACKED || c->mode == MODE_TILE_REC) && acgt && !(pp->flags & KMER_FLAG_BYTE_SCAN);
    c->gen_planes = c->gm_on && acgt && !(pp->flags & KMER_FLAG_BYTE_SCAN);
    if (c->planes || c->gen_planes) {
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
        // [0,64) P and [64,128) rc(P) (tile kernel, truncated), [128, 128+|P|) full P,
        // [128+|P|, 128+2|P|) full rc(P) (general kernels)
        std::vector<uint8_t> pr(2 * KMAX_TILE + 2 * c->prefix.size(), 0);
        memcpy(pr.data(), c->prefix.data(), std::min<size_t>(c->prefix.size(), KMAX_TILE));
        memcpy(pr.data() + KMAX_TILE, c->rprefix.data(), std::min<size_t>(c->rprefix.size(), KMAX_TILE));
        memcpy(pr.data() + 2 * KMAX_TILE, c->prefix.data(), c->prefix.size());
        memcpy(pr.data() + 2 * KMAX_TILE + c->prefix.size(), c->rprefix.data(), c->rprefix.size());
        ok &= dalloc(&c->d_PR, pr.size()) == hipSuccess;
        if (ok) ok &= hipMemcpy(c->d_PR, pr.data(), pr.size(), hipMemcpyHostToDevice) == hipSuccess;
    }
    ok &= dalloc(&c->d_ticket, 4) == hipSuccess;
    ok &= dalloc(&c->d_bticket, 1) == hipSuccess;
    if (ok) ok &= hipMemset(c->d_bticket, 0, sizeof(unsigned int)) == hipSuccess;
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
    for (hipEvent_t &e : c->fa_ev) ok &= hipEventCreate(&e) == hipSuccess;
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
                    &c->xkey, &c->xkey2, &c->ukey, &c->first, &c->cnt_out})
        b->release();
    for (auto *b : {&c->ridx, &c->ridx2, &c->ecnt, &c->bbase, &c->xslot, &c->rkey32, &c->rkey32b, &c->bH, &c->bHs}) b->release();
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
    c->gcand.release();
    c->cpcnt.release();
    c->cpoff.release();
    c->lines.release();
    c->rec_keys.release();
    c->tmp.release();
    c->batch.release();
    for (auto *b : {&c->tb1, &c->tb2, &c->tHs, &c->tstart, &c->tp1, &c->tpb, &c->tsend}) b->release();
    c->tspc.release();
    c->tseg.release();
    c->tpc.release();
    c->tpieces.release();
    c->tH.release();
    c->tnd.release();
    c->epre.release();
    c->tunits.release();
    c->tbig.release();
    c->tstats.release();
    c->tleft.release();
    c->trecv.release();
    c->gm_keys.release();
    c->gm_keys2.release();
    for (auto *b : {&c->gm_cnt, &c->gm_cnt2, &c->gm_first, &c->gm_first2, &c->gm_h1, &c->gm_h2, &c->gm_h1b, &c->gm_h2b})
        b->release();
    for (auto *b : {&c->gm_idx, &c->gm_idx2, &c->gm_head, &c->gm_gid, &c->gm_start}) b->release();
    c->gm_flag.release();
    dfree(c->d_ticket); dfree(c->d_bticket); dfree(c->d_scal); dfree(c->d_pos); dfree(c->d_pos_saved);
    dfree(c->d_P); dfree(c->d_PR);
    if (c->h_small) (void)hipHostFree(c->h_small);
    if (c->h_tail) (void)hipHostFree(c->h_tail);
    for (hipStream_t us : c->up_streams) (void)hipStreamSynchronize(us);
    if (c->up_p) (void)hipHostFree(c->up_p);
    for (hipEvent_t e : {c->ev0, c->ev1, c->ev2, c->ev3, c->ev4, c->evw})
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->tev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->fa_ev)
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
    // (narrow keys: the 32-bit pass-1 keys go out widened to h, the receiving
    // side's table_finish reads 64-bit keys)
    const bool narrow = c->p.k <= TAB_NARROW_K;
    if (nch == 1 && c->t_cbase[0] == 0 && !narrow) {
        *d_send = c->tb1.p;
        return KMER_OK;
    }
    std::vector<TabSeg> segs;
    uint64_t dst = 0;
    for (uint32_t p = 0; p < TAB_NB; ++p)
        for (size_t ch = 0; ch < nch; ++ch) {
            const uint64_t a0 = c->t_coff[ch][p], a1 = c->t_coff[ch][p + 1];
            if (a1 > a0) segs.push_back(TabSeg{c->t_cbase[ch] + a0, dst, a1 - a0, p});
            dst += a1 - a0;
        }
    if (segs.size() >= (1ull << 31)) return fail(c, KMER_E_BAD_PARAM, "too many table segments");
    HIPCHK(c, c->tsend.ensure(n, s));
    HIPCHK(c, c->tseg.ensure(segs.size(), s));
    kmer_status st = upload(c, c->tseg.p, segs.data(), segs.size() * sizeof(TabSeg), s);
    if (st) return st;
    if (narrow)
        HIPCHK(c, launch_tab_widen((const uint32_t *)c->tb1.p, c->tseg.p, (uint32_t)segs.size(), c->tsend.p, s));
    else
        HIPCHK(c, launch_tab_segcopy(c->tb1.p, c->tseg.p, (uint32_t)segs.size(), c->tsend.p, s));
    HIPCHK(c, hipStreamSynchronize(s));        // (the caller's collective follows)
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
    if (c->gm_on && c->gm_n) {              // (general-path entries held on the device travel as records)
        if (hipSetDevice(c->device) != hipSuccess) return KMER_E_DEVICE;
        kmer_status st = general_to_host(c);
        if (st) return st;
    }
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
    const bool narrow = c->p.k <= TAB_NARROW_K;
    HIPCHK(c, launch_tab_digest(c->t_ent, c->tstart.p, c->tnd.p, c->p.k, narrow ? 1u : 0u, d, s));
    uint64_t acc = 0;
    std::vector<TabBig> big(c->t_nbig);
    HIPCHK(c, hipMemcpyAsync(&acc, d, 8, hipMemcpyDeviceToHost, s));
    if (!big.empty())
        HIPCHK(c, hipMemcpyAsync(big.data(), c->tbig.p, big.size() * sizeof(TabBig), hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    for (const TabBig &b : big)   // (entries hold TAB_CMAX)
        acc += (b.count - TAB_CMAX) * tab_digest_mix(tab_digest_key(b.h, c->p.k, narrow));
    *digest = acc;
    return KMER_OK;
}

kmer_status kmer_table_routes(kmer_ctx *c, uint64_t *p1_fixed, uint64_t *p1_merged, uint64_t *p1_counted,
                              uint64_t *p2_fixed) {
    if (!c) return KMER_E_BAD_PARAM;
    uint64_t f = 0, m = 0, n = 0, f2 = 0;
    if (!c->group.empty()) {                         // a group: its children's routes add up
        for (kmer_ctx *x : c->group) {
            if (hipSetDevice(x->device) != hipSuccess) return KMER_E_DEVICE;
            SETTLE(x);
            f += x->t_p1_fixed;
            m += x->t_p1_merged;
            n += x->t_p1_counted;
            f2 += x->t_p2_fixed;
        }
    } else {
        SETTLE(c);
        f = c->t_p1_fixed;
        m = c->t_p1_merged;
        n = c->t_p1_counted;
        f2 = c->t_p2_fixed;
    }
    if (p1_fixed) *p1_fixed = f;
    if (p1_merged) *p1_merged = m;
    if (p1_counted) *p1_counted = n;
    if (p2_fixed) *p2_fixed = f2;
    return KMER_OK;
}

kmer_status kmer_phase_times(kmer_ctx *c, uint32_t max, const char **names, double *ms, uint32_t *n) {
    if (!c || !n || (max && (!names || !ms))) return KMER_E_BAD_PARAM;
    SETTLE(c);
    static const char *tab_names[7] = {"lines", "hist1", "scatter1", "hist2", "scatter2", "final", "fasta"};
    static const char *ord_names[3] = {"scan", "feed", "finish"};
    if (c->mode == MODE_TABLE) {
        *n = c->fasta ? 7 : 6;                   // (fasta: the FASTA rewrite of the chunks)
        for (uint32_t i = 0; i < *n && i < max; ++i) {
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
