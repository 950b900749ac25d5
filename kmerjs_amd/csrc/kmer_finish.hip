// kmer_finish.hip — the ordered finish: cross-list placement, key sort / bucket heads,
// emit in first-occurrence (Map) order, host results.
#include "kmer_host.hpp"

namespace kmerhip {

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

// bucket partition + per-bucket LDS tables (keys of <= BKT_LOW + 11 bits):
// histogram per (bucket, block), offsets (one kernel), scatter, tables
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
    HIPCHK(c, c->bbase.ensure(2 * BKT_MAX + 2, s));   // bucket totals [0, nb), starts [BKT_MAX, BKT_MAX + nb]
    uint32_t *btot = c->bbase.p, *bstart = c->bbase.p + BKT_MAX;
    HIPCHK(c, launch_bucket_hist(c->rkey32.p, n, invalid, shift, nb, nblk, c->bH.p, c->hcnt.p, s));
    HIPCHK(c, launch_bucket_offsets(c->bH.p, nb, nblk, c->bHs.p, btot, bstart, c->d_bticket, s));
    HIPCHK(c, launch_bucket_scatter(c->rkey32.p, n, invalid, shift, nb, nblk, c->bHs.p, bstart, c->pkey16.p, c->ridx2.p, s));
    HIPCHK(c, launch_bucket_heads(c->pkey16.p, c->ridx2.p, bstart, nb, shift, c->hcnt.p, s));
    return KMER_OK;
}


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
    const uint64_t nb = (n + CP_BLOCK - 1) / CP_BLOCK;
    // per-workgroup counts -> offsets (+ the total at [nb]) -> valid pairs written in rank order
    HIPCHK(c, c->cpcnt.ensure(nb + 1, s));
    HIPCHK(c, c->cpoff.ensure(nb + 1, s));
    HIPCHK(c, hipMemsetAsync(c->cpcnt.p + nb, 0, sizeof(uint32_t), s));
    const uint32_t *k32 = c->narrow ? c->rkey32.p : nullptr;
    const uint64_t *k64 = c->narrow ? nullptr : c->rkey.p;
    HIPCHK(c, launch_compact_count(k32, k64, n, invalid, c->cpcnt.p, s));
    ROCPRIM_RUN(c, rocprim::exclusive_scan(t, b, c->cpcnt.p, c->cpoff.p, (uint64_t)0, (size_t)nb + 1,
                                           rocprim::plus<uint64_t>(), s));
    HIPCHK(c, hipMemcpyAsync(c->h_small + 20, c->cpoff.p + nb, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    const uint64_t n2 = c->h_small[20];
    if (n2 >= n) return KMER_OK;
    // written into the second buffers, copied back (the session buffers keep their size)
    if (c->narrow) HIPCHK(c, c->rkey32b.ensure(n2 + 1, s));
    else HIPCHK(c, c->rkey2.ensure(n2 + 1, s));
    HIPCHK(c, c->rord2.ensure(n2 + 1, s));
    HIPCHK(c, launch_compact_write(k32, k64, c->rord.p, n, invalid, c->cpoff.p, c->narrow ? c->rkey32b.p : nullptr,
                                   c->narrow ? nullptr : c->rkey2.p, c->rord2.p, s));
    if (c->narrow) HIPCHK(c, hipMemcpyAsync(c->rkey32.p, c->rkey32b.p, n2 * 4, hipMemcpyDeviceToDevice, s));
    else HIPCHK(c, hipMemcpyAsync(c->rkey.p, c->rkey2.p, n2 * 8, hipMemcpyDeviceToDevice, s));
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
// first-occurrence order: the keys grouped (bucket tables or a radix sort of
// (key, rank)); group heads flag their rank with the count; the emit kernel
// gives each flagged rank its output position (heads before it).
// partial: (code, {first, count}) into ukey/uval; else decoded keys, counts
// and firsts into keys_out / cnt_out / first.  Returns the unique count.
// sync = false: the unique count is copied back asynchronously (resolve_out).
kmer_status rank_finish(kmer_ctx *c, uint64_t n, bool partial, bool with_counts, uint64_t *nu_out, bool sync) {
    hipStream_t s = c->stream;
    *nu_out = 0;
    if (n == 0) return KMER_OK;
    if (c->narrow) HIPCHK(c, c->rkey32b.ensure(n, s));
    else HIPCHK(c, c->rkey2.ensure(n, s));
    HIPCHK(c, c->ridx2.ensure(n, s));
    if (with_counts) HIPCHK(c, c->hrec.ensure(n, s));
    HIPCHK(c, c->hcnt.ensure(n + 4, s));
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
    // heads per emit workgroup; their prefixes (summed in the emit kernel, or
    // scanned here when there are many workgroups)
    const uint64_t nbe = emit_blocks(n);
    HIPCHK(c, c->ecnt.ensure(nbe, s));
    HIPCHK(c, launch_head_count(c->hcnt.p, n, c->ecnt.p, s));
    EmitArgs e;
    memset(&e, 0, sizeof(e));
    e.ecnt = c->ecnt.p;
    if (nbe > EMIT_DIRECT_MAX) {
        HIPCHK(c, c->epre.ensure(nbe, s));
        ROCPRIM_RUN(c, rocprim::exclusive_scan(t, b, c->ecnt.p, c->epre.p, (uint64_t)0, (size_t)nbe,
                                               rocprim::plus<uint64_t>(), s));
        e.epre = c->epre.p;
    }
    e.hcnt = c->hcnt.p;
    e.hrec = with_counts ? c->hrec.p : nullptr;
    e.rkey32 = c->narrow ? c->rkey32.p : nullptr;
    e.rkey64 = c->narrow ? nullptr : c->rkey.p;
    e.rkeyh = c->wide ? c->rkeyh.p : nullptr;
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

// ---------------------------------------------------------------------------
// general path, device merge (step 1): k > 64, unprefixed k > 31, any prefix
// bytes -- no host merge of the records (lib/kmers.js:88-100 has no k limit)
// ---------------------------------------------------------------------------
constexpr uint64_t GM_MERGE_AT = 1ull << 25;   // entries held before an intermediate merge

// a chunk's records (c->recs) -> session entries (key bytes, count 1, first)
kmer_status general_append(kmer_ctx *c, const uint8_t *d, uint64_t nrec, hipStream_t s) {
    const uint64_t k = c->p.k;
    // (an intermediate merge when the entries reach twice the last merge's
    // output: distinct-heavy inputs are not re-sorted once per 2^25 entries)
    if (c->gm_n && c->gm_n + nrec > std::max<uint64_t>(GM_MERGE_AT, 2 * c->gm_last)) {
        kmer_status st = general_merge(c);
        if (st) return st;
    }
    const uint64_t n = c->gm_n + nrec;
    HIPCHK(c, c->gm_keys.ensure(n * k, s, true, c->gm_n * k));
    HIPCHK(c, c->gm_cnt.ensure(n, s, true, c->gm_n));
    HIPCHK(c, c->gm_first.ensure(n, s, true, c->gm_n));
    HIPCHK(c, launch_gen_append(c->recs.p, nrec, d, (uint32_t)k, c->gm_keys.p + c->gm_n * k, c->gm_cnt.p + c->gm_n,
                                c->gm_first.p + c->gm_n, s));
    c->gm_n = n;
    c->gm_merged = false;
    return KMER_OK;
}

// entries -> unique entries: 128-bit hash of the key bytes, stable LSD radix
// sort by (h1, h2), groups where the hash changes (neighbours with equal
// hashes compared byte for byte: a collision redoes the merge with another
// seed), one thread per group sums counts and takes the min first.  The
// entries stay in hash order (general_finish puts them in Map order).
kmer_status general_merge(kmer_ctx *c) {
    if (c->gm_merged || c->gm_n == 0) {
        c->gm_merged = true;
        return KMER_OK;
    }
    hipStream_t s = c->stream;
    const uint64_t n = c->gm_n, k = c->p.k;
    if (n >= 0xFFFFFFFFull) return fail(c, KMER_E_TOO_MANY_KEYS, "more than 2^32 - 1 general-path entries");
    HIPCHK(c, c->gm_h1.ensure(n, s));
    HIPCHK(c, c->gm_h2.ensure(n, s));
    HIPCHK(c, c->gm_h1b.ensure(n, s));
    HIPCHK(c, c->gm_h2b.ensure(n, s));
    HIPCHK(c, c->gm_idx.ensure(n, s));
    HIPCHK(c, c->gm_idx2.ensure(n, s));
    HIPCHK(c, c->gm_head.ensure(n, s));
    HIPCHK(c, c->gm_gid.ensure(n, s));
    HIPCHK(c, c->gm_start.ensure(n + 1, s));
    HIPCHK(c, c->gm_flag.ensure(1, s));
    for (uint64_t attempt = 0; attempt < 4; ++attempt) {
        HIPCHK(c, hipMemsetAsync(c->gm_flag.p, 0, sizeof(unsigned int), s));
        HIPCHK(c, launch_gen_hash(c->gm_keys.p, n, (uint32_t)k, 0x6A09E667F3BCC909ull + attempt, c->gm_h1.p, c->gm_h2.p,
                                  c->gm_idx.p, s));
        // first attempt: one radix sort by h1 (a 64-bit collision between two
        // distinct keys -- p ~ n^2 / 2^65 -- is caught by the byte check and
        // redone); later attempts: the LSD pair (h2, then h1, stable)
        const uint32_t *idx_sorted;
        if (attempt == 0) {
            ROCPRIM_RUN(c, rocprim::radix_sort_pairs(t, b, c->gm_h1.p, c->gm_h1b.p, c->gm_idx.p, c->gm_idx2.p,
                                                     (size_t)n, 0, 64, s));
            HIPCHK(c, launch_gen_heads(c->gm_h1b.p, c->gm_h1b.p, c->gm_idx2.p, n, c->gm_keys.p, (uint32_t)k,
                                       c->gm_head.p, c->gm_flag.p, s));
            idx_sorted = c->gm_idx2.p;
        } else {
            ROCPRIM_RUN(c, rocprim::radix_sort_pairs(t, b, c->gm_h2.p, c->gm_h2b.p, c->gm_idx.p, c->gm_idx2.p,
                                                     (size_t)n, 0, 64, s));
            HIPCHK(c, launch_gather_u64(c->gm_h1.p, c->gm_idx2.p, n, c->gm_h1b.p, s));
            ROCPRIM_RUN(c, rocprim::radix_sort_pairs(t, b, c->gm_h1b.p, c->gm_h1.p, c->gm_idx2.p, c->gm_idx.p,
                                                     (size_t)n, 0, 64, s));
            HIPCHK(c, launch_gather_u64(c->gm_h2.p, c->gm_idx.p, n, c->gm_h2b.p, s));   // (h2 of each sorted entry)
            HIPCHK(c, launch_gen_heads(c->gm_h1.p, c->gm_h2b.p, c->gm_idx.p, n, c->gm_keys.p, (uint32_t)k,
                                       c->gm_head.p, c->gm_flag.p, s));
            idx_sorted = c->gm_idx.p;
        }
        ROCPRIM_RUN(c, rocprim::inclusive_scan(t, b, c->gm_head.p, c->gm_gid.p, (size_t)n, rocprim::plus<uint32_t>(), s));
        uint32_t hv[2] = {0, 0};
        HIPCHK(c, hipMemcpyAsync(&hv[0], c->gm_flag.p, 4, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(&hv[1], c->gm_gid.p + n - 1, 4, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        if (attempt == 0 && (c->p.flags & KMER_FLAG_GEN_COLLIDE_TEST)) hv[0] = 1;   // (debug: force the retry)
        if (hv[0]) continue;                       // a hash collision: another seed
        const uint64_t ng = hv[1];
        HIPCHK(c, c->gm_keys2.ensure(ng * k, s));
        HIPCHK(c, c->gm_cnt2.ensure(ng, s));
        HIPCHK(c, c->gm_first2.ensure(ng, s));
        HIPCHK(c, launch_gen_starts(c->gm_head.p, c->gm_gid.p, n, c->gm_start.p, s));
        HIPCHK(c, launch_gen_reduce(c->gm_start.p, ng, idx_sorted, c->gm_keys.p, c->gm_cnt.p, c->gm_first.p,
                                    (uint32_t)k, c->gm_keys2.p, c->gm_cnt2.p, c->gm_first2.p, s));
        std::swap(c->gm_keys, c->gm_keys2);
        std::swap(c->gm_cnt, c->gm_cnt2);
        std::swap(c->gm_first, c->gm_first2);
        c->gm_n = ng;
        c->gm_last = ng;
        c->gm_merged = true;
        if (c->p.max_keys) {
            // host records of k bytes may also be among the device entries
            // (kmer_records_export / _import): only the other lengths are
            // certainly distinct here; general_finish folds the k-byte ones
            // in first, so its merge counts every key exactly once
            uint64_t other = 0;
            for (const auto &kv : c->exotic) other += kv.first.size() != k;
            if (ng + other > c->p.max_keys)
                return fail(c, KMER_E_TOO_MANY_KEYS, "more distinct keys than max_keys (reference Map limit)");
        }
        return KMER_OK;
    }
    return fail(c, KMER_E_DEVICE, "general-path key hashes kept colliding");
}

// merged entries in first-occurrence (Map) order -> the context's result arrays.
// Host records of k bytes (imported from other ranks, or folded by an earlier
// kmer_records_export) join the entries first, so a key never appears twice.
kmer_status general_finish(kmer_ctx *c) {
    const uint64_t k = c->p.k;
    if (!c->exotic.empty()) {
        std::vector<char> hk;
        std::vector<uint64_t> hc, hf;
        for (auto it = c->exotic.begin(); it != c->exotic.end();) {
            if (it->first.size() != k) {
                ++it;
                continue;
            }
            hk.insert(hk.end(), it->first.begin(), it->first.end());
            hc.push_back(it->second.count);
            hf.push_back(it->second.first);
            it = c->exotic.erase(it);
        }
        const uint64_t m = hc.size(), n0 = c->gm_n;
        if (m) {
            hipStream_t s = c->stream;
            HIPCHK(c, c->gm_keys.ensure((n0 + m) * k, s, true, n0 * k));
            HIPCHK(c, c->gm_cnt.ensure(n0 + m, s, true, n0));
            HIPCHK(c, c->gm_first.ensure(n0 + m, s, true, n0));
            kmer_status st = upload(c, c->gm_keys.p + n0 * k, hk.data(), m * k, s);
            if (!st) st = upload(c, c->gm_cnt.p + n0, hc.data(), m * 8, s);
            if (!st) st = upload(c, c->gm_first.p + n0, hf.data(), m * 8, s);
            if (st) return st;
            c->gm_n = n0 + m;
            c->gm_merged = false;
        }
    }
    kmer_status st = general_merge(c);
    if (st) return st;
    const uint64_t n = c->gm_n;
    c->n_out = n;
    if (n == 0) return KMER_OK;
    hipStream_t s = c->stream;
    HIPCHK(c, c->xord2.ensure(n, s));
    HIPCHK(c, c->ridx2.ensure(n, s));
    HIPCHK(c, c->keys_out.ensure(n * k, s));
    HIPCHK(c, c->cnt_out.ensure(n, s));
    HIPCHK(c, c->first.ensure(n, s));
    rocprim::counting_iterator<uint32_t> iota(0u);
    ROCPRIM_RUN(c, rocprim::radix_sort_pairs(t, b, c->gm_first.p, c->xord2.p, iota, c->ridx2.p, (size_t)n, 0, 64, s));
    HIPCHK(c, launch_permute_rows(c->gm_keys.p, c->gm_cnt.p, c->gm_first.p, c->ridx2.p, n, (uint32_t)k, c->keys_out.p,
                                  c->cnt_out.p, c->first.p, s));
    c->gm_n = 0;
    return KMER_OK;
}

// the session's entries folded into the host record map (kmer_records_export
// before a multi-rank gather: the ranks' general-path keys travel as records)
kmer_status general_to_host(kmer_ctx *c) {
    kmer_status st = general_merge(c);
    if (st) return st;
    const uint64_t n = c->gm_n, k = c->p.k;
    if (n == 0) return KMER_OK;
    std::vector<char> keys(n * k);
    std::vector<uint64_t> cnt(n), fst(n);
    hipStream_t s = c->stream;
    HIPCHK(c, hipMemcpyAsync(keys.data(), c->gm_keys.p, n * k, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(cnt.data(), c->gm_cnt.p, n * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(fst.data(), c->gm_first.p, n * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    for (uint64_t i = 0; i < n; ++i) {
        std::string key(keys.data() + i * k, k);
        auto it = c->exotic.find(key);
        if (it == c->exotic.end()) {
            c->exotic.emplace(std::move(key), Ent{cnt[i], fst[i]});
        } else {
            it->second.count += cnt[i];
            it->second.first = std::min(it->second.first, fst[i]);
        }
    }
    c->gm_n = 0;
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
        if (c->mode == MODE_WINDOWS && !c->prefix.empty() && c->win_slots) {
            st = compact_windows(c);
            if (st) return st;
        }
        st = rank_finish(c, c->n_hits, false, false, &nu, sync);
        if (st) return st;
        c->n_out = nu;
    } else if (c->mode == MODE_TABLE) {
        st = table_finish(c);
        if (st) return st;
    } else if (c->mode == MODE_GENERAL && c->gm_on) {
        st = general_finish(c);
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


}  // namespace kmerhip
