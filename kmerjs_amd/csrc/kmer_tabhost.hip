// kmer_tabhost.hip — table mode orchestration (kernels: kmer_table.hip): pass 1 per chunk,
// pass 2 + final at finish, host results of a table.
#include "kmer_host.hpp"

namespace kmerhip {

// ---------------------------------------------------------------------------
// table mode feed (kernels: kmer_table.hip)
// ---------------------------------------------------------------------------
// Pass 1 of one chunk: its sequence lines, then per workgroup share of lines
// a histogram of keys by partition, a scan, and the scatter into tb1 after
// the session's earlier keys.  Non-ACGT windows go to the host map.
float ev_ms(kmer_ctx *c, hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) ms = 0.f;
    return ms;
}

// The pass-1 scatter of a chunk (records of non-ACGT windows: the attempt is
// redone with a larger record list until it fits), then its records drained.
kmer_status table_scatter1(kmer_ctx *c, TabArgs &a, hipStream_t s, hipError_t (*launch)(const TabArgs &, hipStream_t)) {
    for (int attempt = 0;; ++attempt) {
        a.recs = c->recs.p;
        a.rec_count = c->d_rec_count;
        a.rec_cap = c->recs.cap;
        HIPCHK(c, hipMemsetAsync(c->d_rec_count, 0, 8, s));
        if (attempt && a.pcur) HIPCHK(c, hipMemsetAsync(a.pcur, 0, (TAB_NB + 1) * 8, s));   // (a redo: the spill areas again)
        HIPCHK(c, hipEventRecord(c->tev[2], s));
        HIPCHK(c, launch(a, s));
        HIPCHK(c, hipEventRecord(c->tev[3], s));
        HIPCHK(c, hipMemcpyAsync(c->h_small, c->d_scal, 8 * 8, hipMemcpyDeviceToHost, s));
        if (a.pcur)                                  // (fixed runs: the spill overflow count, same wait)
            HIPCHK(c, hipMemcpyAsync(c->h_small + 17, a.pcur + TAB_NB, 8, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        const float ms_s1 = ev_ms(c, c->tev[2], c->tev[3]);
        const uint32_t e = (uint32_t)c->h_small[5];
        kmer_status st = check_err(c, e);
        if (st) return st;
        if (!(e & ERR_REC_OVERFLOW)) {         // (a redo rewrites the same key ranges)
            c->t_ms[2] += ms_s1;
            break;
        }
        if (attempt == 7) return fail(c, KMER_E_OOM, "record list kept overflowing");
        HIPCHK(c, hipMemsetAsync(c->d_err, 0, 4, s));
        st = ensure_records(c, c->h_small[0] + 1024);
        if (st) return st;
    }
    return KMER_OK;
}

kmer_status table_pass1_counted(kmer_ctx *c, TabArgs &a, hipStream_t s) {
    const uint64_t nh = (uint64_t)TAB_NB * a.nwg;
    a.H1 = c->tH.p;
    HIPCHK(c, launch_tab_hist1(a, s));
    ROCPRIM_RUN(c, rocprim::exclusive_scan(t, b, c->tH.p, c->tHs.p, (uint64_t)0, (size_t)nh,
                                           rocprim::plus<uint64_t>(), s));
    HIPCHK(c, launch_tab_p1_offsets(c->tHs.p, a.nwg, c->tp1.p, s));
    std::vector<uint64_t> off(TAB_NB + 1);
    HIPCHK(c, hipMemcpyAsync(off.data(), c->tp1.p, TAB_NB * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(c->h_small + 14, c->tHs.p + nh - 1, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(c->h_small + 15, c->tH.p + nh - 1, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipEventRecord(c->tev[2], s));
    HIPCHK(c, hipStreamSynchronize(s));
    c->t_ms[0] += ev_ms(c, c->tev[0], c->tev[1]);
    c->t_ms[1] += ev_ms(c, c->tev[1], c->tev[2]);
    const uint64_t n_c = c->h_small[14] + (uint32_t)c->h_small[15];
    off[TAB_NB] = n_c;
    HIPCHK(c, c->tb1.ensure(c->t_keys + n_c, s, true, c->t_keys));
    a.H1s = c->tHs.p;
    a.base = c->t_keys;
    a.B1 = c->tb1.p;
    kmer_status st = table_scatter1(c, a, s, launch_tab_scatter1);
    if (st) return st;
    c->t_cbase.push_back(c->t_keys);
    c->t_coff.push_back(std::move(off));
    c->t_keys += n_c;
    c->t_p1_counted += 1;
    return KMER_OK;
}

// Pass 1 with fixed runs (tab_scatter1f): workgroup w's run in partition p
// holds its mean share of keys + 2 standard deviations + 4, rounded up to 8 (a
// hash partition's count is ~Poisson; at C3 ~5 % of the slots are filler, ~2 %
// of the runs spill a few keys), sized from the workgroups' window counts.
// Each partition's runs are followed by a spill area of S = R / 64 slots
// (>= 256), so the chunk's partition p is one contiguous range [p PS,
// (p + 1) PS) for pass 2, its unused slots TAB_SENT.  *done false: the runs
// would be more than 1/12 filler (small shares), or a spill area overflowed
// (crowded partitions: repeated k-mers); nothing of the chunk is kept and the
// caller runs the counted pass.
kmer_status table_pass1_fixed(kmer_ctx *c, TabArgs &a, hipStream_t s, bool *done) {
    *done = false;
    uint64_t *W = c->tHs.p, *pcw = c->tHs.p + a.nwg;
    HIPCHK(c, launch_tab_wg_windows(a.lines, a.n_lines, a.lpw, a.k, a.nwg, W, s));
    std::vector<uint64_t> hw(a.nwg), hp(a.nwg + 1);
    HIPCHK(c, hipMemcpyAsync(hw.data(), W, a.nwg * 8ull, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipEventRecord(c->tev[2], s));
    HIPCHK(c, hipStreamSynchronize(s));
    const float ms0 = ev_ms(c, c->tev[0], c->tev[1]), ms1 = ev_ms(c, c->tev[1], c->tev[2]);
    uint64_t tot = 0;
    hp[0] = 0;
    double sig = 2.0;                          // (KMERHIP_TAB_SIGMA: A/B experiments)
    if (const char *e = exp_env("KMERHIP_TAB_SIGMA")) sig = atof(e);
    uint64_t sdiv = 64;                        // spill area: R / sdiv slots (KMERHIP_TAB_SPILLDIV: A/B experiments)
    if (const char *e = exp_env("KMERHIP_TAB_SPILLDIV")) sdiv = std::max<uint64_t>(1, strtoull(e, nullptr, 10));
    for (uint32_t w = 0; w < a.nwg; ++w) tot += hw[w];
    // (runs of whole 64-B blocks: 8 keys, narrow keys 16)
    const uint64_t al = a.narrow ? 16 : 8;
    auto sized = [&](const std::vector<uint64_t> &ww, uint32_t nwg) {
        hp.assign(nwg + 1, 0);
        for (uint32_t w = 0; w < nwg; ++w) {
            const double mu = (double)ww[w] / TAB_NB;
            hp[w + 1] = hp[w] + (ww[w] ? ((uint64_t)(mu + sig * std::sqrt(mu)) + 4 + al - 1) & ~(al - 1) : 0);
        }
        const uint64_t R = hp[nwg];
        return (uint64_t)TAB_NB * (R + ((std::max<uint64_t>(256, R / sdiv) + al - 1) & ~(al - 1)));
    };
    uint64_t region = sized(hw, a.nwg);
    // small shares (C5's 1 GB of contigs cut into 4,096-window pieces: ~60
    // keys per run) are mostly filler: merge the workgroups' shares in groups
    // of 2, 4, ... (the sums of the window counts already measured -- share w'
    // is shares w' f .. w' f + f - 1) while at least one workgroup per CU
    // remains, until the filler is at most 1/12 of the keys (C5: down to one
    // per CU beat two per CU by ~1 %, A/B: less filler through pass 2)
    const uint32_t min_wg = (uint32_t)std::max(c->n_cu, 1);
    bool merged = false;
    while (region > tot + tot / 12 && a.nwg >= 2 * min_wg && !(c->p.flags & KMER_FLAG_TABLE_FIXED_TEST)) {
        const uint32_t nwg2 = (a.nwg + 1) / 2;
        std::vector<uint64_t> h2(nwg2, 0);
        for (uint32_t w = 0; w < a.nwg; ++w) h2[w / 2] += hw[w];
        hw.swap(h2);
        a.nwg = nwg2;
        a.lpw *= 2;
        region = sized(hw, a.nwg);
        merged = true;
    }
    // (still more than 1/8 filler: the counting pass moves fewer bytes through
    // pass 2 -- filler costs ~3 x 8 B per slot, the counting pass one more
    // formation of every window)
    if (region > tot + tot / 8 && !(c->p.flags & KMER_FLAG_TABLE_FIXED_TEST)) return KMER_OK;
    const uint64_t R = hp[a.nwg];
    const uint64_t S = (std::max<uint64_t>(256, R / sdiv) + al - 1) & ~(al - 1), PS = R + S;
    const uint64_t cb = (c->t_keys + al - 1) & ~(al - 1);   // (runs of whole blocks start at 64-B boundaries)
    HIPCHK(c, c->tb1.ensure(cb + region, s, true, c->t_keys));
    HIPCHK(c, c->tspc.ensure(TAB_NB + 1, s));
    kmer_status st = upload(c, pcw, hp.data(), hp.size() * 8, s);
    if (st) return st;
    a.pcw = pcw;
    a.R = R;
    a.S = S;
    a.PS = PS;
    a.base = cb;
    a.B1 = c->tb1.p;
    a.pcur = c->tspc.p;
    HIPCHK(c, hipMemsetAsync(c->tspc.p, 0, (TAB_NB + 1) * 8, s));
    st = table_scatter1(c, a, s, launch_tab_scatter1f);
    if (st) return st;
    const unsigned long long over = c->h_small[17];   // (read with table_scatter1's wait)
    if (over) {                                // (records of the attempt are dropped: the counted pass redoes them)
        if (exp_env("KMERHIP_TAB_SPILL_LOG")) fprintf(stderr, "tab pass 1: spill area overflow (%llu)\n", over);
        return KMER_OK;
    }
    HIPCHK(c, launch_tab_spill_fill(a.narrow != 0, c->tb1.p, cb, R, S, PS, c->tspc.p, s));
    std::vector<uint64_t> off(TAB_NB + 1);
    for (uint32_t p = 0; p <= TAB_NB; ++p) off[p] = (uint64_t)p * PS;
    c->t_cbase.push_back(cb);
    c->t_coff.push_back(std::move(off));
    c->t_keys = cb + region;
    c->t_fill += region - std::min<uint64_t>(region, tot);
    if (exp_env("KMERHIP_TAB_SPILL_LOG"))
        fprintf(stderr, "tab pass 1: %llu keys, %llu slots (spill areas of %llu)\n", (unsigned long long)tot,
                (unsigned long long)region, (unsigned long long)S);
    c->t_ms[0] += ms0;
    c->t_ms[1] += ms1;
    c->t_p1_fixed += 1;
    c->t_p1_merged += merged ? 1 : 0;
    *done = true;
    return KMER_OK;
}

kmer_status table_feed(kmer_ctx *c, const uint8_t *d, uint64_t len, uint32_t n_tiles, hipStream_t s) {
    const uint64_t li0 = c->host_lines;
    HIPCHK(c, hipEventRecord(c->ev0, s));
    HIPCHK(c, hipEventRecord(c->tev[0], s));
    uint64_t n_nl = 0, n_seq = 0;
    kmer_status st = chunk_lines(c, d, len, n_tiles, s, false, &n_nl, &n_seq);
    if (st) return st;
    HIPCHK(c, launch_pos_after(c->d_pos, li0 + n_nl, d, len, c->d_ends_open, s));
    c->host_lines = li0 + n_nl;
    // long lines -> pieces of <= TAB_PIECE windows (balance pass 1's shares)
    const SeqLine *plines = c->lines.p;
    uint64_t n_items = n_seq;
    if (n_seq) {
        HIPCHK(c, c->tpc.ensure(n_seq + 1, s));
        HIPCHK(c, c->tpb.ensure(n_seq, s));
        uint32_t *split = c->tpc.p + n_seq;             // set when a line is not exactly one piece
        HIPCHK(c, hipMemsetAsync(split, 0, 4, s));
        HIPCHK(c, launch_tab_piece_count(c->wcount.p, n_seq, c->tpc.p, split, s));
        HIPCHK(c, hipMemcpyAsync(c->h_small + 16, split, 4, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        uint64_t n_pieces = n_seq;                // (no split: one piece per line)
        if ((uint32_t)c->h_small[16]) {
            ROCPRIM_RUN(c, rocprim::exclusive_scan(t, b, c->tpc.p, c->tpb.p, (uint64_t)0, (size_t)n_seq,
                                                   rocprim::plus<uint64_t>(), s));
            HIPCHK(c, hipMemcpyAsync(c->h_small + 12, c->tpb.p + n_seq - 1, 8, hipMemcpyDeviceToHost, s));
            HIPCHK(c, hipMemcpyAsync(c->h_small + 13, c->tpc.p + n_seq - 1, 4, hipMemcpyDeviceToHost, s));
            HIPCHK(c, hipStreamSynchronize(s));
            n_pieces = c->h_small[12] + (uint32_t)c->h_small[13];
        }
        if (n_pieces == 0) {
            n_items = 0;                          // no line holds a window
        } else if ((uint32_t)c->h_small[16]) {    // long lines (or empty ones, dropped on the way)
            HIPCHK(c, c->tpieces.ensure(std::max<uint64_t>(n_pieces, 1), s));
            HIPCHK(c, launch_tab_piece_write(c->lines.p, c->wcount.p, c->tpb.p, n_seq, c->p.k, c->tpieces.p, s));
            plines = c->tpieces.p;
            n_items = n_pieces;
        }
    }
    HIPCHK(c, hipEventRecord(c->tev[1], s));
    if (n_items) {
        TabArgs a;
        memset(&a, 0, sizeof(a));
        a.data = d;
        a.len = len;
        a.lines = plines;
        a.n_lines = n_items;
        const uint64_t nwg0 = std::min<uint64_t>(8192, (n_items + 63) / 64);
        a.lpw = (n_items + nwg0 - 1) / nwg0;
        a.nwg = (uint32_t)((n_items + a.lpw - 1) / a.lpw);
        a.k = c->p.k;
        for (size_t i = 0; i < c->prefix.size(); ++i) {
            const uint8_t ch = (uint8_t)c->prefix[i];
            a.plo |= ((((uint32_t)ch >> 1) ^ ((uint32_t)ch >> 2)) & 1u) << i;
            a.phi |= (((uint32_t)ch >> 2) & 1u) << i;
        }
        a.pmask = c->prefix.size() >= 32 ? ~0u : ((1u << c->prefix.size()) - 1u);
        a.canonical = (c->p.flags & KMER_FLAG_CANONICAL) ? 1u : 0u;
        a.narrow = c->p.k <= TAB_NARROW_K ? 1u : 0u;
        if (const char *hx = exp_env("KMERHIP_TAB_HASH"))   // (A/B experiments: shift = no mix, results wrong)
            if (a.narrow && strcmp(hx, "shift") == 0) a.narrow = 2;
        a.err = c->d_err;
        const uint64_t nh = (uint64_t)TAB_NB * a.nwg;
        HIPCHK(c, c->tH.ensure(nh, s));
        HIPCHK(c, c->tHs.ensure(nh, s));
        HIPCHK(c, c->tp1.ensure(TAB_NB, s));
        // no prefix and k <= 31: pass 1 without the counting pass (fixed runs,
        // tab_scatter1f); an overfull spill list falls back to the counted pass
        // (KMERHIP_TAB_P1=count: always counted, A/B experiments)
        const char *p1 = exp_env("KMERHIP_TAB_P1");
        bool done = false;
        if (a.pmask == 0 && a.k <= 31 && !(p1 && strcmp(p1, "count") == 0)) {
            st = table_pass1_fixed(c, a, s, &done);
            if (st) return st;
        }
        if (!done) {
            st = table_pass1_counted(c, a, s);
            if (st) return st;
        }
        const uint64_t nrec = c->h_small[0];
        if (nrec) {
            st = drain_records(c, d, nrec, s);
            if (st) return st;
        }
    }
    HIPCHK(c, hipEventRecord(c->ev1, s));
    HIPCHK(c, hipMemcpyAsync(c->h_small, c->d_scal, 8 * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    float ms = 0.f;
    HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
    c->scan_ms += ms;
    c->feed_ms += ms;
    c->chunk_open = c->h_small[7] != 0;
    c->abs_offset += len;
    return KMER_OK;
}


// Pass 2 + final of the session: pass-1 partitions (one run per chunk) are
// cut into units; each unit's keys go to their 2^20 buckets in tb2; the
// final kernel merges each bucket in LDS and writes its entries into tb1.
// B1: the pass-1 keys (default: this session's, tb1); [qlo, qhi): the buckets
// present (multi-GPU: this rank's partitions; the others are left empty).
kmer_status table_finish(kmer_ctx *c, const uint64_t *B1, uint32_t qlo, uint32_t qhi) {
    // this session's own pass-1 keys (B1 null) are 32 bits for narrow keys;
    // received ones (exchanged) are 64-bit h
    const bool b1n = !B1 && c->p.k <= TAB_NARROW_K;
    hipStream_t s = c->stream;
    c->t_canon = c->t_nkeys = c->t_sum = c->t_nbig = 0;
    c->t_done = true;
    const uint64_t n = c->t_keys;
    if (n == 0) return KMER_OK;
    // the table is written over the pass-1 keys (dead after pass 2)
    if (!B1) B1 = c->tb1.p;
    c->t_ent = const_cast<uint64_t *>(B1);
    std::vector<TabUnit> units;
    std::vector<TabUnit> heads(TAB_NB);
    std::vector<uint32_t> ufirst(TAB_NB);
    uint64_t ubase = 0;
    // a partition's run in a chunk is cut into ceil(len / cap) units of equal
    // length (KMERHIP_TAB_UNIT: the cap, A/B experiments)
    uint64_t ucap = TAB_UNIT;
    if (const char *e = exp_env("KMERHIP_TAB_UNIT")) ucap = std::max<uint64_t>(8192, strtoull(e, nullptr, 10));
    for (uint32_t p = 0; p < TAB_NB; ++p) {
        const size_t first = units.size();
        for (size_t ch = 0; ch < c->t_cbase.size(); ++ch) {
            const uint64_t a0 = c->t_coff[ch][p], a1 = c->t_coff[ch][p + 1];
            if (a1 <= a0) continue;
            const uint64_t nu = (a1 - a0 + ucap - 1) / ucap, ul = (a1 - a0 + nu - 1) / nu;
            for (uint64_t o = a0; o < a1; o += ul) {
                TabUnit u{};
                u.start = c->t_cbase[ch] + o;
                u.len = (uint32_t)std::min<uint64_t>(ul, a1 - o);
                u.part = p;
                units.push_back(u);
            }
        }
        if (units.size() == first) units.push_back(TabUnit{});   // empty partition: zero histogram row
        const uint32_t nun = (uint32_t)(units.size() - first);
        for (size_t i = first; i < units.size(); ++i) {
            units[i].u = (uint32_t)(i - first);
            units[i].nunits = nun;
            units[i].hbase = ubase * TAB_NB;
        }
        heads[p] = units[first];
        ufirst[p] = (uint32_t)first;
        ubase += nun;
    }
    const uint64_t n_units = units.size();
    if (n_units >= (1ull << 31)) return fail(c, KMER_E_BAD_PARAM, "too many table units");
    units.insert(units.end(), heads.begin(), heads.end());
    HIPCHK(c, c->tunits.ensure(units.size(), s));
    kmer_status st = upload(c, c->tunits.p, units.data(), units.size() * sizeof(TabUnit), s);
    if (st) return st;
    const uint64_t nh = n_units * TAB_NB;
    HIPCHK(c, c->tH.ensure(nh, s));
    HIPCHK(c, c->tHs.ensure(nh, s));
    HIPCHK(c, c->tstart.ensure(TAB_NQ + 1, s));
    HIPCHK(c, c->tnd.ensure(TAB_NQ, s));
    HIPCHK(c, c->tbig.ensure(1 << 16, s));
    HIPCHK(c, c->tstats.ensure(5, s));
    // Pass 2 with fixed capacities (tab_scatter2f, no histogram pass): a
    // REGION of qg consecutive buckets of a partition holds mean + 6 sigma +
    // 16 slots (a count near its mean).  Large buckets (mean >= 2,048: C3's
    // ~11.4 K, the sort final's one-bucket units) get a region each; small
    // ones (C5: ~480 keys) share one, as many as keep its capacity within a
    // sort-final group (TS_CAPG keys: C5 11 buckets).  Else (small tables,
    // < 2^24 keys) or after a capacity overflow, the counted route:
    // tab_hist2, a scan, tab_scatter2c, bucket starts.
    // KMER_FLAG_TABLE_FIXED_TEST: from any table size.  (KMERHIP_TAB_P2=count:
    // always counted, A/B experiments.)
    const uint64_t n_est = n - std::min(n, c->t_fill);             // keys (filler slots excluded; an upper bound)
    const double mu = (double)n_est / TAB_NQ;
    const char *p2 = exp_env("KMERHIP_TAB_P2");
    // Narrow keys (k <= 21, tab_mix_n): B2 holds 32-bit keys, and the sort
    // final takes a region of up to TAB_SORT_KEYS of them (C5: 24 buckets).
    const bool narrow = c->p.k <= TAB_NARROW_K;
    const uint64_t al = narrow ? 16 : 8;            // (64-B blocks of keys)
    auto cap6 = [&](double m) { return ((uint64_t)(m + 6.0 * std::sqrt(m)) + 16 + al - 1) & ~(al - 1); };
    const bool sort_ok = !exp_env("KMERHIP_TAB_FINAL") && !exp_env("KMERHIP_TAB_PROF");   // (general final alone: qg 1)
    uint32_t qg = 0;
    if (mu >= 2048.0 && !narrow) {
        qg = 1;
    } else {
        const uint64_t lim = narrow ? TAB_SORT_KEYS_BIG : TAB_SORT_GROUP_KEYS;
        for (uint32_t g = sort_ok ? 64 : 1; g >= 1 && !qg; --g)
            if (cap6(g * mu) <= lim && (g >= 2 || narrow)) qg = g;
    }
    // (a crowded region sets ERR_TAB_CAP: the finals then do nothing, and the
    // check after them -- no wait between the passes -- redoes pass 2 and the
    // finals on the counted route)
    const uint64_t *B1w = nullptr;                 // (narrow pass-1 keys widened for the counted route)
    for (bool try_fixed = true;; try_fixed = false) {
    uint64_t capq = 0;
    uint32_t rpp = TAB_NB, gmag = 1u << 20;
    if (try_fixed && qg && (n_est >= (1ull << 24) || (c->p.flags & KMER_FLAG_TABLE_FIXED_TEST)) &&
        !(c->p.flags & KMER_FLAG_TABLE_SPLIT_TEST) && !(p2 && strcmp(p2, "count") == 0) &&
        (qlo & (TAB_NB - 1)) == 0 && (qhi & (TAB_NB - 1)) == 0) {
        capq = cap6(qg * mu);
        rpp = (TAB_NB + qg - 1) / qg;
        gmag = ((1u << 20) + qg - 1) / qg;
        for (uint32_t b = 0; b < TAB_NB; ++b)      // (the region map is exact)
            if (tab_region(b, rpp, gmag) != b / qg) return fail(c, KMER_E_DEVICE, "table region map");
        const uint64_t nr = (uint64_t)TAB_NB * rpp;
        HIPCHK(c, c->tb2.ensure(narrow ? nr * capq / 2 : nr * capq, s));
        HIPCHK(c, c->tH.ensure(nr + 1, s));
        HIPCHK(c, c->tHs.ensure(TAB_NB / 2 + nr + 1, s));   // ufirst (u32), then the region starts
        st = upload(c, c->tHs.p, ufirst.data(), TAB_NB * sizeof(uint32_t), s);
        if (st) return st;
        uint32_t *blen = c->tH.p;
        HIPCHK(c, hipMemsetAsync(blen, 0, (nr + 1) * sizeof(uint32_t), s));
        HIPCHK(c, hipEventRecord(c->tev[4], s));
        HIPCHK(c, hipEventRecord(c->tev[5], s));
        HIPCHK(c, launch_tab_scatter2f(B1, c->tunits.p, (const uint32_t *)c->tHs.p, qlo >> TAB_L2,
                                       (qhi - qlo) >> TAB_L2, capq, rpp, gmag, narrow, b1n, c->tb2.p, blen, c->d_err,
                                       s));
        HIPCHK(c, hipEventRecord(c->tev[6], s));
        // entries go out compactly: region starts = the scan of the regions'
        // key counts (one bucket per region: the bucket starts themselves)
        uint64_t *rst = qg == 1 ? c->tstart.p : c->tHs.p + TAB_NB / 2;
        ROCPRIM_RUN(c, rocprim::exclusive_scan(t, b, blen, rst, (uint64_t)0, (size_t)(nr + 1),
                                               rocprim::plus<uint64_t>(), s));
        if (qg > 1) HIPCHK(c, launch_tab_region_starts(rst, rpp, gmag, c->tstart.p, s));
    }
    if (!capq) {
        if (b1n && !B1w) {
            // the counted route reads 64-bit keys: widen the 32-bit pass-1
            // keys once (h rebuilt from each unit's partition), the table then
            // goes over the widened copy
            std::vector<TabSeg> segs;
            for (uint64_t i = 0; i < n_units; ++i)
                if (units[i].len) segs.push_back(TabSeg{units[i].start, units[i].start, units[i].len, units[i].part});
            HIPCHK(c, c->tsend.ensure(n, s));
            HIPCHK(c, c->tseg.ensure(std::max<size_t>(segs.size(), 1), s));
            st = upload(c, c->tseg.p, segs.data(), segs.size() * sizeof(TabSeg), s);
            if (st) return st;
            HIPCHK(c, launch_tab_widen((const uint32_t *)B1, c->tseg.p, (uint32_t)segs.size(), c->tsend.p, s));
            B1w = c->tsend.p;
        }
        const uint64_t *B1c = b1n ? B1w : B1;
        c->t_ent = const_cast<uint64_t *>(B1c);
        HIPCHK(c, c->tb2.ensure(n, s));
        HIPCHK(c, hipEventRecord(c->tev[4], s));
        HIPCHK(c, launch_tab_hist2(B1c, c->tunits.p, (uint32_t)n_units, c->tH.p, s));
        ROCPRIM_RUN(c, rocprim::exclusive_scan(t, b, c->tH.p, c->tHs.p, (uint64_t)0, (size_t)nh,
                                               rocprim::plus<uint64_t>(), s));
        HIPCHK(c, hipEventRecord(c->tev[5], s));
        HIPCHK(c, launch_tab_scatter2(B1c, c->tunits.p, (uint32_t)n_units, c->tHs.p, c->tb2.p, s));
        HIPCHK(c, hipEventRecord(c->tev[6], s));
        HIPCHK(c, launch_tab_starts(c->tHs.p, c->tH.p, nh, c->tunits.p + n_units, c->tstart.p, s));
    }
    HIPCHK(c, hipMemsetAsync(c->tstats.p, 0, 4 * sizeof(unsigned long long), s));
    TabFinal f;
    memset(&f, 0, sizeof(f));
    f.B2 = c->tb2.p;
    f.start = c->tstart.p;
    f.capq = capq;
    f.inlen = capq ? c->tH.p : nullptr;
    f.qg = capq ? qg : 1;
    f.rpp = rpp;
    f.gmag = gmag;
    f.rstart = capq ? (qg == 1 ? c->tstart.p : c->tHs.p + TAB_NB / 2) : nullptr;
    f.wstart = c->tstart.p;
    f.out = c->t_ent;
    f.nd = c->tnd.p;
    const uint64_t mean = (n - std::min(n, c->t_fill)) / TAB_NQ;   // (keys, not filler slots)
    uint64_t range_keys = 3000;               // mean keys per LDS range (load ~0.37: short probes; measured best at C3)
    if (const char *rk = exp_env("KMERHIP_TAB_RANGE")) range_keys = std::max<uint64_t>(64, strtoull(rk, nullptr, 10));
    while (f.sub_bits < 16 && (mean >> f.sub_bits) > range_keys) ++f.sub_bits;
    f.range_keys = (uint32_t)std::min<uint64_t>(range_keys, TAB_CAP);
    f.cap = (c->p.flags & KMER_FLAG_TABLE_SPLIT_TEST) ? 64 : TAB_CAP;
    if (const char *ab = exp_env("KMERHIP_TAB_ABLATE")) f.ablate = (uint32_t)atoi(ab);   // experiments only
    f.big = c->tbig.p;
    f.big_count = c->tstats.p + 3;
    f.big_cap = c->tbig.cap;
    f.err = c->d_err;
    f.k = c->p.k;
    for (size_t i = 0; i < c->prefix.size(); ++i) {
        const uint8_t ch = (uint8_t)c->prefix[i];
        f.plo |= ((((uint32_t)ch >> 1) ^ ((uint32_t)ch >> 2)) & 1u) << i;
        f.phi |= (((uint32_t)ch >> 2) & 1u) << i;
    }
    f.pmask = c->prefix.size() >= 32 ? ~0u : ((1u << c->prefix.size()) - 1u);
    f.inv = TAB_INV;
    f.narrow = narrow ? 1u : 0u;
    f.b2n = narrow && capq ? 1u : 0u;
    f.canonical = (c->p.flags & KMER_FLAG_CANONICAL) ? 1u : 0u;
    f.stats = c->tstats.p;
    f.qlo = qlo;
    f.qhi = qhi;
    if (qlo != 0 || qhi != TAB_NQ) HIPCHK(c, hipMemsetAsync(c->tnd.p, 0, TAB_NQ * sizeof(uint32_t), s));
    const uint32_t fgrid = (uint32_t)std::max(c->n_cu, 1);
    std::vector<uint64_t> hprof;
#ifdef TAB_PROF
    if (exp_env("KMERHIP_TAB_PROF")) {         // experiments (-DTAB_PROF build): per-phase clocks of the final kernel
#else
    if (false) {
#endif
        HIPCHK(c, hipMalloc((void **)&f.prof, fgrid * 64ull));
        HIPCHK(c, hipMemsetAsync(f.prof, 0, fgrid * 64ull, s));
        hprof.resize(fgrid * 8ull);
    }
    // the sort kernel (two workgroups per CU) takes every unit it can; the
    // general kernel (hash path, range splits) takes the ones it leaves
    // (crowded buckets, many copies of a key).  KMERHIP_TAB_FINAL=general: the
    // general kernel alone (A/B experiments).
    const char *fk = exp_env("KMERHIP_TAB_FINAL");
    const bool sort_first = !(fk && strcmp(fk, "general") == 0) && !f.prof &&
                            !(c->p.flags & KMER_FLAG_TABLE_SPLIT_TEST);
    HIPCHK(c, hipEventRecord(c->tev[2], s));
    if (sort_first) {
        HIPCHK(c, c->tleft.ensure(2ull * TAB_NQ + 1, s));
        f.left = c->tleft.p + 1;
        f.left_n = c->tleft.p;
        HIPCHK(c, hipMemsetAsync(c->tleft.p, 0, 4, s));
        HIPCHK(c, launch_tab_sort_final(f, 2 * fgrid, s));
    }
    HIPCHK(c, launch_tab_final(f, fgrid, s));
    HIPCHK(c, hipEventRecord(c->tev[7], s));
    if (f.prof) {
        HIPCHK(c, hipMemcpyAsync(hprof.data(), f.prof, fgrid * 64ull, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        (void)hipFree(f.prof);
        double ph[6] = {0, 0, 0, 0, 0, 0};
        uint64_t ranges = 0, buckets = 0;
        for (uint32_t g = 0; g < fgrid; ++g) {
            for (int i = 0; i < 6; ++i) ph[i] += i == 4 ? 0 : (double)hprof[g * 8 + i] * 0.01 / fgrid;   // us
            ranges += hprof[g * 8 + 4] >> 32;
            buckets += hprof[g * 8 + 4] & 0xFFFFFFFFull;
        }
        fprintf(stderr, "tab_final prof (us per workgroup): load+setup %.0f range-syncs %.0f insert %.0f emit %.0f "
                        "empty %.0f | buckets %llu ranges %llu sub_bits %u\n", ph[0], ph[1], ph[2], ph[3], ph[5],
                (unsigned long long)buckets, (unsigned long long)ranges, f.sub_bits);
    }
    HIPCHK(c, hipMemcpyAsync(c->h_small + 8, c->tstats.p, 4 * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(c->h_small, c->d_scal, 8 * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    c->t_ms[3] += ev_ms(c, c->tev[4], c->tev[5]);
    c->t_ms[4] += ev_ms(c, c->tev[5], c->tev[6]);
    c->t_ms[5] += ev_ms(c, c->tev[2], c->tev[7]);
    const uint32_t e = (uint32_t)c->h_small[5];
    if (capq && (e & ERR_TAB_CAP)) {             // (a crowded region: the counted route)
        HIPCHK(c, hipMemsetD32Async((hipDeviceptr_t)c->d_err, (int)(e & ~ERR_TAB_CAP), 1, s));
        continue;
    }
    if (capq) c->t_p2_fixed += 1;
    break;
    }
    const uint32_t e = (uint32_t)c->h_small[5];
    if (e & ERR_COUNT_OVERFLOW) return fail(c, KMER_E_TOO_MANY_KEYS, "a k-mer count exceeds 2^32 - 1");
    if (e & ERR_BIG_OVERFLOW) return fail(c, KMER_E_OOM, "too many k-mers with counts >= 2^20");
    if (e & ERR_TAB_SPLIT) return fail(c, KMER_E_DEVICE, "table bucket could not be split");
    c->t_canon = c->h_small[8];
    c->t_nkeys = c->h_small[9];
    c->t_sum = c->h_small[10];
    c->t_nbig = c->h_small[11];
    c->n_out = c->t_nkeys;
    return KMER_OK;
}

// Canonical classes of the record keys (KMER_FLAG_CANONICAL: forward windows)
std::unordered_map<std::string, uint64_t> canonical_records(const kmer_ctx *c) {
    std::unordered_map<std::string, uint64_t> cls;
    for (auto &kv : c->exotic) {
        std::string r(kv.first.rbegin(), kv.first.rend());
        for (char &ch : r) ch = (char)comp((uint8_t)ch);
        cls[std::min(kv.first, r)] += kv.second.count;
    }
    return cls;
}

// Host result of a table finish: every canonical entry expanded into its Map
// keys (c and rc c, prefix-filtered; palindromes counted twice), plus the
// record keys; entries sorted by key bytes (the table has no order).
kmer_status build_table_result(kmer_ctx *c, uint64_t lines, kmer_result **out) {
    kmer_result *r = new (std::nothrow) kmer_result();
    if (!r) return fail(c, KMER_E_OOM, "host allocation failed");
    r->lines = lines;
    std::vector<std::pair<std::string, uint64_t>> ents;
    const uint32_t k = c->p.k;
    if (c->t_keys) {
        hipStream_t s = c->stream;
        std::vector<uint64_t> start(TAB_NQ + 1), ent;
        std::vector<uint32_t> nd(TAB_NQ);
        std::vector<TabBig> big(c->t_nbig);
        // (the table's extent is start[TAB_NQ], the keys pass 2 counted: t_keys
        // also holds the filler slots of a fixed-run pass 1)
        bool ok = hipMemcpyAsync(start.data(), c->tstart.p, start.size() * 8, hipMemcpyDeviceToHost, s) == hipSuccess &&
                  hipMemcpyAsync(nd.data(), c->tnd.p, nd.size() * 4, hipMemcpyDeviceToHost, s) == hipSuccess &&
                  hipStreamSynchronize(s) == hipSuccess && start[TAB_NQ] <= c->t_keys;
        if (ok) {
            ent.resize(start[TAB_NQ]);
            ok = hipMemcpyAsync(ent.data(), c->t_ent, ent.size() * 8, hipMemcpyDeviceToHost, s) == hipSuccess;
        }
        if (ok && !big.empty())
            ok = hipMemcpyAsync(big.data(), c->tbig.p, big.size() * sizeof(TabBig), hipMemcpyDeviceToHost, s) == hipSuccess;
        if (!ok || hipStreamSynchronize(s) != hipSuccess) {
            delete r;
            return fail(c, KMER_E_DEVICE, "result copy failed");
        }
        std::unordered_map<uint64_t, uint64_t> bigc;
        for (auto &b : big) bigc[b.h] = b.count;
        const bool narrow = k <= TAB_NARROW_K;
        const bool canon = (c->p.flags & KMER_FLAG_CANONICAL) != 0;
        const uint64_t kmask = k >= 32 ? 0xFFFFFFFFull : ((1ull << k) - 1);
        std::string key(k, 'A'), rkey(k, 'A');
        for (uint32_t q = 0; q < TAB_NQ; ++q) {
            for (uint32_t i = 0; i < nd[q]; ++i) {
                const uint64_t w = ent[start[q] + i];
                const uint64_t h = ((uint64_t)q << TAB_RBITS) | (w >> 20);
                uint64_t cnt = w & TAB_CMAX;
                if (cnt == TAB_CMAX) cnt = bigc[h];
                const uint64_t x = tab_code(h, k, narrow, TAB_INV);
                const uint64_t lo = x & kmask, hi = (x >> k) & kmask;
                for (uint32_t j = 0; j < k; ++j) {
                    const uint32_t v = (uint32_t)(((hi >> j) & 1u) << 1 | ((lo >> j) & 1u));
                    key[j] = "ACGT"[v];
                    rkey[k - 1 - j] = "TGCA"[v];
                }
                const bool pal = key == rkey;
                if (canon) {                          // one key per class, counted once per window
                    const std::string &ck = key < rkey ? key : rkey;
                    if (ck.compare(0, c->prefix.size(), c->prefix) == 0) ents.emplace_back(ck, cnt);
                    continue;
                }
                if (key.compare(0, c->prefix.size(), c->prefix) == 0) ents.emplace_back(key, pal ? 2 * cnt : cnt);
                if (!pal && rkey.compare(0, c->prefix.size(), c->prefix) == 0) ents.emplace_back(rkey, cnt);
            }
        }
    }
    if (c->p.flags & KMER_FLAG_CANONICAL) {
        // record keys (non-ACGT windows; forward windows only, unfiltered):
        // classed under min(x, rc x), then the prefix is tested on that key
        for (auto &kv : canonical_records(c))
            if (kv.first.compare(0, c->prefix.size(), c->prefix) == 0) ents.emplace_back(kv.first, kv.second);
    } else {
        for (auto &kv : c->exotic) ents.emplace_back(kv.first, kv.second.count);
    }
    std::sort(ents.begin(), ents.end());
    r->keys.reserve(ents.size() * k);
    r->offsets.reserve(ents.size() + 1);
    r->counts.reserve(ents.size());
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
