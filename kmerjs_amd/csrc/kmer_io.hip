// kmer_io.hip — host input: batches of a buffer or a file (read ahead on a
// reader thread; FIFOs and pipes; gzip), feed_host, and the whole-input counts
// kmer_count_buffer / kmer_count_file (replace readFile(), lib/kmers.js:106-185)
// with their long-line retry.
#include "kmer_host.hpp"

namespace kmerhip {

// Where a batch of input may end (chunks are cut at line ends; FASTA chunks
// before a header line, so that no record spans two chunks).
// batch_cut: the last cut inside [p, p + n), 0 = none;
// batch_extend: the first cut at or after b + from, else len.
uint64_t batch_cut(const uint8_t *p, uint64_t n, bool fasta) {
    if (!fasta) {
        const void *q = n ? memrchr(p, '\n', n) : nullptr;
        return q ? (uint64_t)((const uint8_t *)q - p) + 1 : 0;
    }
    uint64_t e = n ? n - 1 : 0;                  // a '\n' at j < n - 1 with p[j + 1] == '>'
    while (e > 0) {
        const void *q = memrchr(p, '\n', e);
        if (!q) return 0;
        const uint64_t j = (uint64_t)((const uint8_t *)q - p);
        if (p[j + 1] == '>') return j + 1;
        e = j;
    }
    return 0;
}

uint64_t batch_extend(const uint8_t *b, uint64_t from, uint64_t len, bool fasta) {
    uint64_t i = from;
    while (i < len) {
        const void *q = memchr(b + i, '\n', len - i);
        if (!q) return len;
        i = (uint64_t)((const uint8_t *)q - b) + 1;
        if (!fasta || (i < len && b[i] == '>')) return i;
    }
    return len;
}

// Feed host bytes through the device in batches cut at '\n' boundaries.
kmer_status feed_host(kmer_ctx *c, const uint8_t *bytes, uint64_t len, bool report) {
    const uint64_t batch = c->p.batch_bytes ? c->p.batch_bytes : DEFAULT_BATCH;
    uint64_t pos = 0;
    while (pos < len) {
        uint64_t end = std::min(len, pos + batch);
        if (end < len) {
            // cut after the last '\n' in [pos, end) (FASTA: before the last header
            // line); a line (record) longer than the batch extends it
            const uint64_t cut = batch_cut(bytes + pos, end - pos, c->fasta);
            end = cut ? pos + cut : batch_extend(bytes, end, len, c->fasta);
        }
        const uint64_t n = end - pos;
        kmer_status st0 = settle(c);            // the previous batch is done with the staging buffer
        if (st0) return st0;
        HIPCHK(c, c->batch.ensure(n, c->stream));
        // (the caller's bytes, read in place -- a batch is too large to stage
        // through the upload arena: on an error the copy is waited for before
        // returning, so the caller may release them; on success the caller's
        // settle / finish waits for it)
        HIPCHK(c, hipMemcpyAsync(c->batch.p, bytes + pos, n, hipMemcpyHostToDevice, c->stream));
        kmer_status st = feed(c, c->batch.p, n, c->stream);
        if (st) {
            (void)hipStreamSynchronize(c->stream);
            return st;
        }
        pos = end;
        if (report) report_progress(c, pos, len);
    }
    if (report && len == 0) report_progress(c, 0, 0);
    return KMER_OK;
}



// batches of a caller's buffer
struct MemSrc : GroupSrc {
    const uint8_t *b;
    uint64_t len, batch, pos = 0;
    bool fasta;
    MemSrc(const uint8_t *b_, uint64_t len_, uint64_t batch_, bool fasta_)
        : b(b_), len(len_), batch(std::max<uint64_t>(batch_, 1)), fasta(fasta_) {}
    void progress(uint64_t *d, uint64_t *t) override {
        *d = pos;
        *t = len;
    }
    bool next(const uint8_t **p, uint64_t *n, kmer_status *, std::string *) override {
        if (pos >= len) return false;
        uint64_t end = std::min(len, pos + batch);
        if (end < len) {                             // (a line / record longer than the batch extends it)
            const uint64_t cut = batch_cut(b + pos, end - pos, fasta);
            end = cut ? pos + cut : batch_extend(b, end, len, fasta);
        }
        *p = b + pos;
        *n = end - pos;
        pos = end;
        return true;
    }
};

// Batches of a file cut at '\n', read ahead: a reader thread fills a ring of
// host buffers with the next raw ranges of the file (plain files: several
// preads in parallel per range; gzip: zlib) while the caller counts the
// batches it already has, so the file read overlaps the device work
// (lib/kmers.js:108-139 streams the file in chunks too).  A batch is the
// carry of the previous range (the bytes after its last '\n', copied into the
// headroom in front of the next range) plus this range up to its last '\n'.
// Several batches may be outstanding (group counts); each is released when
// its bytes have been consumed.
struct FileBatches : GroupSrc {
    static constexpr uint64_t HEAD = 1ull << 20;     // headroom for the carry
    struct Slot {
        std::unique_ptr<uint8_t[]> buf;
        uint64_t cap = 0, len = 0;
        uint64_t zoff = 0;                           // gzip: compressed bytes read when the slot was filled
        int state = 0;                               // 0 free, 1 filled, 2 in use
        bool last = false;
    };
    int fd = -1;
    gzFile gz = nullptr;
    uint64_t batch = 0, size = 0, rd_off = 0;
    int threads = 1;
    std::vector<Slot> ring;
    std::mutex m;
    std::condition_variable cv;
    std::thread reader;
    bool stop = false, rd_eof = false;
    kmer_status rd_st = KMER_OK;
    std::string rd_err;
    uint64_t next_fill = 0, next_take = 0, consumed = 0;
    uint64_t consumed_z = 0;                         // gzip: compressed offset of the last batch taken
    std::vector<uint8_t> carry;
    std::unordered_map<const uint8_t *, std::unique_ptr<uint8_t[]>> big;   // batches of lines longer than HEAD
    std::unordered_map<const uint8_t *, size_t> slot_of;
    bool done = false;
    bool fasta = false;                              // batches cut before header lines

    ~FileBatches() override {
        {
            std::lock_guard<std::mutex> lk(m);
            stop = true;
        }
        cv.notify_all();
        if (reader.joinable()) reader.join();
        if (gz) gzclose(gz);
        if (fd >= 0) close(fd);
    }

    kmer_status open(const char *path, uint64_t batch_, size_t nslots, std::string *err) {
        fd = ::open(path, O_RDONLY);
        if (fd < 0) {
            *err = std::string("cannot open ") + path;
            return KMER_E_IO;
        }
        struct stat sb;
        const bool regular = fstat(fd, &sb) == 0 && S_ISREG(sb.st_mode);
        if (regular) size = (uint64_t)sb.st_size;
        unsigned char magic[2] = {0, 0};
        // a pipe, FIFO, socket or terminal (fs.createReadStream reads those too)
        // cannot be pread: zlib reads it sequentially on the reader thread, and
        // passes it through unchanged when it is not gzip (transparent mode)
        const bool gzip = !regular || (pread(fd, magic, 2, 0) == 2 && magic[0] == 0x1f && magic[1] == 0x8b);
        batch = std::max<uint64_t>(batch_, 1);
        if (gzip) {
            gz = gzdopen(dup(fd), "rb");
            if (!gz) {
                *err = std::string("cannot read gzip stream ") + path;
                return KMER_E_IO;
            }
            gzbuffer(gz, 1 << 20);
        } else if (size) {
            batch = std::min<uint64_t>(batch, size);  // a small file takes one small buffer
        }
        const unsigned hc = std::thread::hardware_concurrency();
        threads = gzip ? 1 : (int)std::max(1u, std::min(8u, hc ? hc / 2 : 1u));
        ring.resize(std::max<size_t>(nslots, 2));
        reader = std::thread([this] { read_loop(); });
        return KMER_OK;
    }

    // raw range r into slot r % R (plain: `threads` preads in parallel)
    void read_loop() {
        while (true) {
            size_t si;
            {
                std::unique_lock<std::mutex> lk(m);
                si = (size_t)(next_fill % ring.size());
                cv.wait(lk, [&] { return stop || ring[si].state == 0; });
                if (stop) return;
            }
            Slot &S = ring[si];
            if (S.cap < HEAD + batch) {
                S.buf.reset(new (std::nothrow) uint8_t[HEAD + batch]);
                S.cap = S.buf ? HEAD + batch : 0;
            }
            kmer_status st = S.buf ? KMER_OK : KMER_E_OOM;
            uint64_t got = 0;
            bool eof = false;
            if (!st && gz) {
                while (got < batch) {
                    const unsigned want = (unsigned)std::min<uint64_t>(batch - got, 1u << 30);
                    const int r = gzread(gz, S.buf.get() + HEAD + got, want);
                    if (r < 0) {
                        st = KMER_E_IO;
                        break;
                    }
                    got += (uint64_t)r;
                    if ((unsigned)r < want) break;
                }
                int zerr = 0;
                gzerror(gz, &zerr);
                if (zerr != Z_OK && zerr != Z_BUF_ERROR) st = KMER_E_IO;
                eof = got < batch;
                S.zoff = (uint64_t)std::max<z_off_t>(gzoffset(gz), 0);   // (gz is this thread's alone)
            } else if (!st) {
                // parallel preads of [rd_off, rd_off + batch); a short read (end of
                // file, or a file that is not regular) ends the input
                const int T = threads;
                const uint64_t piece = (batch + T - 1) / T;
                std::vector<uint64_t> gotv(T, 0);
                std::vector<int> errv(T, 0);
                auto job = [&](int t) {
                    const uint64_t a = (uint64_t)t * piece, b = std::min<uint64_t>(batch, a + piece);
                    uint64_t o = a;
                    while (o < b) {
                        const ssize_t r = pread(fd, S.buf.get() + HEAD + o, (size_t)(b - o), (off_t)(rd_off + o));
                        if (r < 0) {
                            errv[t] = 1;
                            break;
                        }
                        if (r == 0) break;
                        o += (uint64_t)r;
                    }
                    gotv[t] = o - a;
                };
                std::vector<std::thread> th;
                for (int t = 1; t < T; ++t) th.emplace_back(job, t);
                job(0);
                for (auto &x : th) x.join();
                for (int t = 0; t < T; ++t) {
                    if (errv[t]) st = KMER_E_IO;
                    const uint64_t a = (uint64_t)t * piece, b = std::min<uint64_t>(batch, a + piece);
                    got += gotv[t];
                    if (gotv[t] < b - a) {               // the file ends inside this piece
                        eof = true;
                        break;
                    }
                }
                rd_off += got;
            }
            std::lock_guard<std::mutex> lk(m);
            S.len = got;
            S.last = eof || st;
            S.state = 1;
            if (st) {
                rd_st = st;
                rd_err = "read error";
            }
            ++next_fill;
            cv.notify_all();
            if (S.last) return;
        }
    }

    bool next(const uint8_t **p, uint64_t *n, kmer_status *st, std::string *err) override {
        while (!done) {
            size_t si;
            {
                std::unique_lock<std::mutex> lk(m);
                si = (size_t)(next_take % ring.size());
                cv.wait(lk, [&] { return ring[si].state == 1; });
                ring[si].state = 2;
                ++next_take;
                if (rd_st) {
                    *st = rd_st;
                    *err = rd_err;
                    done = true;
                    return false;
                }
            }
            Slot &S = ring[si];
            consumed += S.len;
            consumed_z = S.zoff;
            const bool last = S.last;
            uint8_t *start;
            uint64_t have;
            std::unique_ptr<uint8_t[]> own;
            if (carry.size() <= HEAD) {
                start = S.buf.get() + HEAD - carry.size();
                if (!carry.empty()) memcpy(start, carry.data(), carry.size());
                have = carry.size() + S.len;
            } else {                                      // a line longer than the headroom
                own.reset(new (std::nothrow) uint8_t[carry.size() + S.len]);
                if (!own) {
                    *st = KMER_E_OOM;
                    *err = "host batch buffer";
                    done = true;
                    return false;
                }
                memcpy(own.get(), carry.data(), carry.size());
                memcpy(own.get() + carry.size(), S.buf.get() + HEAD, S.len);
                start = own.get();
                have = carry.size() + S.len;
            }
            const uint64_t cut = last ? have : batch_cut(start, have, fasta);
            carry.assign(start + cut, start + have);
            if (last) done = true;
            if (cut == 0) {                               // (no '\n' yet: all of it is carry)
                release_slot(si);
                if (last) return false;
                continue;
            }
            *p = start;
            *n = cut;
            std::lock_guard<std::mutex> lk(m);
            if (own) {
                release_slot_locked(si);
                big[start] = std::move(own);
            } else {
                slot_of[start] = si;
            }
            return true;
        }
        return false;
    }

    void release_slot_locked(size_t si) {
        ring[si].state = 0;
        cv.notify_all();
    }
    void release_slot(size_t si) {
        std::lock_guard<std::mutex> lk(m);
        release_slot_locked(si);
    }
    void release(const uint8_t *q) override {
        std::lock_guard<std::mutex> lk(m);
        auto b = big.find(q);
        if (b != big.end()) {
            big.erase(b);
            return;
        }
        auto it = slot_of.find(q);
        if (it != slot_of.end()) {
            release_slot_locked(it->second);
            slot_of.erase(it);
        }
    }
    // progress: (bytes taken, file size) -- for gzip the compressed offset of the
    // batches taken and the compressed size.  Called on the consuming thread
    // only (never touches the gzFile, which the reader thread owns)
    void progress(uint64_t *d, uint64_t *t) override {
        *d = gz ? consumed_z : consumed;
        *t = size;
        if (*d > *t && *t) *d = *t;
    }
};


constexpr uint64_t GROUP_FILE_BATCH = 256ull << 20;

kmer_status group_count_buffer(kmer_ctx *g, const uint8_t *bytes, uint64_t len, kmer_result **out) {
    const size_t N = g->group.size();
    // default: one batch per child (a buffer is already in host memory)
    const uint64_t batch = g->p.batch_bytes ? g->p.batch_bytes : std::max<uint64_t>(1, (len + N - 1) / N);
    MemSrc src(bytes, len, batch, (g->p.flags & KMER_FLAG_FASTA) != 0);
    return group_count(g, src, out);
}

kmer_status group_count_file(kmer_ctx *g, const char *path, kmer_result **out) {
    const size_t N = g->group.size();
    FileBatches src;
    src.fasta = (g->p.flags & KMER_FLAG_FASTA) != 0;
    std::string err;
    const kmer_status st = src.open(path, g->p.batch_bytes ? g->p.batch_bytes : GROUP_FILE_BATCH, N + 2, &err);
    if (st) return fail(g, st, err);
    return group_count(g, src, out);
}



// A whole-input count that met a sequence line longer than the default
// order key's position field (2^23 bytes: a FASTA contig or chromosome) is
// redone once in long-line mode (2^40-byte lines, up to 2^23 lines).
// A group context redoes it on every device.
void set_pbits(kmer_ctx *c, uint32_t pbits) {
    c->pbits = pbits;
    for (kmer_ctx *x : c->group) x->pbits = pbits;
}

kmer_status with_long_line_retry(kmer_ctx *c, const std::function<kmer_status()> &count) {
    c->progress_any = false;
    c->progress_hw = 0;
    kmer_status st = count();
    if (st == KMER_E_LINE_TOO_LONG && c->pbits == PBITS_DEFAULT && c->mode != MODE_TABLE) {
        set_pbits(c, PBITS_LONG);
        st = count();
        set_pbits(c, PBITS_DEFAULT);
    }
    return st;
}

kmer_status count_buffer_once(kmer_ctx *c, const uint8_t *bytes, size_t len, kmer_result **out) {
    kmer_status st = reset(c);
    if (st) return st;
    st = feed_host(c, bytes, len, true);
    if (st) {
        c->open_stream = false;
        return st;
    }
    return finish(c, out);
}

kmer_status count_file_once(kmer_ctx *c, const char *path, kmer_result **out);



kmer_status count_file_once(kmer_ctx *c, const char *path, kmer_result **out) {
    if (hipSetDevice(c->device) != hipSuccess) return KMER_E_DEVICE;
    // the file is read ahead (FileBatches: a reader thread, parallel preads)
    // in batches of batch_bytes (default 256 MiB; no larger than the file),
    // while the device counts the batch before; gzip input (magic 1f 8b) is
    // read through zlib, the count being that of the decompressed FASTQ
    FileBatches src;
    src.fasta = c->fasta;
    std::string err;
    kmer_status st = src.open(path, c->p.batch_bytes ? c->p.batch_bytes : FILE_BATCH, 3, &err);
    if (st) return fail(c, st, err);
    st = reset(c);
    const uint8_t *p = nullptr;
    uint64_t n = 0;
    kmer_status rst = KMER_OK;
    while (!st && src.next(&p, &n, &rst, &err)) {
        st = feed_host(c, p, n);
        if (!st) st = settle(c);
        if (!st && hipStreamSynchronize(c->stream) != hipSuccess) st = fail(c, KMER_E_DEVICE, "stream sync");
        src.release(p);                           // (the batch's bytes are on the device)
        if (!st && c->p.progress) {
            uint64_t d = 0, t = 0;
            src.progress(&d, &t);
            report_progress(c, d, t);
        }
    }
    if (!st && rst) st = fail(c, rst, err + " on " + path);
    if (st) {
        c->open_stream = false;
        return st;
    }
    if (c->p.progress && src.consumed == 0) {        // (an empty file: one event, as progress-stream's end)
        uint64_t d = 0, t = 0;
        src.progress(&d, &t);
        report_progress(c, d, t);
    }
    return finish(c, out);
}


}  // namespace kmerhip

using namespace kmerhip;

extern "C" {


kmer_status kmer_count_buffer(kmer_ctx *c, const uint8_t *bytes, size_t len, kmer_result **out) {
    if (!c || !out || (!bytes && len)) return KMER_E_BAD_PARAM;
    *out = nullptr;
    if (!c->group.empty()) return with_long_line_retry(c, [&] { return group_count_buffer(c, bytes, len, out); });
    if (hipSetDevice(c->device) != hipSuccess) return KMER_E_DEVICE;
    return with_long_line_retry(c, [&] { return count_buffer_once(c, bytes, len, out); });
}

kmer_status kmer_count_file(kmer_ctx *c, const char *path, kmer_result **out) {
    if (!c || !path || !out) return KMER_E_BAD_PARAM;
    *out = nullptr;
    if (!c->group.empty()) return with_long_line_retry(c, [&] { return group_count_file(c, path, out); });
    return with_long_line_retry(c, [&] { return count_file_once(c, path, out); });
}


}  // extern "C"
