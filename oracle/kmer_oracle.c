/*
 * kmer_oracle.c — CPU restatement of the kmerjs FASTQ k-mer hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
 * product path (kmerjs_amd/csrc).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it; the product never links, calls or
 * falls back to it.
 *
 * Parity pinned: the outputs of this restatement are compared bit-for-bit
 * (ordered key/count lists) against golden vectors produced by running the
 * UNMODIFIED reference lib/kmers.js under node in the build container
 * (tools/ref_loader.js, tests/golden/gen_golden.py), and against the
 * reference's own known-answer tests (test/kmers.js:12-52) — see
 * tests/test_oracle.py.
 *
 * Semantics followed, byte for byte (reference = /root/reference):
 *   lines    lib/kmers.js:114-136  split on '\n' only; carry partial lines;
 *                                  trailing segment emitted only if non-empty;
 *                                  empty lines ARE lines; '\r' stays in a line.
 *   records  lib/kmers.js:143-171  line counter i cycles 0..3; a line is a
 *                                  sequence line iff i==1 && line.length>1.
 *   strands  lib/kmers.js:152-155  kmersInLine(line) then
 *                                  kmersInLine(complement(line)).
 *   revcomp  lib/kmers.js:12-17,31-38  map A<->T, G<->C only (other bytes,
 *                                  including N, X, lowercase and '\r', kept),
 *                                  then reverse.
 *   windows  lib/kmers.js:88-100   for index=0..L-k: key = substring(ini,
 *                                  ini+k) (clamped to L), kept iff
 *                                  key.startsWith(preffix); ini += step.
 *   order    lib/kmers.js:76,95    Map insertion order = first occurrence.
 * Input bytes >= 0x80 are rejected (ORACLE_E_NONASCII): the reference decodes
 * chunks as UTF-8 (lib/kmers.js:116) and non-ASCII data would change lengths.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORACLE_OK 0
#define ORACLE_E_NONASCII 1
#define ORACLE_E_OOM 2

typedef struct {
    uint8_t *keys;      /* packed key bytes, entry i at keys[key_off[i]] */
    uint64_t *key_off;
    uint32_t *key_len;
    uint64_t *counts;
    uint64_t *first;    /* ordinal of the first occurrence (monotone) */
    uint64_t n;         /* distinct keys */
    uint64_t lines;     /* lines seen (kmerObj.lines, lib/kmers.js:165) */
    uint64_t windows;   /* windows examined on both strands */
    uint64_t seq_lines; /* sequence lines processed */
    /* private */
    uint64_t cap, keys_cap, keys_used;
    uint64_t *slots;    /* hash slots: entry index + 1, 0 = empty */
    uint64_t slot_mask;
    uint64_t *hashes;
    uint64_t ordinal;
} oracle_result;

static uint64_t hash_bytes(const uint8_t *p, size_t n) {
    uint64_t h = 0xcbf29ce484222325ull ^ (n * 0x9E3779B97F4A7C15ull);
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        memcpy(&w, p + i, 8);
        h = (h ^ w) * 0x100000001b3ull;
        h ^= h >> 29;
    }
    for (; i < n; ++i) h = (h ^ p[i]) * 0x100000001b3ull;
    h ^= h >> 31;
    h *= 0xbf58476d1ce4e5b9ull;
    h ^= h >> 27;
    return h;
}

static int res_init(oracle_result *r) {
    memset(r, 0, sizeof(*r));
    r->cap = 1024;
    r->keys_cap = 1 << 16;
    r->key_off = malloc(r->cap * sizeof(uint64_t));
    r->key_len = malloc(r->cap * sizeof(uint32_t));
    r->counts = malloc(r->cap * sizeof(uint64_t));
    r->first = malloc(r->cap * sizeof(uint64_t));
    r->hashes = malloc(r->cap * sizeof(uint64_t));
    r->keys = malloc(r->keys_cap);
    r->slot_mask = 2048 - 1;
    r->slots = calloc(r->slot_mask + 1, sizeof(uint64_t));
    if (!r->key_off || !r->key_len || !r->counts || !r->first || !r->hashes || !r->keys || !r->slots)
        return ORACLE_E_OOM;
    return ORACLE_OK;
}

void oracle_free(oracle_result *r) {
    free(r->keys); free(r->key_off); free(r->key_len); free(r->counts);
    free(r->first); free(r->slots); free(r->hashes);
    memset(r, 0, sizeof(*r));
}

static int rehash(oracle_result *r) {
    uint64_t nslots = (r->slot_mask + 1) * 2;
    uint64_t *s = calloc(nslots, sizeof(uint64_t));
    if (!s) return ORACLE_E_OOM;
    for (uint64_t e = 0; e < r->n; ++e) {
        uint64_t j = r->hashes[e] & (nslots - 1);
        while (s[j]) j = (j + 1) & (nslots - 1);
        s[j] = e + 1;
    }
    free(r->slots);
    r->slots = s;
    r->slot_mask = nslots - 1;
    return ORACLE_OK;
}

/* Map.set(kmer, (Map.get(kmer) || 0) + 1)  — lib/kmers.js:95 */
static int map_incr(oracle_result *r, const uint8_t *key, size_t n) {
    uint64_t h = hash_bytes(key, n);
    uint64_t j = h & r->slot_mask;
    for (;;) {
        uint64_t e = r->slots[j];
        if (!e) break;
        e -= 1;
        if (r->hashes[e] == h && r->key_len[e] == n && memcmp(r->keys + r->key_off[e], key, n) == 0) {
            r->counts[e] += 1;
            r->ordinal++;
            return ORACLE_OK;
        }
        j = (j + 1) & r->slot_mask;
    }
    if (r->n == r->cap) {
        uint64_t c = r->cap * 2;
        void *a = realloc(r->key_off, c * sizeof(uint64_t)); if (!a) return ORACLE_E_OOM; r->key_off = a;
        a = realloc(r->key_len, c * sizeof(uint32_t)); if (!a) return ORACLE_E_OOM; r->key_len = a;
        a = realloc(r->counts, c * sizeof(uint64_t)); if (!a) return ORACLE_E_OOM; r->counts = a;
        a = realloc(r->first, c * sizeof(uint64_t)); if (!a) return ORACLE_E_OOM; r->first = a;
        a = realloc(r->hashes, c * sizeof(uint64_t)); if (!a) return ORACLE_E_OOM; r->hashes = a;
        r->cap = c;
    }
    if (r->keys_used + n > r->keys_cap) {
        uint64_t c = r->keys_cap * 2;
        while (c < r->keys_used + n) c *= 2;
        void *a = realloc(r->keys, c); if (!a) return ORACLE_E_OOM;
        r->keys = a; r->keys_cap = c;
    }
    uint64_t e = r->n++;
    memcpy(r->keys + r->keys_used, key, n);
    r->key_off[e] = r->keys_used;
    r->key_len[e] = (uint32_t)n;
    r->keys_used += n;
    r->counts[e] = 1;
    r->first[e] = r->ordinal++;
    r->hashes[e] = h;
    r->slots[j] = e + 1;
    if (r->n * 2 > r->slot_mask + 1) return rehash(r);
    return ORACLE_OK;
}

/* complementMap (lib/kmers.js:12-17): only A,T,G,C are mapped. */
static inline uint8_t comp_byte(uint8_t c) {
    switch (c) {
    case 'A': return 'T';
    case 'T': return 'A';
    case 'G': return 'C';
    case 'C': return 'G';
    default: return c;
    }
}

/* complement(string) — lib/kmers.js:31-38: replace then reverse. */
void oracle_complement(const uint8_t *in, size_t n, uint8_t *out) {
    for (size_t i = 0; i < n; ++i) out[n - 1 - i] = comp_byte(in[i]);
}

/* KmerJS.kmersInLine(line) — lib/kmers.js:88-100. */
static int kmers_in_line(oracle_result *r, const uint8_t *t, size_t L,
                         const uint8_t *prefix, size_t plen, uint64_t k, uint64_t step) {
    if (L < k) return ORACLE_OK;              /* stop = L - k < 0: no iteration */
    uint64_t stop = L - k;
    uint64_t ini = 0;
    for (uint64_t index = 0; index <= stop; ++index) {
        /* substring(ini, ini + k) clamps both ends to L (ES2015 21.1.3.19) */
        uint64_t a = ini < L ? ini : L;
        uint64_t b = ini + k < L ? ini + k : L;
        size_t klen = (size_t)(b - a);
        r->windows++;
        if (klen >= plen && memcmp(t + a, prefix, plen) == 0) {
            int st = map_incr(r, t + a, klen);
            if (st) return st;
        }
        ini += step;
    }
    return ORACLE_OK;
}

int oracle_kmers_in_line(const uint8_t *line, size_t n, const uint8_t *prefix, size_t plen,
                         uint32_t k, uint32_t step, oracle_result *out) {
    int st = res_init(out);
    if (st) return st;
    return kmers_in_line(out, line, n, prefix, plen, k, step);
}

/* The line loop of readFile() (lib/kmers.js:114-171) over one piece of the
 * stream; *li is `i` of lib/kmers.js:143, carried across pieces (pieces end at
 * a '\n' -- a whole number of lines -- except the stream's last). */
static int count_lines(oracle_result *out, const uint8_t *buf, size_t len, int *li, uint8_t **rc, size_t *rc_cap,
                       const uint8_t *prefix, size_t plen, uint32_t k, uint32_t step) {
    int st = ORACLE_OK;
    size_t pos = 0;
    while (pos < len) {
        const uint8_t *nl = memchr(buf + pos, '\n', len - pos);
        size_t end = nl ? (size_t)(nl - buf) : len;
        size_t L = end - pos;
        if (!nl && L == 0) break;   /* _flush: empty trailing segment dropped (:131) */
        const uint8_t *line = buf + pos;
        if (*li == 1 && L > 1) {    /* :151 */
            out->seq_lines++;
            st = kmers_in_line(out, line, L, prefix, plen, k, step);
            if (st) break;
            if (L > *rc_cap) {
                free(*rc);
                *rc_cap = L * 2;
                *rc = malloc(*rc_cap);
                if (!*rc) { st = ORACLE_E_OOM; break; }
            }
            oracle_complement(line, L, *rc);
            st = kmers_in_line(out, *rc, L, prefix, plen, k, step);
            if (st) break;
        } else if (*li == 3) {
            *li = -1;               /* :160-161 */
        }
        *li += 1;
        out->lines++;
        pos = nl ? end + 1 : len;
    }
    return st;
}

/* readFile() — lib/kmers.js:106-185, over an in-memory byte buffer. */
int oracle_count_buffer(const uint8_t *buf, size_t len, const uint8_t *prefix, size_t plen,
                        uint32_t k, uint32_t step, oracle_result *out) {
    int st = res_init(out);
    if (st) return st;
    for (size_t i = 0; i < len; ++i)
        if (buf[i] >= 0x80) return ORACLE_E_NONASCII;
    uint8_t *rc = NULL;
    size_t rc_cap = 0;
    int li = 0;
    st = count_lines(out, buf, len, &li, &rc, &rc_cap, prefix, plen, k, step);
    free(rc);
    return st;
}

void oracle_synth_fastq(uint64_t seed, uint64_t first_read, uint64_t n_reads, uint8_t *out);

/* readFile() over the synthetic FASTQ of reads [first_read, first_read +
 * n_reads) (oracle_synth_fastq), generated and counted in
 * blocks of whole records, so full-size workloads (C2, the C4 shard) need no
 * copy of their input in memory.  The same line loop as oracle_count_buffer. */
int oracle_count_synth(uint64_t seed, uint64_t first_read, uint64_t n_reads, const uint8_t *prefix, size_t plen,
                       uint32_t k, uint32_t step, oracle_result *out) {
    int st = res_init(out);
    if (st) return st;
    const uint64_t B = 8192;
    uint8_t *buf = malloc(B * 317), *rc = NULL;
    if (!buf) return ORACLE_E_OOM;
    size_t rc_cap = 0;
    int li = 0;
    for (uint64_t r = 0; r < n_reads && !st; r += B) {
        const uint64_t n = n_reads - r < B ? n_reads - r : B;
        oracle_synth_fastq(seed, first_read + r, n, buf);
        st = count_lines(out, buf, n * 317, &li, &rc, &rc_cap, prefix, plen, k, step);
    }
    free(buf);
    free(rc);
    return st;
}

/* FASTA mode (KMER_FLAG_FASTA) — an EXTENSION, parity unpinned by the
 * reference: it has no FASTA parser (test/kmers.js:53-61 "TODO: FASTA tests
 * missing!", test/kmerFinderServer.js:158 "TODO: FIX FASTA parser").  Records
 * start at lines beginning with '>' (the header is not counted); lines before
 * the first header form a headerless record; a record's sequence is its other
 * lines, each without one trailing '\r', concatenated; each sequence is then
 * counted exactly as readFile() counts a sequence line (lib/kmers.js:151-155:
 * length > 1, kmersInLine of the sequence and of its complement).  `lines`
 * counts input lines as lib/kmers.js:114-136 splits them. */
static int fasta_flush(oracle_result *r, const uint8_t *seq, size_t L, uint8_t **rc, size_t *rc_cap,
                       const uint8_t *prefix, size_t plen, uint32_t k, uint32_t step) {
    if (L <= 1) return ORACLE_OK;
    r->seq_lines++;
    int st = kmers_in_line(r, seq, L, prefix, plen, k, step);
    if (st) return st;
    if (L > *rc_cap) {
        free(*rc);
        *rc_cap = L * 2;
        *rc = malloc(*rc_cap);
        if (!*rc) return ORACLE_E_OOM;
    }
    oracle_complement(seq, L, *rc);
    return kmers_in_line(r, *rc, L, prefix, plen, k, step);
}

int oracle_count_fasta(const uint8_t *buf, size_t len, const uint8_t *prefix, size_t plen,
                       uint32_t k, uint32_t step, oracle_result *out) {
    int st = res_init(out);
    if (st) return st;
    for (size_t i = 0; i < len; ++i)
        if (buf[i] >= 0x80) return ORACLE_E_NONASCII;
    uint8_t *seq = NULL, *rc = NULL;
    size_t seq_len = 0, seq_cap = 0, rc_cap = 0;
    size_t pos = 0;
    while (pos < len && !st) {
        const uint8_t *nl = memchr(buf + pos, '\n', len - pos);
        size_t end = nl ? (size_t)(nl - buf) : len;
        size_t L = end - pos;
        if (!nl && L == 0) break;
        const uint8_t *line = buf + pos;
        out->lines++;
        pos = nl ? end + 1 : len;
        if (L > 0 && line[L - 1] == '\r') --L;
        if (L > 0 && line[0] == '>') {                 /* a header: the record before it ends */
            st = fasta_flush(out, seq, seq_len, &rc, &rc_cap, prefix, plen, k, step);
            seq_len = 0;
            continue;
        }
        if (seq_len + L > seq_cap) {
            seq_cap = (seq_len + L) * 2 + 64;
            uint8_t *q = realloc(seq, seq_cap);
            if (!q) { st = ORACLE_E_OOM; break; }
            seq = q;
        }
        if (L) memcpy(seq + seq_len, line, L);
        seq_len += L;
    }
    if (!st) st = fasta_flush(out, seq, seq_len, &rc, &rc_cap, prefix, plen, k, step);
    free(seq);
    free(rc);
    return st;
}

/* ---- synthetic FASTQ, identical to the device generator ----
 * Record i: "@r%010llu\n" + 150 bases + "\n+\n" + 150 x 'I' + "\n" = 317 B.
 * Base b of read i = "ACGT"[(mix(seed*G + i*8 + b/32) >> 2*(b%32)) & 3]. */
static inline uint64_t splitmix_mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void oracle_synth_fastq(uint64_t seed, uint64_t first_read, uint64_t n_reads, uint8_t *out) {
    static const char B[4] = {'A', 'C', 'G', 'T'};
    for (uint64_t r = 0; r < n_reads; ++r) {
        uint64_t i = first_read + r;
        uint8_t *p = out + r * 317;
        p[0] = '@'; p[1] = 'r';
        uint64_t v = i;
        for (int d = 9; d >= 0; --d) { p[2 + d] = (uint8_t)('0' + v % 10); v /= 10; }
        p[12] = '\n';
        uint8_t *s = p + 13;
        for (int m = 0; m < 5; ++m) {
            uint64_t w = splitmix_mix(seed * 0x9E3779B97F4A7C15ull + i * 8 + (uint64_t)m);
            for (int b = 0; b < 32 && m * 32 + b < 150; ++b) s[m * 32 + b] = (uint8_t)B[(w >> (2 * b)) & 3];
        }
        s[150] = '\n'; s[151] = '+'; s[152] = '\n';
        memset(s + 153, 'I', 150);
        s[303] = '\n';
    }
}

/* ---- table digest (kmer_table_digest's definition), streaming ----
 * Table mode stores one entry per canonical class {x, rc x} (SURVEY.md App.
 * A.6), counted once per FORWARD window of a sequence line (lines as
 * readFile() splits them, lib/kmers.js:114-171; windows lib/kmers.js:88-100
 * with step 1); windows holding a byte outside A/C/G/T are records, outside
 * the digest.  With the planar code of a k-mer (base i at bit i of two planes,
 * A/C/G/T = (hi, lo) 00/01/10/11, code = hi << k | lo) and h = min(code(w),
 * code(rc w)) * 0x9E3779B97F4A7C15, the digest is
 *     sum over classes of count x mix(h) = sum over forward windows of mix(h)
 * (mod 2^64; mix = splitmix64's finaliser): linear, so no map is needed.
 * Codes are rolled: one new base per window on the forward planes (shift
 * down) and on the reverse-complement planes (shift up). */
static inline uint64_t digest_mix(uint64_t h) {
    h ^= h >> 30;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 27;
    h *= 0x94D049BB133111EBull;
    return h ^ (h >> 31);
}

static void digest_line(const uint8_t *t, size_t L, uint32_t k, uint64_t *dig, uint64_t *win) {
    const uint64_t mask = k >= 64 ? ~0ull : (1ull << k) - 1;
    uint64_t flo = 0, fhi = 0, rlo = 0, rhi = 0, acc = 0, n = 0;
    uint32_t run = 0;                        /* A/C/G/T bytes ending here */
    for (size_t i = 0; i < L; ++i) {
        const uint8_t b = t[i];
        if (b == 'A' || b == 'C' || b == 'G' || b == 'T') {
            const uint64_t lo = ((b >> 1) ^ (b >> 2)) & 1u, hi = (b >> 2) & 1u;
            flo = (flo >> 1) | (lo << (k - 1));
            fhi = (fhi >> 1) | (hi << (k - 1));
            rlo = ((rlo << 1) | (lo ^ 1u)) & mask;
            rhi = ((rhi << 1) | (hi ^ 1u)) & mask;
            if (run < k) ++run;
        } else {
            run = 0;
        }
        if (i + 1 >= k) {                    /* window [i + 1 - k, i] */
            ++n;
            if (run >= k) {
                const uint64_t cf = fhi << k | flo, cr = rhi << k | rlo;
                acc += digest_mix((cf < cr ? cf : cr) * 0x9E3779B97F4A7C15ull);
            }
        }
    }
    *dig += acc;
    *win += n;
}

/* over a buffer: sequence lines as readFile() finds them (k <= 31) */
static void digest_lines(const uint8_t *buf, size_t len, int *li, uint32_t k, uint64_t *dig, uint64_t *win) {
    size_t pos = 0;
    while (pos < len) {
        const uint8_t *nl = memchr(buf + pos, '\n', len - pos);
        size_t end = nl ? (size_t)(nl - buf) : len;
        size_t L = end - pos;
        if (!nl && L == 0) break;
        if (*li == 1 && L > 1) digest_line(buf + pos, L, k, dig, win);
        else if (*li == 3) *li = -1;
        *li += 1;
        pos = nl ? end + 1 : len;
    }
}

int oracle_table_digest_buffer(const uint8_t *buf, size_t len, uint32_t k, uint64_t *digest, uint64_t *windows) {
    if (k == 0 || k > 31) return ORACLE_E_NONASCII + 2;
    int li = 0;
    *digest = 0;
    *windows = 0;
    digest_lines(buf, len, &li, k, digest, windows);
    return ORACLE_OK;
}

/* the table digest of FASTA records (KMER_FLAG_FASTA; the record rules of
 * oracle_count_fasta above: '>' opens a record, its other lines joined with one
 * trailing '\r' each dropped, sequences of length > 1 counted) -- BASELINE C5's
 * .fsa-style contigs in table mode */
int oracle_table_digest_fasta(const uint8_t *buf, size_t len, uint32_t k, uint64_t *digest, uint64_t *windows) {
    if (k == 0 || k > 31) return ORACLE_E_NONASCII + 2;
    *digest = 0;
    *windows = 0;
    uint8_t *seq = NULL;
    size_t seq_len = 0, seq_cap = 0, pos = 0;
    while (pos < len) {
        const uint8_t *nl = memchr(buf + pos, '\n', len - pos);
        size_t end = nl ? (size_t)(nl - buf) : len;
        size_t L = end - pos;
        if (!nl && L == 0) break;
        const uint8_t *line = buf + pos;
        pos = nl ? end + 1 : len;
        if (L > 0 && line[L - 1] == '\r') --L;
        if (L > 0 && line[0] == '>') {
            if (seq_len > 1) digest_line(seq, seq_len, k, digest, windows);
            seq_len = 0;
            continue;
        }
        if (seq_len + L > seq_cap) {
            seq_cap = (seq_len + L) * 2 + 64;
            uint8_t *q = realloc(seq, seq_cap);
            if (!q) { free(seq); return ORACLE_E_OOM; }
            seq = q;
        }
        if (L) memcpy(seq + seq_len, line, L);
        seq_len += L;
    }
    if (seq_len > 1) digest_line(seq, seq_len, k, digest, windows);
    free(seq);
    return ORACLE_OK;
}

#include <pthread.h>

typedef struct {
    uint64_t seed, r0, r1, dig, win;
    uint32_t k;
    int st;
} digest_job;

static void *digest_worker(void *arg) {
    digest_job *j = arg;
    const uint64_t B = 4096;
    uint8_t *buf = malloc(B * 317);
    if (!buf) { j->st = ORACLE_E_OOM; return NULL; }
    for (uint64_t r = j->r0; r < j->r1; r += B) {
        const uint64_t n = j->r1 - r < B ? j->r1 - r : B;
        int li = 0;                          /* blocks are whole records */
        oracle_synth_fastq(j->seed, r, n, buf);
        digest_lines(buf, n * 317, &li, j->k, &j->dig, &j->win);
    }
    free(buf);
    return NULL;
}

/* the table digest of the synthetic FASTQ reads [first_read, first_read +
 * n_reads) on `threads` threads (full-size C3: 100 M reads, 24 G windows) */
int oracle_table_digest_synth(uint64_t seed, uint64_t first_read, uint64_t n_reads, uint32_t k, uint32_t threads,
                              uint64_t *digest, uint64_t *windows) {
    if (k == 0 || k > 31) return ORACLE_E_NONASCII + 2;
    if (threads == 0) threads = 1;
    if (threads > 256) threads = 256;
    digest_job jobs[256];
    pthread_t tid[256];
    int st = ORACLE_OK;
    for (uint32_t t = 0; t < threads; ++t) {
        jobs[t] = (digest_job){seed, first_read + n_reads * t / threads, first_read + n_reads * (t + 1) / threads,
                               0, 0, k, ORACLE_OK};
        if (pthread_create(&tid[t], NULL, digest_worker, &jobs[t])) { threads = t; st = ORACLE_E_OOM; break; }
    }
    *digest = 0;
    *windows = 0;
    for (uint32_t t = 0; t < threads; ++t) {
        pthread_join(tid[t], NULL);
        *digest += jobs[t].dig;
        *windows += jobs[t].win;
        if (jobs[t].st) st = jobs[t].st;
    }
    return st;
}
