/*
 * kmer_api.h — C-ABI of libkmerhip, the MI355X (gfx950) k-mer counter that
 * replaces the FASTQ sliding-window loop of kmerjs (lib/kmers.js).
 *
 * The reference has no native interface; these entry points are what a
 * kmerjs binding (the N-API addon in kmerjs_amd/node/, or ctypes) needs to
 * implement the reference's KmerJS surface unchanged:
 *
 *   reference                                    replaced by
 *   -------------------------------------------  ------------------------------------
 *   new KmerJS(fastq, preffix, length, step, ..) kmer_open(params)        lib/kmers.js:67-82
 *   KmerJS.readFile() -> {promise: Map, event}   kmer_count_file()        lib/kmers.js:106-185
 *     (stream -> liner -> mod-4 -> kmersInLine)  kmer_count_buffer()      lib/kmers.js:114-171
 *   kmersInLine(line), complement(line)          (inside the kernels)     lib/kmers.js:88-100,31-38
 *   Map insertion order / size / entries         kmer_result_*            lib/kmers.js:76,95,177
 *   kmerObj.lines                                kmer_result_lines()      lib/kmers.js:145,165
 *
 * Results are bit-exact with the reference: identical keys (byte strings,
 * including non-ACGT bytes such as N, X, lowercase or '\r'), identical counts,
 * and entries in the reference Map's insertion (first-occurrence) order.
 *
 * Device-resident entry points (kmer_reset / kmer_feed_device /
 * kmer_finish_device) let a caller that already holds the FASTQ bytes in HBM
 * count them without any host copy; kmer_partial_device / kmer_finish_merged
 * merge per-GPU partial results (shards of one input, RCCL over xGMI).
 *
 * Threading: a kmer_ctx is used by one thread at a time (one in-flight call
 * per context); distinct contexts are independent.  All calls return a
 * kmer_status; kmer_last_error() gives a message for the last failure.
 */
#ifndef KMER_API_H
#define KMER_API_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    KMER_OK = 0,
    KMER_E_IO = 1,            /* file missing/unreadable (reference: uncaught stream error) */
    KMER_E_BAD_PARAM = 2,     /* k == 0, step == 0, NULL pointers, ... */
    KMER_E_OOM = 3,           /* host or device allocation failed */
    KMER_E_DEVICE = 4,        /* HIP runtime error */
    KMER_E_TOO_MANY_KEYS = 5, /* more than max_keys distinct keys (reference: RangeError at 2^24, lib/kmers.js:95) */
    KMER_E_NONASCII = 6,      /* input byte >= 0x80 (reference decodes UTF-8, lib/kmers.js:116) */
    KMER_E_LINE_TOO_LONG = 7, /* a sequence line longer than the order key holds (KMER_FLAG_LONG_LINES) */
    KMER_E_STATE = 8          /* call out of sequence (e.g. finish without reset) */
} kmer_status;

enum {
    KMER_FLAG_TWO_PASS = 1u << 0,  /* debug: exact two-pass line scan instead of single-pass look-back */
    KMER_FLAG_NO_DENSE = 1u << 1,  /* debug: records instead of packed keys (host merge) */
    KMER_FLAG_BYTE_SCAN = 1u << 2, /* debug: byte-SWAR prefix scan instead of the bit-plane scan */
    KMER_FLAG_SORT_FINISH = 1u << 3, /* debug: radix-sort finish instead of the bucket-table finish */
    /* Table mode: the result need not be in Map insertion order.  For step 1,
     * k <= 32 and an empty or A/C/G/T prefix the counts go to a hash-partitioned
     * table of canonical k-mers in HBM (no 2^32-hit session limit; host results
     * sorted by key bytes); other configurations keep the ordered paths. */
    KMER_FLAG_UNORDERED = 1u << 4,
    KMER_FLAG_TABLE_SPLIT_TEST = 1u << 5, /* debug: table mode with 64-key LDS ranges (exercises range splits) */
    /* Canonical k-mers (BASELINE C5; an extension, not the reference's Map):
     * table mode whose result holds one key per {x, rc x} class -- the
     * lexicographically smaller string -- counted once per forward window of
     * the class (jellyfish -C).  Step 1, k <= 32, empty or A/C/G/T prefix
     * (tested on the canonical key); KMER_E_BAD_PARAM otherwise. */
    KMER_FLAG_CANONICAL = 1u << 6,
    /* Long-line mode: order keys with a 40-bit position field, so ordered
     * counts take sequence lines up to 2^40 bytes (FASTA contigs and
     * chromosomes; the reference has no limit, lib/kmers.js:88-100) at up to
     * 2^23 lines.  Default: lines up to 2^23 bytes, 2^40 lines.
     * kmer_count_file / kmer_count_buffer switch to it by themselves when a
     * longer line turns up (the count is redone once); the device-resident
     * calls and multi-GPU group contexts need the flag. */
    KMER_FLAG_LONG_LINES = 1u << 7,
    /* bits 8..15 are reserved (kmer_open rejects them) */
    /* FASTA input (an extension; the reference has no FASTA parser:
     * test/kmers.js:53-61, test/kmerFinderServer.js:158, so its readFile()
     * counts only lines with index % 4 == 1 of a .fsa file, lib/kmers.js:151).
     * A line starting with '>' opens a record (the header is not counted);
     * lines before the first header form a headerless record; a record's
     * sequence is its other lines joined (one trailing '\r' per line dropped),
     * so windows span line breaks; each sequence is counted as the reference
     * counts a sequence line (length > 1; windows of it and of its complement;
     * first-occurrence order by record).  Every mode (ordered, UNORDERED,
     * CANONICAL, any k / step / prefix; records longer than 2^23 bytes through
     * the long-line retry).  kmer_result_lines = input lines.  Device feeds
     * must cut chunks before a header line (offset 0, or a '>' after '\n'). */
    KMER_FLAG_FASTA = 1u << 16,
    /* debug: table pass 1 always with fixed per-workgroup runs (by default
     * only when their filler slots are <= 1/12 of the keys: large inputs), and
     * pass 2 with fixed region capacities at any table size (by default from
     * 2^24 keys) */
    KMER_FLAG_TABLE_FIXED_TEST = 1u << 17,
    /* debug: the general path's first merge attempt reports a hash collision,
     * so the two-hash (h2, h1) retry runs (exercises the collision route) */
    KMER_FLAG_GEN_COLLIDE_TEST = 1u << 18
};

typedef struct {
    uint32_t k;               /* kmerLength (reference default 16) */
    uint32_t step;            /* step (reference default 1) */
    const uint8_t *prefix;    /* preffix bytes (reference default "ATGAC"); may be NULL if prefix_len == 0 */
    uint32_t prefix_len;
    int32_t device;           /* HIP device ordinal */
    uint32_t flags;           /* KMER_FLAG_* */
    uint64_t max_keys;        /* 0 = unlimited; 16777216 reproduces the reference Map cap */
    uint64_t batch_bytes;     /* host->device batch size for file/buffer input; 0 = default (files:
                               * 256 MiB, read ahead on a reader thread; buffers: 1 GiB) */
    /* Multi-GPU (SURVEY.md §8b `ndev`): ndev > 1 makes a group context over
     * `devices` (ndev HIP ordinals; NULL = 0..ndev-1; an ordinal may repeat).
     * kmer_count_file / kmer_count_buffer then split the input into ndev
     * line-aligned shards counted concurrently, one per device, and merge the
     * per-device partials (copied to devices[0] over xGMI) into one result in
     * Map order -- bit-exact with a single-device count.  The input is read
     * as a stream of batches cut at '\n' (batch_bytes; default for files
     * 256 MiB, for buffers one share per device) dealt round robin to the
     * devices, so a file never has to fit in host memory.  Table and
     * canonical mode: every device's pass-1 keys go to the device that owns
     * their slice of the hash space, which builds that slice of the table;
     * kmer_table_stats / kmer_table_digest of a group add up its devices'.
     * Every ordered configuration with packed keys is sharded too (any prefix
     * bytes, step > 1).  Only the configurations without packed partials run
     * on devices[0] alone: k > 64 and unprefixed k > 31 (the general path),
     * keys of 64 bits or more (k - |P| >= 32), and KMER_FLAG_NO_DENSE.  A
     * group count that meets a line longer than 2^23 bytes is redone in
     * long-line mode on every device, as a single-device count is.  The other
     * device-resident entry
     * points are single-device only (KMER_E_STATE on a group).  0 or 1 =
     * single device `device`. */
    uint32_t ndev;
    const int32_t *devices;
    /* Progress of kmer_count_file / kmer_count_buffer (replaces the
     * progress-stream of readFile(), lib/kmers.js:108-110): called on the
     * counting thread after each input batch with the input bytes consumed so
     * far and the input's size (for gzip: compressed bytes read and the
     * compressed size).  NULL = none. */
    void (*progress)(void *user, uint64_t done, uint64_t total);
    void *progress_user;
} kmer_params;

typedef struct kmer_ctx kmer_ctx;
typedef struct kmer_result kmer_result;

/* Context lifecycle (replaces `new KmerJS(...)`, lib/kmers.js:67-82). */
kmer_status kmer_open(const kmer_params *params, kmer_ctx **out);
kmer_status kmer_close(kmer_ctx *ctx);

/* Whole-input calls (replace readFile(), lib/kmers.js:106-185). */
/* kmer_count_file also reads gzip-compressed FASTQ (magic 1f 8b) through zlib:
 * the count is that of the decompressed bytes. */
kmer_status kmer_count_file(kmer_ctx *ctx, const char *path, kmer_result **out);
kmer_status kmer_count_buffer(kmer_ctx *ctx, const uint8_t *bytes, size_t len, kmer_result **out);

/* Device-resident streaming: bytes already in HBM.  Each fed chunk must start
 * at a line start (offset 0 of the input, or just after a '\n'); all chunks
 * but the last must end with '\n'.  `stream` is the hipStream_t that produced
 * the bytes (NULL = the legacy default stream): the count waits for the work
 * queued on it so far.  kmer_finish_device leaves the ordered result in
 * device memory (kmer_result_device) and also returns it as a host result
 * when `out` is non-NULL. */
kmer_status kmer_reset(kmer_ctx *ctx);
kmer_status kmer_feed_device(kmer_ctx *ctx, const void *d_bytes, size_t len, void *stream);
kmer_status kmer_finish_device(kmer_ctx *ctx, kmer_result **out);
/* kmer_feed_device returns once the chunk is queued on the context's stream
 * (packed paths); the chunk is settled -- its counters read back, an overflow
 * of the hit lists redone, its errors reported -- by the next call on the
 * context, or explicitly by kmer_sync.  The bytes must stay valid and
 * unchanged until then.  While a chunk is in flight the caller may queue
 * work on other contexts (e.g. another session's finish), which then
 * overlaps the scan on the device.  (lib/kmers.js:148-171 reads the stream
 * chunk by chunk; errors surface at the next call instead of the feed.) */
kmer_status kmer_sync(kmer_ctx *ctx);

/* Multi-GPU merge.  kmer_partial_device reduces this context's session to its
 * unique packed keys: keys = uint64[n] 2-bit suffix codes (the k-|P| bases
 * after the prefix, first base most significant), vals = n x {uint64 first,
 * uint64 count} (first-occurrence order, count).  Keys of 64 bits or more
 * (k - |P| >= 32, counted on the packed path as two words) have no partial:
 * KMER_E_STATE here and in the hit exchange below.  Device pointers, valid until
 * the next call on the context.  Concatenate the partials of every rank on one
 * device (e.g. RCCL gather over xGMI) and hand them to kmer_finish_merged,
 * which reduces again (min first, sum count), orders by first occurrence and
 * decodes.  Record keys (non-ACGT windows) stay on the host: move them with
 * kmer_records_export / kmer_records_import.  KMER_E_STATE when the
 * configuration has no packed keys. */
kmer_status kmer_partial_device(kmer_ctx *ctx, const void **d_keys, const void **d_vals, uint64_t *n);
kmer_status kmer_finish_merged(kmer_ctx *ctx, const void *d_keys, const void *d_vals, uint64_t n,
                               uint64_t total_lines, kmer_result **out);
/* Multi-GPU hit exchange (the default multi-GPU finish).  After the feeds,
 * kmer_exchange_prepare partitions this session's counting hits by owning
 * rank -- equal slices of the packed-key space over `world` ranks (world <=
 * 256) -- into d_send: per owner a contiguous run of 16-byte records {uint64
 * first-occurrence order key, uint64 packed key}, runs in owner order, each
 * run in first-occurrence order; counts[o] (host array of `world`) = records
 * for owner o.  d_send is valid until the next call on the context.  Exchange
 * the runs (all-to-all over xGMI) and hand each rank's received records,
 * concatenated in source-rank order, to kmer_finish_exchanged, which counts
 * them (this rank's key range of the result, in first-occurrence order,
 * device-resident: kmer_result_device).  `wait_stream` (hipStream_t; NULL =
 * the legacy default stream): the context's stream waits for the work queued
 * so far on that stream (the collective that wrote d_recv) before reading it.  Shards must be fed in
 * line order (kmer_set_position) so that order keys are global. */
kmer_status kmer_exchange_prepare(kmer_ctx *ctx, uint32_t world, const void **d_send, uint64_t *counts);
kmer_status kmer_finish_exchanged(kmer_ctx *ctx, const void *d_recv, uint64_t n, uint64_t total_lines,
                                  void *wait_stream, kmer_result **out);
/* One result in Map order from every rank's ordered key range (the device
 * result of kmer_finish_exchanged on each rank), gathered to this context's
 * device and concatenated (any order): n rows of keys (n * k bytes), counts
 * (uint64) and first-occurrence keys (uint64).  Re-orders them by first
 * occurrence into this context's device result (kmer_result_device) and,
 * when `out` is non-NULL, returns the host result with this context's record
 * keys merged in (import the other ranks' records first). */
kmer_status kmer_merge_ordered(kmer_ctx *ctx, const void *d_keys, const void *d_counts, const void *d_firsts,
                               uint64_t n, uint64_t total_lines, kmer_result **out);
kmer_status kmer_records_export(kmer_ctx *ctx, kmer_result **out);
kmer_status kmer_records_import(kmer_ctx *ctx, const char *keys, const uint64_t *offsets,
                                const uint64_t *counts, const uint64_t *firsts, uint64_t n);
/* Drop this session's record keys (after they were moved to another rank). */
kmer_status kmer_records_clear(kmer_ctx *ctx);
/* Ordered result of the last finish, still in device memory (packed path):
 * keys = n * k bytes, counts = uint64[n], firsts = uint64[n]. */
kmer_status kmer_result_device(kmer_ctx *ctx, const void **d_keys, const void **d_counts,
                               const void **d_firsts, uint64_t *n);
/* Set the running line/byte position (lines already consumed, absolute byte
 * offset of the next fed chunk) — used when one input is sharded over ranks. */
kmer_status kmer_set_position(kmer_ctx *ctx, uint64_t lines_before, uint64_t byte_offset);
/* Lines consumed so far (reference kmerObj.lines). */
kmer_status kmer_lines(kmer_ctx *ctx, uint64_t *lines);

/* Ordered result (Map insertion order). */
uint64_t kmer_result_size(const kmer_result *r);
uint64_t kmer_result_lines(const kmer_result *r);
kmer_status kmer_result_get(const kmer_result *r, uint64_t i, const char **key, uint32_t *klen,
                            uint64_t *count);
/* Bulk view: keys packed back to back; key i = keys[offsets[i] .. offsets[i+1]). */
kmer_status kmer_result_arrays(const kmer_result *r, const char **keys, const uint64_t **offsets,
                               const uint64_t **counts);
/* First-occurrence order key of every entry (monotone in Map order). */
kmer_status kmer_result_firsts(const kmer_result *r, const uint64_t **firsts);
/* Write a result to a file, in Map order: KMER_WRITE_JSON = JSON.stringify of
 * mapToJSON(map) (lib/kmers.js:46-54); KMER_WRITE_LEGACY = the npm main's
 * "{\n key: count, ... }\n" dump (lib/index.js:381-388). */
enum { KMER_WRITE_JSON = 0, KMER_WRITE_LEGACY = 1 };
kmer_status kmer_result_write(const kmer_result *r, const char *path, uint32_t format);
void kmer_result_free(kmer_result *r);

/* Benchmark utility: write n_reads synthetic 317-byte FASTQ records (SURVEY.md
 * §8d generator, splitmix64 of (seed, read index)) to device memory. */
kmer_status kmer_synth_fastq_device(void *d_out, uint64_t seed, uint64_t first_read, uint64_t n_reads,
                                    void *stream);

/* Table mode (KMER_FLAG_UNORDERED), after a finish.  The counts replace the
 * reference Map (lib/kmers.js:95) when it would be too large to build:
 *   canonical = distinct canonical k-mers in the table,
 *   keys      = distinct Map keys (both orientations, prefix-filtered, + records),
 *   total     = sum of the Map's counts (= counted windows on both strands). */
kmer_status kmer_table_stats(kmer_ctx *ctx, uint64_t *canonical, uint64_t *keys, uint64_t *total);
/* The table itself, in device memory.  2^20 buckets; bucket q holds
 * bucket_len[q] (uint32) entries at entries[bucket_start[q] ..] (uint64 each:
 * remainder << 20 | count, count == 0xFFFFF meaning "see the big list").
 * h = q << 44 | remainder = c * 0x9E3779B97F4A7C15 (mod 2^64), a bijection of the canonical
 * planar code c = min(code(w), code(rc w)) with code = hi_plane << k | lo_plane,
 * base i of the k-mer at bit i of each plane, A/C/G/T = (hi,lo) 00/01/10/11.
 * k <= 21 (narrow keys): h = f(c') << 23, f(x) = (x ^ (x >> 21)) *
 * 0x9E3779B97F4A7C15 mod 2^41 (the remainder's low 23 bits are 0), where c'
 * is, for even k, c; for odd k, the planar code of the orientation (w or
 * rc w) whose middle base is A or C, with that base's high-plane bit (bit
 * k + (k - 1) / 2, zero) taken out.  Inverse: x = z ^ (z >> 21), z = (h >>
 * 23) * 0x9E3779B97F4A7C15^-1 mod 2^41, then (odd k) a zero bit put back at
 * k + (k - 1) / 2.  (The digest weighs c * 0x9E3779B97F4A7C15 for every k.)
 * big = n_big {uint64 h, uint64 count} pairs.  Valid until the next reset. */
kmer_status kmer_table_device(kmer_ctx *ctx, const void **d_entries, const void **d_bucket_start,
                              const void **d_bucket_len, const void **d_big, uint64_t *n_big);
/* Linear digest of the table (after a finish): sum over its canonical entries
 * of count x mix(h) mod 2^64, mix = the splitmix64 finalizer
 * (z ^= z >> 30; z *= 0xBF58476D1CE4E5B9; z ^= z >> 27; z *= 0x94D049BB133111EB;
 * z ^= z >> 31).  Linear in the counts: the digest of a count over input
 * A + B is the sum of the digests over A and over B, and the ranks' digests
 * of an exchanged table add up -- a size-independent check of a table that is
 * too large to compare entry by entry.  Record keys are not included. */
kmer_status kmer_table_digest(kmer_ctx *ctx, uint64_t *digest);
/* Diagnostics of table mode's routes since the last reset.  Pass 1: chunks
 * whose keys went out in fixed-capacity runs (p1_fixed), of them the chunks
 * whose workgroup shares were merged first (p1_merged: small shares, e.g. long
 * contigs cut into pieces), and chunks counted by the two-pass route
 * (p1_counted).  Pass 2: finishes that ran with fixed bucket capacities and no
 * histogram pass (p2_fixed: large buckets).  Lets a test assert which route a
 * workload took. */
kmer_status kmer_table_routes(kmer_ctx *ctx, uint64_t *p1_fixed, uint64_t *p1_merged, uint64_t *p1_counted,
                              uint64_t *p2_fixed);
/* Table mode across ranks (replaces the one Map.set stream of lib/kmers.js:95
 * when the count is sharded over GPUs; reads are independent, :151-155).
 * Rank o (of `world` <= 1024) owns the pass-1 partitions [o*1024/world,
 * (o+1)*1024/world) -- a contiguous slice of the hash space h and its
 * buckets.  After the feeds, kmer_table_exchange_prepare returns in d_send,
 * per owner, a contiguous run of uint64 pass-1 keys (runs in owner order, each
 * partition-major); counts[o] (host, `world`) = keys for owner o; parts[p]
 * (host, 1024) = this session's keys per partition.  d_send is valid until the
 * next call on the context.  Exchange the runs (all-to-all over xGMI) and the
 * parts tables (all-gather), then hand the received runs, concatenated in
 * source-rank order (n keys), and parts (world x 1024, source-rank order) to
 * kmer_table_finish_exchanged: pass 2 + final over this rank's buckets
 * (others empty).  The table is written over d_recv, which must stay alive
 * until the next reset; kmer_table_stats / kmer_table_device then describe
 * this rank's share (the ranks' stats add up: partitions are disjoint; move
 * record keys to one rank first, kmer_records_export / _import / _clear).
 * `wait_stream` as for kmer_finish_exchanged. */
kmer_status kmer_table_exchange_prepare(kmer_ctx *ctx, uint32_t world, const void **d_send, uint64_t *counts,
                                        uint64_t *parts);
kmer_status kmer_table_finish_exchanged(kmer_ctx *ctx, void *d_recv, uint64_t n, const uint64_t *parts,
                                        uint32_t world, uint32_t rank, void *wait_stream);

/* Device time (HIP events on the context's stream, ms) since the last reset:
 * scan_ms = the streaming tile-scan kernel(s) alone, feed_ms = every kernel of
 * the feeds (scan + line scans + hit resolution), finish_ms = the last finish
 * (compaction + sort + decode).  Waits for the last finish only when
 * finish_ms is non-NULL. */
kmer_status kmer_last_timing(kmer_ctx *ctx, double *scan_ms, double *feed_ms, double *finish_ms);

/* Device time per phase since the last reset (HIP events on the context's
 * stream, ms; feeds summed).  Table mode: "lines" (newline array, sequence
 * lines), "hist1" (+ its scan), "scatter1", "hist2" (+ scan), "scatter2",
 * "final"; ordered modes: "scan", "feed", "finish" as kmer_last_timing.
 * Up to `max` entries are written; *n = the number of phases. */
kmer_status kmer_phase_times(kmer_ctx *ctx, uint32_t max, const char **names, double *ms, uint32_t *n);

const char *kmer_status_string(kmer_status s);
const char *kmer_last_error(const kmer_ctx *ctx);
const char *kmer_version(void);

#ifdef __cplusplus
}
#endif
#endif /* KMER_API_H */
