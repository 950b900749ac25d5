/*
 * kmer_match.h — C-ABI of the k-mer -> template matcher in libkmerhip
 * (SURVEY.md §8f row 3): kmerFinder's hash-join of a query k-mer Map against
 * a template database, on the GPU.
 *
 *   reference                                             replaced by
 *   ----------------------------------------------------  ---------------------------
 *   Redis kmer -> [template] lists, Mongo `reads`         kmer_db_open
 *     (src/kmerPyToMongo.py:21-42)
 *   findKmersMatchesRedis: one lrange per query k-mer,    kmer_match_open
 *     templates scored in first-hit order                 (+ kmer_match_templates)
 *     (lib/kmerFinderServer.js:171-226)
 *   findWinner: templates sorted by uScore, first wins    kmer_match_winner
 *     (:741-752, sortKmerMatches :700-709)
 *   removeWinnerKmers + getMatches: the winner's k-mers   kmer_match_remove
 *     leave the query, every template is re-scored
 *     (:778-830)
 *   findMatchesMongoAggregation: templates in DB order    kmer_match_templates(.., DB order)
 *     (:452-522)
 *
 * The statistics of a winner (lib/stats.js zScore / fastp, matchSummary
 * lib/kmerFinderServer.js:625-676, bignumber.js decimals) are scalar host work
 * done by the caller (kmerjs_amd/node/kmerfinder.js, kmerjs_amd/kmerfinder.py)
 * between kmer_match_winner and kmer_match_remove.
 *
 * K-mers are byte strings of length k <= 32 over A/C/G/T (upper case).  A
 * query key of another length or with another byte never matches (the
 * reference compares strings).  Within one k-mer's template list, templates
 * are in ascending DB order; a template's duplicate k-mers count once
 * (the ETL's list(set(...)), src/kmerPyToMongo.py:23).
 */
#ifndef KMER_MATCH_H
#define KMER_MATCH_H

#include <stddef.h>
#include <stdint.h>

#include "kmer_api.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct kmer_db kmer_db;
typedef struct kmer_match kmer_match;

/* Template DB on `device`: n_keys k-mers (keys = n_keys * k bytes back to
 * back); template t owns keys [template_start[t], template_start[t + 1]),
 * template_start has n_templates + 1 entries (0 ... n_keys).
 * KMER_E_BAD_PARAM for k == 0 or k > 32, a byte outside A/C/G/T, or bad
 * offsets. */
kmer_status kmer_db_open(int32_t device, uint32_t k, const char *keys, uint64_t n_keys,
                         const uint64_t *template_start, uint32_t n_templates, kmer_db **out);
/* distinct = distinct k-mers, entries = (k-mer, template) pairs after dedup. */
kmer_status kmer_db_info(const kmer_db *db, uint32_t *k, uint32_t *n_templates, uint64_t *distinct,
                         uint64_t *entries);
/* Matches of the DB that are still open keep it alive: its device data is then
 * freed by the last kmer_match_close.  Do not pass `db` to any call afterwards
 * (offsets passed to kmer_match_open must start at 0 and not decrease:
 * KMER_E_BAD_PARAM otherwise). */
kmer_status kmer_db_close(kmer_db *db);

/* Round 1 (findKmersMatchesRedis): a query Map in iteration order — key i =
 * keys[offsets[i] .. offsets[i + 1]), counts[i] its value.  Scores every
 * template: uScore = query k-mers it holds, tScore = the sum of their counts;
 * hits = (k-mer, template) pairs.  The query is copied; the DB must outlive
 * the match. */
kmer_status kmer_match_open(kmer_db *db, const char *keys, const uint64_t *offsets, const uint64_t *counts,
                            uint64_t n, kmer_match **out);
/* The same from device memory (e.g. kmer_result_device of a count): n keys of
 * klen bytes back to back, uint64 counts.  `stream` (hipStream_t, NULL = the
 * legacy default stream): the match waits for the work queued on it so far. */
kmer_status kmer_match_open_device(kmer_db *db, const void *d_keys, uint32_t klen, const void *d_counts,
                                   uint64_t n, void *stream, kmer_match **out);
/* Current hits (sum of uScore) and templates with uScore > 0. */
kmer_status kmer_match_info(kmer_match *m, uint64_t *hits, uint32_t *n_templates);

enum { KMER_ORDER_FIRST_HIT = 0, KMER_ORDER_DB = 1 };
/* The templates with uScore > 0 and their current scores, in first-hit order
 * (the Redis path's templates Map) or DB order (the Mongo aggregation's).
 * Up to `cap` entries; *n = the number of such templates. */
kmer_status kmer_match_templates(kmer_match *m, uint32_t order, uint32_t cap, uint32_t *tmpl, uint64_t *uscore,
                                 uint64_t *tscore, uint32_t *n);

/* The round-1 query k-mers of template `tmpl` as query indices, ascending
 * (the `kmers` Set of its templates-Map entry, lib/kmerFinderServer.js:190-198).
 * Up to `cap` entries; *n = their number. */
kmer_status kmer_match_template_kmers(kmer_match *m, uint32_t tmpl, uint64_t cap, uint32_t *qidx, uint64_t *n);

typedef struct {
    uint32_t tmpl;          /* template index; UINT32_MAX when no template has hits */
    uint32_t reserved;
    uint64_t uscore, tscore; /* current scores of the winner */
    uint64_t hits;           /* current hits (results.hits of this round) */
    uint64_t first_uscore, first_tscore; /* its round-1 scores (kmerObject.firstMatches) */
} kmer_winner;
/* findWinner's pick: the largest uScore, ties to the earliest first hit. */
kmer_status kmer_match_winner(kmer_match *m, kmer_winner *w);
/* removeWinnerKmers(tmpl) + getMatches: every query k-mer of template `tmpl`
 * still in the query leaves it; all scores drop accordingly.  *hits = the
 * hits left. */
kmer_status kmer_match_remove(kmer_match *m, uint32_t tmpl, uint64_t *hits);
/* flags[i] = 1 iff query k-mer i was removed (n bytes). */
kmer_status kmer_match_removed(kmer_match *m, uint8_t *flags);
kmer_status kmer_match_close(kmer_match *m);

/* Message of the last failed kmer_db_* / kmer_match_* call on this thread. */
const char *kmer_match_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* KMER_MATCH_H */
