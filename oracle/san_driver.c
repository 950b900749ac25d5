/*
 * san_driver.c — runs the CPU restatement (kmer_oracle.c, compiled into this
 * one translation unit) under AddressSanitizer + UndefinedBehaviorSanitizer
 * (SURVEY.md §5 race/memory checks, host code only).  TEST INFRASTRUCTURE
 * ONLY, built by `make -C oracle san` into oracle/_san/ and driven by
 * tests/test_sanitizers.py.
 *
 * usage: san_driver FILE PREFIX K STEP  -> "n sum lines fnv" on stdout, where
 * fnv = FNV-1a 64 over every entry's key bytes, a 0 byte and the count's 8
 * little-endian bytes, in Map order.
 */
#include <stdio.h>

#include "kmer_oracle.c"

int main(int argc, char **argv) {
    if (argc != 5) {
        fprintf(stderr, "usage: %s FILE PREFIX K STEP\n", argv[0]);
        return 2;
    }
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 3;
    fseek(f, 0, SEEK_END);
    const long len = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *buf = (uint8_t *)malloc(len > 0 ? (size_t)len : 1);
    if (!buf || fread(buf, 1, (size_t)len, f) != (size_t)len) return 4;
    fclose(f);
    oracle_result r;
    memset(&r, 0, sizeof(r));
    const int st = oracle_count_buffer(buf, (size_t)len, (const uint8_t *)argv[2], strlen(argv[2]),
                                       (uint32_t)atoi(argv[3]), (uint32_t)atoi(argv[4]), &r);
    if (st) {
        printf("error %d\n", st);
        oracle_free(&r);
        free(buf);
        return 0;
    }
    uint64_t h = 1469598103934665603ull, sum = 0;
    for (uint64_t i = 0; i < r.n; ++i) {
        for (uint32_t j = 0; j < r.key_len[i]; ++j) h = (h ^ r.keys[r.key_off[i] + j]) * 1099511628211ull;
        h = (h ^ 0) * 1099511628211ull;
        for (int j = 0; j < 8; ++j) h = (h ^ ((r.counts[i] >> (8 * j)) & 0xFF)) * 1099511628211ull;
        sum += r.counts[i];
    }
    printf("%llu %llu %llu %llu\n", (unsigned long long)r.n, (unsigned long long)sum, (unsigned long long)r.lines,
           (unsigned long long)h);
    oracle_free(&r);
    free(buf);
    return 0;
}
