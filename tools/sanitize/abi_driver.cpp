// abi_driver.cpp -- drives the C-ABI (include/kmer_api.h) under a host-side
// AddressSanitizer + UBSan build of libkmerhip (tools/sanitize_abi.sh; SURVEY.md
// §5).  For every input file and configuration it counts with one context,
// with a 3-way device group (ordinal 0 repeated: one host thread per shard)
// and through kmer_count_file, and requires the three results to be equal.
// Exit status 0 = every case equal and no sanitizer report.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "kmer_api.h"

static uint64_t fnv(const kmer_result *r) {
    uint64_t h = 1469598103934665603ull;
    const uint64_t n = kmer_result_size(r);
    for (uint64_t i = 0; i < n; ++i) {
        const char *key = nullptr;
        uint32_t klen = 0;
        uint64_t cnt = 0;
        if (kmer_result_get(r, i, &key, &klen, &cnt) != KMER_OK) return 0;
        for (uint32_t j = 0; j < klen; ++j) h = (h ^ (uint8_t)key[j]) * 1099511628211ull;
        h = (h ^ 0) * 1099511628211ull;
        for (int j = 0; j < 8; ++j) h = (h ^ ((cnt >> (8 * j)) & 0xFF)) * 1099511628211ull;
    }
    return (h ^ kmer_result_lines(r)) * 1099511628211ull;
}

struct Cfg {
    const char *prefix;
    uint32_t k, step, flags;
};

int main(int argc, char **argv) {
    const Cfg cfgs[] = {{"ATGAC", 16, 1, 0}, {"", 16, 1, 0}, {"", 31, 1, KMER_FLAG_UNORDERED},
                        {"", 21, 1, KMER_FLAG_CANONICAL}, {"N", 5, 1, 0}, {"AT", 21, 2, 0}, {"ACG", 40, 1, 0}};
    int bad = 0, cases = 0;
    for (int a = 1; a < argc; ++a) {
        FILE *f = fopen(argv[a], "rb");
        if (!f) return 3;
        std::vector<uint8_t> data;
        uint8_t tmp[1 << 16];
        size_t got;
        while ((got = fread(tmp, 1, sizeof(tmp), f)) > 0) data.insert(data.end(), tmp, tmp + got);
        fclose(f);
        for (const Cfg &c : cfgs) {
            uint64_t d[3] = {0, 0, 0};
            kmer_status st[3] = {KMER_OK, KMER_OK, KMER_OK};
            for (int v = 0; v < 3; ++v) {
                const int32_t devs[3] = {0, 0, 0};
                kmer_params p;
                memset(&p, 0, sizeof(p));
                p.k = c.k;
                p.step = c.step;
                p.prefix = (const uint8_t *)c.prefix;
                p.prefix_len = (uint32_t)strlen(c.prefix);
                p.flags = c.flags;
                p.batch_bytes = v == 2 ? 4096 : 0;          // count_file in small batches
                if (v == 1) {
                    p.ndev = 3;
                    p.devices = devs;
                }
                kmer_ctx *ctx = nullptr;
                st[v] = kmer_open(&p, &ctx);
                if (st[v] != KMER_OK) continue;
                kmer_result *r = nullptr;
                st[v] = v == 2 ? kmer_count_file(ctx, argv[a], &r) : kmer_count_buffer(ctx, data.data(), data.size(), &r);
                if (st[v] == KMER_OK) d[v] = fnv(r);
                kmer_result_free(r);
                kmer_close(ctx);
            }
            ++cases;
            if (st[0] != KMER_OK || st[0] != st[1] || st[0] != st[2] || d[0] != d[1] || d[0] != d[2]) {
                ++bad;
                fprintf(stderr, "MISMATCH %s '%s' k=%u step=%u flags=%u: st %d %d %d digest %llx %llx %llx\n", argv[a],
                        c.prefix, c.k, c.step, c.flags, st[0], st[1], st[2], (unsigned long long)d[0],
                        (unsigned long long)d[1], (unsigned long long)d[2]);
            }
        }
    }
    printf("abi_driver: %d cases, %d mismatches\n", cases, bad);
    return bad ? 1 : 0;
}
