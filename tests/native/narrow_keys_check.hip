// Host-side check of table mode's narrow keys (k <= 21, kmer_internal.hpp):
// for random windows w of every k, the key code of {w, rc w} is the same from
// either orientation, fits 41 bits, h = tab_mix_n(code) has 23 zero low bits
// and a 31-bit key below its partition (never the filler mark), the key round
// trips through the 32-bit form, tab_code(h) is w or rc w, and the digest key
// is tab_mix(min(code(w), code(rc w))) -- the wide keys' h, so the pinned
// digests hold for both.  Built and run by tests/test_narrow_keys.py.
#include "kmer_internal.hpp"
#include <cstdio>
#include <random>
using namespace kmerhip;
int main() {
    std::mt19937_64 g(1);
    long bad = 0, n = 0;
    for (uint32_t k = 1; k <= TAB_NARROW_K; ++k) {
        for (int it = 0; it < 100000; ++it, ++n) {
            const uint64_t cf = g() & ((1ull << (2 * k)) - 1);
            const uint64_t cr = tab_rc_code(cf, k);
            const uint64_t c = tab_canon_n(cf, cr, k);
            const uint64_t h = tab_mix_n(c);
            const uint32_t x = (uint32_t)(h >> TAB_NSH) & 0x7FFFFFFFu;
            const uint64_t code = tab_code(h, k, true, TAB_INV);
            const bool ok = tab_rc_code(cr, k) == cf && (c >> 41) == 0 && c == tab_canon_n(cr, cf, k) &&
                            (h & ((1ull << TAB_NSH) - 1)) == 0 && x != TAB_SENT32 &&
                            (((h >> 54) << 54) | ((uint64_t)x << TAB_NSH)) == h && (code == cf || code == cr) &&
                            tab_digest_key(h, k, true) == tab_mix(cf < cr ? cf : cr);
            if (!ok && bad++ < 5) printf("k %u w %llx\n", k, (unsigned long long)cf);
        }
    }
    printf("narrow keys: %ld of %ld bad\n", bad, n);
    return bad != 0;
}
