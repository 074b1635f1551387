/* Empirical check that the Markstein correction with a correctly rounded
 * reciprocal reproduces IEEE binary32 division exactly:
 *     y = RN(1/d); q = RN(a*y); r = fma(-q, d, a); q' = fma(r, y, q) == RN(a/d)
 * for |d| in [2^-60, 2^60] and a = 0 or |a| in [2^-100, 2^100].
 * Sweeps every d mantissa (2^23) against a set of a mantissas per d, plus
 * random exponents.  Build: gcc -O2 -ffp-contract=off -mfma verify_markstein.c -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>

static inline float bits2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t f2bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static uint64_t s = 0x9E3779B97F4A7C15ull;
static inline uint32_t rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (uint32_t)(s >> 11); }

int main(int argc, char** argv) {
    long per_d = argc > 1 ? atol(argv[1]) : 64;
    uint64_t tested = 0, bad = 0;
    for (uint32_t m = 0; m < (1u << 23); ++m) {
        int ed = (int)(rnd() % 121) - 60;                /* d exponent in [-60, 60] */
        float d = bits2f(((uint32_t)(127 + ed) << 23) | m);
        if (rnd() & 1) d = -d;
        volatile float one = 1.0f;
        float y = one / d;
        for (long k = 0; k < per_d; ++k) {
            uint32_t am;
            switch (k) {
                case 0: am = 0; break;               /* a mantissa 1.0   */
                case 1: am = 0x7FFFFF; break;        /* all ones         */
                case 2: am = m; break;               /* a = d (q = 1)    */
                case 3: am = (m + 1) & 0x7FFFFF; break;
                default: am = rnd() & 0x7FFFFF;
            }
            int ea = (int)(rnd() % 125) - 63;           /* a exponent in [-63, 61] */
            float a = bits2f(((uint32_t)(127 + ea) << 23) | am);
            if (rnd() & 1) a = -a;
            volatile float av = a, dv = d;
            float want = av / dv;
            float q = a * y;
            float r = fmaf(-q, d, a);
            float q2 = fmaf(r, y, q);
            ++tested;
            if (f2bits(q2) != f2bits(want)) {
                if (bad < 10) printf("MISMATCH a=%a d=%a want=%a got=%a\n", a, d, want, q2);
                ++bad;
            }
        }
    }
    printf("tested %llu pairs, mismatches %llu\n", (unsigned long long)tested, (unsigned long long)bad);
    return bad != 0;
}
