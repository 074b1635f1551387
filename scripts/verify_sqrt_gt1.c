/* Exhaustive check of the rejection-loop rewrite in shade_step (mm_trace.h):
 *     RN(sqrt(x)) > 1.0f   <=>   x > 0x1.000002p0f   (= 1 + 2^-23)
 * for every binary32 x (both signs, zeros, denormals, infinities, NaNs).
 * sqrtf is IEEE correctly rounded on x86-64 (sqrtss).
 * Build: gcc -O2 -ffp-contract=off verify_sqrt_gt1.c -lm && ./a.out */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

int main(void) {
    uint64_t bad = 0;
    for (uint64_t u = 0; u <= 0xFFFFFFFFull; ++u) {
        uint32_t b = (uint32_t)u;
        float x;
        memcpy(&x, &b, 4);
        volatile float vx = x;
        const int ref = sqrtf(vx) > 1.0f;
        const int got = x > 0x1.000002p0f;
        if (ref != got) {
            if (bad < 10) printf("mismatch x=%a ref=%d got=%d\n", x, ref, got);
            ++bad;
        }
    }
    printf("%llu mismatches over 2^32 inputs\n", (unsigned long long)bad);
    return bad != 0;
}
