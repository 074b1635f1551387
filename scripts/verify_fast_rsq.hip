// verify_fast_rsq.hip — exhaustive GPU checks of the exact fast forms of two
// IEEE operations on the path, compiled with the product library's flags
// (built by mirror-maze_amd/Makefile into lib/verify_fast_rsq, run by
// tests/test_gpu_arith.py):
//   rsq          mm::rsq (mm_device.h: hardware sqrt / rcp with exact
//                corrections on [2^-40, 2^40]) against the IEEE expansion
//                1.0f / sqrtf(x) -- the reference's fast_rsqrt with its IEEE
//                meaning -- for EVERY float x in [2^-44, 2^44] (the range and
//                4 binades either side, which take the IEEE path);
//   rcp_guarded  mm::rcp_guarded (mm_trace.h: one fma Newton step on v_rcp_f32,
//                the per-ray y = RN(1/d) the Markstein quotients read) against
//                1.0f / d for EVERY float d of either sign with |d| in
//                [2^-40, 2^40] (the guard's range; outside it y is never read);
//   ray_guard    mm::ray_fast_ok_boxed (mm_trace.h: the per-query guard in
//                integer form) against mm::ray_fast_ok for EVERY 32-bit
//                pattern on one axis of the direction (the others 1), and on
//                one axis of the origin wherever the grid box check can pass
//                (|o| <= 2^60, not NaN; grid_build.cpp builds no grid past it).
// Prints one line per check:  <name> checked <n> mismatches <m> [first 0x<bits>]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>

#include "mm_trace.h"

template <int kWhich>
__global__ void k_check(uint32_t lo, uint32_t hi, unsigned long long* bad, uint32_t* first) {
    const uint64_t n = (uint64_t)hi - lo + 1;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t b = lo + (uint32_t)i;
        const float x = __uint_as_float(b);
        bool diff;
        if constexpr (kWhich == 0) {
            diff = __float_as_uint(mm::rsq(x)) != __float_as_uint(mm::rsq_ieee(x));
        } else if constexpr (kWhich == 2) {
            mm::Ray rd{}, ro{};
            rd.o = mm::F3{1.0f, 1.0f, 1.0f};
            rd.d = mm::F3{1.0f, x, 1.0f};
            ro.o = mm::F3{1.0f, 1.0f, x};
            ro.d = mm::F3{1.0f, 1.0f, 1.0f};
            diff = mm::ray_fast_ok_boxed(rd) != mm::ray_fast_ok(rd);
            if (!(fabsf(x) > 0x1p60f) && x == x) diff |= mm::ray_fast_ok_boxed(ro) != mm::ray_fast_ok(ro);
        } else {
            const float a = mm::rcp_guarded(x), e = 1.0f / x;
            const float an = mm::rcp_guarded(-x), en = 1.0f / -x;
            diff = __float_as_uint(a) != __float_as_uint(e) || __float_as_uint(an) != __float_as_uint(en);
        }
        if (diff) {
            atomicAdd(bad, 1ull);
            atomicMin(first, b);
        }
    }
}

template <int kWhich>
static int check_bits(const char* name, uint32_t lo, uint32_t hi, unsigned long long* bad, uint32_t* first) {
    (void)hipMemset(bad, 0, 8);
    (void)hipMemset(first, 0xFF, 4);
    hipLaunchKernelGGL(k_check<kWhich>, dim3(65536), dim3(256), 0, 0, lo, hi, bad, first);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    unsigned long long h_bad = 0;
    uint32_t h_first = 0;
    (void)hipMemcpy(&h_bad, bad, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&h_first, first, 4, hipMemcpyDeviceToHost);
    printf("%s checked %llu mismatches %llu", name, (unsigned long long)hi - lo + 1, h_bad);
    if (h_bad) printf(" first 0x%08x", h_first);
    printf("\n");
    return h_bad ? 1 : 0;
}
template <int kWhich>
static int check(const char* name, float lo_f, float hi_f, unsigned long long* bad, uint32_t* first) {
    uint32_t lo, hi;
    memcpy(&lo, &lo_f, 4);
    memcpy(&hi, &hi_f, 4);
    return check_bits<kWhich>(name, lo, hi, bad, first);
}

int main() {
    unsigned long long* bad = nullptr;
    uint32_t* first = nullptr;
    if (hipMalloc(&bad, 8) != hipSuccess || hipMalloc(&first, 4) != hipSuccess) return 2;
    int rc = check<0>("rsq", 0x1p-44f, 0x1p44f, bad, first);
    rc |= check<1>("rcp_guarded", 0x1p-40f, 0x1p40f, bad, first);
    rc |= check_bits<2>("ray_guard", 0u, 0xFFFFFFFFu, bad, first);
    return rc;
}
