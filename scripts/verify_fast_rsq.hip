// verify_fast_rsq.hip — exhaustive GPU check that mm::rsq (mm_device.h: the
// hardware sqrt / rcp with exact corrections on [2^-40, 2^40]) returns the bits
// of the IEEE expansion 1.0f / sqrtf(x) -- the reference's fast_rsqrt with its
// IEEE meaning -- for EVERY float x in [2^-40, 2^40], plus a margin of binades
// either side (which take the IEEE path and must match trivially), compiled
// with the product library's flags.  Built by mirror-maze_amd/Makefile into
// lib/verify_fast_rsq; run by tests/test_gpu_arith.py.  Prints one line:
//   checked <n> mismatches <m> [first <hex x> fast <hex> ieee <hex>]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <cstring>

#include "mm_device.h"

__global__ void k_check(uint32_t lo, uint32_t hi, unsigned long long* bad, uint32_t* first) {
    const uint64_t n = (uint64_t)hi - lo + 1;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t b = lo + (uint32_t)i;
        const float x = __uint_as_float(b);
        const float f = mm::rsq(x), e = mm::rsq_ieee(x);
        if (__float_as_uint(f) != __float_as_uint(e)) {
            atomicAdd(bad, 1ull);
            atomicMin(first, b);
        }
    }
}

int main() {
    unsigned long long* bad = nullptr;
    uint32_t* first = nullptr;
    if (hipMalloc(&bad, 8) != hipSuccess || hipMalloc(&first, 4) != hipSuccess) return 2;
    (void)hipMemset(bad, 0, 8);
    (void)hipMemset(first, 0xFF, 4);
    float lo_f = 0x1p-44f, hi_f = 0x1p44f;  // the fast range [2^-40, 2^40] and 4 binades either side
    uint32_t lo, hi;
    memcpy(&lo, &lo_f, 4);
    memcpy(&hi, &hi_f, 4);
    hipLaunchKernelGGL(k_check, dim3(65536), dim3(256), 0, 0, lo, hi, bad, first);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    unsigned long long h_bad = 0;
    uint32_t h_first = 0;
    (void)hipMemcpy(&h_bad, bad, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&h_first, first, 4, hipMemcpyDeviceToHost);
    printf("checked %llu mismatches %llu", (unsigned long long)hi - lo + 1, h_bad);
    if (h_bad) printf(" first 0x%08x", h_first);
    printf("\n");
    return h_bad ? 1 : 0;
}
