// probe_sqrt_exact.hip -- is the hardware v_sqrt_f32 (__builtin_amdgcn_sqrtf) already correctly rounded on
// [2^-40, 2^40], the range mm::rsq takes its fast form on (mm_device.h)?  If it is, rsq's two fma corrections
// of the square root could go.  Compares, for EVERY float x in the range, the bare hardware square root with
// the corrected one (mm::rsq's first half: the hardware root stepped down / up by one ulp where the residuals
// say so -- LLVM's correctly rounded expansion); and the bare v_rcp_f32 against rsq's Newton-corrected
// reciprocal on [2^-20, 2^20] (the square roots of that range).  Diagnostics only, not part of the product build:
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I mirror-maze_amd/csrc -I include scripts/probe_sqrt_exact.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__device__ __forceinline__ float sqrt_corrected(float x) {
    float s = __builtin_amdgcn_sqrtf(x);
    const float sd = __uint_as_float(__float_as_uint(s) - 1u), su = __uint_as_float(__float_as_uint(s) + 1u);
    const float vd = __builtin_fmaf(-sd, s, x), vu = __builtin_fmaf(-su, s, x);
    s = vd <= 0.0f ? sd : s;
    s = vu > 0.0f ? su : s;
    return s;
}

__device__ __forceinline__ float rcp_corrected(float s) {  // mm::rsq's second half (one fma Newton step)
    const float y = __builtin_amdgcn_rcpf(s);
    const float e = __builtin_fmaf(-s, y, 1.0f);
    return __builtin_fmaf(e, y, y);
}

template <int kWhich>
__global__ void k_probe(uint32_t lo, uint32_t hi, unsigned long long* bad, uint32_t* first) {
    const uint64_t n = (uint64_t)hi - lo + 1;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t b = lo + (uint32_t)i;
        const float x = __uint_as_float(b);
        const bool diff = kWhich == 0 ? __float_as_uint(__builtin_amdgcn_sqrtf(x)) != __float_as_uint(sqrt_corrected(x))
                                      : __float_as_uint(__builtin_amdgcn_rcpf(x)) != __float_as_uint(rcp_corrected(x));
        if (diff) {
            atomicAdd(bad, 1ull);
            atomicMin(first, b);
        }
    }
}

int main() {
    unsigned long long* bad;
    uint32_t* first;
    if (hipMalloc(&bad, 8) != hipSuccess || hipMalloc(&first, 4) != hipSuccess) return 2;
    auto run = [&](auto kern, const char* name, uint32_t lo, uint32_t hi) {
        (void)hipMemset(bad, 0, 8);
        (void)hipMemset(first, 0xFF, 4);
        hipLaunchKernelGGL(kern, dim3(65536), dim3(256), 0, 0, lo, hi, bad, first);
        if (hipDeviceSynchronize() != hipSuccess) return false;
        unsigned long long h_bad = 0;
        uint32_t h_first = 0;
        (void)hipMemcpy(&h_bad, bad, 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(&h_first, first, 4, hipMemcpyDeviceToHost);
        printf("%s checked %llu mismatches %llu first 0x%08x\n", name, (unsigned long long)hi - lo + 1, h_bad, h_first);
        return true;
    };
    if (!run(k_probe<0>, "sqrt_hw_vs_corrected [2^-40, 2^40]", 0x2B800000u, 0x53800000u)) return 3;
    if (!run(k_probe<1>, "rcp_hw_vs_corrected [2^-20, 2^20]", 0x35800000u, 0x49800000u)) return 3;
    return 0;
}
