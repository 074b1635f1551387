// isa_rates.hip — microbenchmark: issue cost of the VALU instructions the
// trace kernel's hot loops use (v_mul_lo_u32 in the RNG, v_sqrt / v_rcp in
// the correctly rounded sqrt and divide, v_cvt_f32_u32, v_cndmask), relative
// to v_add_u32.  Each kernel runs a dependent-free unrolled loop of one
// instruction kind at full occupancy; the time per instruction per wave gives
// the rate.  Diagnostics only (not part of the product library).
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/isa_rates scripts/isa_rates.hip && /tmp/isa_rates
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 4096;

#define KERNEL(NAME, T, INIT, OP)                                                         \
    __global__ __launch_bounds__(256) void NAME(T* out, T seed) {                         \
        T a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;                 \
        T a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                            \
        INIT;                                                                             \
        for (int i = 0; i < kIters; ++i) {                                                \
            OP(a0); OP(a1); OP(a2); OP(a3); OP(a4); OP(a5); OP(a6); OP(a7);               \
        }                                                                                 \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7; \
    }

#define OP_ADD(a) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(k))
#define OP_MUL(a) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a) : "v"(k))
#define OP_MUL24(a) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a) : "v"(k))
#define OP_CVT(a) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a))
#define OP_FMUL(a) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a) : "v"(kf))
#define OP_FMA(a) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a) : "v"(kf))
#define OP_SQRT(a) asm volatile("v_sqrt_f32 %0, %0" : "+v"(a))
#define OP_RCP(a) asm volatile("v_rcp_f32 %0, %0" : "+v"(a))
#define OP_RSQ(a) asm volatile("v_rsq_f32 %0, %0" : "+v"(a))
#define OP_CND(a) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a) : "v"(k))
#define OP_PKMUL(a) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(a) : "v"(kf2))

KERNEL(k_add, unsigned, const unsigned k = seed | 1u, OP_ADD)
KERNEL(k_mul, unsigned, const unsigned k = seed | 1u, OP_MUL)
KERNEL(k_mul24, unsigned, const unsigned k = seed | 1u, OP_MUL24)
KERNEL(k_cvt, unsigned, , OP_CVT)
KERNEL(k_fmul, float, const float kf = seed * 0.5f, OP_FMUL)
KERNEL(k_fma, float, const float kf = seed * 0.5f, OP_FMA)
KERNEL(k_sqrt, float, , OP_SQRT)
KERNEL(k_rcp, float, , OP_RCP)
KERNEL(k_rsq, float, , OP_RSQ)
KERNEL(k_cnd, unsigned, const unsigned k = seed | 1u, OP_CND)

template <typename K, typename T>
float run(K kern, T* out, T seed, int blocks) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, seed);  // warm
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, seed);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 8;  // 8 blocks x 4 waves = 8 waves per SIMD
    void* out = nullptr;
    (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
    const double waves = blocks * 4.0, instr = 8.0 * kIters;
    struct { const char* name; float ms; } rows[] = {
        {"v_add_u32", run(k_add, (unsigned*)out, 3u, blocks)},
        {"v_mul_lo_u32", run(k_mul, (unsigned*)out, 3u, blocks)},
        {"v_mul_u32_u24", run(k_mul24, (unsigned*)out, 3u, blocks)},
        {"v_cvt_f32_u32", run(k_cvt, (unsigned*)out, 3u, blocks)},
        {"v_mul_f32", run(k_fmul, (float*)out, 0.75f, blocks)},
        {"v_fma_f32", run(k_fma, (float*)out, 0.75f, blocks)},
        {"v_sqrt_f32", run(k_sqrt, (float*)out, 0.75f, blocks)},
        {"v_rcp_f32", run(k_rcp, (float*)out, 0.75f, blocks)},
        {"v_rsq_f32", run(k_rsq, (float*)out, 0.75f, blocks)},
        {"v_cndmask_b32", run(k_cnd, (unsigned*)out, 3u, blocks)},
    };
    const float base = rows[0].ms;
    printf("%d CUs, %d blocks x 256 threads, %d x 8 instructions per thread\n", cus, blocks, kIters);
    for (auto& r : rows) {
        // cycles per wave-instruction per SIMD at the 2.4 GHz peak clock
        const double cyc = r.ms * 1e-3 * 2.4e9 * (cus * 4.0) / (waves * instr);
        printf("%-14s %8.3f ms  %5.2f x add  ~%5.2f SIMD cycles per wave64 instruction\n", r.name, r.ms, r.ms / base, cyc);
    }
    (void)hipFree(out);
    return 0;
}
