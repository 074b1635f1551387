// isa_dual.hip — microbenchmark: VALU issue rate and dual issue per
// instruction form on gfx950, for the trace kernel's issue attribution
// (DESIGN.md §10).  A SIMD-32 runs a wave64 VALU op in
// two clocks, so the SIMD reaches its peak only by issuing two VALU ops (from
// two waves) in one quad-cycle -- SQ_ACTIVE_INST_VALU2 counts those quads.
// Each kernel runs one instruction form on 8 independent accumulators per
// lane at 8 waves per SIMD over the whole chip; under
//   rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE ...
// its counters give the form's dual-issue share, and its time the clocks per
// wave64 instruction per SIMD.  Diagnostics only (not part of the library).
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/isa_dual scripts/isa_dual.hip && /tmp/isa_dual
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 256;  // x 16 steps x 8 instructions per lane

#define ACC "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
#define IN "v"(k1), "v"(k2), "s"(m), "s"(ks)
// %0..%7 accumulators, %8 %9 VGPR operands, %10 SGPR pair, %11 SGPR
#define EIGHT(T) T(0) T(1) T(2) T(3) T(4) T(5) T(6) T(7)

#define F_ADD(n) "v_add_f32 %" #n ", %" #n ", %8\n\t"
#define F_MUL(n) "v_mul_f32 %" #n ", %" #n ", %8\n\t"
#define F_FMA(n) "v_fma_f32 %" #n ", %" #n ", %8, %9\n\t"
#define F_FMAC(n) "v_fmac_f32 %" #n ", %8, %9\n\t"
#define F_FMA_S(n) "v_fma_f32 %" #n ", %" #n ", %11, %9\n\t"
#define F_SUB_S(n) "v_sub_f32 %" #n ", %11, %" #n "\n\t"
#define F_ADDU(n) "v_add_u32 %" #n ", %" #n ", %8\n\t"
#define F_LSHLADD(n) "v_lshl_add_u32 %" #n ", %" #n ", 1, %8\n\t"
#define F_AND(n) "v_and_b32 %" #n ", %" #n ", %8\n\t"
#define F_MOV(n) "v_mov_b32 %" #n ", %8\n\t"
#define F_CND_VCC(n) "v_cndmask_b32 %" #n ", %" #n ", %8, vcc\n\t"
#define F_CND_E64(n) "v_cndmask_b32_e64 %" #n ", %" #n ", %8, %10\n\t"
#define F_CMP_VCC(n) "v_cmp_lt_f32 vcc, %" #n ", %8\n\t"
#define F_CMP_E64(n) "v_cmp_lt_f32_e64 s[40:41], %" #n ", %8\n\t"
#define F_RFL(n) "v_readfirstlane_b32 s40, %" #n "\n\t"
#define F_CVT(n) "v_cvt_f32_i32 %" #n ", %" #n "\n\t"
#define F_MIN3(n) "v_min3_f32 %" #n ", %" #n ", %8, %9\n\t"
#define F_BFE(n) "v_bfe_u32 %" #n ", %" #n ", 3, 3\n\t"
#define F_RCP(n) "v_rcp_f32 %" #n ", %" #n "\n\t"
#define F_MULLO(n) "v_mul_lo_u32 %" #n ", %" #n ", %8\n\t"
#define F_LSHL_K(n) "v_lshlrev_b32 %" #n ", 4, %" #n "\n\t"
#define F_ADD_K(n) "v_add_u32 %" #n ", 2, %" #n "\n\t"
#define F_AND_LIT(n) "v_and_b32 %" #n ", 0x3f0, %" #n "\n\t"
#define F_MIN(n) "v_min_f32 %" #n ", %" #n ", %8\n\t"
#define F_SUB(n) "v_sub_f32 %" #n ", %" #n ", %8\n\t"
#define F_XOR(n) "v_xor_b32 %" #n ", %" #n ", %8\n\t"
#define F_LSHR_V(n) "v_lshrrev_b32 %" #n ", %8, %" #n "\n\t"
#define F_LSHL_V(n) "v_lshlrev_b32 %" #n ", %8, %" #n "\n\t"
#define F_LSHR_K(n) "v_lshrrev_b32 %" #n ", 4, %" #n "\n\t"
#define F_ADDU_LIT(n) "v_add_u32 %" #n ", 0xd4800000, %" #n "\n\t"
#define F_ADDU_SELF(n) "v_add_u32 %" #n ", %" #n ", %" #n "\n\t"
#define F_MAX3U(n) "v_max3_u32 %" #n ", %" #n ", %8, %9\n\t"
#define F_OR3(n) "v_or3_b32 %" #n ", %" #n ", %8, %9\n\t"
#define F_OR(n) "v_or_b32 %" #n ", %" #n ", %8\n\t"
#define F_MULU24(n) "v_mul_u32_u24 %" #n ", %" #n ", %8\n\t"
#define F_FMA_NEG(n) "v_fma_f32 %" #n ", -%" #n ", %8, %9\n\t"
#define F_MUL_K(n) "v_mul_f32 %" #n ", 0x3dcccccd, %" #n "\n\t"
#define F_ADDCO(n) "v_add_co_u32 %" #n ", vcc, %" #n ", %8\n\t"
#define F_CNDV(n) "v_cmp_lt_f32 vcc, %" #n ", %8\n\tv_cndmask_b32 %" #n ", %" #n ", %9, vcc\n\t"
#define F_MIX_SS(n) "v_cmp_lt_f32 vcc, %" #n ", %8\n\tv_cndmask_b32_e64 %" #n ", %" #n ", %9, %10\n\t"
#define F_MIX(n) "v_fma_f32 %" #n ", %" #n ", %8, %9\n\tv_add_f32 %" #n ", %" #n ", %8\n\t"
#define F_MIX_CMP(n) "v_cmp_lt_f32 vcc, %" #n ", %8\n\tv_add_f32 %" #n ", %" #n ", %8\n\t"

#define KERNEL(NAME, PRE, T)                                                                       \
    __global__ __launch_bounds__(256) void NAME(float* out, float seed, unsigned long long m, float ks) { \
        float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;                       \
        float a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                  \
        const float k1 = seed * 0.5f, k2 = seed * 0.25f;                                           \
        for (int i = 0; i < kIters; ++i) {                                                         \
            for (int s = 0; s < 16; ++s)                                                           \
                asm volatile(PRE EIGHT(T) : ACC : IN : "vcc", "s40", "s41");                        \
        }                                                                                          \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;        \
    }

KERNEL(d_add_f32, "", F_ADD)
KERNEL(d_mul_f32, "", F_MUL)
KERNEL(d_fma_f32, "", F_FMA)
KERNEL(d_fmac_f32, "", F_FMAC)
KERNEL(d_fma_f32_sgpr, "", F_FMA_S)
KERNEL(d_sub_f32_sgpr, "", F_SUB_S)
KERNEL(d_add_u32, "", F_ADDU)
KERNEL(d_lshl_add_u32, "", F_LSHLADD)
KERNEL(d_and_b32, "", F_AND)
KERNEL(d_mov_b32, "", F_MOV)
KERNEL(d_cndmask_vcc, "s_mov_b64 vcc, %10\n\t", F_CND_VCC)
KERNEL(d_cndmask_e64, "", F_CND_E64)
KERNEL(d_cmp_vcc, "", F_CMP_VCC)
KERNEL(d_cmp_e64, "", F_CMP_E64)
KERNEL(d_readfirstlane, "", F_RFL)
KERNEL(d_cvt_f32_i32, "", F_CVT)
KERNEL(d_min3_f32, "", F_MIN3)
KERNEL(d_bfe_u32, "", F_BFE)
KERNEL(d_rcp_f32, "", F_RCP)
KERNEL(d_mul_lo_u32, "", F_MULLO)
KERNEL(d_lshl_k, "", F_LSHL_K)
KERNEL(d_add_k, "", F_ADD_K)
KERNEL(d_and_lit, "", F_AND_LIT)
KERNEL(d_min_f32, "", F_MIN)
KERNEL(d_sub_f32, "", F_SUB)
KERNEL(d_xor_b32, "", F_XOR)
KERNEL(d_lshr_v, "", F_LSHR_V)
KERNEL(d_fma_neg, "", F_FMA_NEG)
KERNEL(d_lshl_v, "", F_LSHL_V)
KERNEL(d_lshr_k, "", F_LSHR_K)
KERNEL(d_addu_lit, "", F_ADDU_LIT)
KERNEL(d_addu_self, "", F_ADDU_SELF)
KERNEL(d_max3_u32, "", F_MAX3U)
KERNEL(d_or3_b32, "", F_OR3)
KERNEL(d_or_b32, "", F_OR)
KERNEL(d_mul_u24, "", F_MULU24)
KERNEL(d_mul_lit, "", F_MUL_K)
KERNEL(d_add_co, "", F_ADDCO)
KERNEL(d_cmp_cnd, "", F_CNDV)
KERNEL(d_mix_cmp_cnd64, "", F_MIX_SS)
KERNEL(d_mix_fma_add, "", F_MIX)
KERNEL(d_mix_cmp_add, "", F_MIX_CMP)

typedef void (*kfn)(float*, float, unsigned long long, float);

static float run(kfn k, float* out, int blocks) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 0.75f, 0x5555555555555555ull, 1.5f);  // warm
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < 5; ++r)
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, 0.75f, 0x5555555555555555ull, 1.5f);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return ms / 5;
}

int main() {
    int cus = 0, clk_khz = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    (void)hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
    const int blocks = cus * 8;  // 8 blocks x 4 waves = 8 waves per SIMD
    float* out = nullptr;
    (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
    struct Row { const char* name; kfn k; int per; } rows[] = {
        {"v_add_f32", d_add_f32, 1}, {"v_mul_f32", d_mul_f32, 1}, {"v_fma_f32", d_fma_f32, 1},
        {"v_fmac_f32", d_fmac_f32, 1}, {"v_fma_f32 (sgpr src)", d_fma_f32_sgpr, 1},
        {"v_sub_f32 (sgpr src)", d_sub_f32_sgpr, 1}, {"v_add_u32", d_add_u32, 1},
        {"v_lshl_add_u32", d_lshl_add_u32, 1}, {"v_and_b32", d_and_b32, 1}, {"v_mov_b32", d_mov_b32, 1},
        {"v_cndmask_b32 vcc", d_cndmask_vcc, 1}, {"v_cndmask_b32_e64 s[]", d_cndmask_e64, 1},
        {"v_cmp_lt_f32 vcc", d_cmp_vcc, 1}, {"v_cmp_lt_f32_e64 s[]", d_cmp_e64, 1},
        {"v_readfirstlane_b32", d_readfirstlane, 1}, {"v_cvt_f32_i32", d_cvt_f32_i32, 1},
        {"v_min3_f32", d_min3_f32, 1}, {"v_bfe_u32", d_bfe_u32, 1}, {"v_rcp_f32", d_rcp_f32, 1},
        {"v_mul_lo_u32", d_mul_lo_u32, 1}, {"v_lshlrev_b32 inline k", d_lshl_k, 1},
        {"v_add_u32 inline k", d_add_k, 1}, {"v_and_b32 literal", d_and_lit, 1}, {"v_min_f32", d_min_f32, 1},
        {"v_sub_f32", d_sub_f32, 1}, {"v_xor_b32", d_xor_b32, 1}, {"v_lshrrev_b32 vgpr", d_lshr_v, 1},
        {"v_fma_f32 neg src", d_fma_neg, 1}, {"v_mul_f32 literal", d_mul_lit, 1},
        {"v_add_co_u32 (vcc out)", d_add_co, 1}, {"cmp vcc + cndmask vcc", d_cmp_cnd, 2},
        {"cmp vcc + cndmask_e64", d_mix_cmp_cnd64, 2},
        {"fma + add", d_mix_fma_add, 2}, {"cmp vcc + add", d_mix_cmp_add, 2},
        {"v_lshlrev_b32 vgpr", d_lshl_v, 1}, {"v_lshrrev_b32 inline k", d_lshr_k, 1},
        {"v_add_u32 literal", d_addu_lit, 1}, {"v_add_u32 x + x", d_addu_self, 1}, {"v_max3_u32", d_max3_u32, 1},
        {"v_or3_b32", d_or3_b32, 1}, {"v_or_b32", d_or_b32, 1}, {"v_mul_u32_u24", d_mul_u24, 1},
    };
    printf("%d CUs, %d blocks x 256 threads (8 waves per SIMD), %d VALU per lane per kernel; clock attr %d MHz\n",
           cus, blocks, kIters * 16 * 8, clk_khz / 1000);
    const double waves_per_simd = 8.0;
    for (auto& r : rows) {
        const float ms = run(r.k, out, blocks);
        const double instr = (double)kIters * 16 * 8 * r.per * waves_per_simd;  // wave-instructions per SIMD
        const double clocks = ms * 1e-3 * 2.4e9;  // at the 2.4 GHz peak clock
        printf("%-24s %8.3f ms  %5.2f clocks per wave64 VALU op per SIMD (2.00 = dual issue every quad)\n", r.name,
               ms, clocks / instr);
    }
    (void)hipFree(out);
    return 0;
}
