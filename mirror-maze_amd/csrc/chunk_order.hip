// chunk_order.hip — longest-first chunk order for the wave-persistent kernel
// (MM_OPT_CHUNK_ORDER).
//
// A launch ends when its last wave finishes its last 64-path chunk; with the
// queue in pixel order the waves that drew expensive chunks late run alone for
// up to ~0.4 ms (profiles/r01_timeline_probe.txt).  Handing out the chunks
// longest first (LPT scheduling) leaves the cheap ones for the end.  The
// durations come from the previous launch of the same tile (the kernel writes
// cost[chunk]); frame-to-frame they differ only by the per-frame RNG.
//
// Sort: a counting sort on 512 bins of 1/16 octave (float exponent and top 4
// mantissa bits of the duration), descending.  Two launches: a histogram
// (LDS bins, one global atomic per non-empty bin and block), then a scatter
// (each block scans the global histogram, reserves its range per bin with one
// global atomic, and places its chunks by LDS rank).  Order within a bin
// depends on block timing; any permutation gives the same samples.
#include <hip/hip_runtime.h>

#include "mm_launch.h"

namespace mm {

namespace {

constexpr uint32_t kBins = 512;
constexpr uint32_t kThreads = 256;
constexpr uint32_t kPerThread = 4;
constexpr uint32_t kPerBlock = kThreads * kPerThread;

// descending: bin 0 holds the longest chunks
__device__ __forceinline__ uint32_t cost_bin(uint32_t c) {
    const uint32_t b = (__float_as_uint((float)(c | 1u)) >> 19) - (127u << 4);  // c >= 1: exponent >= 127
    return kBins - 1u - min(b, kBins - 1u);
}

__global__ __launch_bounds__(kThreads) void k_order_hist(const uint32_t* __restrict__ cost, uint32_t n,
                                                         uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[kBins];
    for (uint32_t i = threadIdx.x; i < kBins; i += kThreads) h[i] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * kPerBlock;
    for (uint32_t k = 0; k < kPerThread; ++k) {
        const uint32_t e = base + k * kThreads + threadIdx.x;
        if (e < n) atomicAdd(&h[cost_bin(cost[e])], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < kBins; i += kThreads)
        if (h[i]) atomicAdd(&hist[i], h[i]);
}

__global__ __launch_bounds__(kThreads) void k_order_scatter(const uint32_t* __restrict__ cost, uint32_t n,
                                                            const uint32_t* __restrict__ hist,
                                                            uint32_t* __restrict__ cursor,
                                                            uint32_t* __restrict__ order) {
    __shared__ uint32_t start[kBins];  // exclusive prefix of hist, then + this block's reservation
    __shared__ uint32_t cnt[kBins];
    // exclusive scan of the 512 global bins: two per thread, Hillis-Steele on the pair sums
    __shared__ uint32_t pair[kThreads];
    const uint32_t t = threadIdx.x;
    const uint32_t h0 = hist[2 * t], h1 = hist[2 * t + 1];
    pair[t] = h0 + h1;
    cnt[2 * t] = 0;
    cnt[2 * t + 1] = 0;
    __syncthreads();
    for (uint32_t off = 1; off < kThreads; off <<= 1) {
        const uint32_t v = t >= off ? pair[t - off] : 0u;
        __syncthreads();
        pair[t] += v;
        __syncthreads();
    }
    const uint32_t excl = pair[t] - (h0 + h1);
    start[2 * t] = excl;
    start[2 * t + 1] = excl + h0;
    uint32_t bin[kPerThread], rank[kPerThread];
    const uint32_t base = blockIdx.x * kPerBlock;
    for (uint32_t k = 0; k < kPerThread; ++k) {
        const uint32_t e = base + k * kThreads + t;
        bin[k] = e < n ? cost_bin(cost[e]) : kBins;
        rank[k] = bin[k] < kBins ? atomicAdd(&cnt[bin[k]], 1u) : 0u;
    }
    __syncthreads();
    for (uint32_t i = t; i < kBins; i += kThreads)
        if (cnt[i]) start[i] += atomicAdd(&cursor[i], cnt[i]);
    __syncthreads();
    for (uint32_t k = 0; k < kPerThread; ++k)
        if (bin[k] < kBins) order[start[bin[k]] + rank[k]] = base + k * kThreads + t;
}

}  // namespace

hipError_t launch_chunk_order(const uint32_t* cost, uint32_t n, uint32_t* order, uint32_t* tmp, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(tmp, 0, 2 * kBins * sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    const uint32_t grid = (n + kPerBlock - 1) / kPerBlock;
    hipLaunchKernelGGL(k_order_hist, dim3(grid), dim3(kThreads), 0, s, cost, n, tmp);
    hipLaunchKernelGGL(k_order_scatter, dim3(grid), dim3(kThreads), 0, s, cost, n, tmp, tmp + kBins, order);
    return hipGetLastError();
}

}  // namespace mm
