// mm_wave_util.h — wave-level helpers shared by the throughput kernels
// (trace_kernels.hip, trace_block.hip): per-wave counter flush and the fused
// per-pixel resolve.
#pragma once

#include "mm_launch.h"
#include "mm_trace.h"

namespace mm {

// Sum per-thread counters over the wave, one atomic per wave.
__device__ __forceinline__ void flush_stats(unsigned long long* stats, const Counters& c, uint32_t paths) {
    unsigned long long v[4] = {c.rays, c.visits, c.rtests, paths};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        unsigned long long x = v[i];
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
        v[i] = x;
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&stats[0], v[0]);
        atomicAdd(&stats[1], v[1]);
        atomicAdd(&stats[2], v[2]);
        atomicAdd(&stats[3], v[3]);
    }
}

// The per-pixel reduction of k_resolve done inside a wave: with 64 % spp == 0
// and chunks starting at multiples of 64, a wave's 64 paths are 64/spp whole
// pixels (lanes [p*spp, (p+1)*spp)).  spp % 8 == 0: pairwise tree in blocks of
// 8 by xor-shuffles (a+b == b+a exactly), blocks added left to right by the
// pixel's first lane; otherwise a left-to-right sum.  Then / spp -- the same
// operations in the same order as k_resolve, so the pixel is bit-identical.
// Called by all 64 lanes (uniform control flow); `valid` lanes' pixels written
// to out (the job's output, or its frame's slice of it in a multi-frame launch).
// Pixel pix of a launch's output: float4 (alpha 1, or += the frame value with
// MM_EXT_ACCUMULATE), or with MM_EXT_RGBA8 its texture-write conversion in 4
// bytes -- mm_quantize_rgba8's (k_quantize) on that float4, fused into the
// store so the float frame never goes to HBM.
__device__ __forceinline__ void store_pixel(const TileJob& job, void* __restrict__ out, size_t pix, F3 v) {
    if (job.e.flags & MM_EXT_RGBA8) {
        reinterpret_cast<uint32_t*>(out)[pix] =
            unorm8(v.x) | (unorm8(v.y) << 8) | (unorm8(v.z) << 16) | (unorm8(1.0f) << 24);
    } else if (job.e.flags & MM_EXT_ACCUMULATE) {
        float4* o = reinterpret_cast<float4*>(out) + pix;
        const float4 p = *o;
        *o = make_float4(p.x + v.x, p.y + v.y, p.z + v.z, p.w + 1.0f);
    } else {
        reinterpret_cast<float4*>(out)[pix] = make_float4(v.x, v.y, v.z, 1.0f);
    }
}

// The pixel's mean, sum / spp: when spp = 2^k as sum * 2^-k (both are the
// exact sum x 2^-k rounded once: the same float, without three IEEE divisions).
__device__ __forceinline__ F3 pixel_mean(F3 acc, uint32_t spp) {
    if ((spp & (spp - 1u)) == 0u) {
        const float r = __uint_as_float((127u - (31u - (uint32_t)__clz(spp))) << 23);  // 2^-log2(spp), exact
        return F3{acc.x * r, acc.y * r, acc.z * r};
    }
    const float m = (float)spp;
    return F3{acc.x / m, acc.y / m, acc.z / m};
}

// (out: the launch's output base; pixel path / spp + pix0 of it)
__device__ __forceinline__ void resolve_in_wave(const TileJob& job, F3 s, uint32_t path, bool valid,
                                                void* __restrict__ out, size_t pix0) {
    const uint32_t spp = job.e.spp, lane = threadIdx.x & 63u;
    F3 acc;
    if (spp % 8 == 0) {
        s = s + F3{__shfl_xor(s.x, 1), __shfl_xor(s.y, 1), __shfl_xor(s.z, 1)};
        s = s + F3{__shfl_xor(s.x, 2), __shfl_xor(s.y, 2), __shfl_xor(s.z, 2)};
        s = s + F3{__shfl_xor(s.x, 4), __shfl_xor(s.y, 4), __shfl_xor(s.z, 4)};
        acc = s;
        for (uint32_t b = 8; b < spp; b += 8)
            acc = acc + F3{__shfl(s.x, (int)(lane + b)), __shfl(s.y, (int)(lane + b)), __shfl(s.z, (int)(lane + b))};
    } else {
        acc = s;
        for (uint32_t k = 1; k < spp; ++k)
            acc = acc + F3{__shfl(s.x, (int)(lane + k)), __shfl(s.y, (int)(lane + k)), __shfl(s.z, (int)(lane + k))};
    }
    if (valid && (lane & (spp - 1)) == 0) store_pixel(job, out, pix0 + path / spp, pixel_mean(acc, spp));
}

}  // namespace mm
