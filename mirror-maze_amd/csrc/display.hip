// display.hip — the stages either side of the trace kernels in the reference's
// frame (src/main.rs:860-894): the presentation blur, the streaming packet
// format and the RGBA8 quantisation of offline frames.
//
//   k_present_blur   fragment_shader (src/shaders.metal:214-225), re-specified
//                    as a Jacobi step (read the old texture, write a new one;
//                    out-of-range neighbours read as 0).  The reference blurs
//                    the texture in place from concurrent fragments, which is
//                    a race; double-buffering makes every frame deterministic.
//                    Operation order of the compiled IR (src/shaders.ir,
//                    fragment_shader): c = (((L + R) + D) + U) * 0.5 + C,
//                    then c * RN(1/3); alpha written as 1.
//   k_chunk_packets  the per-pixel packet of the shaders.air revision of
//                    compute_shader (extra `device float4* pixel_data`):
//                    (rgb, bitcast(x << 16 | y)) at chunk * 16 + pn.
//   k_quantize       float RGBA -> RGBA8 with the texture-write conversion.
// All three are HBM-bound byte streams (4-20 B per pixel).
#include <hip/hip_runtime.h>

#include "mm_launch.h"

namespace mm {

namespace {

// RGBA8Unorm texel -> float, c / 255 (IEEE division, as Metal's unorm read)
__device__ __forceinline__ F3 texel(const uint32_t* __restrict__ tex, int x, int y, int W, int H) {
    if (x < 0 || y < 0 || x >= W || y >= H) return F3{0.0f, 0.0f, 0.0f};
    const uint32_t p = tex[(size_t)y * W + x];
    return F3{(float)(p & 0xFFu) / 255.0f, (float)((p >> 8) & 0xFFu) / 255.0f, (float)((p >> 16) & 0xFFu) / 255.0f};
}

__global__ void k_present_blur(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, int W, int H) {
    const int x = (int)(blockIdx.x * blockDim.x + threadIdx.x), y = (int)(blockIdx.y * blockDim.y + threadIdx.y);
    if (x >= W || y >= H) return;
    const F3 c = texel(in, x, y, W, H);
    const F3 r = texel(in, x + 1, y, W, H), l = texel(in, x - 1, y, W, H);
    const F3 d = texel(in, x, y + 1, W, H), u = texel(in, x, y - 1, W, H);
    F3 s = ((l + r) + d) + u;
    s = 0.5f * s;
    s = s + c;
    s = 0x1.555556p-2f * s;  // fdiv by 3.0 folded to a multiply in the IR
    out[(size_t)y * W + x] = unorm8(s.x) | (unorm8(s.y) << 8) | (unorm8(s.z) << 16) | (255u << 24);
}

__global__ void k_chunk_packets(const float4* __restrict__ fb, const uint32_t* __restrict__ chunks,
                                uint32_t n_chunks, uint32_t W, uint32_t H, float4* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_chunks * 16u) return;
    const uint32_t ch = i >> 4, pn = i & 15u;
    const uint32_t x = chunks[2 * ch] + pn / 4u, y = chunks[2 * ch + 1] + pn % 4u;  // shaders.metal:275
    float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (x < W && y < H) v = fb[(size_t)y * W + x];
    v.w = __uint_as_float((x << 16) | y);
    out[i] = v;
}

__global__ void k_quantize(const float4* __restrict__ in, uint32_t* __restrict__ out, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 v = in[i];
    out[i] = unorm8(v.x) | (unorm8(v.y) << 8) | (unorm8(v.z) << 16) | (unorm8(v.w) << 24);
}

}  // namespace

hipError_t launch_present_blur(const uint32_t* in, uint32_t* out, uint32_t W, uint32_t H, hipStream_t s) {
    const dim3 block(64, 4);
    const dim3 grid((W + 63) / 64, (H + 3) / 4);
    hipLaunchKernelGGL(k_present_blur, grid, block, 0, s, in, out, (int)W, (int)H);
    return hipGetLastError();
}

hipError_t launch_chunk_packets(const float4* fb, const uint32_t* chunks, uint32_t n_chunks, uint32_t W, uint32_t H,
                                float4* out, hipStream_t s) {
    const uint32_t n = n_chunks * 16u;
    hipLaunchKernelGGL(k_chunk_packets, dim3((n + 255) / 256), dim3(256), 0, s, fb, chunks, n_chunks, W, H, out);
    return hipGetLastError();
}

hipError_t launch_quantize(const float4* in, uint32_t* out, size_t n, hipStream_t s) {
    hipLaunchKernelGGL(k_quantize, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, out, n);
    return hipGetLastError();
}

}  // namespace mm
