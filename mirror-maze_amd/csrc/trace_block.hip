// trace_block.hip — block-synchronous bounce loop with ray compaction
// (MM_OPT_BLOCKSYNC, experimental).
//
// A resident 1024-thread block owns 1024 paths at a time (one per thread, in
// registers) and runs their bounces in lockstep across the block: every
// bounce, the live paths' rays (o, d) are compacted into the first n_live
// slots of an LDS exchange (wave ballot + per-wave counts), threads 0..n_live-1
// trace them -- so the traversal waves are full however many paths of the
// block have ended -- and write (t, hit) back for the owning threads to shade.
// The wave model (scripts/wave_sim.cpp) prices this at 0.86 of the VALU slots
// of per-wave bounces; the price is three block barriers per bounce and the
// exchange (32 B per slot), which with the BVH (47 KB on C3) still fits two
// blocks per CU (rect records are read through L1/L2, not LDS).
//
// Each path executes exactly the reference's operations (trace_path's
// sequence, split at the closest-hit query), so samples are bit-identical to
// the other kernels.
#include <hip/hip_runtime.h>

#include "mm_launch.h"
#include "mm_trace.h"
#include "mm_wave_util.h"

namespace mm {

namespace {

constexpr uint32_t kNoHit = 0xFFFFFFFFu;  // closest-hit query overflowed its stack

__device__ __forceinline__ uint64_t lanemask_lt_bs() {
    const uint32_t lane = threadIdx.x & 63u;
    return lane ? (~0ull >> (64 - lane)) : 0ull;
}

template <bool kStats>
__global__ __launch_bounds__(1024, 8) void k_trace_blocksync(DevScene sc, TileJob job, float4* __restrict__ samples,
                                                             unsigned long long* stats, uint32_t* err,
                                                             uint32_t* work) {
    extern __shared__ float4 lds[];
    __shared__ uint32_t s_cnt[16];
    __shared__ uint32_t s_base;
    float4* lds_nodes = lds;
    for (uint32_t i = threadIdx.x; i < 2 * sc.n_nodes; i += blockDim.x) lds_nodes[i] = sc.nodes[i];
    float4* xo = lds + 2 * sc.n_nodes;                      // (o.xyz, d.x) per slot
    float2* xd = reinterpret_cast<float2*>(xo + blockDim.x);  // (d.y, d.z)
    float2* xt = xd + blockDim.x;                             // (t, bits(hit))
    __syncthreads();
    const auto v = view(static_cast<const float4*>(lds_nodes), sc.recs);

    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6, nw = blockDim.x >> 6;
    const uint32_t spp = job.e.spp;
    const uint32_t n_paths = job.w * job.h * spp;
    const int bounce_limit = (int)job.e.bounce_limit, mirror_limit = (int)job.e.mirror_limit;
    const F3 cam = F3{job.u.cam.center[0], job.u.cam.center[1], job.u.cam.center[2]};
    Counters c;
    uint32_t paths = 0;
    ScratchStack stack;
    for (;;) {
        if (tid == 0) s_base = atomicAdd(work, blockDim.x);
        __syncthreads();
        const uint32_t base = s_base;
        if (base >= n_paths) break;  // block-uniform
        const uint32_t path = base + tid;
        const bool valid = path < n_paths;
        PathState p;
        p.ori = cam;
        p.dir = F3{0.0f, 0.0f, 0.0f};
        p.T = F3{1.0f, 1.0f, 1.0f};
        p.L = F3{0.0f, 0.0f, 0.0f};
        p.seed = 0;
        p.n = 0;
        p.mh = 0;
        bool live = false;
        if (valid) {
            const uint32_t pix = path / spp, smp = path - pix * spp;
            const uint32_t j = pix / job.w, i = pix - j * job.w;
            const uint32_t px = job.x0 + i, py = job.y0 + j * job.y_stride;
            p.seed = seed_tile(py * job.view_w + px, smp, job.e.frame);
            p.dir = jitter(primary_dir(job.u, px, py), p.seed);
            live = 0 < bounce_limit;
        }
        for (;;) {
            // compaction: slot of every live ray among the block's live rays
            const uint64_t m = __ballot(live);
            if (lane == 0) s_cnt[wid] = (uint32_t)__popcll(m);
            __syncthreads();
            uint32_t off = 0, total = 0;
            for (uint32_t w = 0; w < nw; ++w) {
                const uint32_t cw = s_cnt[w];
                off += w < wid ? cw : 0u;
                total += cw;
            }
            if (total == 0) break;  // block-uniform
            const uint32_t slot = off + (uint32_t)__popcll(m & lanemask_lt_bs());
            if (live) {
                xo[slot] = make_float4(p.ori.x, p.ori.y, p.ori.z, p.dir.x);
                xd[slot] = make_float2(p.dir.y, p.dir.z);
            }
            __syncthreads();
            // closest-hit queries on dense waves
            if (wid * 64u < total && tid < total) {
                const float4 a = xo[tid];
                const float2 b = xd[tid];
                float t = kBig;
                uint32_t k = 0;
                const bool ok = closest_hit<kStats, decltype(v), ScratchStack, 5>(
                    sc, v, F3{a.x, a.y, a.z}, F3{a.w, b.x, b.y}, t, k, stack, c);
                if (kStats) c.rays++;
                xt[tid] = make_float2(t, __uint_as_float(ok ? k : kNoHit));
            }
            __syncthreads();
            // shading by the owners (ori/dir re-read: not live across the query)
            if (live) {
                const float4 a = xo[slot];
                const float2 b = xd[slot];
                p.ori = F3{a.x, a.y, a.z};
                p.dir = F3{a.w, b.x, b.y};
                const float2 r = xt[slot];
                const uint32_t k = __float_as_uint(r.y);
                bool cont;
                if (k == kNoHit) {
                    atomicOr(err, 1u);
                    cont = false;
                } else {
                    cont = shade_step(sc, p, r.x, k, mirror_limit);
                }
                p.n++;
                live = cont && p.n < bounce_limit + p.mh;
            }
        }
        const F3 s = valid ? F3{sqrtf(fmaxf(p.L.x, 0.0f)), sqrtf(fmaxf(p.L.y, 0.0f)), sqrtf(fmaxf(p.L.z, 0.0f))}
                           : F3{0.0f, 0.0f, 0.0f};
        if (valid) paths++;
        if (job.fuse) resolve_in_wave(job, s, path, valid, job.out);
        else if (valid) samples[path] = make_float4(s.x, s.y, s.z, 0.0f);
        __syncthreads();  // s_base is rewritten by the next fetch
    }
    if (kStats) flush_stats(stats, c, paths);
    // self-cleaning counter pair (as k_trace_wavepersist), counted per block
    if (tid == 0) {
        __threadfence();
        if (atomicAdd(work + 1, 1u) == gridDim.x - 1) {
            atomicExch(work, 0u);
            atomicExch(work + 1, 0u);
        }
    }
}

}  // namespace

size_t blocksync_lds_bytes(const DevScene& sc, uint32_t block) {
    return 2 * (size_t)sc.n_nodes * sizeof(float4) + (size_t)block * (sizeof(float4) + 2 * sizeof(float2));
}

hipError_t launch_trace_blocksync(const DevScene& sc, const TileJob& job, float4* samples, unsigned long long* stats,
                                  uint32_t* err, uint32_t* work, bool count_stats, hipStream_t s) {
    constexpr uint32_t block = 1024;
    const size_t lds = blocksync_lds_bytes(sc, block);
    auto kern = count_stats ? k_trace_blocksync<true> : k_trace_blocksync<false>;
    int per_cu = 0, dev = 0, cus = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, (int)block, lds);
    if (e != hipSuccess) return e;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint32_t n_paths = job.w * job.h * job.e.spp;
    uint32_t grid = (uint32_t)std::max(1, per_cu) * (uint32_t)std::max(1, cus);
    grid = std::max(1u, std::min(grid, (n_paths + block - 1) / block));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(block), lds, s, sc, job, samples, stats, err, work);
    return hipGetLastError();
}

}  // namespace mm
