// trace_wave.hip — wavefront pipeline for throughput mode (MM_PIPE_WAVEFRONT).
//
// The bounce loop of shaders.metal:306-340 is flattened into launches over a
// queue of live paths; path state lives in HBM as SoA so every access is a
// coalesced 4-B-per-lane stream:
//   k_wf_generate  primary ray + seed for every path, queue 0 = survivors
//   k_wf_extend    closest hit for each queued path (the dominant kernel)
//   k_wf_shade     shading step; survivors are appended to the other queue
//                  with a wave ballot + prefix popcount and ONE atomic per
//                  wave (stream compaction), so later bounces -- the long
//                  mirror chains -- run dense
// Per ray the kernels move 24 B (o,d) + 8 B hit in extend and 64 B in / 56 B
// out + 4 B queue in shade: ~156 B/ray against SURVEY §8(d)'s 136 B model.
#include <hip/hip_runtime.h>

#include "mm_launch.h"
#include "mm_path.h"

namespace mm {

constexpr uint32_t kHitOverflow = 0xFFFFFFFEu;

__device__ __forceinline__ uint64_t wf_lanemask_lt() {
    const uint32_t lane = threadIdx.x & 63u;
    return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// Append `pid` to queue q (if keep) with one atomic per wave.
__device__ __forceinline__ void wave_append(bool keep, uint32_t pid, uint32_t* __restrict__ queue, uint32_t* count) {
    const uint64_t m = __ballot(keep);
    if (!m) return;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t leader = (uint32_t)__ffsll((unsigned long long)m) - 1u;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(count, (uint32_t)__popcll(m));
    base = __shfl(base, (int)leader);
    if (keep) queue[base + (uint32_t)__popcll(m & wf_lanemask_lt())] = pid;
}

__device__ __forceinline__ void store_state(const WaveState& ws, uint32_t pid, const PathState& p) {
    ws.ox[pid] = p.ori.x; ws.oy[pid] = p.ori.y; ws.oz[pid] = p.ori.z;
    ws.dx[pid] = p.dir.x; ws.dy[pid] = p.dir.y; ws.dz[pid] = p.dir.z;
    ws.tr[pid] = p.T.x; ws.tg[pid] = p.T.y; ws.tb[pid] = p.T.z;
    ws.lr[pid] = p.L.x; ws.lg[pid] = p.L.y; ws.lb[pid] = p.L.z;
    ws.seed[pid] = p.seed;
    ws.nm[pid] = (uint32_t)p.n | ((uint32_t)p.mh << 16);
}

__device__ __forceinline__ void load_state(const WaveState& ws, uint32_t pid, PathState& p) {
    p.ori = F3{ws.ox[pid], ws.oy[pid], ws.oz[pid]};
    p.dir = F3{ws.dx[pid], ws.dy[pid], ws.dz[pid]};
    p.T = F3{ws.tr[pid], ws.tg[pid], ws.tb[pid]};
    p.L = F3{ws.lr[pid], ws.lg[pid], ws.lb[pid]};
    p.seed = ws.seed[pid];
    const uint32_t nm = ws.nm[pid];
    p.n = (int)(nm & 0xFFFFu);
    p.mh = (int)(nm >> 16);
}

__device__ __forceinline__ float4 sample_value(const PathState& p) {
    return make_float4(sqrtf(fmaxf(p.L.x, 0.0f)), sqrtf(fmaxf(p.L.y, 0.0f)), sqrtf(fmaxf(p.L.z, 0.0f)), 0.0f);
}

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_wf_generate(TileJob job, WaveState ws, float4* __restrict__ samples) {
    const uint32_t spp = job.e.spp;
    const uint32_t n_paths = job.w * job.h * spp;
    const F3 cam = F3{job.u.cam.center[0], job.u.cam.center[1], job.u.cam.center[2]};
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t base = blockIdx.x * blockDim.x; base < n_paths; base += stride) {
        const uint32_t path = base + threadIdx.x;
        const bool valid = path < n_paths;
        bool keep = false;
        if (valid) {
            const uint32_t pix = path / spp, smp = path - pix * spp;
            const uint32_t j = pix / job.w, i = pix - j * job.w;
            const uint32_t px = job.x0 + i, py = job.y0 + j * job.y_stride;
            PathState p;
            p.seed = seed_tile(py * job.view_w + px, smp, job.e.frame);
            p.dir = jitter(primary_dir(job.u, px, py), p.seed);
            p.ori = cam;
            p.T = F3{1.0f, 1.0f, 1.0f};
            p.L = F3{0.0f, 0.0f, 0.0f};
            p.n = 0;
            p.mh = 0;
            keep = 0 < (int)job.e.bounce_limit;
            if (keep) store_state(ws, path, p);
            else samples[path] = sample_value(p);
        }
        wave_append(keep, path, ws.queue[0], &ws.counters[0]);
    }
}

// ---------------------------------------------------------------------------
template <bool kStats, typename V>
__device__ __forceinline__ void extend_body(const DevScene& sc, const V& v, const WaveState& ws, int q,
                                            unsigned long long* stats) {
    const uint32_t n_in = ws.counters[q];
    const uint32_t stride = gridDim.x * blockDim.x;
    Counters c;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n_in; i += stride) {
        const uint32_t pid = ws.queue[q][i];
        const F3 o = F3{ws.ox[pid], ws.oy[pid], ws.oz[pid]};
        const F3 d = F3{ws.dx[pid], ws.dy[pid], ws.dz[pid]};
        float t = kBig;
        uint32_t k = 0;
        ScratchStack stack;
        const bool ok = closest_hit_bvh<kStats, kFormIfIf>(sc, v, make_ray(o, d), t, k, stack, c);
        if (kStats) c.rays++;
        ws.hit_t[pid] = t;
        ws.hit_i[pid] = ok ? k : kHitOverflow;
    }
    if (kStats) {
        unsigned long long v[3] = {c.rays, c.visits, c.rtests};
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            unsigned long long x = v[j];
            for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
            v[j] = x;
        }
        if ((threadIdx.x & 63u) == 0) {
            atomicAdd(&stats[0], v[0]);
            atomicAdd(&stats[1], v[1]);
            atomicAdd(&stats[2], v[2]);
        }
    }
}

template <bool kStats, bool kLds>
__global__ __launch_bounds__(512) void k_wf_extend(DevScene sc, WaveState ws, int q, unsigned long long* stats) {
    if (blockIdx.x == 0 && threadIdx.x == 0) ws.counters[q ^ 1] = 0;  // shade's output queue
    if (blockIdx.x * blockDim.x >= ws.counters[q]) return;               // no work: skip the LDS fill
    if constexpr (kLds) {
        extern __shared__ float4 lds_nodes[];
        for (uint32_t i = threadIdx.x; i < 2 * sc.n_nodes; i += blockDim.x) lds_nodes[i] = sc.nodes[i];
        __syncthreads();
        extend_body<kStats>(sc, view(lds_nodes), ws, q, stats);
    } else {
        extend_body<kStats>(sc, view(sc.nodes), ws, q, stats);
    }
}

// ---------------------------------------------------------------------------
template <bool kStats>
__global__ __launch_bounds__(256) void k_wf_shade(DevScene sc, TileJob job, WaveState ws, int q,
                                                  float4* __restrict__ samples, unsigned long long* stats,
                                                  uint32_t* err) {
    const uint32_t n_in = ws.counters[q];
    const int bounce_limit = (int)job.e.bounce_limit, mirror_limit = (int)job.e.mirror_limit;
    const uint32_t stride = gridDim.x * blockDim.x;
    uint32_t done = 0;
    for (uint32_t base = blockIdx.x * blockDim.x; base < n_in; base += stride) {
        const uint32_t i = base + threadIdx.x;
        bool keep = false;
        uint32_t pid = 0;
        if (i < n_in) {
            pid = ws.queue[q][i];
            PathState p;
            load_state(ws, pid, p);
            const float t = ws.hit_t[pid];
            const uint32_t k = ws.hit_i[pid];
            bool cont;
            if (k == kHitOverflow) {
                atomicOr(err, 1u);
                cont = false;
            } else {
                cont = shade_step(sc, p, t, k, mirror_limit);
            }
            p.n++;
            keep = cont && p.n < bounce_limit + p.mh;
            if (keep) {
                store_state(ws, pid, p);
            } else {
                samples[pid] = sample_value(p);
                done++;
            }
        }
        wave_append(keep, pid, ws.queue[q ^ 1], &ws.counters[q ^ 1]);
    }
    if (kStats) {
        unsigned long long x = done;
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
        if ((threadIdx.x & 63u) == 0) atomicAdd(&stats[3], x);
    }
}

// ---------------------------------------------------------------------------
hipError_t launch_wf_generate(const TileJob& job, const WaveState& ws, float4* samples, hipStream_t s) {
    hipError_t e = hipMemsetAsync(ws.counters, 0, 4 * sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    const uint32_t n = job.w * job.h * job.e.spp;
    const uint32_t grid = std::min<uint32_t>((n + 255) / 256, 256u * 16u);
    hipLaunchKernelGGL(k_wf_generate, dim3(grid), dim3(256), 0, s, job, ws, samples);
    return hipGetLastError();
}

hipError_t launch_wf_extend(const DevScene& sc, const WaveState& ws, int q, uint32_t n_upper,
                            unsigned long long* stats, bool count_stats, const WaveOpts& o, hipStream_t s) {
    const uint32_t block = o.block;
    const size_t lds = o.lds_nodes ? 2 * (size_t)sc.n_nodes * sizeof(float4) : 0;
    const uint32_t grid = std::max(1u, std::min<uint32_t>((n_upper + block - 1) / block, o.extend_blocks));
    if (o.lds_nodes) {
        if (count_stats) hipLaunchKernelGGL((k_wf_extend<true, true>), dim3(grid), dim3(block), lds, s, sc, ws, q, stats);
        else hipLaunchKernelGGL((k_wf_extend<false, true>), dim3(grid), dim3(block), lds, s, sc, ws, q, stats);
    } else {
        if (count_stats) hipLaunchKernelGGL((k_wf_extend<true, false>), dim3(grid), dim3(block), 0, s, sc, ws, q, stats);
        else hipLaunchKernelGGL((k_wf_extend<false, false>), dim3(grid), dim3(block), 0, s, sc, ws, q, stats);
    }
    return hipGetLastError();
}

hipError_t launch_wf_shade(const DevScene& sc, const TileJob& job, const WaveState& ws, int q, uint32_t n_upper,
                           float4* samples, unsigned long long* stats, uint32_t* err, bool count_stats,
                           hipStream_t s) {
    const uint32_t grid = std::max(1u, std::min<uint32_t>((n_upper + 255) / 256, 256u * 16u));
    if (count_stats)
        hipLaunchKernelGGL((k_wf_shade<true>), dim3(grid), dim3(256), 0, s, sc, job, ws, q, samples, stats, err);
    else
        hipLaunchKernelGGL((k_wf_shade<false>), dim3(grid), dim3(256), 0, s, sc, job, ws, q, samples, stats, err);
    return hipGetLastError();
}

}  // namespace mm
