// trace_kernels.hip — gfx950 kernels for mirror-maze's per-pixel ray-trace loop.
//
//   k_prep_rects         per-rect subexpressions of ray_rect_intersect
//   k_trace_chunks       parity mode: the reference dispatch (shaders.metal:245-368)
//   k_trace_mega         throughput mode, one thread per (pixel, sample) path
//                        (and MM_PIPE_REFERENCE, the straight statement)
//   k_trace_wavepersist  throughput mode, the production kernel: resident
//                        blocks, waves pull 64-path chunks, pixels resolved in
//                        the wave
//   k_resolve            per-pixel sample reduction in the reference's order
#include <hip/hip_runtime.h>

#include "mm_launch.h"
#include "mm_path.h"
#include "mm_wave_util.h"

namespace mm {

// ---------------------------------------------------------------------------
__global__ void k_prep_rects(const mm_rect* __restrict__ rects, uint32_t n, float4* __restrict__ geo) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const mm_rect r = rects[k];
    const F3 o = F3{r.o[0], r.o[1], r.o[2]};
    const F3 v = F3{r.v[0], r.v[1], r.v[2]};
    const F3 u = F3{r.u[0], r.u[1], r.u[2]};
    const F3 nn = normalize3(cross3(v, u));       // shaders.metal:52 (and :309)
    const float lv = sqrtf(dot3(v, v));           // length(mirror.v), :60
    const float lu = sqrtf(dot3(u, u));           // length(mirror.u), :61
    geo[4 * k + 0] = make_float4(o.x, o.y, o.z, lv);
    geo[4 * k + 1] = make_float4(nn.x, nn.y, nn.z, lu);
    geo[4 * k + 2] = make_float4(v.x, v.y, v.z, 1.0f / lv);
    geo[4 * k + 3] = make_float4(u.x, u.y, u.z, 1.0f / lu);
}

hipError_t launch_prep_rects(const mm_rect* rects, uint32_t n, float4* geo_dev, hipStream_t s) {
    hipLaunchKernelGGL(k_prep_rects, dim3((n + 255) / 256), dim3(256), 0, s, rects, n, geo_dev);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Parity mode.  One workgroup = one reference threadgroup of 32x32 threads;
// flat = gid.x + 32*gid.y, so each wave64 holds exactly the 64 samples of one
// pixel (pixel_number = flat/64, shaders.metal:271-275) and the reference's
// threadgroup-memory tree reduction (shaders.metal:342-367) becomes a
// shuffle reduction inside the wave with the same pairing and order.
template <bool kStats>
__global__ __launch_bounds__(1024) void k_trace_chunks(DevScene sc, mm_uniform u,
                                                       const uint32_t* __restrict__ chunks, float4* __restrict__ fb,
                                                       uint32_t* __restrict__ fb8, unsigned long long* stats,
                                                       uint32_t* err) {
    const uint32_t W = (uint32_t)u.view_w, H = (uint32_t)u.view_h;
    const uint32_t chunk = u.chunk_w, ppc = chunk * chunk;  // 4, 16
    const uint32_t gx = blockIdx.x, gy = blockIdx.y;
    // pixel_buffer_index in float, IR %26-%31
    const uint32_t pbi = cvt_u32_sat(((u.view_w * 0.5f) * (float)gy) / (float)ppc + (float)gx);
    const uint32_t cx = chunks[2 * pbi], cy = chunks[2 * pbi + 1];
    const uint32_t flat = threadIdx.x;          // 0..1023
    const uint32_t lx = flat & 31, ly = flat >> 5;
    const uint32_t pn = flat >> 6;              // flat / (1024 / 16)
    const uint32_t px = cx + pn / chunk, py = cy + pn % chunk;
    uint32_t seed = seed_reference(gx * 32 + lx, gy * 32 + ly, u.time);
    const F3 d = jitter(primary_dir(u, px, py), seed);
    const F3 ori = F3{u.cam.center[0], u.cam.center[1], u.cam.center[2]};
    ScratchStack stack;
    Counters c;
    bool overflow = false;
    const BvhQuery<kStats, kFormIfIf, NodeView<const float4*>> q{sc, view(sc.nodes)};
    F3 s = trace_path<kStats>(sc, q, ori, d, seed, 5, 15, stack, c, overflow);  // shaders.metal:294-295
    if (overflow) atomicOr(err, 1u);
    // level 1..3: test[f] += test[f+1], += test[f+2], += test[f+4]
    s = s + F3{__shfl_xor(s.x, 1), __shfl_xor(s.y, 1), __shfl_xor(s.z, 1)};
    s = s + F3{__shfl_xor(s.x, 2), __shfl_xor(s.y, 2), __shfl_xor(s.z, 2)};
    s = s + F3{__shfl_xor(s.x, 4), __shfl_xor(s.y, 4), __shfl_xor(s.z, 4)};
    // first thread of the pixel: acc = blk0 + blk1 + ... + blk7, then / 64
    F3 acc = s;
#pragma unroll
    for (int i = 1; i < 8; ++i) acc = acc + F3{__shfl(s.x, 8 * i), __shfl(s.y, 8 * i), __shfl(s.z, 8 * i)};
    if (kStats) flush_stats(stats, c, 64);
    if ((flat & 63) == 0 && px < W && py < H) {
        const float m = 64.0f;
        const F3 o = F3{acc.x / m, acc.y / m, acc.z / m};
        fb[(size_t)py * W + px] = make_float4(o.x, o.y, o.z, 1.0f);
        fb8[(size_t)py * W + px] = unorm8(o.x) | (unorm8(o.y) << 8) | (unorm8(o.z) << 16) | (255u << 24);
    }
}

hipError_t launch_trace_chunks(const DevScene& sc, const mm_uniform& u, const uint32_t* chunks_dev,
                               uint32_t grid_w, uint32_t grid_h, float4* fb, uint32_t* fb8,
                               unsigned long long* stats_dev, uint32_t* err, bool count_stats, hipStream_t s) {
    if (count_stats)
        hipLaunchKernelGGL(k_trace_chunks<true>, dim3(grid_w, grid_h), dim3(1024), 0, s, sc, u, chunks_dev, fb, fb8,
                           stats_dev, err);
    else
        hipLaunchKernelGGL(k_trace_chunks<false>, dim3(grid_w, grid_h), dim3(1024), 0, s, sc, u, chunks_dev, fb, fb8,
                           stats_dev, err);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Throughput mode, one thread per path: path = pixel*spp + sample.
//   kRef  : traverse_reference (IEEE division everywhere), for A/B
//   kLds  : stage the node array in LDS (dynamic shared memory) first
template <bool kStats, typename Q>
__device__ __forceinline__ void mega_body(const DevScene& sc, const Q& q, const TileJob& job,
                                          float4* __restrict__ samples, unsigned long long* stats, uint32_t* err) {
    const uint32_t spp = job.e.spp;
    const uint32_t n_paths = job.w * job.h * spp;
    const uint32_t path = blockIdx.x * blockDim.x + threadIdx.x;
    Counters c;
    if (path < n_paths) {
        const uint32_t pix = path / spp, smp = path - pix * spp;
        const uint32_t j = pix / job.w, i = pix - j * job.w;
        const uint32_t px = job.x0 + i, py = job.y0 + j * job.y_stride;
        uint32_t seed = seed_tile(py * job.view_w + px, smp, job.e.frame);
        const F3 d = jitter(primary_dir(job.u, px, py), seed);
        const F3 ori = F3{job.u.cam.center[0], job.u.cam.center[1], job.u.cam.center[2]};
        ScratchStack stack;
        bool overflow = false;
        const F3 s = trace_path<kStats>(sc, q, ori, d, seed, (int)job.e.bounce_limit, (int)job.e.mirror_limit, stack,
                                        c, overflow);
        if (overflow) atomicOr(err, 1u);
        samples[path] = make_float4(s.x, s.y, s.z, 0.0f);
    }
    if (kStats) flush_stats(stats, c, path < n_paths ? 1u : 0u);
}

template <bool kStats, bool kRef, bool kLds>
__global__ __launch_bounds__(1024) void k_trace_mega(DevScene sc, TileJob job, float4* __restrict__ samples,
                                                     unsigned long long* stats, uint32_t* err) {
    if constexpr (kRef) {
        mega_body<kStats>(sc, RefQuery<kStats>{sc}, job, samples, stats, err);
    } else if constexpr (kLds) {
        extern __shared__ float4 lds_nodes[];
        for (uint32_t i = threadIdx.x; i < 2 * sc.n_nodes; i += blockDim.x) lds_nodes[i] = sc.nodes[i];
        __syncthreads();
        mega_body<kStats>(sc, BvhQuery<kStats, kFormIfIf, NodeView<float4*>>{sc, view(lds_nodes)}, job, samples,
                          stats, err);
    } else {
        mega_body<kStats>(sc, BvhQuery<kStats, kFormIfIf, NodeView<const float4*>>{sc, view(sc.nodes)}, job,
                          samples, stats, err);
    }
}

// ---------------------------------------------------------------------------
// Wave-persistent megakernel: resident 1024-thread blocks (two per CU at
// <= 64 VGPRs, 8 waves per SIMD) fill LDS once; each wave takes 64
// consecutive paths at a time from a global counter and traces them, so no
// block waits for its slowest wave before the CU can take more work.  With
// 64 % spp == 0 the wave's 64 paths are whole pixels and it resolves them
// itself (job.fuse).  A multi-frame launch queues frame 0's chunks, then frame
// 1's, ...; a chunk's frame picks its RNG frame and output slice.
template <bool kStats, typename Q>
__device__ __forceinline__ uint32_t wavepersist_body(const DevScene& sc, const Q& q, const TileJob& job,
                                                     float4* __restrict__ samples, unsigned long long* stats,
                                                     uint32_t* err, uint32_t* work) {
    const uint32_t spp = job.e.spp;
    const uint32_t n_paths = job.w * job.h * spp;         // per frame
    const uint32_t cpf = (n_paths + 63u) / 64u;           // 64-path chunks per frame
    const uint32_t n_queue = cpf * 64u * job.n_frames;    // the queue, in paths (chunks padded to 64)
    const uint32_t lane = threadIdx.x & 63u;
    const F3 ori = F3{job.u.cam.center[0], job.u.cam.center[1], job.u.cam.center[2]};
    Counters c;
    ScratchStack stack;
    uint32_t paths = 0, chunks = 0;
    for (;;) {
        uint32_t b = 0;
        if (lane == 0) b = atomicAdd(work, 64u);
        const uint32_t base = __builtin_amdgcn_readfirstlane(b);
        if (base >= n_queue) break;
        ++chunks;
        const uint32_t qc = base >> 6;
        const uint32_t fr = job.n_frames > 1 ? qc / cpf : 0u;
        const uint32_t path = (qc - fr * cpf) * 64u + lane;
        const bool valid = path < n_paths;
        F3 s = F3{0.0f, 0.0f, 0.0f};
        if (valid) {
            const uint32_t pix = path / spp, smp = path - pix * spp;
            const uint32_t j = pix / job.w, i = pix - j * job.w;
            const uint32_t px = job.x0 + i, py = job.y0 + j * job.y_stride;
            uint32_t seed = seed_tile(py * job.view_w + px, smp, job.e.frame + fr);
            const F3 d = jitter(primary_dir(job.u, px, py), seed);
            bool overflow = false;
            s = trace_path<kStats>(sc, q, ori, d, seed, (int)job.e.bounce_limit, (int)job.e.mirror_limit, stack, c,
                                   overflow);
            if (overflow) atomicOr(err, 1u);
            if (!job.fuse) samples[path] = make_float4(s.x, s.y, s.z, 0.0f);
            paths++;
        }
        if (job.fuse) resolve_in_wave(job, s, path, valid, job.out + (size_t)fr * job.w * job.h);
    }
    if (kStats) flush_stats(stats, c, paths);
    return chunks;
}

// LDS modes (what a resident block stages before tracing; the rest is read
// through L1/L2):
//   0  nothing (nodes, records global)           BVH forms 0 / 5
//   1  BVH nodes                                  BVH forms 0 / 5 (general rect test)
//   3  BVH nodes + compact slot records           BVH forms 0 / 5 / 7
//   6  top of the breadth-first node array        BVH forms 5 / 7 (split cache)
//   7  BVH nodes, compact records global          BVH forms 5 / 7
//   10 dictionary-coded nodes, records global     BVH forms 5 / 7
//   11 the whole grid image                       grid search
//   12 grid cells + lists, records + boxes global grid search
//   13 nothing (the grid image global)             grid search
#define MM_TS_STAGED()                                                                                      \
    do {                                                                                                     \
        if (job.wave_ts && (threadIdx.x & 63u) == 0) {                                                       \
            const uint32_t wid_ = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);                      \
            if (wid_ < job.wave_ts_cap) job.wave_ts[4 * wid_ + 1] = (unsigned long long)wall_clock64();     \
        }                                                                                                    \
    } while (0)

template <bool kStats, int kLds, int kForm>
// 1024-thread blocks at 8 waves per SIMD (<= 64 VGPRs).  With the grid search,
// 768-thread blocks at 6 waves (80 VGPRs, no VGPR spills) measured 6.21 vs
// 5.87 ms on C3 (profiles/r02_ab_grid_variants.txt).
__global__ __launch_bounds__(1024, 8) void k_trace_wavepersist(DevScene sc, TileJob job, float4* __restrict__ samples,
                                                               unsigned long long* stats, uint32_t* err,
                                                               uint32_t* work) {
    const unsigned long long t_entry = job.wave_ts ? (unsigned long long)wall_clock64() : 0ull;
    uint32_t chunks = 0;
    extern __shared__ float4 lds[];
    if constexpr (kLds == 11 || kLds == 12) {
        const uint32_t n16 = (kLds == 11 ? sc.grid.bytes : sc.grid.off_recs) / 16u;
        uint4* img = reinterpret_cast<uint4*>(lds);
        for (uint32_t i = threadIdx.x; i < n16; i += blockDim.x) img[i] = sc.grid.image[i];
        __syncthreads();
        MM_TS_STAGED();
        const char* base = reinterpret_cast<const char*>(lds);
        const uint32_t* cells = reinterpret_cast<const uint32_t*>(base);
        const uint16_t* list = reinterpret_cast<const uint16_t*>(base + sc.grid.off_list);
        if constexpr (kLds == 11) {
            const auto gv = grid_view(cells, list, reinterpret_cast<const uint2*>(base + sc.grid.off_recs),
                                      reinterpret_cast<const float2*>(base + sc.grid.off_box));
            chunks = wavepersist_body<kStats>(sc, GridQuery<kStats, decltype(gv)>{sc, gv}, job, samples, stats, err,
                                              work);
        } else {
            const auto gv = grid_view(cells, list, sc.grid.recs, sc.grid.box);
            chunks = wavepersist_body<kStats>(sc, GridQuery<kStats, decltype(gv)>{sc, gv}, job, samples, stats, err,
                                              work);
        }
    } else if constexpr (kLds == 13) {
        const auto gv = grid_view(sc.grid.cells, sc.grid.list, sc.grid.recs, sc.grid.box);
        chunks = wavepersist_body<kStats>(sc, GridQuery<kStats, decltype(gv)>{sc, gv}, job, samples, stats, err,
                                          work);
    } else if constexpr (kLds == 6) {
        for (uint32_t i = threadIdx.x; i < sc.n_lds_f4; i += blockDim.x) lds[i] = sc.nodes[i];
        __syncthreads();
        MM_TS_STAGED();
        const auto v = view(SplitNodes{lds, sc.nodes, sc.n_lds_f4}, sc.recs);
        chunks = wavepersist_body<kStats>(sc, BvhQuery<kStats, kForm, decltype(v)>{sc, v}, job, samples, stats, err,
                                          work);
    } else if constexpr (kLds == 10) {
        float* tab = reinterpret_cast<float*>(lds);
        uint32_t* words = reinterpret_cast<uint32_t*>(tab + 256);
        for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) tab[i] = sc.dict_tab[i];
        for (uint32_t i = threadIdx.x; i < 3 * sc.n_nodes; i += blockDim.x) words[i] = sc.dict_words[i];
        __syncthreads();
        MM_TS_STAGED();
        const auto v = view(DictNodes{words, tab}, sc.recs);
        chunks = wavepersist_body<kStats>(sc, BvhQuery<kStats, kForm, decltype(v)>{sc, v}, job, samples, stats, err,
                                          work);
    } else if constexpr (kLds == 1 || kLds == 3 || kLds == 7) {
        for (uint32_t i = threadIdx.x; i < 2 * sc.n_nodes; i += blockDim.x) lds[i] = sc.nodes[i];
        uint2* lds_recs = reinterpret_cast<uint2*>(lds + 2 * sc.n_nodes);
        if constexpr (kLds == 3)
            for (uint32_t i = threadIdx.x; i < 5 * sc.n_rects; i += blockDim.x) lds_recs[i] = sc.recs[i];
        __syncthreads();
        MM_TS_STAGED();
        if constexpr (kLds == 3) {
            const auto v = view(static_cast<float4*>(lds), lds_recs);
            chunks = wavepersist_body<kStats>(sc, BvhQuery<kStats, kForm, decltype(v)>{sc, v}, job, samples, stats,
                                              err, work);
        } else if constexpr (kLds == 7) {
            const auto v = view(static_cast<float4*>(lds), sc.recs);
            chunks = wavepersist_body<kStats>(sc, BvhQuery<kStats, kForm, decltype(v)>{sc, v}, job, samples, stats,
                                              err, work);
        } else {
            const auto v = view(static_cast<float4*>(lds));
            chunks = wavepersist_body<kStats>(sc, BvhQuery<kStats, kForm, decltype(v)>{sc, v}, job, samples, stats,
                                              err, work);
        }
    } else {
        const auto v = view(sc.nodes);
        chunks = wavepersist_body<kStats>(sc, BvhQuery<kStats, kForm, decltype(v)>{sc, v}, job, samples, stats, err,
                                          work);
    }
    if (job.wave_ts && (threadIdx.x & 63u) == 0) {
        const uint32_t wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        if (wid < job.wave_ts_cap) {
            job.wave_ts[4 * wid + 0] = t_entry;
            job.wave_ts[4 * wid + 2] = (unsigned long long)wall_clock64();
            job.wave_ts[4 * wid + 3] = chunks;
        }
    }
    // Self-cleaning work counter (work[0] = next path, work[1] = waves done):
    // the last wave to finish re-zeroes both, so the next launch needs no
    // memset -- a fill kernel queued between two frames on another stream
    // would wait for free CUs and serialise overlapping frames.
    if ((threadIdx.x & 63u) == 0) {
        __threadfence();
        const uint32_t total = gridDim.x * (blockDim.x >> 6);
        if (atomicAdd(work + 1, 1u) == total - 1) {
            atomicExch(work, 0u);
            atomicExch(work + 1, 0u);
        }
    }
}

size_t wavepersist_lds_bytes(const DevScene& sc, int lds_mode) {
    switch (lds_mode) {
        case 11: return sc.grid.bytes;
        case 12: return sc.grid.off_recs;
        case 6: return (size_t)sc.n_lds_f4 * sizeof(float4);
        case 10: return 256 * sizeof(float) + 3 * (size_t)sc.n_nodes * sizeof(uint32_t);
        case 1: case 7: return 2 * (size_t)sc.n_nodes * sizeof(float4);
        case 3: return 2 * (size_t)sc.n_nodes * sizeof(float4) + 5 * (size_t)sc.n_rects * sizeof(uint2);
        default: return 0;
    }
}

template <int kLds, int kForm>
static hipError_t launch_wavepersist_t(const DevScene& sc, const TileJob& job, float4* samples,
                                       unsigned long long* stats, uint32_t* err, uint32_t* work, bool count_stats,
                                       hipStream_t s) {
    constexpr uint32_t block = 1024;
    const size_t lds = wavepersist_lds_bytes(sc, kLds);
    auto kern = count_stats ? k_trace_wavepersist<true, kLds, kForm> : k_trace_wavepersist<false, kLds, kForm>;
    int per_cu = 0, dev = 0, cus = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, (int)block, lds);
    if (e != hipSuccess) return e;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint64_t n_paths = (uint64_t)job.w * job.h * job.e.spp * job.n_frames;
    // MM_OPT_RESERVE_CUS: leave that many CUs' worth of resident blocks free for other work (collectives)
    const int cus_used = std::max(1, cus - (int)job.reserve_cus);
    uint64_t grid = (uint64_t)std::max(1, per_cu) * (uint64_t)cus_used;
    grid = std::max<uint64_t>(1, std::min<uint64_t>(grid, (n_paths + block - 1) / block));
    hipLaunchKernelGGL(kern, dim3((uint32_t)grid), dim3(block), lds, s, sc, job, samples, stats, err, work);
    return hipGetLastError();
}

hipError_t launch_trace_wavepersist(const DevScene& sc, const TileJob& job, float4* samples,
                                    unsigned long long* stats, uint32_t* err, uint32_t* work, bool count_stats,
                                    int lds_mode, int form, hipStream_t s) {
#define MM_WP(L, F) \
    if (lds_mode == L && form == F) return launch_wavepersist_t<L, F>(sc, job, samples, stats, err, work, count_stats, s);
    MM_WP(11, kFormGrid) MM_WP(12, kFormGrid) MM_WP(13, kFormGrid)
    MM_WP(3, kFormLean) MM_WP(6, kFormLean) MM_WP(7, kFormLean) MM_WP(10, kFormLean)
    MM_WP(0, kFormLeafInterior) MM_WP(1, kFormLeafInterior) MM_WP(3, kFormLeafInterior) MM_WP(6, kFormLeafInterior)
    MM_WP(7, kFormLeafInterior) MM_WP(10, kFormLeafInterior)
    MM_WP(1, kFormIfIf) MM_WP(3, kFormIfIf)
#undef MM_WP
    return hipErrorInvalidValue;
}

template <bool kRef, bool kLds>
static void launch_mega_t(const DevScene& sc, const TileJob& job, float4* samples, unsigned long long* stats,
                          uint32_t* err, bool count_stats, uint32_t block, hipStream_t s) {
    const uint32_t n = job.w * job.h * job.e.spp;
    const dim3 grid((n + block - 1) / block);
    const size_t lds = kLds ? 2 * (size_t)sc.n_nodes * sizeof(float4) : 0;
    if (count_stats)
        hipLaunchKernelGGL((k_trace_mega<true, kRef, kLds>), grid, dim3(block), lds, s, sc, job, samples, stats, err);
    else
        hipLaunchKernelGGL((k_trace_mega<false, kRef, kLds>), grid, dim3(block), lds, s, sc, job, samples, stats, err);
}

hipError_t launch_trace_mega(const DevScene& sc, const TileJob& job, float4* samples, unsigned long long* stats_dev,
                             uint32_t* err, bool count_stats, const MegaOpts& o, hipStream_t s) {
    if (o.reference)
        launch_mega_t<true, false>(sc, job, samples, stats_dev, err, count_stats, o.block, s);
    else if (o.lds_nodes)
        launch_mega_t<false, true>(sc, job, samples, stats_dev, err, count_stats, o.block, s);
    else
        launch_mega_t<false, false>(sc, job, samples, stats_dev, err, count_stats, o.block, s);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Sample reduction: spp % 8 == 0 -> pairwise tree in blocks of 8, blocks added
// left to right (the reference order for 64 spp); otherwise left to right.
__global__ void k_resolve(TileJob job, const float4* __restrict__ samples, float4* __restrict__ out) {
    const uint32_t pix = blockIdx.x * blockDim.x + threadIdx.x;
    if (pix >= job.w * job.h) return;
    const uint32_t spp = job.e.spp;
    const float4* s = samples + (size_t)pix * spp;
    F3 acc;
    if (spp % 8 == 0) {
        for (uint32_t b = 0; b < spp; b += 8) {
            const F3 p0 = xyz(s[b + 0]) + xyz(s[b + 1]), p1 = xyz(s[b + 2]) + xyz(s[b + 3]);
            const F3 p2 = xyz(s[b + 4]) + xyz(s[b + 5]), p3 = xyz(s[b + 6]) + xyz(s[b + 7]);
            const F3 blk = (p0 + p1) + (p2 + p3);
            acc = (b == 0) ? blk : acc + blk;
        }
    } else {
        acc = xyz(s[0]);
        for (uint32_t k = 1; k < spp; ++k) acc = acc + xyz(s[k]);
    }
    const float m = (float)spp;
    const F3 v = F3{acc.x / m, acc.y / m, acc.z / m};
    if (job.e.flags & MM_EXT_ACCUMULATE) {
        float4 o = out[pix];
        out[pix] = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + 1.0f);
    } else {
        out[pix] = make_float4(v.x, v.y, v.z, 1.0f);
    }
}

hipError_t launch_resolve(const TileJob& job, const float4* samples, float4* out, hipStream_t s) {
    const uint32_t n = job.w * job.h;
    hipLaunchKernelGGL(k_resolve, dim3((n + 255) / 256), dim3(256), 0, s, job, samples, out);
    return hipGetLastError();
}

}  // namespace mm
