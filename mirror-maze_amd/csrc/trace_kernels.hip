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
//
// Mirror-tail deferral (job.defer_from < 2^30): once at most defer_lanes of a
// wave's 64 lanes still run -- past bounce_limit only paths that hit mirrors
// continue (shaders.metal:306, `n < bounce_limit + mirror_hits`) -- those
// lanes queue their path state and the wave takes a new chunk; k_trace_tail
// then runs the queued tails 64 to a wave.  On C3 a
// wave otherwise spends ~27 % of its bounce iterations on <= 12 live lanes
// (scripts/grid_sim.c).  Samples are then staged per path and resolved by
// k_resolve (the same operations in the same order as the fused resolve).

// A deferred path's state into its reserved queue entry.
__device__ __forceinline__ void tail_store(const TailQueue& q, uint32_t i, const PathState& p, uint32_t slot) {
    q.f(0)[i] = p.ori.x; q.f(1)[i] = p.ori.y; q.f(2)[i] = p.ori.z;
    q.f(3)[i] = p.dir.x; q.f(4)[i] = p.dir.y; q.f(5)[i] = p.dir.z;
    q.f(6)[i] = p.T.x; q.f(7)[i] = p.T.y; q.f(8)[i] = p.T.z;
    q.f(9)[i] = p.L.x; q.f(10)[i] = p.L.y; q.f(11)[i] = p.L.z;
    q.u(0)[i] = p.seed;
    q.u(1)[i] = (uint32_t)p.n | ((uint32_t)p.mh << 16);
    q.u(2)[i] = slot;
}

__device__ __forceinline__ F3 path_value(const PathState& p) {
    return F3{sqrtf(fmaxf(p.L.x, 0.0f)), sqrtf(fmaxf(p.L.y, 0.0f)), sqrtf(fmaxf(p.L.z, 0.0f))};
}

template <bool kStats, bool kDefer, typename Q>
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
            PathState p;
            p.seed = seed_tile(py * job.view_w + px, smp, job.e.frame + fr);
            p.dir = jitter(primary_dir(job.u, px, py), p.seed);
            p.ori = ori;
            p.T = F3{1.0f, 1.0f, 1.0f};
            p.L = F3{0.0f, 0.0f, 0.0f};
            p.n = 0;
            p.mh = 0;
            bool overflow = false;
            uint32_t qi = 0;
            bool deferred = false;
            if constexpr (kDefer)
                deferred = bounce_loop<kStats>(sc, q, p, (int)job.e.bounce_limit, (int)job.e.mirror_limit, stack, c,
                                               overflow, (int)job.defer_from, job.defer_lanes, job.tail.count,
                                               job.tail.cap, &qi);
            else
                bounce_loop<kStats>(sc, q, p, (int)job.e.bounce_limit, (int)job.e.mirror_limit, stack, c, overflow,
                                    1 << 30, 0u);
            if (overflow) atomicOr(err, 1u);
            const uint32_t slot = fr * n_paths + path;
            if (deferred) tail_store(job.tail, qi, p, slot);
            if (!deferred) {
                s = path_value(p);
                if (!job.fuse) samples[slot] = make_float4(s.x, s.y, s.z, 0.0f);
                paths++;
            }
        }
        if (job.fuse) resolve_in_wave(job, s, path, valid, job.out + (size_t)fr * job.w * job.h);
    }
#ifdef MM_PHASE_CLOCKS
    {  // the wave's time in queries / shading: the max over its lanes (some lane runs every iteration)
        uint64_t qc = c.q_cyc, sc2 = c.s_cyc;
        for (int o = 32; o > 0; o >>= 1) {
            qc = max(qc, (uint64_t)__shfl_xor((unsigned long long)qc, o));
            sc2 = max(sc2, (uint64_t)__shfl_xor((unsigned long long)sc2, o));
        }
        if (job.wave_ts && lane == 0) {
            const uint32_t wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
            if (wid < job.wave_ts_cap) {
                job.wave_ts[4 * wid + 1] = qc;
                job.wave_ts[4 * wid + 3] = sc2;
            }
        }
    }
#endif
    if (kStats) flush_stats(stats, c, paths);
    return chunks;
}

// The deferred tails: waves take 64 queued paths at a time and finish them.
template <bool kStats, typename Q>
__device__ __forceinline__ uint32_t tail_body(const DevScene& sc, const Q& q, const TileJob& job,
                                              float4* __restrict__ samples, unsigned long long* stats,
                                              uint32_t* err, uint32_t*) {
    const TailQueue& tq = job.tail;
    const uint32_t n = min(tq.count[0], tq.cap);  // reservations past cap were not used
    const uint32_t lane = threadIdx.x & 63u;
    Counters c;
    ScratchStack stack;
    uint32_t paths = 0, chunks = 0;
#ifdef MM_TAIL_TIMELINE
    uint32_t wave_iters = 0;
#endif
    for (;;) {
        uint32_t b = 0;
        if (lane == 0) b = atomicAdd(tq.count + 1, 64u);
        const uint32_t base = __builtin_amdgcn_readfirstlane(b);
        if (base >= n) break;
        ++chunks;
        const uint32_t i = base + lane;
#ifdef MM_TAIL_TIMELINE
        int lane_bounces = 0;
#endif
        if (i < n) {
            PathState p;
            p.ori = F3{tq.f(0)[i], tq.f(1)[i], tq.f(2)[i]};
            p.dir = F3{tq.f(3)[i], tq.f(4)[i], tq.f(5)[i]};
            p.T = F3{tq.f(6)[i], tq.f(7)[i], tq.f(8)[i]};
            p.L = F3{tq.f(9)[i], tq.f(10)[i], tq.f(11)[i]};
            p.seed = tq.u(0)[i];
            const uint32_t nm = tq.u(1)[i];
            p.n = (int)(nm & 0xFFFFu);
            p.mh = (int)(nm >> 16);
            bool overflow = false;
#ifdef MM_TAIL_TIMELINE
            const int n0 = p.n;
#endif
            bounce_loop<kStats>(sc, q, p, (int)job.e.bounce_limit, (int)job.e.mirror_limit, stack, c, overflow,
                                1 << 30, 0u);
#ifdef MM_TAIL_TIMELINE
            lane_bounces = p.n - n0 + 1;
#endif
            if (overflow) atomicOr(err, 1u);
            const F3 s = path_value(p);
            samples[tq.u(2)[i]] = make_float4(s.x, s.y, s.z, 0.0f);
            paths++;
        }
#ifdef MM_TAIL_TIMELINE  // the wave's bounce iterations for this chunk: its lanes' maximum
        for (int o = 32; o > 0; o >>= 1) lane_bounces = max(lane_bounces, __shfl_xor(lane_bounces, o));
        wave_iters += (uint32_t)lane_bounces;
#endif
    }
    if (kStats) flush_stats(stats, c, paths);
#ifdef MM_TAIL_TIMELINE
    return wave_iters;
#endif
    return chunks;
}

// LDS modes (what a resident block stages before tracing; the rest is read
// through L1/L2):
//   0  nothing (nodes, records global)           BVH forms 5
//   1  BVH nodes                                  BVH forms 0 / 5 (general rect test)
//   3  BVH nodes + compact slot records           BVH forms 0 / 5 / 7
//   6  top of the breadth-first node array        BVH forms 5 / 7 (split cache)
//   7  BVH nodes, compact records global          BVH forms 5 / 7
//   10 dictionary-coded nodes, records global     BVH forms 5 / 7
//   11 the whole grid image                       grid search
//   12 grid cells + lists, records + boxes global grid search
//   13 nothing (the grid image global)             grid search
// stage_and_run fills the block's LDS for the mode and calls body(query).
template <int kLds, int kForm, bool kStats, typename F>
__device__ __forceinline__ uint32_t stage_and_run(const DevScene& sc, const TileJob& job, F&& body) {
    extern __shared__ float4 lds[];
    auto staged = [&]() {  // diagnostics: time at which the block's LDS staging completed (wave timeline)
        if (job.wave_ts && (threadIdx.x & 63u) == 0) {
            const uint32_t wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
#ifndef MM_PHASE_CLOCKS
            if (wid < job.wave_ts_cap) job.wave_ts[4 * wid + 1] = (unsigned long long)wall_clock64();
#endif
        }
    };
    if constexpr (kLds == 11) {
        // records + boxes first, at LDS address 0 (a constant in the rect test),
        // then cells + lists
        const uint32_t nr16 = (sc.grid.bytes - sc.grid.off_recs) / 16u, ni16 = sc.grid.off_recs / 16u;
        uint4* img = reinterpret_cast<uint4*>(lds);
        const uint4* src = sc.grid.image;
        for (uint32_t i = threadIdx.x; i < nr16; i += blockDim.x) img[i] = src[ni16 + i];
        for (uint32_t i = threadIdx.x; i < ni16; i += blockDim.x) img[nr16 + i] = src[i];
        __syncthreads();
        staged();
        const char* base = reinterpret_cast<const char*>(lds);
        const char* index = base + 16u * nr16;
        const auto gv = grid_view(reinterpret_cast<const char*>(index),
                                  reinterpret_cast<const uint16_t*>(index + sc.grid.off_list),
                                  reinterpret_cast<const uint4*>(lds),
                                  reinterpret_cast<const float2*>(base + (sc.grid.off_box - sc.grid.off_recs)));
        return body(GridQuery<kStats, kForm == kFormGridSlow || kForm == kFormGridWideSlow, kForm >= kFormGridWide, decltype(gv)>{sc, gv});
    } else if constexpr (kLds == 12) {
        const uint32_t n16 = sc.grid.off_recs / 16u;
        uint4* img = reinterpret_cast<uint4*>(lds);
        for (uint32_t i = threadIdx.x; i < n16; i += blockDim.x) img[i] = sc.grid.image[i];
        __syncthreads();
        staged();
        const char* base = reinterpret_cast<const char*>(lds);
        const auto gv = grid_view(reinterpret_cast<const char*>(base),
                                  reinterpret_cast<const uint16_t*>(base + sc.grid.off_list), sc.grid.recs,
                                  sc.grid.box);
        return body(GridQuery<kStats, kForm == kFormGridSlow || kForm == kFormGridWideSlow, kForm >= kFormGridWide, decltype(gv)>{sc, gv});
    } else if constexpr (kLds == 13) {
        const auto gv = grid_view(reinterpret_cast<const char*>(sc.grid.cells), sc.grid.list, sc.grid.recs, sc.grid.box);
        return body(GridQuery<kStats, kForm == kFormGridSlow || kForm == kFormGridWideSlow, kForm >= kFormGridWide, decltype(gv)>{sc, gv});
    } else if constexpr (kLds == 6) {
        for (uint32_t i = threadIdx.x; i < sc.n_lds_f4; i += blockDim.x) lds[i] = sc.nodes[i];
        __syncthreads();
        staged();
        const auto v = view(SplitNodes{lds, sc.nodes, sc.n_lds_f4}, sc.recs);
        return body(BvhQuery<kStats, kForm, decltype(v)>{sc, v});
    } else if constexpr (kLds == 10) {
        float* tab = reinterpret_cast<float*>(lds);
        uint32_t* words = reinterpret_cast<uint32_t*>(tab + 256);
        for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) tab[i] = sc.dict_tab[i];
        for (uint32_t i = threadIdx.x; i < 3 * sc.n_nodes; i += blockDim.x) words[i] = sc.dict_words[i];
        __syncthreads();
        staged();
        const auto v = view(DictNodes{words, tab}, sc.recs);
        return body(BvhQuery<kStats, kForm, decltype(v)>{sc, v});
    } else if constexpr (kLds == 1 || kLds == 3 || kLds == 7) {
        for (uint32_t i = threadIdx.x; i < 2 * sc.n_nodes; i += blockDim.x) lds[i] = sc.nodes[i];
        uint2* lds_recs = reinterpret_cast<uint2*>(lds + 2 * sc.n_nodes);
        if constexpr (kLds == 3)
            for (uint32_t i = threadIdx.x; i < 5 * sc.n_rects; i += blockDim.x) lds_recs[i] = sc.recs[i];
        __syncthreads();
        staged();
        if constexpr (kLds == 3) {
            const auto v = view(static_cast<float4*>(lds), lds_recs);
            return body(BvhQuery<kStats, kForm, decltype(v)>{sc, v});
        } else if constexpr (kLds == 7) {
            const auto v = view(static_cast<float4*>(lds), sc.recs);
            return body(BvhQuery<kStats, kForm, decltype(v)>{sc, v});
        } else {
            const auto v = view(static_cast<float4*>(lds));
            return body(BvhQuery<kStats, kForm, decltype(v)>{sc, v});
        }
    } else {
        const auto v = view(sc.nodes);
        return body(BvhQuery<kStats, kForm, decltype(v)>{sc, v});
    }
}

// Per-wave diagnostics record and the self-cleaning counter pair shared by the
// persistent kernels (counter[0] = next item, counter[1] = waves done; the
// last wave to finish re-zeroes the words, so the next launch needs no memset
// -- a fill kernel queued between two frames on another stream would wait for
// free CUs and serialise overlapping frames).  `extra` (or null): a third word
// the last wave also clears (the tail queue's entry count).
__device__ __forceinline__ void persistent_exit(const TileJob& job, uint32_t chunks, unsigned long long t_entry,
                                                uint32_t* counter, uint32_t* extra) {
    if (job.wave_ts && (threadIdx.x & 63u) == 0) {
        const uint32_t wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        if (wid < job.wave_ts_cap) {
#ifdef MM_PHASE_CLOCKS  // (entry, query cycles, exit, shade cycles), s_memtime
            job.wave_ts[4 * wid + 0] = t_entry;
            job.wave_ts[4 * wid + 2] = (unsigned long long)wall_clock64();
#else
            job.wave_ts[4 * wid + 0] = t_entry;
            job.wave_ts[4 * wid + 2] = (unsigned long long)wall_clock64();
            job.wave_ts[4 * wid + 3] = chunks;
#endif
        }
    }
    if ((threadIdx.x & 63u) == 0) {
        __threadfence();
        const uint32_t total = gridDim.x * (blockDim.x >> 6);
        if (atomicAdd(counter + 1, 1u) == total - 1) {
            atomicExch(counter, 0u);
            atomicExch(counter + 1, 0u);
            if (extra) atomicExch(extra, 0u);
        }
    }
}

// 1024-thread blocks at 8 waves per SIMD (<= 64 VGPRs).  With the grid search,
// 768-thread blocks at 6 waves (80 VGPRs, no VGPR spills) measured 6.21 vs
// 5.87 ms on C3 (profiles/r02_ab_grid_variants.txt).
template <bool kStats, int kLds, int kForm, bool kDefer>
__global__ __launch_bounds__(1024, 8) void k_trace_wavepersist(DevScene sc, TileJob job, float4* __restrict__ samples,
                                                               unsigned long long* stats, uint32_t* err,
                                                               uint32_t* work) {
#ifdef MM_PHASE_CLOCKS
    const unsigned long long t_entry = job.wave_ts ? (unsigned long long)wall_clock64() : 0ull;
#else
    const unsigned long long t_entry = job.wave_ts ? (unsigned long long)wall_clock64() : 0ull;
#endif
    const uint32_t chunks = stage_and_run<kLds, kForm, kStats>(sc, job, [&](const auto& q) {
        return wavepersist_body<kStats, kDefer>(sc, q, job, samples, stats, err, work);
    });
    persistent_exit(job, chunks, t_entry, work, nullptr);
}

template <bool kStats, int kLds, int kForm>
__global__ __launch_bounds__(1024, 8) void k_trace_tail(DevScene sc, TileJob job, float4* __restrict__ samples,
                                                        unsigned long long* stats, uint32_t* err) {
    const unsigned long long t_entry = job.wave_ts ? (unsigned long long)wall_clock64() : 0ull;
    const uint32_t chunks = stage_and_run<kLds, kForm, kStats>(sc, job, [&](const auto& q) {
        return tail_body<kStats>(sc, q, job, samples, stats, err, nullptr);
    });
    persistent_exit(job, chunks, t_entry, job.tail.count + 1, job.tail.count);
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

// Resident grid of a persistent kernel: blocks per CU from the occupancy API x
// CUs (minus MM_OPT_RESERVE_CUS), capped by the work.
template <typename K>
static uint32_t persistent_grid(K kern, size_t lds, uint32_t reserve_cus, uint64_t items) {
    int per_cu = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 1024, lds) != hipSuccess) return 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int cus_used = std::max(1, cus - (int)reserve_cus);
    uint64_t grid = (uint64_t)std::max(1, per_cu) * (uint64_t)cus_used;
    return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(grid, (items + 1023) / 1024));
}

template <int kLds, int kForm, bool kDefer>
static hipError_t launch_wavepersist_t(const DevScene& sc, const TileJob& job, float4* samples,
                                       unsigned long long* stats, uint32_t* err, uint32_t* work, bool count_stats,
                                       hipStream_t s) {
    const size_t lds = wavepersist_lds_bytes(sc, kLds);
    auto kern = count_stats ? k_trace_wavepersist<true, kLds, kForm, kDefer>
                            : k_trace_wavepersist<false, kLds, kForm, kDefer>;
    const uint32_t grid =
        persistent_grid(kern, lds, job.reserve_cus, (uint64_t)job.w * job.h * job.e.spp * job.n_frames);
    if (!grid) return hipErrorInvalidValue;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(1024), lds, s, sc, job, samples, stats, err, work);
    return hipGetLastError();
}

template <int kLds, int kForm>
static hipError_t launch_tail_t(const DevScene& sc, const TileJob& job, float4* samples, unsigned long long* stats,
                                uint32_t* err, bool count_stats, hipStream_t s) {
    const size_t lds = wavepersist_lds_bytes(sc, kLds);
    auto kern = count_stats ? k_trace_tail<true, kLds, kForm> : k_trace_tail<false, kLds, kForm>;
    // the queue length is known on the device only: a full resident grid (each wave drains 64 at a time)
    const uint32_t grid = persistent_grid(kern, lds, job.reserve_cus, ~0ull >> 1);
    if (!grid) return hipErrorInvalidValue;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(1024), lds, s, sc, job, samples, stats, err);
    return hipGetLastError();
}

// (LDS mode, form) pairs; the tail-deferral variant (MM_OPT_DEFER) is built
// for the grid search and the lean BVH form with records in LDS
#define MM_DEFER_INSTANCES(X)                                                                                 \
    X(11, kFormGrid) X(12, kFormGrid) X(13, kFormGrid)                                                        \
    X(11, kFormGridSlow) X(12, kFormGridSlow) X(13, kFormGridSlow)                                            \
    X(11, kFormGridWide) X(13, kFormGridWide) X(11, kFormGridWideSlow) X(13, kFormGridWideSlow)               \
    X(3, kFormLean)
#define MM_WP_INSTANCES(X)                                                                                    \
    MM_DEFER_INSTANCES(X) X(6, kFormLean) X(7, kFormLean) X(10, kFormLean)                                    \
    X(0, kFormLeafInterior) X(1, kFormLeafInterior) X(3, kFormLeafInterior) X(6, kFormLeafInterior)           \
    X(7, kFormLeafInterior) X(10, kFormLeafInterior)                                                          \
    X(1, kFormIfIf) X(3, kFormIfIf)

bool wavepersist_defer_built(int lds_mode, int form) {
#define MM_WP(L, F) if (lds_mode == L && form == F) return true;
    MM_DEFER_INSTANCES(MM_WP)
#undef MM_WP
    return false;
}

hipError_t launch_trace_wavepersist(const DevScene& sc, const TileJob& job, float4* samples,
                                    unsigned long long* stats, uint32_t* err, uint32_t* work, bool count_stats,
                                    int lds_mode, int form, hipStream_t s) {
    const bool defer = job.defer_from < (1u << 30);
#define MM_WP(L, F)                                                                                          \
    if (lds_mode == L && form == F && defer)                                                                 \
        return launch_wavepersist_t<L, F, true>(sc, job, samples, stats, err, work, count_stats, s);
    MM_DEFER_INSTANCES(MM_WP)
#undef MM_WP
#define MM_WP(L, F)                                                                                          \
    if (lds_mode == L && form == F && !defer)                                                                \
        return launch_wavepersist_t<L, F, false>(sc, job, samples, stats, err, work, count_stats, s);
    MM_WP_INSTANCES(MM_WP)
#undef MM_WP
    return hipErrorInvalidValue;
}

hipError_t launch_trace_tail(const DevScene& sc, const TileJob& job, float4* samples, unsigned long long* stats,
                             uint32_t* err, bool count_stats, int lds_mode, int form, hipStream_t s) {
#define MM_WP(L, F) \
    if (lds_mode == L && form == F) return launch_tail_t<L, F>(sc, job, samples, stats, err, count_stats, s);
    MM_DEFER_INSTANCES(MM_WP)
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

// The same reduction when 64 % spp == 0, a wave per 64 consecutive samples
// (64/spp whole pixels): every load is one coalesced 1-KB wave access, and
// resolve_in_wave adds in k_resolve's order (bit-identical).
__global__ __launch_bounds__(256) void k_resolve_wave(TileJob job, const float4* __restrict__ samples,
                                                      float4* __restrict__ out) {
    const uint32_t n = job.w * job.h * job.e.spp;
    const uint32_t path = blockIdx.x * blockDim.x + threadIdx.x;  // waves never straddle the end: n % 64 == 0
    const bool valid = path < n;                                   // unless the tile is ragged
    const float4 v = valid ? samples[path] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    resolve_in_wave(job, F3{v.x, v.y, v.z}, path, valid, out);
}

hipError_t launch_resolve(const TileJob& job, const float4* samples, float4* out, hipStream_t s) {
    const uint32_t n = job.w * job.h;
    if (64 % job.e.spp == 0) {
        const uint32_t paths = n * job.e.spp;
        hipLaunchKernelGGL(k_resolve_wave, dim3((paths + 255) / 256), dim3(256), 0, s, job, samples, out);
    } else {
        hipLaunchKernelGGL(k_resolve, dim3((n + 255) / 256), dim3(256), 0, s, job, samples, out);
    }
    return hipGetLastError();
}

}  // namespace mm
