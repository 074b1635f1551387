// trace_kernels.hip — gfx950 kernels for mirror-maze's per-pixel ray-trace loop.
//
//   k_prep_rects      per-rect subexpressions of ray_rect_intersect
//   k_trace_chunks    parity mode: the reference dispatch (shaders.metal:245-368)
//   k_trace_mega      throughput mode, one thread per (pixel, sample) path
//   k_resolve         per-pixel sample reduction in the reference's order
#include <hip/hip_runtime.h>

#include <type_traits>

#include "mm_launch.h"
#include "mm_trace.h"
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

hipError_t launch_prep_rects(const mm_rect* rects_dev, uint32_t n, float4* geo_dev, hipStream_t s) {
    hipLaunchKernelGGL(k_prep_rects, dim3((n + 255) / 256), dim3(256), 0, s, rects_dev, n, geo_dev);
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
    F3 s = trace_path<kStats, false>(sc, view(sc.nodes), ori, d, seed, 5, 15, stack, c, overflow);  // shaders.metal:294-295
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
// Throughput mode megakernel: path = pixel*spp + sample.
//   kRef  : traverse_reference (IEEE division everywhere), for A/B
//   kLds  : stage the node array in LDS (dynamic shared memory) first
template <bool kStats, bool kRef, bool kLds>
__global__ __launch_bounds__(1024) void k_trace_mega(DevScene sc, TileJob job, float4* __restrict__ samples,
                                                     unsigned long long* stats, uint32_t* err) {
    extern __shared__ float4 lds_nodes[];
    if constexpr (kLds) {
        for (uint32_t i = threadIdx.x; i < 2 * sc.n_nodes; i += blockDim.x) lds_nodes[i] = sc.nodes[i];
        __syncthreads();
    }
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
        F3 s;
        if constexpr (kLds)
            s = trace_path<kStats, kRef>(sc, view(lds_nodes), ori, d, seed, (int)job.e.bounce_limit,
                                         (int)job.e.mirror_limit, stack, c, overflow);
        else
            s = trace_path<kStats, kRef>(sc, view(sc.nodes), ori, d, seed, (int)job.e.bounce_limit,
                                         (int)job.e.mirror_limit, stack, c, overflow);
        if (overflow) atomicOr(err, 1u);
        samples[path] = make_float4(s.x, s.y, s.z, 0.0f);
    }
    if (kStats) flush_stats(stats, c, path < n_paths ? 1u : 0u);
}

// Wave-persistent megakernel: resident blocks (LDS filled once per block);
// each wave takes 64 consecutive paths at a time from a global counter and
// traces them exactly like k_trace_mega, so no block waits for its slowest
// wave before the CU can take more work.
template <bool kStats, int kWW, typename V, typename Stack, typename Cold = NoCold>
__device__ __forceinline__ uint32_t wavepersist_body(const DevScene& sc, const V& v, Stack& stack,
                                                 const TileJob& job, float4* __restrict__ samples,
                                                 unsigned long long* stats, uint32_t* err, uint32_t* work,
                                                 const Cold& cold = Cold{}) {
    const uint32_t spp = job.e.spp;
    const uint32_t n_paths = job.w * job.h * spp;         // per frame
    const uint32_t cpf = (n_paths + 63u) / 64u;           // 64-path chunks per frame
    const uint32_t n_queue = cpf * 64u * job.n_frames;    // the queue, in paths (chunks padded to 64)
    const uint32_t lane = threadIdx.x & 63u;
    const F3 ori = F3{job.u.cam.center[0], job.u.cam.center[1], job.u.cam.center[2]};
    Counters c;
    uint32_t paths = 0, chunks = 0;
    const uint32_t n_waves = gridDim.x * (blockDim.x >> 6);
    const uint32_t grab = 64u * job.grab;   // paths claimed per atomic (MM_OPT_GRAB chunks)
    uint32_t next = 0, end = 0;             // wave-uniform claimed range
    for (;;) {
        if (next >= end) {
            uint32_t b = 0;
            if (lane == 0) b = atomicAdd(work, grab);
            next = __builtin_amdgcn_readfirstlane(b);
            end = min(next + grab, n_queue);
        }
        const uint32_t base = next;
        next += 64u;
        if (base >= n_queue) break;
        // MM_OPT_FAIR: a wave behind the mean chunk count runs at raised issue
        // priority (the SIMD arbiter otherwise favours the oldest waves: chunk
        // counts per wave spread 9-59 on C3, 28-37 with this on; the frame time
        // does not change -- profiles/r01_timeline_probe.txt).
        if (job.fair) {
            if (__builtin_amdgcn_readfirstlane((uint64_t)chunks * n_waves < base / 64u ? 1u : 0u))
                __builtin_amdgcn_s_setprio(1);
            else
                __builtin_amdgcn_s_setprio(0);
        }
        ++chunks;
        // MM_OPT_CHUNK_ORDER: queue position -> chunk through the cost-sorted
        // permutation (paths are keyed by pixel/sample, so any order gives the
        // same samples); the chunk's duration is recorded for the next sort
        // queue position -> (frame, chunk of the frame); one frame: frame 0, chunk = position
        const uint32_t q = base >> 6;
        const uint32_t fr = job.n_frames > 1 ? q / cpf : 0u;
        const uint32_t qc = q - fr * cpf;
        const uint32_t chunk = job.order ? __builtin_amdgcn_readfirstlane(job.order[qc]) : qc;
        const unsigned long long t_chunk = job.cost ? (unsigned long long)wall_clock64() : 0ull;
        const uint32_t path = chunk * 64u + lane;
        const bool valid = path < n_paths;
        F3 s = F3{0.0f, 0.0f, 0.0f};
        if (valid) {
            const uint32_t pix = path / spp, smp = path - pix * spp;
            const uint32_t j = pix / job.w, i = pix - j * job.w;
            const uint32_t px = job.x0 + i, py = job.y0 + j * job.y_stride;
            uint32_t seed = seed_tile(py * job.view_w + px, smp, job.e.frame + fr);
            const F3 d = jitter(primary_dir(job.u, px, py), seed);
            bool overflow = false;
            s = trace_path<kStats, false, V, Stack, kWW>(sc, v, ori, d, seed, (int)job.e.bounce_limit,
                                                         (int)job.e.mirror_limit, stack, c, overflow, cold);
            if (overflow) atomicOr(err, 1u);
            if (!job.fuse) samples[path] = make_float4(s.x, s.y, s.z, 0.0f);
            paths++;
        }
        if (job.fuse) resolve_in_wave(job, s, path, valid, job.out + (size_t)fr * job.w * job.h);
        if (job.cost && lane == 0 && fr == 0)
            job.cost[chunk] = (uint32_t)((unsigned long long)wall_clock64() - t_chunk);
    }
    if (kStats) flush_stats(stats, c, paths);
    return chunks;
}

// Bounce-refill form of the wave-persistent body (loop form 4): a lane whose
// path ends takes the next path of the wave's chunk at the next bounce
// boundary instead of idling until the wave's longest path ends.  The wave
// runs one bounce (closest hit + shade) per iteration for all lanes; every
// path's operation sequence is trace_path's, so samples are bit-identical.
template <bool kStats, typename V, typename Stack, int kTrav = 0, typename Cold = NoCold>
__device__ __forceinline__ uint32_t bouncerefill_body(const DevScene& sc, const V& v, Stack& stack, const TileJob& job,
                                                  float4* __restrict__ samples, unsigned long long* stats,
                                                  uint32_t* err, uint32_t* work) {
    const uint32_t spp = job.e.spp;
    const uint32_t n_paths = job.w * job.h * spp;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    const int bounce_limit = (int)job.e.bounce_limit, mirror_limit = (int)job.e.mirror_limit;
    Counters c;
    uint32_t paths = 0;
    uint32_t chunk_base = 0, chunk_end = 0;  // wave-uniform
    bool more = true, active = false;
    uint32_t pid = 0;
    PathState p;
    for (;;) {
        const uint64_t idle = __ballot(!active);
        if (idle && (more || chunk_base < chunk_end)) {
            const uint32_t need = (uint32_t)__popcll(idle), rank = (uint32_t)__popcll(idle & lt);
            const uint32_t take1 = min(need, chunk_end - chunk_base);
            bool got = !active && rank < take1;
            uint32_t mine = chunk_base + rank;
            chunk_base += take1;
            if (take1 < need && more) {
                uint32_t b = 0;
                if (lane == 0) b = atomicAdd(work, 64u);
                b = __shfl(b, 0);
                if (b >= n_paths) {
                    more = false;
                } else {
                    chunk_base = b;
                    chunk_end = min(b + 64u, n_paths);
                    const uint32_t take2 = min(need - take1, chunk_end - chunk_base);
                    if (!active && rank >= take1 && rank < take1 + take2) {
                        got = true;
                        mine = chunk_base + (rank - take1);
                    }
                    chunk_base += take2;
                }
            }
            if (got) {
                pid = mine;
                const uint32_t pix = mine / spp, smp = mine - pix * spp;
                const uint32_t j = pix / job.w, i = pix - j * job.w;
                const uint32_t px = job.x0 + i, py = job.y0 + j * job.y_stride;
                p.seed = seed_tile(py * job.view_w + px, smp, job.e.frame);
                p.dir = jitter(primary_dir(job.u, px, py), p.seed);
                p.ori = F3{job.u.cam.center[0], job.u.cam.center[1], job.u.cam.center[2]};
                p.T = F3{1.0f, 1.0f, 1.0f};
                p.L = F3{0.0f, 0.0f, 0.0f};
                p.n = 0;
                p.mh = 0;
                active = true;
            }
        }
        if (!__ballot(active)) break;
        if (active) {
            bool fin = !(p.n < bounce_limit + p.mh);
            if (!fin) {  // one bounce: shaders.metal:306-340
                float t = kBig;
                uint32_t k = 0;
                const bool ok = closest_hit<kStats, V, Stack, kTrav>(sc, v, p.ori, p.dir, t, k, stack, c);
                if (kStats) c.rays++;
                if (!ok) atomicOr(err, 1u);
                fin = !ok || !shade_step(sc, p, t, k, mirror_limit);
                p.n++;
                fin = fin || !(p.n < bounce_limit + p.mh);
            }
            if (fin) {
                samples[pid] = make_float4(sqrtf(fmaxf(p.L.x, 0.0f)), sqrtf(fmaxf(p.L.y, 0.0f)),
                                           sqrtf(fmaxf(p.L.z, 0.0f)), 0.0f);
                paths++;
                active = false;
            }
        }
    }
    if (kStats) flush_stats(stats, c, paths);
    return 0;
}

template <bool kStats, int kWW, typename V, typename Stack, typename Cold = NoCold>
__device__ __forceinline__ uint32_t wp_dispatch(const DevScene& sc, const V& v, Stack& stack, const TileJob& job,
                                                float4* __restrict__ samples, unsigned long long* stats,
                                                uint32_t* err, uint32_t* work, const Cold& cold = Cold{}) {
    if constexpr (kWW == 4) return bouncerefill_body<kStats>(sc, v, stack, job, samples, stats, err, work);
    else if constexpr (kWW == 6) return bouncerefill_body<kStats, V, Stack, 5>(sc, v, stack, job, samples, stats, err, work);
    else return wavepersist_body<kStats, kWW>(sc, v, stack, job, samples, stats, err, work, cold);
}

// Traversal stack of the wave-persistent kernel: loop form 3 is the if-if loop
// with the register-top stack (RegTopStack), every other form the scratch array.
template <int kWW> using WpStack = std::conditional_t<kWW == 3, RegTopStack, ScratchStack>;

// kLds: 0 nodes via L1/L2 + scratch stack, 1 nodes in LDS + scratch stack,
// 2 nodes in LDS + u16 stack in LDS (stack_slots entries per thread),
// 3 nodes + compact rect records in LDS, 4 top of the tree in LDS (the first
// sc.n_lds_f4 float4s of the breadth-first node array), the rest via L1/L2,
// 5 nodes in LDS + each path's T and L parked in LDS while it traverses,
// 6 = 4 + compact rect records read through L1/L2, 7 = 1 + the same,
// 8 = 2 + the same (nodes and u16 stack in LDS, rect records via L1/L2),
// 9 = 3 with u16 traversal-stack entries in scratch, 10 dictionary-coded nodes
// in LDS (DictNodes) + compact rect records read through L1/L2.
// Diagnostics: time at which the block's LDS staging completed (wave timeline).
#define MM_TS_STAGED()                                                                                      \
    do {                                                                                                     \
        if (job.wave_ts && (threadIdx.x & 63u) == 0) {                                                       \
            const uint32_t wid_ = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);                      \
            if (wid_ < job.wave_ts_cap) job.wave_ts[4 * wid_ + 1] = (unsigned long long)wall_clock64();     \
        }                                                                                                    \
    } while (0)

template <bool kStats, int kLds, int kBlock, int kMinWaves, int kWW>
__global__ __launch_bounds__(kBlock, kMinWaves) void k_trace_wavepersist(DevScene sc, TileJob job,
                                                                         float4* __restrict__ samples,
                                                                         unsigned long long* stats, uint32_t* err,
                                                                         uint32_t* work, uint32_t stack_slots) {
    const unsigned long long t_entry = job.wave_ts ? (unsigned long long)wall_clock64() : 0ull;
    uint32_t chunks = 0;
    if constexpr (kLds == 4 || kLds == 6) {
        extern __shared__ float4 lds_top[];
        for (uint32_t i = threadIdx.x; i < sc.n_lds_f4; i += blockDim.x) lds_top[i] = sc.nodes[i];
        __syncthreads();
        MM_TS_STAGED();
        WpStack<kWW> st;
        const SplitNodes nodes{lds_top, sc.nodes, sc.n_lds_f4};
        if constexpr (kLds == 6)
            chunks = wp_dispatch<kStats, kWW>(sc, view(nodes, sc.recs), st, job, samples, stats, err, work);
        else
            chunks = wp_dispatch<kStats, kWW>(sc, view(nodes), st, job, samples, stats, err, work);
    } else if constexpr (kLds == 10) {  // dictionary-coded nodes in LDS, compact rect records via L1/L2
        extern __shared__ float4 lds_dict[];
        float* tab = reinterpret_cast<float*>(lds_dict);
        uint32_t* words = reinterpret_cast<uint32_t*>(tab + 256);
        for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) tab[i] = sc.dict_tab[i];
        for (uint32_t i = threadIdx.x; i < 3 * sc.n_nodes; i += blockDim.x) words[i] = sc.dict_words[i];
        __syncthreads();
        MM_TS_STAGED();
        WpStack<kWW> st;
        chunks = wp_dispatch<kStats, kWW>(sc, view(DictNodes{words, tab}, sc.recs), st, job, samples, stats, err,
                                          work);
    } else if constexpr (kLds == 7) {
        extern __shared__ float4 lds_nodes7[];
        for (uint32_t i = threadIdx.x; i < 2 * sc.n_nodes; i += blockDim.x) lds_nodes7[i] = sc.nodes[i];
        __syncthreads();
        MM_TS_STAGED();
        WpStack<kWW> st;
        chunks = wp_dispatch<kStats, kWW>(sc, view(lds_nodes7, sc.recs), st, job, samples, stats, err, work);
    } else if constexpr (kLds > 0) {
        extern __shared__ float4 lds_nodes[];
        for (uint32_t i = threadIdx.x; i < 2 * sc.n_nodes; i += blockDim.x) lds_nodes[i] = sc.nodes[i];
        uint2* lds_recs = reinterpret_cast<uint2*>(lds_nodes + 2 * sc.n_nodes);
        if constexpr (kLds == 3 || kLds == 9)
            for (uint32_t i = threadIdx.x; i < 5 * sc.n_rects; i += blockDim.x) lds_recs[i] = sc.recs[i];
        __syncthreads();
        MM_TS_STAGED();
        if constexpr (kLds == 3) {
            WpStack<kWW> st;
            chunks = wp_dispatch<kStats, kWW>(sc, view(lds_nodes, lds_recs), st, job, samples, stats, err, work);
        } else if constexpr (kLds == 9) {  // = 3 with u16 stack entries in scratch
            ScratchStack16 st;
            chunks = wp_dispatch<kStats, kWW>(sc, view(lds_nodes, lds_recs), st, job, samples, stats, err, work);
        } else if constexpr (kLds == 5) {
            WpStack<kWW> st;
            const LdsCold cold{reinterpret_cast<float*>(lds_recs) + threadIdx.x, blockDim.x};
            chunks = wp_dispatch<kStats, kWW>(sc, view(lds_nodes), st, job, samples, stats, err, work, cold);
        } else if constexpr (kLds == 2 || kLds == 8) {
            LdsStack16 st;
            st.base = reinterpret_cast<uint16_t*>(lds_recs) + threadIdx.x;
            st.stride = blockDim.x;
            st.cap = stack_slots;
            if constexpr (kLds == 8)  // + compact rect records through L1/L2
                chunks = wp_dispatch<kStats, kWW>(sc, view(lds_nodes, sc.recs), st, job, samples, stats, err, work);
            else
                chunks = wp_dispatch<kStats, kWW>(sc, view(lds_nodes), st, job, samples, stats, err, work);
        } else {
            WpStack<kWW> st;
            chunks = wp_dispatch<kStats, kWW>(sc, view(lds_nodes), st, job, samples, stats, err, work);
        }
    } else {
        WpStack<kWW> st;
        chunks = wp_dispatch<kStats, kWW>(sc, view(sc.nodes), st, job, samples, stats, err, work);
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

template <int kLds, int kBlock, int kMinWaves, int kWW>
static hipError_t launch_wavepersist_t(const DevScene& sc, const TileJob& job, float4* samples,
                                       unsigned long long* stats, uint32_t* err, uint32_t* work, bool count_stats,
                                       uint32_t stack_slots, hipStream_t s) {
    const uint32_t block = kBlock;
    const size_t lds = kLds == 10 ? 256 * sizeof(float) + 3 * (size_t)sc.n_nodes * sizeof(uint32_t)
                     : (kLds == 4 || kLds == 6) ? (size_t)sc.n_lds_f4 * sizeof(float4)
                                 : (kLds ? 2 * (size_t)sc.n_nodes * sizeof(float4) : 0) +
                                       (kLds == 5 ? 6 * (size_t)block * sizeof(float) : 0) +
                                       (kLds == 2 || kLds == 8 ? (size_t)stack_slots * block * sizeof(uint16_t) : 0) +
                                       (kLds == 3 || kLds == 9 ? 5 * (size_t)sc.n_rects * sizeof(uint2) : 0);
    auto kern = count_stats ? k_trace_wavepersist<true, kLds, kBlock, kMinWaves, kWW>
                            : k_trace_wavepersist<false, kLds, kBlock, kMinWaves, kWW>;
    int per_cu = 0, dev = 0, cus = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, (int)block, lds);
    if (e != hipSuccess) return e;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint32_t n_paths = job.w * job.h * job.e.spp;
    // MM_OPT_RESERVE_CUS: leave that many CUs' worth of resident blocks free for other work (collectives)
    const int cus_used = std::max(1, cus - (int)job.reserve_cus);
    uint32_t grid = (uint32_t)std::max(1, per_cu) * (uint32_t)cus_used;
    grid = std::max(1u, std::min(grid, (n_paths + block - 1) / block));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(block), lds, s, sc, job, samples, stats, err, work, stack_slots);
    return hipGetLastError();
}

// Register budget by launch bounds: waves/SIMD = 8 -> <= 64 VGPRs.
hipError_t launch_trace_wavepersist(const DevScene& sc, const TileJob& job, float4* samples,
                                    unsigned long long* stats, uint32_t* err, uint32_t* work, bool count_stats,
                                    int lds_mode, uint32_t stack_slots, uint32_t block, uint32_t min_waves,
                                    int loop_form, hipStream_t s) {
#define MM_WP2(L, B, W, WW) \
    if (lds_mode == L) return launch_wavepersist_t<L, B, W, WW>(sc, job, samples, stats, err, work, count_stats, stack_slots, s);
#define MM_WP3(B, W, WW) \
    if (loop_form == WW) { MM_WP2(3, B, W, WW) MM_WP2(2, B, W, WW) MM_WP2(1, B, W, WW) MM_WP2(0, B, W, WW) }
#define MM_WP(B, W) \
    if (block == B && min_waves == W) {                                                              \
        if (loop_form == 0) { MM_WP2(4, B, W, 0) }                                                    \
        if (loop_form == 2) { MM_WP2(4, B, W, 2) }                                                    \
        if (loop_form == 3) { MM_WP2(4, B, W, 3) }                                                    \
        if (loop_form == 0) { MM_WP2(5, B, W, 0) MM_WP2(6, B, W, 0) MM_WP2(7, B, W, 0) }              \
        if (loop_form == 4) { MM_WP2(4, B, W, 4) MM_WP2(3, B, W, 4) MM_WP2(1, B, W, 4) MM_WP2(0, B, W, 4) }  \
        MM_WP3(B, W, 0) MM_WP3(B, W, 1) MM_WP3(B, W, 2) MM_WP3(B, W, 3) MM_WP3(B, W, 8) MM_WP3(B, W, 16)  \
        MM_WP3(B, W, 32) }
    MM_WP(256, 8) MM_WP(512, 6) MM_WP(512, 8) MM_WP(1024, 1) MM_WP(1024, 8)
    if (block == 1024 && min_waves == 8 && loop_form == 5) {
        MM_WP2(4, 1024, 8, 5) MM_WP2(6, 1024, 8, 5) MM_WP2(7, 1024, 8, 5) MM_WP2(8, 1024, 8, 5) MM_WP2(9, 1024, 8, 5)
        MM_WP2(10, 1024, 8, 5)
        MM_WP3(1024, 8, 5)
    }
    if (block == 1024 && min_waves == 8 && loop_form == 6) { MM_WP2(3, 1024, 8, 6) MM_WP2(4, 1024, 8, 6) }
    if (block == 1024 && min_waves == 8 && loop_form == 7) {
        MM_WP2(3, 1024, 8, 7) MM_WP2(6, 1024, 8, 7) MM_WP2(7, 1024, 8, 7) MM_WP2(10, 1024, 8, 7)
    }
    if (block == 1024 && min_waves == 8 && loop_form == 9) { MM_WP2(3, 1024, 8, 9) MM_WP2(6, 1024, 8, 9) MM_WP2(7, 1024, 8, 9) }
    // 768-thread blocks at 6 waves/SIMD (80 VGPRs): two blocks per CU still fit the LDS
    if (block == 768 && min_waves == 6 && loop_form == 5) { MM_WP2(3, 768, 6, 5) MM_WP2(6, 768, 6, 5) }
#undef MM_WP
#undef MM_WP3
#undef MM_WP2
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
// Tail gate: a one-wave no-op queued ahead of a frame's trace kernel when
// frames from several contexts share the GPU.  It can only be dispatched once
// a wave slot frees up, i.e. once the frame already running starts to drain,
// so the next frame's resident blocks fill exactly the CUs the previous
// frame's tail leaves idle instead of splitting the GPU with it from the start
// (measured: profiles/r01_overlap_probe.txt).
__global__ void k_tail_gate() {}

hipError_t launch_tail_gate(hipStream_t s) {
    hipLaunchKernelGGL(k_tail_gate, dim3(1), dim3(64), 0, s);
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
