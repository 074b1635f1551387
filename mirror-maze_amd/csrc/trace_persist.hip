// trace_persist.hip — persistent megakernel for throughput mode.
//
// Each lane runs one path at a time as a small state machine:
//     TRAV  (one intersect_bvh_iterative step per round)
//  -> SHADE (shaders.metal:308-340 for the finished closest-hit query)
//  -> TRAV  (next bounce) or IDLE (path done: sample written)
//  IDLE  -> TRAV with a new path taken from the wave's 64-path chunk; chunks
//           come from one global counter (one atomic per 64 paths).
// A wave keeps stepping traversals while more than `threshold` lanes are in
// TRAV (or nothing else is waiting), then shades every finished lane and
// refills idle lanes at once.  This keeps the SIMD busy across the very
// uneven traversal lengths (5-60 node visits) and path lengths (1-16 rays)
// that leave a one-path-per-thread kernel at ~40 % lane utilisation
// (profiles/r01_*).  Every path still executes exactly the reference's
// sequence of operations, so the output is bit-identical.
#include <hip/hip_runtime.h>

#include "mm_launch.h"
#include "mm_trace.h"

namespace mm {

enum : uint32_t { kIdle = 0, kTrav = 1, kShade = 2 };
constexpr uint32_t kChunk = 64;
constexpr uint32_t kNone = 0xFFFFFFFFu;

__device__ __forceinline__ uint64_t lanemask_lt() {
    const uint32_t lane = threadIdx.x & 63u;
    return lane ? (~0ull >> (64 - lane)) : 0ull;
}

template <bool kStats, typename V>
__device__ __forceinline__ void persist_body(const DevScene& sc, const V& v, const TileJob& job,
                                             float4* __restrict__ samples, unsigned long long* stats,
                                             uint32_t* err, uint32_t* work, uint32_t threshold) {
    const uint32_t spp = job.e.spp;
    const uint32_t n_paths = job.w * job.h * spp;
    const int bounce_limit = (int)job.e.bounce_limit, mirror_limit = (int)job.e.mirror_limit;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t lt = lanemask_lt();
    const F3 cam = F3{job.u.cam.center[0], job.u.cam.center[1], job.u.cam.center[2]};

    // wave-uniform chunk bookkeeping (identical in every lane)
    uint32_t chunk_base = 0, chunk_end = 0;
    bool more = true;

    // lane state
    uint32_t status = kIdle, pid = kNone;
    PathState p;
    Ray ray;
    bool fast = false, ovf = false;
    float t = kBig;
    uint32_t hit = 0, cur = 0, head = 0;
    ScratchStack stack;
    Counters c;
    uint32_t done_paths = 0;

    auto start_ray = [&]() {
        ray = make_ray(p.ori, p.dir);
        fast = sc.fast_ok && ray_fast_ok(ray);
        t = kBig;
        hit = 0;
        cur = sc.root_packed;
        head = 0;
        status = kTrav;
    };
    auto finish_path = [&]() {
        samples[pid] = make_float4(sqrtf(fmaxf(p.L.x, 0.0f)), sqrtf(fmaxf(p.L.y, 0.0f)),
                                   sqrtf(fmaxf(p.L.z, 0.0f)), 0.0f);
        if (ovf) atomicOr(err, 1u);
        done_paths++;
        status = kIdle;
        pid = kNone;
    };
    auto start_path = [&](uint32_t path) {
        pid = path;
        const uint32_t pix = path / spp, smp = path - pix * spp;
        const uint32_t j = pix / job.w, i = pix - j * job.w;
        const uint32_t px = job.x0 + i, py = job.y0 + j * job.y_stride;
        p.seed = seed_tile(py * job.view_w + px, smp, job.e.frame);
        p.dir = jitter(primary_dir(job.u, px, py), p.seed);
        p.ori = cam;
        p.T = F3{1.0f, 1.0f, 1.0f};
        p.L = F3{0.0f, 0.0f, 0.0f};
        p.n = 0;
        p.mh = 0;
        ovf = false;
        if (0 < bounce_limit) start_ray();
        else finish_path();
    };

    for (;;) {
        // ---- refill idle lanes --------------------------------------------
        const uint64_t idle = __ballot(status == kIdle);
        if (idle && (more || chunk_base < chunk_end)) {
            const uint32_t need = (uint32_t)__popcll(idle);
            const uint32_t rank = (uint32_t)__popcll(idle & lt);
            uint32_t take1 = min(need, chunk_end - chunk_base);
            uint32_t mine = kNone;
            if (status == kIdle && rank < take1) mine = chunk_base + rank;
            chunk_base += take1;
            if (take1 < need && more) {
                uint32_t b = 0;
                if (lane == 0) b = atomicAdd(work, kChunk);
                b = __shfl(b, 0);
                if (b >= n_paths) {
                    more = false;
                } else {
                    chunk_base = b;
                    chunk_end = min(b + kChunk, n_paths);
                    const uint32_t take2 = min(need - take1, chunk_end - chunk_base);
                    if (status == kIdle && rank >= take1 && rank < take1 + take2) mine = chunk_base + (rank - take1);
                    chunk_base += take2;
                }
            }
            if (mine != kNone) start_path(mine);
        }
        const uint64_t busy = __ballot(status != kIdle);
        if (!busy) {
            if (!more && chunk_base >= chunk_end) break;
            continue;
        }
        // ---- traversal rounds ----------------------------------------------
        for (;;) {
            const uint64_t trav = __ballot(status == kTrav);
            const uint32_t ntrav = (uint32_t)__popcll(trav);
            if (ntrav == 0) break;
            const bool refill = more || chunk_base < chunk_end;
            const uint64_t waiting = __ballot(status == kShade || (refill && status == kIdle));
            if (waiting && ntrav <= threshold) break;
            if (status == kTrav) {
                bool fin;
                if (fast) fin = trav_step<true, kStats>(sc, v, ray, t, hit, cur, head, stack, c, ovf);
                else fin = trav_step<false, kStats>(sc, v, ray, t, hit, cur, head, stack, c, ovf);
                if (fin) status = kShade;
            }
        }
        // ---- shade finished queries -----------------------------------------
        if (status == kShade) {
            if (kStats) c.rays++;
            const bool cont = !ovf && shade_step(sc, p, t, hit, mirror_limit);
            p.n++;
            if (cont && p.n < bounce_limit + p.mh) start_ray();
            else finish_path();
        }
    }
    if (kStats) {
        unsigned long long v[4] = {c.rays, c.visits, c.rtests, done_paths};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            unsigned long long x = v[i];
            for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
            v[i] = x;
        }
        if (lane == 0) {
            atomicAdd(&stats[0], v[0]);
            atomicAdd(&stats[1], v[1]);
            atomicAdd(&stats[2], v[2]);
            atomicAdd(&stats[3], v[3]);
        }
    }
}

template <bool kStats, bool kLds>
__global__ __launch_bounds__(512) void k_trace_persist(DevScene sc, TileJob job, float4* __restrict__ samples,
                                                       unsigned long long* stats, uint32_t* err, uint32_t* work,
                                                       uint32_t threshold) {
    if constexpr (kLds) {
        extern __shared__ float4 lds_nodes[];
        for (uint32_t i = threadIdx.x; i < 2 * sc.n_nodes; i += blockDim.x) lds_nodes[i] = sc.nodes[i];
        __syncthreads();
        persist_body<kStats>(sc, view(lds_nodes), job, samples, stats, err, work, threshold);
    } else {
        persist_body<kStats>(sc, view(sc.nodes), job, samples, stats, err, work, threshold);
    }
}

template <bool kLds>
static hipError_t launch_persist_t(const DevScene& sc, const TileJob& job, float4* samples,
                                   unsigned long long* stats, uint32_t* err, uint32_t* work, bool count_stats,
                                   const PersistOpts& o, hipStream_t s) {
    const size_t lds = kLds ? 2 * (size_t)sc.n_nodes * sizeof(float4) : 0;
    auto kern = count_stats ? k_trace_persist<true, kLds> : k_trace_persist<false, kLds>;
    int per_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, (int)o.block, lds);
    if (e != hipSuccess) return e;
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint32_t n_paths = job.w * job.h * job.e.spp;
    uint32_t grid = (uint32_t)std::max(1, per_cu) * (uint32_t)std::max(1, cus) * std::max(1u, o.grid_mult);
    const uint32_t needed = (n_paths + o.block - 1) / o.block;
    grid = std::max(1u, std::min(grid, needed));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(o.block), lds, s, sc, job, samples, stats, err, work, o.threshold);
    return hipGetLastError();
}

hipError_t launch_trace_persist(const DevScene& sc, const TileJob& job, float4* samples, unsigned long long* stats,
                                uint32_t* err, uint32_t* work, bool count_stats, const PersistOpts& o,
                                hipStream_t s) {
    hipError_t e = hipMemsetAsync(work, 0, sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    return o.lds_nodes ? launch_persist_t<true>(sc, job, samples, stats, err, work, count_stats, o, s)
                       : launch_persist_t<false>(sc, job, samples, stats, err, work, count_stats, o, s);
}

}  // namespace mm
