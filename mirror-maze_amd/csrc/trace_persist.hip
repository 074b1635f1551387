// trace_persist.hip — lane-refill persistent megakernel (MM_OPT_PERSIST = 1).
//
// Each lane runs one path at a time as a small state machine:
//     TRAV  one intersect_bvh_iterative step per round
//  -> SHADE shaders.metal:308-340 for the finished closest-hit query
//  -> TRAV  (next bounce) or IDLE (path done: sample written)
//  IDLE  -> TRAV with a new path from the wave's 64-path chunk; chunks come
//           from one global counter (one atomic per 64 paths).
// A wave keeps stepping traversals while more than `threshold` lanes are in
// TRAV (or nothing else waits), then shades every finished lane, refills idle
// lanes and starts their rays together, so a lane whose query ended early does
// not idle until the wave's longest query ends (the one-path-per-thread
// kernels run at ~40 % lane utilisation, profiles/r01_pmc_*).
//
// Register budget: the stepping loop holds only the fast (Markstein-guarded)
// step; the rare rays outside the guard are traversed to completion with IEEE
// division when they start.  Per-lane control lives in one status word.  Every
// path executes exactly the reference's sequence of operations, so the output
// is bit-identical to the other pipelines.
#include <hip/hip_runtime.h>

#include "mm_launch.h"
#include "mm_trace.h"

namespace mm {

namespace {

constexpr uint32_t kChunk = 64;
// status word: bits 0-1 state, bit 2 stack overflow, bit 3 ray start pending
constexpr uint32_t kIdle = 0, kTrav = 1, kShade = 2, kOvf = 4, kStart = 8;

__device__ __forceinline__ uint64_t lanemask_lt() {
    const uint32_t lane = threadIdx.x & 63u;
    return lane ? (~0ull >> (64 - lane)) : 0ull;
}

template <bool kStats, typename V>
__device__ __forceinline__ void refill_body(const DevScene& sc, const V& v, const TileJob& job,
                                            float4* __restrict__ samples, unsigned long long* stats, uint32_t* err,
                                            uint32_t* work, uint32_t threshold) {
    const uint32_t spp = job.e.spp;
    const uint32_t n_paths = job.w * job.h * spp;
    const int bounce_limit = (int)job.e.bounce_limit, mirror_limit = (int)job.e.mirror_limit;
    const uint32_t lane = threadIdx.x & 63u;

    uint32_t chunk_base = 0, chunk_end = 0;  // wave-uniform
    bool more = true;

    uint32_t st = kIdle, pid = 0;
    PathState p;
    Ray ray;
    float t = kBig;
    uint32_t hit = 0, cur = 0, head = 0;
    ScratchStack stack;
    Counters c;
    uint32_t done_paths = 0;

    for (;;) {
        // ---- shade finished queries; finish paths -----------------------------
        if ((st & 3u) == kShade) {
            if (kStats) c.rays++;
            p.ori = ray.o;  // ori/dir live only in the ray while it traverses
            p.dir = ray.d;
            const bool cont = !(st & kOvf) && shade_step(sc, p, t, hit, mirror_limit);
            p.n++;
            if (cont && p.n < bounce_limit + p.mh) {
                st = kShade | kStart;
            } else {
                samples[pid] = make_float4(sqrtf(fmaxf(p.L.x, 0.0f)), sqrtf(fmaxf(p.L.y, 0.0f)),
                                           sqrtf(fmaxf(p.L.z, 0.0f)), 0.0f);
                if (st & kOvf) atomicOr(err, 1u);
                done_paths++;
                st = kIdle;
            }
        }
        // ---- refill idle lanes with new paths ---------------------------------
        const uint64_t idle = __ballot(st == kIdle);
        if (idle && (more || chunk_base < chunk_end)) {
            const uint32_t need = (uint32_t)__popcll(idle);
            const uint32_t rank = (uint32_t)__popcll(idle & lanemask_lt());
            const uint32_t take1 = min(need, chunk_end - chunk_base);
            uint32_t mine = 0;
            bool got = st == kIdle && rank < take1;
            if (got) mine = chunk_base + rank;
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
                    if (st == kIdle && rank >= take1 && rank < take1 + take2) {
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
                if (0 < bounce_limit) {
                    st = kShade | kStart;
                } else {  // no bounce at all: the sample is sqrt(0)
                    samples[pid] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                    done_paths++;
                }
            }
        }
        // ---- start rays --------------------------------------------------------
        if (st & kStart) {
            ray = make_ray(p.ori, p.dir);
            t = kBig;
            hit = 0;
            if (sc.fast_ok && ray_fast_ok(ray)) {
                cur = sc.root_packed;
                head = 0;
                st = kTrav;
            } else {  // rare: the whole query with IEEE division; shaded next round
                st = traverse<false, kStats>(sc, v, ray, t, hit, stack, c) ? kShade : (kShade | kOvf);
            }
        }
        if (!__ballot(st != kIdle)) {
            if (!more && chunk_base >= chunk_end) break;
            continue;
        }
        // ---- traversal rounds -------------------------------------------------
        const bool refill = more || chunk_base < chunk_end;
        for (;;) {
            const uint32_t ntrav = (uint32_t)__popcll(__ballot(st == kTrav));
            if (ntrav == 0) break;
            if (ntrav <= threshold && __ballot(st != kTrav && (st != kIdle || refill))) break;
            if (st == kTrav) {
                bool ovf = false;
                if (trav_step<true, kStats>(sc, v, ray, t, hit, cur, head, stack, c, ovf))
                    st = ovf ? (kShade | kOvf) : kShade;
            }
        }
    }
    if (kStats) {
        unsigned long long vv[4] = {c.rays, c.visits, c.rtests, done_paths};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            unsigned long long x = vv[i];
            for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
            vv[i] = x;
        }
        if (lane == 0) {
            atomicAdd(&stats[0], vv[0]);
            atomicAdd(&stats[1], vv[1]);
            atomicAdd(&stats[2], vv[2]);
            atomicAdd(&stats[3], vv[3]);
        }
    }
}

// kLds: 0 nodes via L1/L2, 1 nodes in LDS, 3 nodes + compact rect records in LDS
template <bool kStats, int kLds, int kBlock, int kMinWaves>
__global__ __launch_bounds__(kBlock, kMinWaves) void k_trace_persist(DevScene sc, TileJob job,
                                                                     float4* __restrict__ samples,
                                                                     unsigned long long* stats, uint32_t* err,
                                                                     uint32_t* work, uint32_t threshold) {
    if constexpr (kLds > 0) {
        extern __shared__ float4 lds_nodes[];
        for (uint32_t i = threadIdx.x; i < 2 * sc.n_nodes; i += blockDim.x) lds_nodes[i] = sc.nodes[i];
        uint2* lds_recs = reinterpret_cast<uint2*>(lds_nodes + 2 * sc.n_nodes);
        if constexpr (kLds == 3)
            for (uint32_t i = threadIdx.x; i < 5 * sc.n_rects; i += blockDim.x) lds_recs[i] = sc.recs[i];
        __syncthreads();
        if constexpr (kLds == 3)
            refill_body<kStats>(sc, view(lds_nodes, lds_recs), job, samples, stats, err, work, threshold);
        else
            refill_body<kStats>(sc, view(lds_nodes), job, samples, stats, err, work, threshold);
    } else {
        refill_body<kStats>(sc, view(sc.nodes), job, samples, stats, err, work, threshold);
    }
}

template <int kLds, int kBlock, int kMinWaves>
hipError_t launch_persist_t(const DevScene& sc, const TileJob& job, float4* samples, unsigned long long* stats,
                            uint32_t* err, uint32_t* work, bool count_stats, uint32_t threshold, hipStream_t s) {
    const size_t lds = (kLds ? 2 * (size_t)sc.n_nodes * sizeof(float4) : 0) +
                       (kLds == 3 ? 5 * (size_t)sc.n_rects * sizeof(uint2) : 0);
    auto kern = count_stats ? k_trace_persist<true, kLds, kBlock, kMinWaves>
                            : k_trace_persist<false, kLds, kBlock, kMinWaves>;
    int per_cu = 0, dev = 0, cus = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kBlock, lds);
    if (e != hipSuccess) return e;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint32_t n_paths = job.w * job.h * job.e.spp;
    uint32_t grid = (uint32_t)std::max(1, per_cu) * (uint32_t)std::max(1, cus);
    grid = std::max(1u, std::min(grid, (n_paths + kBlock - 1) / kBlock));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), lds, s, sc, job, samples, stats, err, work, threshold);
    return hipGetLastError();
}

}  // namespace

bool persist_instantiated(uint32_t block, uint32_t min_waves) {
    return (block == 1024 && (min_waves == 8 || min_waves == 1)) || (block == 512 && min_waves == 6);
}

hipError_t launch_trace_persist(const DevScene& sc, const TileJob& job, float4* samples, unsigned long long* stats,
                                uint32_t* err, uint32_t* work, bool count_stats, const PersistOpts& o,
                                hipStream_t s) {
    hipError_t e = hipMemsetAsync(work, 0, sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
#define MM_P(L, B, W)                                                                                     \
    if (o.lds_mode == L && o.block == B && o.min_waves == W)                                               \
        return launch_persist_t<L, B, W>(sc, job, samples, stats, err, work, count_stats, o.threshold, s);
    MM_P(0, 1024, 8) MM_P(1, 1024, 8) MM_P(3, 1024, 8)
    MM_P(0, 1024, 1) MM_P(1, 1024, 1) MM_P(3, 1024, 1)
    MM_P(0, 512, 6) MM_P(1, 512, 6) MM_P(3, 512, 6)
#undef MM_P
    return hipErrorInvalidValue;
}

}  // namespace mm
