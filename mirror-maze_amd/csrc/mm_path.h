// mm_path.h — closest-hit query policies and the bounce loop
// (shaders.metal:302-344) every throughput / parity kernel runs.
#pragma once

#include "mm_grid.h"

namespace mm {

// The straight reference walk (MM_PIPE_REFERENCE: IEEE division everywhere).
template <bool kStats>
struct RefQuery {
    const DevScene& sc;
    __device__ __forceinline__ bool operator()(F3 o, F3 d, bool, float& t, uint32_t& k, ScratchStack& st,
                                               Counters& c) const {
        return traverse_reference<kStats>(sc, make_ray(o, d), t, k, st, c);
    }
};

// A production BVH loop form over view V (nodes / records in LDS or global).
template <bool kStats, int kForm, typename V>
struct BvhQuery {
    const DevScene& sc;
    V v;
    __device__ __forceinline__ bool operator()(F3 o, F3 d, bool, float& t, uint32_t& k, ScratchStack& st,
                                               Counters& c) const {
        return closest_hit_bvh<kStats, kForm>(sc, v, make_ray(o, d), t, k, st, c);
    }
};

// The certified grid search (mm_grid.h); the reference walk of the BVH in
// global memory (lean loop form, compact records) when the search cannot
// certify its answer (a tie, a failed leaf-box check) or the ray is outside
// the Markstein guards or the grid.  hit_origin: the ray starts at a hit
// point (a bounce ray), which lies inside the grid box -- the point is on a
// rect up to the rounding of the reference's bounds test and of ori + t dir
// (a few u C), and the grid box is the box of every rect corner widened by
// eps = 2^-14 C (grid_build.cpp) -- so the box check runs only in a wave
// holding a ray from the camera.
template <bool kStats, bool kSlow, bool kWide, bool kFlat, typename GV>
struct GridQuery {
    const DevScene& sc;
    GV gv;
    __device__ __forceinline__ bool operator()(F3 o, F3 d, bool hit_origin, float& t, uint32_t& k,
                                               ScratchStack& st, Counters& c) const {
        const Ray r = make_ray(o, d);
        // sc.fast_ok holds wherever a grid exists (mm_runtime.hip builds none
        // otherwise), and the box check bounds |o| (ray_fast_ok_boxed)
        bool guards = ray_fast_ok_boxed(r);  // one branch for the guards
        if (__builtin_amdgcn_ballot_w64(!hit_origin)) guards &= grid_ray_ok(sc.grid, r);
        if (guards && grid_search<kStats, kSlow, kWide, kFlat>(sc.grid, gv, sc.geo, r, t, k, c)) return true;
        MM_LANE_STAT(kLpFallback);
        t = kBig;  // (an out-of-line walk costs 73 VGPR spills of call ABI)
        return closest_hit_bvh<kStats, kSlow ? kFormLeafInterior : kFormLean>(sc, view(sc.nodes, sc.recs), r, t, k,
                                                                              st, c);
    }
};

// The bounce loop of shaders.metal:306-340 from state p (p.n bounces done).
// Deferral: at the top of a bounce n >= defer_from, if at most defer_lanes
// lanes of the wave are still in the loop and reserve() (called by those
// lanes together) grants them queue entries, those lanes stop and return true
// with p holding the state the next bounce starts from.  defer_from >= 2^30:
// never.  The loop is rotated so that every exit follows the shading step
// (then only the updated state is live, and the compiler keeps one copy of it
// instead of copying it between register sets every bounce): the test at the
// top of bounce n > p.n runs at the end of bounce n - 1, and the one at the
// top of the first bounce is left out -- it never defers: the kernels call
// this with p.n = 0 < defer_from (>= 1) for new paths, and a claimed tail
// chunk has more than defer_lanes live lanes or runs with deferral off
// (trace_kernels.hip wavepersist_ring_body).
template <bool kStats, typename Q, typename Reserve>
__device__ __forceinline__ bool bounce_loop_r(const DevScene& sc, const Q& query, PathState& p, int bounce_limit,
                                              int mirror_limit, ScratchStack& stack, Counters& c, bool& overflow,
                                              int defer_from, uint32_t defer_lanes, Reserve&& reserve) {
    if (!(p.n < bounce_limit + p.mh)) return false;
    for (;;) {
        MM_LANE_STAT(kLpBounce);
        float t = kBig;
        uint32_t k = 0;
#ifdef MM_PHASE_CLOCKS
        const uint64_t t0 = (uint64_t)wall_clock64();
#endif
        const bool ok = query(p.ori, p.dir, p.n != 0, t, k, stack, c);  // (bounce n >= 1 starts at a hit)
#ifdef MM_PHASE_CLOCKS
        const uint64_t t1 = (uint64_t)wall_clock64();
        c.q_cyc += t1 - t0;
#endif
        if (kStats) c.rays++;
        // a failed query (the BVH stack overflowed) ends the path as a miss
        // does -- L kept -- so that no exit bypasses the shading step
        overflow |= !ok;
        const bool more = shade_step(sc, p, ok ? t : kBig, k, mirror_limit);
#ifdef MM_PHASE_CLOCKS
        c.s_cyc += (uint64_t)wall_clock64() - t1;
#endif
        if (!more) break;
        ++p.n;
        if (!(p.n < bounce_limit + p.mh)) break;
        if (p.n >= defer_from && (uint32_t)__popcll(__ballot(1)) <= defer_lanes && reserve()) return true;
    }
    return false;
}

// The bounce loop without deferral.
template <bool kStats, typename Q>
__device__ __forceinline__ void bounce_loop(const DevScene& sc, const Q& query, PathState& p, int bounce_limit,
                                            int mirror_limit, ScratchStack& stack, Counters& c, bool& overflow) {
    bounce_loop_r<kStats>(sc, query, p, bounce_limit, mirror_limit, stack, c, overflow, 1 << 30, 0u,
                          []() { return false; });
}

// Whole path (shaders.metal:302-344): returns sqrt(max(L, 0)).
template <bool kStats, typename Q>
__device__ __forceinline__ F3 trace_path(const DevScene& sc, const Q& query, F3 ori, F3 dir, uint32_t seed,
                                         int bounce_limit, int mirror_limit, ScratchStack& stack, Counters& c,
                                         bool& overflow) {
    PathState p;
    p.ori = ori; p.dir = dir; p.seed = seed;
    p.T = F3{1.0f, 1.0f, 1.0f};
    p.L = F3{0.0f, 0.0f, 0.0f};
    p.n = 0;
    p.mh = 0;
    p.bank = 0u;
    p.s1 = 0u;
    bounce_loop<kStats>(sc, query, p, bounce_limit, mirror_limit, stack, c, overflow);
    return F3{sqrtf(fmaxf(p.L.x, 0.0f)), sqrtf(fmaxf(p.L.y, 0.0f)), sqrtf(fmaxf(p.L.z, 0.0f))};
}

}  // namespace mm
