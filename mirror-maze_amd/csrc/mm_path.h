// mm_path.h — closest-hit query policies and the bounce loop
// (shaders.metal:302-344) every throughput / parity kernel runs.
#pragma once

#include "mm_grid.h"

namespace mm {

// The straight reference walk (MM_PIPE_REFERENCE: IEEE division everywhere).
template <bool kStats>
struct RefQuery {
    const DevScene& sc;
    __device__ __forceinline__ bool operator()(F3 o, F3 d, float& t, uint32_t& k, ScratchStack& st,
                                               Counters& c) const {
        return traverse_reference<kStats>(sc, make_ray(o, d), t, k, st, c);
    }
};

// A production BVH loop form over view V (nodes / records in LDS or global).
template <bool kStats, int kForm, typename V>
struct BvhQuery {
    const DevScene& sc;
    V v;
    __device__ __forceinline__ bool operator()(F3 o, F3 d, float& t, uint32_t& k, ScratchStack& st,
                                               Counters& c) const {
        return closest_hit_bvh<kStats, kForm>(sc, v, make_ray(o, d), t, k, st, c);
    }
};

// The certified grid search (mm_grid.h); the reference walk of the BVH in
// global memory (lean loop form, compact records) when the search cannot
// certify its answer (a tie, a failed leaf-box check) or the ray is outside
// the Markstein guards or the grid.
template <bool kStats, typename GV>
struct GridQuery {
    const DevScene& sc;
    GV gv;
    __device__ __forceinline__ bool operator()(F3 o, F3 d, float& t, uint32_t& k, ScratchStack& st,
                                               Counters& c) const {
        const Ray r = make_ray(o, d);
        if (sc.fast_ok && ray_fast_ok(r) && grid_ray_ok(sc.grid, r) && grid_search<kStats>(sc.grid, gv, r, t, k, c))
            return true;
        t = kBig;  // (an out-of-line walk costs 73 VGPR spills of call ABI)
        return closest_hit_bvh<kStats, kFormLean>(sc, view(sc.nodes, sc.recs), r, t, k, st, c);
    }
};

// Whole path (shaders.metal:302-344): returns sqrt(max(L, 0)).
template <bool kStats, typename Q>
__device__ __forceinline__ F3 trace_path(const DevScene& sc, const Q& query, F3 ori, F3 dir, uint32_t seed,
                                         int bounce_limit, int mirror_limit, ScratchStack& stack, Counters& c,
                                         bool& overflow) {
    PathState p;
    p.ori = ori; p.dir = dir; p.seed = seed;
    p.T = F3{1.0f, 1.0f, 1.0f};
    p.L = F3{0.0f, 0.0f, 0.0f};
    p.mh = 0;
    for (p.n = 0; p.n < bounce_limit + p.mh; ++p.n) {
        float t = kBig;
        uint32_t k = 0;
        const bool ok = query(p.ori, p.dir, t, k, stack, c);
        if (kStats) c.rays++;
        if (!ok) { overflow = true; break; }
        if (!shade_step(sc, p, t, k, mirror_limit)) break;
    }
    return F3{sqrtf(fmaxf(p.L.x, 0.0f)), sqrtf(fmaxf(p.L.y, 0.0f)), sqrtf(fmaxf(p.L.z, 0.0f))};
}

}  // namespace mm
