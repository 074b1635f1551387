// mm_trace.h — the per-ray and per-path device code of the reference kernel:
// ray_rect_intersect (shaders.metal:51-67), intersect_aabb (87-95),
// intersect_bvh_iterative (115-156) and the bounce loop (302-340).
// Operation order follows src/shaders.ir; see oracle/mm_oracle.c for the CPU
// statement the parity tests compare against.
#pragma once

#include "mm_device.h"

namespace mm {

struct Counters {
    uint32_t rays = 0, visits = 0, rtests = 0;
};

// ray_rect_intersect with the per-rect subexpressions (n, |v|, |u|) loaded
// from g0/g1 instead of recomputed (same IEEE ops, same values).
__device__ __forceinline__ void rect_test(const float4* __restrict__ geo, uint32_t k, F3 ori, F3 dir,
                                          float& t, uint32_t& index) {
    const float4 g0 = geo[4 * k + 0], g1 = geo[4 * k + 1], g2 = geo[4 * k + 2], g3 = geo[4 * k + 3];
    const F3 o = xyz(g0), n = xyz(g1), v = xyz(g2), u = xyz(g3);
    const float lv = g0.w, lu = g1.w;
    const float nc = dot3(dir, n);
    const float a = dot3(o - ori, n) / nc;
    const F3 rv = (ori - o) + a * dir;
    const float d1 = dot3(rv, v) / lv;
    const float d2 = dot3(rv, u) / lu;
    if (d1 >= 0.0f && d1 <= lv && d2 >= 0.0f && d2 <= lu && nc != 0.0f && a > 0.1f && a < t) {
        t = a;
        index = k;
    }
}

// intersect_aabb; a = (mn.xyz, mx.x), b = (mx.y, mx.z, ., .)
__device__ __forceinline__ float aabb_test(float4 a, float4 b, F3 ori, F3 dir, float t) {
    const float tx1 = (a.x - ori.x) / dir.x, tx2 = (a.w - ori.x) / dir.x;
    float tmin = fminf(tx1, tx2), tmax = fmaxf(tx1, tx2);
    const float ty1 = (a.y - ori.y) / dir.y, ty2 = (b.x - ori.y) / dir.y;
    tmin = fmaxf(tmin, fminf(ty1, ty2));
    tmax = fminf(tmax, fmaxf(ty1, ty2));
    const float tz1 = (a.z - ori.z) / dir.z, tz2 = (b.y - ori.z) / dir.z;
    tmin = fmaxf(tmin, fminf(tz1, tz2));
    tmax = fminf(tmax, fmaxf(tz1, tz2));
    return (tmax >= tmin && tmin < t && tmax > 0.0f) ? tmin : kBig;
}

// intersect_bvh_iterative.  `stack` is any indexable storage of >= 50 u32.
// Returns false on stack overflow (the reference would write out of bounds).
template <bool kStats, typename Stack>
__device__ __forceinline__ bool intersect_bvh(const DevScene& sc, F3 ori, F3 dir, float& t, uint32_t& index,
                                              Stack& stack, Counters& c) {
    const float4* __restrict__ nodes = sc.nodes;
    uint32_t node = 0, head = 0;
    for (;;) {
        const float4 nb = nodes[2 * node + 1];
        const uint32_t lf = __float_as_uint(nb.z), count = __float_as_uint(nb.w);
        if (count > 0) {
            for (uint32_t i = 0; i < count; ++i) rect_test(sc.geo, sc.idx[lf + i], ori, dir, t, index);
            if (kStats) c.rtests += count;
            if (head == 0) break;
            node = stack[--head];
            continue;
        }
        if (kStats) c.visits++;
        uint32_t l = lf, r = lf + 1;
        float d1 = aabb_test(nodes[2 * l], nodes[2 * l + 1], ori, dir, t);
        float d2 = aabb_test(nodes[2 * r], nodes[2 * r + 1], ori, dir, t);
        if (d1 > d2) {
            const float tt = d1; d1 = d2; d2 = tt;
            const uint32_t x = l; l = r; r = x;
        }
        if (d1 == kBig) {
            if (head == 0) break;
            node = stack[--head];
        } else {
            node = l;
            if (d2 != kBig) {
                if (head >= (uint32_t)kStackMax) return false;
                stack[head++] = r;
            }
        }
    }
    return true;
}

// Path state carried across bounces.
struct PathState {
    F3 ori, dir, T, L;
    uint32_t seed;
    int n, mh;
};

// One shading step after a closest-hit query (the body of shaders.metal:306-340
// after line 307).  Returns false when the path terminates.
__device__ __forceinline__ bool shade_step(const DevScene& sc, PathState& p, float t, uint32_t k, int mirror_limit) {
    if (!(t < kBig)) return false;                           // miss, shaders.metal:336-338
    const F3 nn = xyz(sc.geo[4 * k + 1]);                    // normalize(cross(v,u)), %238
    const float4 s0 = sc.shade[2 * k + 0];                   // color, is_mirror
    const float sg = msign(dot3(p.dir, nn));
    const float side = -sg;
    if (s0.w == 0.0f || sg == 1.0f) {
        const float4 e = sc.shade[2 * k + 1];
        const F3 contrib = (e.w * p.T) * xyz(e);             // %253, %254
        const F3 newT = xyz(s0) * p.T;                       // %264
        float rx = rand_pm1(p.seed), ry = rand_pm1(p.seed), rz = rand_pm1(p.seed);
        F3 rd = F3{rx, ry, rz};
        float len2 = dot3(rd, rd);
        while (sqrtf(len2) > 1.0f) {                         // shaders.metal:316-318
            rx = rand_pm1(p.seed); ry = rand_pm1(p.seed); rz = rand_pm1(p.seed);
            rd = F3{rx, ry, rz};
            len2 = dot3(rd, rd);
        }
        const F3 rn = rsq(len2) * rd;                        // %358
        p.ori = p.ori + t * p.dir;                           // %363
        const F3 nd = rn + side * nn;                        // %367
        p.dir = rsq(dot3(nd, nd)) * nd;                      // %372
        p.L = contrib + p.L;                                 // %409
        p.T = newT;
    } else {
        if (!(p.mh + 1 < mirror_limit)) return false;        // shaders.metal:326, 333
        const F3 contrib = 0.005f * xyz(s0);                 // %386
        p.ori = p.ori + t * p.dir;
        const float dd = dot3(nn, p.dir) * 2.0f;             // reflect, %392-%397
        const F3 rf = p.dir - dd * nn;
        p.dir = rsq(dot3(rf, rf)) * rf;
        p.L = contrib + p.L;
        p.mh += 1;
    }
    return true;
}

// Whole path (shaders.metal:302-344): returns sqrt(max(L, 0)).
template <bool kStats, typename Stack>
__device__ __forceinline__ F3 trace_path(const DevScene& sc, F3 ori, F3 dir, uint32_t seed, int bounce_limit,
                                         int mirror_limit, Stack& stack, Counters& c, bool& overflow) {
    PathState p;
    p.ori = ori; p.dir = dir; p.seed = seed;
    p.T = F3{1.0f, 1.0f, 1.0f};
    p.L = F3{0.0f, 0.0f, 0.0f};
    p.mh = 0;
    for (p.n = 0; p.n < bounce_limit + p.mh; ++p.n) {
        float t = kBig;
        uint32_t k = 0;
        const bool ok = intersect_bvh<kStats>(sc, p.ori, p.dir, t, k, stack, c);
        if (kStats) c.rays++;
        if (!ok) { overflow = true; break; }
        if (!shade_step(sc, p, t, k, mirror_limit)) break;
    }
    return F3{sqrtf(fmaxf(p.L.x, 0.0f)), sqrtf(fmaxf(p.L.y, 0.0f)), sqrtf(fmaxf(p.L.z, 0.0f))};
}

}  // namespace mm
