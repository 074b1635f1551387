// mm_trace.h — the per-ray and per-path device code of the reference kernel:
// ray_rect_intersect (shaders.metal:51-67), intersect_aabb (87-95),
// intersect_bvh_iterative (115-156) and the bounce loop (302-340).
// Operation order follows src/shaders.ir; oracle/mm_oracle.c is the CPU
// statement the parity tests compare against, bit for bit.
//
// Closest-hit queries come in two families:
//   BVH traversals   the reference's own walk of its SAH tree (near child
//                    first, far child pushed, no re-test on pop), as
//                    traverse_reference (the straight statement, IEEE
//                    division everywhere: MM_PIPE_REFERENCE) and the
//                    production loop forms below.  With kFast every slab
//                    division (bound - o) / d uses a per-ray correctly rounded
//                    reciprocal y = RN(1/d) and Markstein's correction
//                        q = a*y;  r = fma(-q, d, a);  q' = fma(r, y, q)
//                    which equals RN(a/d) when no under/overflow occurs
//                    (Markstein 1990; Cornea-Hasegan, Golliver, Markstein
//                    1999; scripts/verify_markstein.c checks 1.6e9 pairs
//                    over every divisor mantissa).  The exponent ranges that
//                    theorem needs are enforced by ray_fast_ok() per ray and
//                    by the scene check at upload; a ray outside them takes
//                    traverse<false> (IEEE division).
//   grid search      (mm_grid.h) a certified search that returns the same
//                    (t, index) as the reference walk without walking it.
#pragma once

#include "mm_device.h"

namespace mm {

struct Counters {
    uint32_t rays = 0, visits = 0, rtests = 0;
#ifdef MM_PHASE_CLOCKS  // diagnostics build (scripts/phase_probe.py): wall_clock64 ticks (100 MHz) per phase
    uint64_t q_cyc = 0, s_cyc = 0;
#endif
};

struct Ray {
    F3 o, d;
    F3 y;  // (1/d.x, 1/d.y, 1/d.z): RN(1/d) wherever it is read (see make_ray)
};

// y = RN(1/d) is read only by the Markstein quotients (qdiv) and the grid
// walk, both only under ray_fast_ok -- |d| in [2^-40, 2^40] on every axis.
// There one fma Newton step on the hardware v_rcp_f32 gives RN(1/d) exactly
// (scripts/verify_fast_rsq.hip checks every float of either sign in
// [2^-44, 2^44]); outside, the value is never used.
__device__ __forceinline__ float rcp_guarded(float d) {
    const float y = __builtin_amdgcn_rcpf(d);
    const float e = __builtin_fmaf(-d, y, 1.0f);
    return __builtin_fmaf(e, y, y);
}

__device__ __forceinline__ Ray make_ray(F3 o, F3 d) {
    Ray r;
    r.o = o;
    r.d = d;
    r.y = F3{rcp_guarded(d.x), rcp_guarded(d.y), rcp_guarded(d.z)};
    return r;
}

// Exponent guards for the Markstein quotient (see header comment).
__device__ __forceinline__ bool dir_ok(float x) {
    const float a = fabsf(x);
    bool ok = a >= 0x1p-40f;
    ok &= a <= 0x1p40f;
    return ok;
}
__device__ __forceinline__ bool org_ok(float x) {
    const float a = fabsf(x);
    bool in = a >= 0x1p-30f;
    in &= a <= 0x1p60f;
    in |= a == 0.0f;
    return in;
}
__device__ __forceinline__ bool ray_fast_ok(const Ray& r) {
    // (&=, not &&: a short-circuit chain is one exec-mask branch per clause,
    // each holding a saved mask in SGPRs that the grid search then spills)
    bool ok = dir_ok(r.d.x);
    ok &= dir_ok(r.d.y);
    ok &= dir_ok(r.d.z);
    ok &= org_ok(r.o.x);
    ok &= org_ok(r.o.y);
    ok &= org_ok(r.o.z);
    return ok;
}

// ray_fast_ok for a ray whose origin the grid box check (grid_ray_ok) holds
// inside [mn, mx], with |mn|, |mx| <= 2^60 (grid_build.cpp builds no grid past
// that): org_ok's upper bound then follows from the box, and the rest is the
// same predicate on the magnitudes' bits as unsigned integers --
//   |d| in [2^-40, 2^40]    <=>  bits(|d|) - bits(2^-40) <= bits(2^40) - bits(2^-40)
//                                (NaN and inf lie above 2^40, smaller |d| wrap),
//   |o| == 0 or >= 2^-30    <=>  bits(|o|) - 1 >= bits(2^-30) - 1   (0 wraps to the top;
//                                a NaN origin passes here and fails the box),
// one max / min over the axes and one compare each: 4 single-slot ops instead
// of 15 compares (dual issue).
__device__ __forceinline__ uint32_t mag_bits(float x) { return __float_as_uint(x) & 0x7FFFFFFFu; }
__device__ __forceinline__ bool ray_fast_ok_boxed(const Ray& r) {
    constexpr uint32_t kDirLo = 0x2B800000u;                 // 2^-40
    constexpr uint32_t kDirSpan = 0x53800000u - kDirLo;      // 2^40
    constexpr uint32_t kOrgLo = 0x30800000u;                 // 2^-30
    const uint32_t dm = max(max(mag_bits(r.d.x) - kDirLo, mag_bits(r.d.y) - kDirLo), mag_bits(r.d.z) - kDirLo);
    const uint32_t om = min(min(mag_bits(r.o.x) - 1u, mag_bits(r.o.y) - 1u), mag_bits(r.o.z) - 1u);
    bool ok = dm <= kDirSpan;
    ok &= om >= kOrgLo - 1u;
    return ok;
}

// RN(a / d) given y = RN(1/d), inside the guarded ranges.
__device__ __forceinline__ float qdiv(float a, float d, float y) {
    const float q = a * y;
    const float r = __builtin_fmaf(-q, d, a);
    return __builtin_fmaf(r, y, q);
}
template <bool kFast>
__device__ __forceinline__ float sdiv(float a, float d, float y) {
    if constexpr (kFast) return qdiv(a, d, y);
    else return a / d;
}

// ---------------------------------------------------------------------------
// ray_rect_intersect.  g0 = (o, |v|), g1 = (n, |u|), g2 = (v, 1/|v|),
// g3 = (u, 1/|u|): n, |v|, |u| are the reference's per-rect subexpressions
// (same IEEE ops, computed once by k_prep_rects).
template <bool kFast>
__device__ __forceinline__ void rect_test(const float4* __restrict__ geo, uint32_t k, const Ray& r, float& t,
                                          uint32_t& index) {
    const float4 g0 = geo[4 * k + 0], g1 = geo[4 * k + 1], g2 = geo[4 * k + 2], g3 = geo[4 * k + 3];
    const F3 o = xyz(g0), n = xyz(g1), v = xyz(g2), u = xyz(g3);
    const float lv = g0.w, lu = g1.w;
    const float nc = dot3(r.d, n);
    const float a = dot3(o - r.o, n) / nc;
    const F3 rv = (r.o - o) + a * r.d;
    const float d1 = sdiv<kFast>(dot3(rv, v), lv, g2.w);
    const float d2 = sdiv<kFast>(dot3(rv, u), lu, g3.w);
    if (d1 >= 0.0f && d1 <= lv && d2 >= 0.0f && d2 <= lu && nc != 0.0f && a > 0.1f && a < t) {
        t = a;
        index = k;
    }
}

// intersect_aabb; a = (mn.xyz, mx.x), b = (mx.y, mx.z, ., .)
template <bool kFast>
__device__ __forceinline__ float aabb_test(float4 a, float4 b, const Ray& r, float t) {
    const float tx1 = sdiv<kFast>(a.x - r.o.x, r.d.x, r.y.x), tx2 = sdiv<kFast>(a.w - r.o.x, r.d.x, r.y.x);
    float tmin = fminf(tx1, tx2), tmax = fmaxf(tx1, tx2);
    const float ty1 = sdiv<kFast>(a.y - r.o.y, r.d.y, r.y.y), ty2 = sdiv<kFast>(b.x - r.o.y, r.d.y, r.y.y);
    tmin = fmaxf(tmin, fminf(ty1, ty2));
    tmax = fminf(tmax, fmaxf(ty1, ty2));
    const float tz1 = sdiv<kFast>(a.z - r.o.z, r.d.z, r.y.z), tz2 = sdiv<kFast>(b.y - r.o.z, r.d.z, r.y.z);
    tmin = fmaxf(tmin, fminf(tz1, tz2));
    tmax = fminf(tmax, fmaxf(tz1, tz2));
    return (tmax >= tmin && tmin < t && tmax > 0.0f) ? tmin : kBig;
}

// Slab test on the production node layout, bounds as (min, max) pairs per
// axis: a = (mn.x, mx.x, mn.y, mx.y), b = (mn.z, mx.z, packed, 0).  Scalar
// ops: gfx950's v_pk_fma_f32 runs at the same FLOP rate as v_fma_f32 and the
// register pairs cost occupancy (measured 13.6 vs 12.85 ms/frame on C3,
// profiles/r01/ab_packed.txt).  Same values as aabb_test.
template <bool kFast>
__device__ __forceinline__ float aabb_pairs(float4 a, float4 b, const Ray& r, float t) {
    const float tx1 = sdiv<kFast>(a.x - r.o.x, r.d.x, r.y.x), tx2 = sdiv<kFast>(a.y - r.o.x, r.d.x, r.y.x);
    float tmin = fminf(tx1, tx2), tmax = fmaxf(tx1, tx2);
    const float ty1 = sdiv<kFast>(a.z - r.o.y, r.d.y, r.y.y), ty2 = sdiv<kFast>(a.w - r.o.y, r.d.y, r.y.y);
    tmin = fmaxf(tmin, fminf(ty1, ty2));
    tmax = fminf(tmax, fmaxf(ty1, ty2));
    const float tz1 = sdiv<kFast>(b.x - r.o.z, r.d.z, r.y.z), tz2 = sdiv<kFast>(b.y - r.o.z, r.d.z, r.y.z);
    tmin = fmaxf(tmin, fminf(tz1, tz2));
    tmax = fminf(tmax, fmaxf(tz1, tz2));
    return (tmax >= tmin && tmin < t && tmax > 0.0f) ? tmin : kBig;
}

// ---------------------------------------------------------------------------
// The reference's 50-entry private traversal stack (scratch).  Entries are
// packed child words (count << 24 | left_first); the stack never holds more
// entries than the tree is deep (one pending far child per level).
struct ScratchStack {
    uint32_t s[kStackMax];
    static constexpr uint32_t kCap = kStackMax;
    __device__ __forceinline__ void push(uint32_t i, uint32_t v) { s[i] = v; }
    __device__ __forceinline__ uint32_t pop(uint32_t i) const { return s[i]; }
};

// ---------------------------------------------------------------------------
// Scene views: where a traversal reads nodes and (optionally) the compact,
// leaf-ordered rect records from (global memory or LDS).
template <typename NodesT>
struct NodeView {
    NodesT nodes;
    static constexpr bool kCompact = false;
};
template <typename NodesT, typename RecsT>
struct CompactView {
    NodesT nodes;
    RecsT recs;  // 5 x uint2 per slot (rect_compact.cpp)
    static constexpr bool kCompact = true;
};
template <typename N> __device__ __forceinline__ NodeView<N> view(N n) { return NodeView<N>{n}; }
template <typename N, typename R> __device__ __forceinline__ CompactView<N, R> view(N n, R r) {
    return CompactView<N, R>{n, r};
}

// The two children of an interior node: one adjacent 64-B pair at 2*lf.
__device__ __forceinline__ void node_pair(const float4* n, uint32_t lf, float4& la, float4& lb, float4& ra,
                                          float4& rb) {
    la = n[2 * lf]; lb = n[2 * lf + 1]; ra = n[2 * lf + 2]; rb = n[2 * lf + 3];
}
__device__ __forceinline__ float sel3(uint32_t a, F3 v) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }

// ray_rect_intersect on a compact record (FAST kind) for a fast-guarded ray;
// the derivation and the thresholds are in rect_compact.cpp.  SKIP records
// can never hit; SLOW records run the general test from global memory.
template <typename R>
__device__ __forceinline__ void rect_test_compact(const DevScene& sc, const R& recs, uint32_t slot, const Ray& r,
                                                  float& t, uint32_t& index) {
    const uint2 w89 = recs[5 * slot + 4];
    const uint32_t meta = w89.y, kind = meta >> 30;
    if (kind == 1u) return;
    const uint32_t k = meta & 0xFFFFFu;
    if (kind == 2u) {
        rect_test<true>(sc.geo, k, r, t, index);
        return;
    }
    const uint2 w01 = recs[5 * slot + 0], w23 = recs[5 * slot + 1], w45 = recs[5 * slot + 2],
                w67 = recs[5 * slot + 3];
    const uint32_t ak = (meta >> 20) & 3u, av = (meta >> 22) & 3u, au = (meta >> 24) & 3u;
    const float a = qdiv(__uint_as_float(w01.x) - sel3(ak, r.o), sel3(ak, r.d), sel3(ak, r.y));
    const float x1 = ((sel3(av, r.o) - __uint_as_float(w01.y)) + a * sel3(av, r.d)) * __uint_as_float(w23.y);
    const float x2 = ((sel3(au, r.o) - __uint_as_float(w23.x)) + a * sel3(au, r.d)) * __uint_as_float(w45.x);
    if (x1 >= __uint_as_float(w45.y) && x1 <= __uint_as_float(w67.x) && x2 >= __uint_as_float(w67.y) &&
        x2 <= __uint_as_float(w89.x) && a > 0.1f && a < t) {
        t = a;
        index = k;
    }
}

// Branch-free leaf test for scenes whose records are all FAST or SKIP (SKIP
// records carry thresholds no x1 passes, rect_compact.cpp): the same
// operations as rect_test_compact's FAST case.
template <typename R>
__device__ __forceinline__ void rect_test_compact_lean(const R& recs, uint32_t slot, const Ray& r, float& t,
                                                       uint32_t& index) {
    const uint2 w01 = recs[5 * slot + 0], w23 = recs[5 * slot + 1], w45 = recs[5 * slot + 2],
                w67 = recs[5 * slot + 3], w89 = recs[5 * slot + 4];
    const uint32_t meta = w89.y;
    const uint32_t ak = (meta >> 20) & 3u, av = (meta >> 22) & 3u, au = (meta >> 24) & 3u;
    const float a = qdiv(__uint_as_float(w01.x) - sel3(ak, r.o), sel3(ak, r.d), sel3(ak, r.y));
    const float x1 = ((sel3(av, r.o) - __uint_as_float(w01.y)) + a * sel3(av, r.d)) * __uint_as_float(w23.y);
    const float x2 = ((sel3(au, r.o) - __uint_as_float(w23.x)) + a * sel3(au, r.d)) * __uint_as_float(w45.x);
    if (x1 >= __uint_as_float(w45.y) && x1 <= __uint_as_float(w67.x) && x2 >= __uint_as_float(w67.y) &&
        x2 <= __uint_as_float(w89.x) && a > 0.1f && a < t) {
        t = a;
        index = meta & 0xFFFFFu;
    }
}

template <bool kFast, typename V>
__device__ __forceinline__ void leaf_tests(const DevScene& sc, const V& v, uint32_t lf, uint32_t cnt, const Ray& r,
                                           float& t, uint32_t& index) {
    if constexpr (V::kCompact && kFast) {
        for (uint32_t i = 0; i < cnt; ++i) rect_test_compact(sc, v.recs, lf + i, r, t, index);
    } else {
        for (uint32_t i = 0; i < cnt; ++i) rect_test<kFast>(sc.geo, sc.idx[lf + i], r, t, index);
    }
}

// ---------------------------------------------------------------------------
// intersect_bvh_iterative, production form.  Device node layout (built at
// upload from the reference's 32-B BVHNode):
//     a = (mn.x, mx.x, mn.y, mx.y)   b = (mn.z, mx.z, bits(packed), 0)
// packed = count << 24 | left_first.  Children are adjacent, so an interior
// visit loads one 64-B pair and already holds each child's (lf, count); the
// stack holds packed words, so a pop needs no node load.  Visit order,
// pruning and pushes are exactly the reference's.
//
// If-if loop (form 0): ONE iteration of the reference's while(true) loop
// (shaders.metal:126-155) per loop trip.
template <bool kFast, bool kStats, typename V>
__device__ __forceinline__ bool traverse(const DevScene& sc, const V& v, const Ray& r, float& t, uint32_t& index,
                                         ScratchStack& stack, Counters& c) {
    uint32_t cur = sc.root_packed, head = 0;
    for (;;) {
        const uint32_t lf = cur & 0xFFFFFFu, cnt = cur >> 24;
        if (cnt > 0) {
            leaf_tests<kFast>(sc, v, lf, cnt, r, t, index);
            if (kStats) c.rtests += cnt;
            if (head == 0) return true;
            cur = stack.pop(--head);
            continue;
        }
        if (kStats) c.visits++;
        float4 la, lb, ra, rb;
        node_pair(v.nodes, lf, la, lb, ra, rb);
        float d1 = aabb_pairs<kFast>(la, lb, r, t);
        float d2 = aabb_pairs<kFast>(ra, rb, r, t);
        uint32_t pl = __float_as_uint(lb.z), pr = __float_as_uint(rb.z);
        if (d1 > d2) {
            const float tt = d1; d1 = d2; d2 = tt;
            const uint32_t x = pl; pl = pr; pr = x;
        }
        if (d1 == kBig) {
            if (head == 0) return true;
            cur = stack.pop(--head);
        } else {
            cur = pl;
            if (d2 != kBig) {
                if (head >= ScratchStack::kCap) return false;
                stack.push(head++, pr);
            }
        }
    }
}

// Leaf-then-interior form (form 5): one iteration runs a lane's leaf tests (if
// it sits at a leaf) and pops, and then, if the lane is now at an interior
// node, that node's step.  Per lane the sequence of leaf tests, node visits,
// pushes and pops is exactly the if-if loop's; a leaf visit just no longer
// costs the wave an iteration of its own (C3 11.06 -> 10.37 ms,
// profiles/r01/ab_leafinterior.txt).
template <bool kFast, bool kStats, typename V>
__device__ __forceinline__ bool traverse_li(const DevScene& sc, const V& v, const Ray& r, float& t,
                                            uint32_t& index, ScratchStack& stack, Counters& c) {
    uint32_t cur = sc.root_packed, head = 0;
    for (;;) {
        if ((cur >> 24) != 0) {
            const uint32_t lf = cur & 0xFFFFFFu, cnt = cur >> 24;
            leaf_tests<kFast>(sc, v, lf, cnt, r, t, index);
            if (kStats) c.rtests += cnt;
            if (head == 0) break;
            cur = stack.pop(--head);
        }
        if ((cur >> 24) == 0) {
            const uint32_t lf = cur & 0xFFFFFFu;
            if (kStats) c.visits++;
            float4 la, lb, ra, rb;
            node_pair(v.nodes, lf, la, lb, ra, rb);
            const float d1 = aabb_pairs<kFast>(la, lb, r, t);
            const float d2 = aabb_pairs<kFast>(ra, rb, r, t);
            const uint32_t pl = __float_as_uint(lb.z), pr = __float_as_uint(rb.z);
            const bool sw = d1 > d2;
            const float dn = sw ? d2 : d1, df = sw ? d1 : d2;
            if (dn == kBig) {
                if (head == 0) break;
                cur = stack.pop(--head);
            } else {
                cur = sw ? pr : pl;
                if (df != kBig) {
                    if (head >= ScratchStack::kCap) return false;
                    stack.push(head++, sw ? pl : pr);
                }
            }
        }
    }
    return true;
}

// Lean leaf-then-interior form (form 7) for scenes without SLOW rect records
// (mm_upload_scene sets lean_ok): the leaf test is rect_test_compact_lean (no
// kind branches) and pushes skip the overflow test (upload rejects trees
// deeper than the stack; near-first traversal holds at most one pending far
// child per level).  Per lane the operation sequence is traverse_li's
// (C3 10.40 -> 9.53 ms, profiles/r01/ab_lean.txt).
template <bool kStats, typename V>
__device__ __forceinline__ bool traverse_lil(const DevScene& sc, const V& v, const Ray& r, float& t,
                                             uint32_t& index, ScratchStack& stack, Counters& c) {
    uint32_t cur = sc.root_packed, head = 0;
    for (;;) {
        if ((cur >> 24) != 0) {
            const uint32_t lf = cur & 0xFFFFFFu, cnt = cur >> 24;
            for (uint32_t i = 0; i < cnt; ++i) rect_test_compact_lean(v.recs, lf + i, r, t, index);
            if (kStats) c.rtests += cnt;
            if (head == 0) break;
            cur = stack.pop(--head);
        }
        if ((cur >> 24) == 0) {
            const uint32_t lf = cur & 0xFFFFFFu;
            if (kStats) c.visits++;
            float4 la, lb, ra, rb;
            node_pair(v.nodes, lf, la, lb, ra, rb);
            const float d1 = aabb_pairs<true>(la, lb, r, t);
            const float d2 = aabb_pairs<true>(ra, rb, r, t);
            const uint32_t pl = __float_as_uint(lb.z), pr = __float_as_uint(rb.z);
            const bool sw = d1 > d2;
            const float dn = sw ? d2 : d1, df = sw ? d1 : d2;
            if (dn == kBig) {
                if (head == 0) break;
                cur = stack.pop(--head);
            } else {
                cur = sw ? pr : pl;
                if (df != kBig) stack.push(head++, sw ? pl : pr);
            }
        }
    }
    return true;
}

// The straight statement of intersect_bvh_iterative over the reference node
// layout (sc.nodes_ref, 2 float4 per node: a, (mx.yz, lf, count)).
template <bool kStats>
__device__ __forceinline__ bool traverse_reference(const DevScene& sc, const Ray& r, float& t, uint32_t& index,
                                                   ScratchStack& stack, Counters& c) {
    const float4* __restrict__ nodes = sc.nodes_ref;
    uint32_t node = 0, head = 0;
    for (;;) {
        const float4 nb = nodes[2 * node + 1];
        const uint32_t lf = __float_as_uint(nb.z), count = __float_as_uint(nb.w);
        if (count > 0) {
            for (uint32_t i = 0; i < count; ++i) rect_test<false>(sc.geo, sc.idx[lf + i], r, t, index);
            if (kStats) c.rtests += count;
            if (head == 0) break;
            node = stack.pop(--head);
            continue;
        }
        if (kStats) c.visits++;
        uint32_t l = lf, rr = lf + 1;
        float d1 = aabb_test<false>(nodes[2 * l], nodes[2 * l + 1], r, t);
        float d2 = aabb_test<false>(nodes[2 * rr], nodes[2 * rr + 1], r, t);
        if (d1 > d2) {
            const float tt = d1; d1 = d2; d2 = tt;
            const uint32_t x = l; l = rr; rr = x;
        }
        if (d1 == kBig) {
            if (head == 0) break;
            node = stack.pop(--head);
        } else {
            node = l;
            if (d2 != kBig) {
                if (head >= (uint32_t)kStackMax) return false;
                stack.push(head++, rr);
            }
        }
    }
    return true;
}

// Closest hit for one ray by the BVH: production traversal with the exact
// (IEEE-division) fallback for rays outside the Markstein guards.
template <bool kStats, int kForm, typename V>
__device__ __forceinline__ bool closest_hit_bvh(const DevScene& sc, const V& v, const Ray& r, float& t,
                                                uint32_t& index, ScratchStack& stack, Counters& c) {
    const bool fast = sc.fast_ok && ray_fast_ok(r);
    if constexpr (kForm == kFormLean) {
        if (fast) return traverse_lil<kStats>(sc, v, r, t, index, stack, c);
        return traverse_li<false, kStats>(sc, v, r, t, index, stack, c);
    } else if constexpr (kForm == kFormLeafInterior) {
        if (fast) return traverse_li<true, kStats>(sc, v, r, t, index, stack, c);
        return traverse_li<false, kStats>(sc, v, r, t, index, stack, c);
    } else {
        if (fast) return traverse<true, kStats>(sc, v, r, t, index, stack, c);
        return traverse<false, kStats>(sc, v, r, t, index, stack, c);
    }
}

// Path state carried across bounces.  bank (0..2): accepted rejection-sampling
// trials already drawn from the RNG for the path's next diffuse bounces
// (shade_step): with bank >= 1 the first ends at s1 (its three numbers are the
// three draws before state s1), with bank = 2 the second ends at `seed`; with
// bank = 1 `seed` may lie past s1 by rejected trials only.
struct PathState {
    F3 ori, dir, T, L;
    uint32_t seed;
    int n, mh;
    uint32_t bank, s1;
};

// random()'s state step s -> a s + c (shaders.metal:181-186, rand_pm1), and the
// inverse of three steps: s0 = A s3 + C with A = a^-3, C = -A c (1 + a + a^2)
// mod 2^32 (a is odd, so invertible), rewinding one trial's three draws.
constexpr uint32_t kLcgA = 747796405u, kLcgC = 291336453u;
constexpr uint32_t lcg_inv(uint32_t a) {  // Newton's iteration for the inverse of an odd a mod 2^32
    uint32_t x = a;
    for (int i = 0; i < 5; ++i) x *= 2u - a * x;
    return x;
}
constexpr uint32_t kLcgBack3A = lcg_inv(kLcgA * kLcgA * kLcgA);
constexpr uint32_t kLcgBack3C = 0u - kLcgBack3A * (kLcgC * (1u + kLcgA + kLcgA * kLcgA));
static_assert(kLcgA * kLcgA * kLcgA * kLcgBack3A == 1u, "a^3 * a^-3 = 1 mod 2^32");
static_assert(kLcgBack3A * (((kLcgA * 12345u + kLcgC) * kLcgA + kLcgC) * kLcgA + kLcgC) + kLcgBack3C == 12345u,
              "three steps rewound");

// One shading step after a closest-hit query (the body of shaders.metal:306-340
// after line 307).  Returns false when the path terminates.
// A terminating path (a miss, shaders.metal:336-338, or a mirror bounce past
// the limit, 326 / 333) keeps its L, the one field read after the bounce loop,
// and runs the rest of the step on rect 0 as a mirror bounce with its results
// discarded: every field but L is then dead, so the step writes the state
// unconditionally and the bounce loop carries one copy of it (with early
// returns the old and the new state were live together and the compiler copied
// the whole state between register sets twice per bounce).
__device__ __forceinline__ bool shade_step(const DevScene& sc, PathState& p, float t, uint32_t k, int mirror_limit) {
    const bool hit = t < kBig;
    k = hit ? k : 0u;
    MM_LANE_STAT(kLpShade);
    const F3 nn = xyz(sc.geo[4 * k + 1]);                    // normalize(cross(v,u)), %238
    const float4 s0 = sc.shade[2 * k + 0];                   // color, is_mirror
    const float sg = msign(dot3(p.dir, nn));
    const bool lit = s0.w == 0.0f || sg == 1.0f;
    const bool more = hit & (lit | (p.mh + 1 < mirror_limit));
    const bool diffuse = more & lit;
    // Both branches end in ori += t dir, dir = normalize(X), L = contrib + L;
    // those run once after the branch (a wave holding diffuse and mirror lanes
    // would otherwise execute the correctly rounded 1/sqrt of each branch).
    F3 x, contrib;
    if (diffuse) {
        MM_LANE_STAT(kLpDiffuse);
        const float side = -sg;
        const float4 e = sc.shade[2 * k + 1];
        contrib = (e.w * p.T) * xyz(e);                      // %253, %254
        p.T = xyz(s0) * p.T;                                 // %264
        // shaders.metal:316-318, length(r) > 1: RN(sqrt(x)) > 1 <=> x > 1 + 2^-23
        // for every binary32 x (exhaustive check: scripts/verify_sqrt_gt1.c).
        // The path's direction samples are its RNG stream's accepted trials in
        // order -- nothing else draws from it after the primary jitter -- so a
        // lane may draw ahead, and may skip rejected trials it already drew.
        // The first trial: the first banked one (its draws rewound from s1 and
        // redrawn: the same numbers; the stream goes on from `seed`, past any
        // rejected trials after it), else a fresh one.  Lanes whose trial is
        // rejected loop; while they do, the wave's other diffuse lanes draw
        // their NEXT bounces' trials until two are accepted (the bank), so those
        // bounces' first trials are accepted on those lanes and the wave's loop
        // runs for fewer lanes -- a wave runs its unluckiest lane's trials (~5.8
        // iterations per bounce on C3 where a lane needs 0.9; a CPU model of 64
        // lanes: 3.3 with a bank of one, 2.6 with two).  (A wave-pooled form --
        // trials spread over the lanes with jumps of the state -- was bit-exact
        // and slower: 12 % on C3 in round 2, 3.5 % in round 3,
        // profiles/r03/ab_pool_trials.txt.)
        uint32_t s = p.bank ? p.s1 : p.seed;
        if (p.bank) s = s * kLcgBack3A + kLcgBack3C;
        float rx = rand_pm1(s), ry = rand_pm1(s), rz = rand_pm1(s);
        p.seed = p.bank ? p.seed : s;
        p.s1 = p.seed;  // (the second banked trial, if any, ends there: it is the first now)
        uint32_t bank = p.bank ? p.bank - 1u : 0u;
        F3 rd = F3{rx, ry, rz};
        float len2 = dot3(rd, rd);
        uint32_t need = len2 > 0x1.000002p0f ? 1u : 0u;
        if (__builtin_amdgcn_ballot_w64(need != 0u)) do {  // (do-while: no copies of the carried values)
            MM_LANE_STAT(kLpTrial);
            // every lane draws (no branch: the loop is one block); a lane whose
            // bank is full keeps its state (need = 1 implies bank = 0)
            uint32_t t = p.seed;
            rx = rand_pm1(t); ry = rand_pm1(t); rz = rand_pm1(t);
            const float q2 = dot3(F3{rx, ry, rz}, F3{rx, ry, rz});
            // accepted <=> !(q2 > 1 + 2^-23) <=> q2 < 1 + 2^-22 <=> the sign of the exact difference
            // (q2 is finite) -- two pairable ops instead of a compare and a select
            const uint32_t acc = __float_as_uint(q2 - 0x1.000004p0f) >> 31;
            const uint32_t act = (bank >> 1) ^ 1u;  // bank < 2: still drawing
            p.seed = act ? t : p.seed;
            const uint32_t take = need & acc;
            rd.x = take ? rx : rd.x;
            rd.y = take ? ry : rd.y;
            rd.z = take ? rz : rd.z;
            len2 = take ? q2 : len2;
            const uint32_t gain = (acc & act) - take;  // accepted on a lane that did not need it
            p.s1 = gain > bank ? t : p.s1;              // the first banked trial's end
            bank += gain;
            need -= take;
        } while (__builtin_amdgcn_ballot_w64(need != 0u));
        p.bank = bank;
        const F3 rn = rsq(len2) * rd;                        // %358
        x = rn + side * nn;                                  // %367
    } else {
        MM_LANE_STAT(kLpMirror);
        contrib = 0.005f * xyz(s0);                          // %386
        const float dd = dot3(nn, p.dir) * 2.0f;             // reflect, %392-%397
        x = p.dir - dd * nn;
        p.mh += 1;
    }
    p.ori = p.ori + t * p.dir;                               // %363
    p.dir = rsq(dot3(x, x)) * x;                             // %372 / reflect's normalize
    const F3 l = contrib + p.L;                              // %409
    p.L = F3{more ? l.x : p.L.x, more ? l.y : p.L.y, more ? l.z : p.L.z};
    return more;
}

}  // namespace mm
