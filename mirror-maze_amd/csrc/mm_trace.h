// mm_trace.h — the per-ray and per-path device code of the reference kernel:
// ray_rect_intersect (shaders.metal:51-67), intersect_aabb (87-95),
// intersect_bvh_iterative (115-156) and the bounce loop (302-340).
// Operation order follows src/shaders.ir; oracle/mm_oracle.c is the CPU
// statement the parity tests compare against, bit for bit.
//
// Two traversals are provided:
//   traverse_reference  the straight statement (IEEE division everywhere);
//                       kept as MM_PIPE_REFERENCE for A/B measurement.
//   traverse<kFast>     the production path.  With kFast every slab division
//                       (bound - o) / d uses a per-ray correctly rounded
//                       reciprocal y = RN(1/d) and Markstein's correction
//                           q = a*y;  r = fma(-q, d, a);  q' = fma(r, y, q)
//                       which equals RN(a/d) when no under/overflow occurs
//                       (Markstein 1990; Cornea-Hasegan, Golliver, Markstein
//                       1999).  scripts/verify_markstein.c checks 1.6e9 pairs
//                       over every divisor mantissa: 0 mismatches.  The
//                       exponent ranges that theorem needs are enforced by
//                       ray_fast_ok() per ray and by the scene check at upload;
//                       a ray outside them takes traverse<false> (IEEE
//                       division), so results are always the reference's.
#pragma once

#include "mm_device.h"

namespace mm {

struct Counters {
    uint32_t rays = 0, visits = 0, rtests = 0;
};

struct Ray {
    F3 o, d;
    F3 y;  // (1/d.x, 1/d.y, 1/d.z), IEEE division
};

__device__ __forceinline__ Ray make_ray(F3 o, F3 d) {
    Ray r;
    r.o = o;
    r.d = d;
    r.y = F3{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
    return r;
}

// Exponent guards for the Markstein quotient (see header comment).
__device__ __forceinline__ bool dir_ok(float x) {
    const float a = fabsf(x);
    return a >= 0x1p-40f && a <= 0x1p40f;
}
__device__ __forceinline__ bool org_ok(float x) {
    const float a = fabsf(x);
    return a == 0.0f || (a >= 0x1p-30f && a <= 0x1p60f);
}
__device__ __forceinline__ bool ray_fast_ok(const Ray& r) {
    return dir_ok(r.d.x) && dir_ok(r.d.y) && dir_ok(r.d.z) && org_ok(r.o.x) && org_ok(r.o.y) && org_ok(r.o.z);
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
// profiles/r01_ab_packed.txt).  Same values as aabb_test.
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
// Traversal stack policies.  Entries are packed child words
// (count << 24 | left_first).  The stack never holds more entries than the
// tree is deep (one pending far child per level of the current path).
struct ScratchStack {          // the reference's 50-entry private array
    uint32_t s[kStackMax];
    static constexpr uint32_t kCap = kStackMax;
    __device__ __forceinline__ void push(uint32_t i, uint32_t v) { s[i] = v; }
    __device__ __forceinline__ uint32_t pop(uint32_t i) const { return s[i]; }
};
// The reference stack with u16 entries (count << 12 | left_first; needs
// count < 16 and left_first < 4096, checked at upload): half the scratch
// footprint, so the traversal stacks of all resident waves stay in L2.
struct ScratchStack16 {
    uint16_t s[kStackMax];
    static constexpr uint32_t kCap = kStackMax;
    __device__ __forceinline__ void push(uint32_t i, uint32_t v) {
        s[i] = (uint16_t)(((v >> 24) << 12) | (v & 0xFFFu));
    }
    __device__ __forceinline__ uint32_t pop(uint32_t i) const {
        const uint32_t p = s[i];
        return ((p >> 12) << 24) | (p & 0xFFFu);
    }
};
// The same stack with its top entry held in a register: a pop returns the
// register and reloads the next entry from scratch, whose latency then
// overlaps the following traversal step instead of stalling the next node
// fetch.  mem[k] holds entry k-1 (mem[0] is a dummy), so push and pop are
// unconditional.
struct RegTopStack {
    uint32_t top = 0;
    uint32_t mem[kStackMax + 1];
    static constexpr uint32_t kCap = kStackMax;
    __device__ __forceinline__ void push(uint32_t i, uint32_t v) { mem[i] = top; top = v; }
    __device__ __forceinline__ uint32_t pop(uint32_t i) {
        const uint32_t r = top;
        top = mem[i];
        return r;
    }
};
// u16 entries in LDS, [slot][thread] so a wave's same-slot accesses are
// contiguous: (count << 12 | left_first) needs count < 16, left_first < 4096
// and slots >= tree depth -- all checked at upload.
struct LdsStack16 {
    uint16_t* base;            // &lds[slot 0][this thread]
    uint32_t stride;           // threads per block
    uint32_t cap;
    __device__ __forceinline__ void push(uint32_t i, uint32_t v) {
        base[i * stride] = (uint16_t)(((v >> 24) << 12) | (v & 0xFFFu));
    }
    __device__ __forceinline__ uint32_t pop(uint32_t i) const {
        const uint32_t p = base[i * stride];
        return ((p >> 12) << 24) | (p & 0xFFFu);
    }
};
template <typename S> __device__ __forceinline__ uint32_t stack_cap(const S& st) { return st.kCap; }
template <> __device__ __forceinline__ uint32_t stack_cap<LdsStack16>(const LdsStack16& st) { return st.cap; }

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

// Top-of-tree cache for scenes whose nodes exceed the LDS budget: production
// float4s [0, n_lds) are staged in LDS, the rest are read from global memory.
// Child pairs are numbered breadth-first at upload (mm_runtime.hip), so the
// LDS part holds the top levels every traversal visits.
struct SplitNodes {
    const float4* lds;
    const float4* glob;
    uint32_t n_lds;
};

// The two children of an interior node: one adjacent 64-B pair at 2*lf.
__device__ __forceinline__ void node_pair(const float4* n, uint32_t lf, float4& la, float4& lb, float4& ra,
                                          float4& rb) {
    la = n[2 * lf]; lb = n[2 * lf + 1]; ra = n[2 * lf + 2]; rb = n[2 * lf + 3];
#ifdef MM_FORCE_B128
    asm volatile("" ::"v"(lb.w), "v"(rb.w));  // experiment: 16-B reads instead of 12-B (ds_read_b96)
#endif
}
__device__ __forceinline__ void node_pair(const SplitNodes& n, uint32_t lf, float4& la, float4& lb, float4& ra,
                                          float4& rb) {
    if (2 * lf < n.n_lds) node_pair(n.lds, lf, la, lb, ra, rb);
    else node_pair(n.glob, lf, la, lb, ra, rb);
}

// Dictionary-coded nodes in LDS (mode 10): 12 B per node, so the N=64 tree
// (5534 nodes, 66 KB + a 1 KB value table) fits the LDS budget.  Decoding
// returns the production layout's values exactly (the table holds the
// original floats).  Left children sit at even production indices, so a pair
// (24 B at 12 * lf) is 8-B aligned.
struct DictNodes {
    const uint32_t* w;   // 3 words per node
    const float* tab;    // 256 bound values
};
__device__ __forceinline__ void node_pair(const DictNodes& n, uint32_t lf, float4& la, float4& lb, float4& ra,
                                          float4& rb) {
    const uint2* p = reinterpret_cast<const uint2*>(n.w + 3 * lf);
    const uint2 q0 = p[0], q1 = p[1], q2 = p[2];
    // left child: q0.x (4 indices), q0.y (2 indices), q1.x packed; right: q1.y, q2.x, q2.y
    la = make_float4(n.tab[q0.x & 255u], n.tab[(q0.x >> 8) & 255u], n.tab[(q0.x >> 16) & 255u], n.tab[q0.x >> 24]);
    lb = make_float4(n.tab[q0.y & 255u], n.tab[(q0.y >> 8) & 255u], __uint_as_float(q1.x), 0.0f);
    ra = make_float4(n.tab[q1.y & 255u], n.tab[(q1.y >> 8) & 255u], n.tab[(q1.y >> 16) & 255u], n.tab[q1.y >> 24]);
    rb = make_float4(n.tab[q2.x & 255u], n.tab[(q2.x >> 8) & 255u], __uint_as_float(q2.y), 0.0f);
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
// trav_step runs ONE iteration of the reference's while(true) loop
// (shaders.metal:126-155) on explicit state (cur, head, stack) and returns
// true when the traversal is over (ovf set on stack overflow), so a caller
// can interleave traversal steps of different rays (k_trace_persist).
template <bool kFast, bool kStats, typename V, typename Stack>
__device__ __forceinline__ bool trav_step(const DevScene& sc, const V& v, const Ray& r, float& t,
                                          uint32_t& index, uint32_t& cur, uint32_t& head, Stack& stack,
                                          Counters& c, bool& ovf) {
    const uint32_t lf = cur & 0xFFFFFFu, cnt = cur >> 24;
    if (cnt > 0) {
        leaf_tests<kFast>(sc, v, lf, cnt, r, t, index);
        if (kStats) c.rtests += cnt;
        if (head == 0) return true;
        cur = stack.pop(--head);
        return false;
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
            if (head >= stack_cap(stack)) { ovf = true; return true; }
            stack.push(head++, pr);
        }
    }
    return false;
}

template <bool kFast, bool kStats, typename V, typename Stack>
__device__ __forceinline__ bool traverse(const DevScene& sc, const V& v, const Ray& r, float& t,
                                         uint32_t& index, Stack& stack, Counters& c) {
    uint32_t cur = sc.root_packed, head = 0;
    bool ovf = false;
    while (!trav_step<kFast, kStats>(sc, v, r, t, index, cur, head, stack, c, ovf)) {
    }
    return !ovf;
}

// Lean form (MM_OPT_TRAVERSAL 2): the same iteration with one pop site and no
// overflow test.  mm_upload_scene rejects trees deeper than the stack (50
// entries, or the LDS stack's depth-sized slots), and near-first traversal
// holds at most one pending far child per level of the current root-to-node
// path, so a push can never overflow.  Per lane the visits, pushes and pops
// are exactly trav_step's.
template <bool kFast, bool kStats, typename V, typename Stack>
__device__ __forceinline__ bool traverse_lean(const DevScene& sc, const V& v, const Ray& r, float& t,
                                              uint32_t& index, Stack& stack, Counters& c) {
    uint32_t cur = sc.root_packed, head = 0;
    for (;;) {
        const uint32_t lf = cur & 0xFFFFFFu, cnt = cur >> 24;
        bool pop;
        if (cnt > 0) {
            leaf_tests<kFast>(sc, v, lf, cnt, r, t, index);
            if (kStats) c.rtests += cnt;
            pop = true;
        } else {
            if (kStats) c.visits++;
            float4 la, lb, ra, rb;
            node_pair(v.nodes, lf, la, lb, ra, rb);
            const float d1 = aabb_pairs<kFast>(la, lb, r, t);
            const float d2 = aabb_pairs<kFast>(ra, rb, r, t);
            const uint32_t pl = __float_as_uint(lb.z), pr = __float_as_uint(rb.z);
            const bool sw = d1 > d2;
            const float dn = sw ? d2 : d1, df = sw ? d1 : d2;
            cur = sw ? pr : pl;
            pop = dn == kBig;
            if (!pop && df != kBig) stack.push(head++, sw ? pl : pr);
        }
        if (pop) {
            if (head == 0) break;
            cur = stack.pop(--head);
        }
    }
    return true;
}

// Leaf-then-interior form (MM_OPT_TRAVERSAL 5): one iteration runs a lane's
// leaf tests (if it sits at a leaf) and pops, and then, if the lane is now at
// an interior node, that node's step.  Per lane the sequence of leaf tests,
// node visits, pushes and pops is exactly trav_step's; a leaf visit just no
// longer costs the wave an iteration of its own (wave model,
// scripts/wave_sim.cpp: 7 % fewer iterations on C3).
template <bool kFast, bool kStats, typename V, typename Stack>
__device__ __forceinline__ bool traverse_li(const DevScene& sc, const V& v, const Ray& r, float& t,
                                            uint32_t& index, Stack& stack, Counters& c) {
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
                    if (head >= stack_cap(stack)) return false;
                    stack.push(head++, sw ? pl : pr);
                }
            }
        }
    }
    return true;
}

// Lean leaf-then-interior form (MM_OPT_TRAVERSAL 7) for scenes without SLOW
// rect records (mm_upload_scene sets lean_ok): the leaf test is
// rect_test_compact_lean (no kind branches) and pushes skip the overflow test (upload rejects trees
// deeper than the stack; near-first traversal holds at most one pending far
// child per level).  Per lane the operation sequence is traverse_li's.
template <bool kStats, typename V, typename Stack>
__device__ __forceinline__ bool traverse_lil(const DevScene& sc, const V& v, const Ray& r, float& t,
                                             uint32_t& index, Stack& stack, Counters& c) {
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

// ---------------------------------------------------------------------------
// Verified conservative closest hit (MM_OPT_TRAVERSAL 9).
//
// Search: the same BVH with every box expanded by an absolute margin E
// (mm_upload_scene) and slab quotients RN(RN(b - o) * RN(1/d)) -- two
// operations instead of the exact quotient's four -- culling only boxes whose
// approximate interval starts beyond the best hit so far (<=, so ties
// survive).  Every rect reached gets the exact reference test (the compact
// record's operations) without its `a < t` clause; the minimum a* and its slot
// are kept with a tie flag.
//
// Why the search cannot miss the reference's answer: a rect the reference
// accepts at a has o + a*d within delta <= ~10u*C of the rect per axis
// (u = 2^-24, C >= every |coordinate| and |origin component|), so inside its
// leaf box, and every ancestor box, expanded by E, with margin E - delta; an
// approximate quotient is within 3u*|b - o|/|d| <= 6u*C/|d| of the exact one,
// so with E >= 64*(10u + 6u)*C the approximate interval of every expanded
// ancestor contains a.  Hence a* is the minimum over ALL rects the reference
// would accept at any t, and a tie flag is exact.
//
// Verification (exactness of the answer, not of the search): with a* unique,
// the reference's current best is > a* whenever it tests a box on R*'s path,
// and the exact (reference-arithmetic) slab values of every ancestor box
// bracket those of R*'s leaf box (RN and Markstein division are monotone,
// ancestors contain the leaf).  So if the leaf box's exact test gives
// tmax >= tmin, tmax > 0 and tmin <= a*, the reference reaches R*, accepts it,
// and never replaces it: its answer is (a*, R*).  A tie, a failed check, or a
// ray outside the guards runs traverse_li on the exact nodes instead.
// scripts/cons_sim.cpp replays C3 / C5 / P0 frames on the CPU: 0 mismatches
// in 37 M queries, ties only where coplanar rects overlap (P0's outer walls).

// RN(RN(b - o) * y): the approximate slab quotient
__device__ __forceinline__ float qapprox(float b, float o, float y) { return (b - o) * y; }

__device__ __forceinline__ float aabb_cons(float4 a, float4 b, const Ray& r, float best) {
    const float tx1 = qapprox(a.x, r.o.x, r.y.x), tx2 = qapprox(a.y, r.o.x, r.y.x);
    float tmin = fminf(tx1, tx2), tmax = fmaxf(tx1, tx2);
    const float ty1 = qapprox(a.z, r.o.y, r.y.y), ty2 = qapprox(a.w, r.o.y, r.y.y);
    tmin = fmaxf(tmin, fminf(ty1, ty2));
    tmax = fminf(tmax, fmaxf(ty1, ty2));
    const float tz1 = qapprox(b.x, r.o.z, r.y.z), tz2 = qapprox(b.y, r.o.z, r.y.z);
    tmin = fmaxf(tmin, fminf(tz1, tz2));
    tmax = fminf(tmax, fmaxf(tz1, tz2));
    return (tmax >= tmin && tmin <= best && tmax > 0.0f) ? tmin : kBig;
}

// Exact compact rect test (FAST / SKIP records) without the `a < t` clause:
// a if the reference would accept the rect at a large enough t, else kBig.
template <typename R>
__device__ __forceinline__ float rect_a_compact(const R& recs, uint32_t slot, const Ray& r) {
    const uint2 w01 = recs[5 * slot + 0], w23 = recs[5 * slot + 1], w45 = recs[5 * slot + 2],
                w67 = recs[5 * slot + 3], w89 = recs[5 * slot + 4];
    const uint32_t meta = w89.y;
    const uint32_t ak = (meta >> 20) & 3u, av = (meta >> 22) & 3u, au = (meta >> 24) & 3u;
    const float a = qdiv(__uint_as_float(w01.x) - sel3(ak, r.o), sel3(ak, r.d), sel3(ak, r.y));
    const float x1 = ((sel3(av, r.o) - __uint_as_float(w01.y)) + a * sel3(av, r.d)) * __uint_as_float(w23.y);
    const float x2 = ((sel3(au, r.o) - __uint_as_float(w23.x)) + a * sel3(au, r.d)) * __uint_as_float(w45.x);
    const bool hit = x1 >= __uint_as_float(w45.y) && x1 <= __uint_as_float(w67.x) &&
                     x2 >= __uint_as_float(w67.y) && x2 <= __uint_as_float(w89.x) && a > 0.1f;
    return hit ? a : kBig;
}

__device__ __forceinline__ bool cons_ray_ok(const DevScene& sc, const Ray& r) {
    return fabsf(r.o.x) <= sc.cons_bound && fabsf(r.o.y) <= sc.cons_bound && fabsf(r.o.z) <= sc.cons_bound;
}

template <bool kStats, typename V, typename Stack>
__device__ __forceinline__ bool traverse_cons(const DevScene& sc, const V& v, const Ray& r, float& t,
                                              uint32_t& index, Stack& stack, Counters& c) {
    uint32_t cur = sc.root_packed, head = 0, bslot = 0;
    float best = kBig;
    bool tie = false;
    for (;;) {
        if ((cur >> 24) != 0) {
            const uint32_t lf = cur & 0xFFFFFFu, cnt = cur >> 24;
            for (uint32_t i = 0; i < cnt; ++i) {
                const float a = rect_a_compact(v.recs, lf + i, r);
                tie = tie || (a == best && a != kBig);
                if (a < best) {
                    best = a;
                    bslot = lf + i;
                    tie = false;
                }
            }
            if (kStats) c.rtests += cnt;
            if (head == 0) break;
            cur = stack.pop(--head);
        }
        if ((cur >> 24) == 0) {
            const uint32_t lf = cur & 0xFFFFFFu;
            if (kStats) c.visits++;
            float4 la, lb, ra, rb;
            node_pair(v.nodes, lf, la, lb, ra, rb);
            const float d1 = aabb_cons(la, lb, r, best);
            const float d2 = aabb_cons(ra, rb, r, best);
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
    if (best == kBig) return true;  // no rect hit: (kBig, index untouched)
    if (!tie) {
        const float4 a = sc.slot_box[2 * bslot], b = sc.slot_box[2 * bslot + 1];
        const float tx1 = qdiv(a.x - r.o.x, r.d.x, r.y.x), tx2 = qdiv(a.y - r.o.x, r.d.x, r.y.x);
        float tmin = fminf(tx1, tx2), tmax = fmaxf(tx1, tx2);
        const float ty1 = qdiv(a.z - r.o.y, r.d.y, r.y.y), ty2 = qdiv(a.w - r.o.y, r.d.y, r.y.y);
        tmin = fmaxf(tmin, fminf(ty1, ty2));
        tmax = fminf(tmax, fmaxf(ty1, ty2));
        const float tz1 = qdiv(b.x - r.o.z, r.d.z, r.y.z), tz2 = qdiv(b.y - r.o.z, r.d.z, r.y.z);
        tmin = fmaxf(tmin, fminf(tz1, tz2));
        tmax = fminf(tmax, fmaxf(tz1, tz2));
        if (tmax >= tmin && tmax > 0.0f && tmin <= best) {
            t = best;
            index = v.recs[5 * bslot + 4].y & 0xFFFFFu;
            return true;
        }
    }
    // tie or unverified: the reference query on the exact nodes (global memory)
    return traverse_li<true, false>(sc, view(sc.nodes_exact, v.recs), r, t, index, stack, c);
}

// "while-while" form of the same traversal: each lane runs interior steps
// until it reaches a leaf (or finishes), then the wave's leaves are processed
// together.  Per lane the sequence of node visits, rect tests, pushes and
// pops is exactly trav_step's (no speculation: a leaf is always tested
// before the next node is visited), so results are identical; only the
// interleaving of lanes' work inside a wave changes.
template <bool kFast, bool kStats, typename V, typename Stack>
__device__ __forceinline__ bool traverse_ww(const DevScene& sc, const V& v, const Ray& r, float& t,
                                            uint32_t& index, Stack& stack, Counters& c) {
    uint32_t cur = sc.root_packed, head = 0;
    for (;;) {
        // interior phase
        bool done = false;
        while ((cur >> 24) == 0) {
            const uint32_t lf = cur & 0xFFFFFFu;
            if (kStats) c.visits++;
            float4 la, lb, ra, rb;
            node_pair(v.nodes, lf, la, lb, ra, rb);
            const float d1 = aabb_pairs<kFast>(la, lb, r, t);
            const float d2 = aabb_pairs<kFast>(ra, rb, r, t);
            const uint32_t pl = __float_as_uint(lb.z), pr = __float_as_uint(rb.z);
            const bool sw = d1 > d2;
            const float dn = sw ? d2 : d1, df = sw ? d1 : d2;
            const uint32_t pn = sw ? pr : pl, pf = sw ? pl : pr;
            if (dn == kBig) {
                if (head == 0) { done = true; break; }
                cur = stack.pop(--head);
            } else {
                cur = pn;
                if (df != kBig) {
                    if (head >= stack_cap(stack)) return false;
                    stack.push(head++, pf);
                }
            }
        }
        if (done) break;
        // leaf phase
        const uint32_t lf = cur & 0xFFFFFFu, cnt = cur >> 24;
        leaf_tests<kFast>(sc, v, lf, cnt, r, t, index);
        if (kStats) c.rtests += cnt;
        if (head == 0) break;
        cur = stack.pop(--head);
    }
    return true;
}

// Leaf-batched form: every iteration the wave runs EITHER one interior step
// for the lanes inside the tree OR the leaf tests for the lanes waiting at a
// leaf -- the latter once at least `kBatch` lanes wait (or every unfinished
// lane does).  A lane at a leaf does nothing until its leaf is tested, so per
// lane the operation sequence is exactly trav_step's; only the interleaving
// between lanes changes.  Avoids paying the leaf body (rect records, ~40 VALU)
// in nearly every iteration as the if-if loop does (P(some lane of 64 at a
// leaf) ~ 99 % at 1.47 leaf visits per 18.3 interior visits).
template <bool kFast, bool kStats, uint32_t kBatch, typename V, typename Stack>
__device__ __forceinline__ bool traverse_lb(const DevScene& sc, const V& v, const Ray& r, float& t,
                                            uint32_t& index, Stack& stack, Counters& c) {
    uint32_t cur = sc.root_packed, head = 0;
    bool done = false, ovf = false;
    for (;;) {
        const bool at_leaf = !done && (cur >> 24) != 0;
        const uint64_t live = __ballot(!done);
        if (live == 0) break;
        const uint64_t leaves = __ballot(at_leaf);
        const bool do_leaves = leaves != 0 && (leaves == live || (uint32_t)__popcll(leaves) >= kBatch);
        if (do_leaves) {
            if (at_leaf) {
                const uint32_t lf = cur & 0xFFFFFFu, cnt = cur >> 24;
                leaf_tests<kFast>(sc, v, lf, cnt, r, t, index);
                if (kStats) c.rtests += cnt;
                if (head == 0) done = true;
                else cur = stack.pop(--head);
            }
        } else if (!done && !at_leaf) {
            const uint32_t lf = cur & 0xFFFFFFu;
            if (kStats) c.visits++;
            float4 la, lb, ra, rb;
            node_pair(v.nodes, lf, la, lb, ra, rb);
            const float d1 = aabb_pairs<kFast>(la, lb, r, t);
            const float d2 = aabb_pairs<kFast>(ra, rb, r, t);
            const uint32_t pl = __float_as_uint(lb.z), pr = __float_as_uint(rb.z);
            const bool sw = d1 > d2;
            const float dn = sw ? d2 : d1, df = sw ? d1 : d2;
            const uint32_t pn = sw ? pr : pl, pf = sw ? pl : pr;
            if (dn == kBig) {
                if (head == 0) done = true;
                else cur = stack.pop(--head);
            } else {
                cur = pn;
                if (df != kBig) {
                    if (head >= stack_cap(stack)) { ovf = true; done = true; }
                    else stack.push(head++, pf);
                }
            }
        }
    }
    return !ovf;
}

// The straight statement of intersect_bvh_iterative over the reference node
// layout (sc.nodes_ref, 2 float4 per node: a, (mx.yz, lf, count)).
template <bool kStats, typename Stack>
__device__ __forceinline__ bool traverse_reference(const DevScene& sc, const Ray& r, float& t, uint32_t& index,
                                                   Stack& stack, Counters& c) {
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

// Closest hit for one ray: production traversal with the exact fallback.
// kWW selects the while-while loop structure.
template <bool kStats, typename V, typename Stack, int kWW = 0>
__device__ __forceinline__ bool closest_hit(const DevScene& sc, const V& v, F3 o, F3 d, float& t,
                                            uint32_t& index, Stack& stack, Counters& c) {
    const Ray r = make_ray(o, d);
    if constexpr (kWW == 2) {
        if (sc.fast_ok && ray_fast_ok(r)) return traverse_lean<true, kStats>(sc, v, r, t, index, stack, c);
        return traverse_lean<false, kStats>(sc, v, r, t, index, stack, c);
    } else if constexpr (kWW >= 8 && kWW != 9) {
        if (sc.fast_ok && ray_fast_ok(r)) return traverse_lb<true, kStats, (uint32_t)kWW>(sc, v, r, t, index, stack, c);
        return traverse_lb<false, kStats, (uint32_t)kWW>(sc, v, r, t, index, stack, c);
    } else if constexpr (kWW == 9) {
        if (sc.fast_ok && ray_fast_ok(r) && cons_ray_ok(sc, r))
            return traverse_cons<kStats>(sc, v, r, t, index, stack, c);
        return traverse_li<false, kStats>(sc, view(sc.nodes_exact, v.recs), r, t, index, stack, c);
    } else if constexpr (kWW == 7) {
        if (sc.fast_ok && ray_fast_ok(r)) return traverse_lil<kStats>(sc, v, r, t, index, stack, c);
        return traverse_li<false, kStats>(sc, v, r, t, index, stack, c);
    } else if constexpr (kWW == 5) {
        if (sc.fast_ok && ray_fast_ok(r)) return traverse_li<true, kStats>(sc, v, r, t, index, stack, c);
        return traverse_li<false, kStats>(sc, v, r, t, index, stack, c);
    } else if constexpr (kWW == 1) {
        if (sc.fast_ok && ray_fast_ok(r)) return traverse_ww<true, kStats>(sc, v, r, t, index, stack, c);
        return traverse_ww<false, kStats>(sc, v, r, t, index, stack, c);
    } else {
        if (sc.fast_ok && ray_fast_ok(r)) return traverse<true, kStats>(sc, v, r, t, index, stack, c);
        return traverse<false, kStats>(sc, v, r, t, index, stack, c);
    }
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
        // shaders.metal:316-318, length(r) > 1: RN(sqrt(x)) > 1 <=> x > 1 + 2^-23
        // for every binary32 x (exhaustive check: scripts/verify_sqrt_gt1.c)
        while (len2 > 0x1.000002p0f) {
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

// Where a path's throughput T and radiance L live while its ray traverses
// (they are only touched by shading): in registers (NoCold), or parked in LDS,
// [field][thread], which frees six VGPRs for the traversal loop.
struct NoCold {
    __device__ __forceinline__ void save(const F3&, const F3&) const {}
    __device__ __forceinline__ void restore(F3&, F3&) const {}
};
struct LdsCold {
    float* base;        // &lds[field 0][this thread]
    uint32_t stride;    // threads per block
    __device__ __forceinline__ void save(const F3& T, const F3& L) const {
        base[0] = T.x; base[stride] = T.y; base[2 * stride] = T.z;
        base[3 * stride] = L.x; base[4 * stride] = L.y; base[5 * stride] = L.z;
    }
    __device__ __forceinline__ void restore(F3& T, F3& L) const {
        T = F3{base[0], base[stride], base[2 * stride]};
        L = F3{base[3 * stride], base[4 * stride], base[5 * stride]};
    }
};

// Whole path (shaders.metal:302-344): returns sqrt(max(L, 0)).
// kRef selects traverse_reference (MM_PIPE_REFERENCE).
template <bool kStats, bool kRef, typename V, typename Stack, int kWW = 0, typename Cold = NoCold>
__device__ __forceinline__ F3 trace_path(const DevScene& sc, const V& v, F3 ori, F3 dir, uint32_t seed,
                                         int bounce_limit, int mirror_limit, Stack& stack, Counters& c,
                                         bool& overflow, const Cold& cold = Cold{}) {
    PathState p;
    p.ori = ori; p.dir = dir; p.seed = seed;
    p.T = F3{1.0f, 1.0f, 1.0f};
    p.L = F3{0.0f, 0.0f, 0.0f};
    p.mh = 0;
    for (p.n = 0; p.n < bounce_limit + p.mh; ++p.n) {
        float t = kBig;
        uint32_t k = 0;
        bool ok;
        cold.save(p.T, p.L);
        if constexpr (kRef) ok = traverse_reference<kStats>(sc, make_ray(p.ori, p.dir), t, k, stack, c);
        else ok = closest_hit<kStats, V, Stack, kWW>(sc, v, p.ori, p.dir, t, k, stack, c);
        cold.restore(p.T, p.L);
        if (kStats) c.rays++;
        if (!ok) { overflow = true; break; }
        if (!shade_step(sc, p, t, k, mirror_limit)) break;
    }
    return F3{sqrtf(fmaxf(p.L.x, 0.0f)), sqrtf(fmaxf(p.L.y, 0.0f)), sqrtf(fmaxf(p.L.z, 0.0f))};
}

}  // namespace mm
