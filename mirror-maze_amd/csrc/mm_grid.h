// mm_grid.h — certified grid search: the closest hit of the reference's BVH
// walk (intersect_bvh_iterative, shaders.metal:115-156) without walking it.
//
// Why the answer is the reference's.  Let A be the set of rects that pass
// ray_rect_intersect (shaders.metal:51-67) with every clause except `a < t`,
// a* = min over A of a, attained by R* only, and L* the reference BVH leaf
// holding R*.  If L*'s box passes intersect_aabb (shaders.metal:87-95) at
// every t > a* -- tmax >= tmin, tmax > 0, tmin <= a* -- then the reference
// returns (a*, R*) whatever order it visits nodes in:
//   * t starts at 1e30 and only a rect of A can lower it, so t >= a* always,
//     and t > a* until R* itself is accepted (a* is attained once);
//   * every ancestor box of L* contains L*'s box, and the slab quotients
//     RN((b - o)/d) are monotone in b, so an ancestor's [tmin, tmax]
//     contains L*'s; each box on the root -> L* path is tested at some
//     t > a* and passes, so L* is reached and R* is tested at t > a* and
//     accepted; nothing in A can replace it afterwards.
// So it suffices to find a*, R* and to know that a* is attained once.
//
// The search.  The scene bounds, widened by eps = C * 2^-14 (C = the largest
// |coordinate|), are cut into a uniform grid; each cell lists every rect whose
// box comes within eps of it; rects that cover more than half of the cells
// (the maze floor) are tested by every query instead.  A query tests the
// global rects, then walks the cells the ray crosses (3-D DDA) and tests each
// cell's list, and stops once the best a found is below the exit time of the
// current cell (or the ray leaves the grid).  Every rect of A with a <= the
// final best is tested: its hit point P = o + a d lies within
// delta ~ 10 u C of the rect (the rounding of the reference's bounds test,
// u = 2^-24), and the computed crossing times (one fma per step, see
// grid_search) put the ray at any t <= (the last exit time) within
// eta ~ 8 u C of a visited cell, so the
// rect comes within delta + eta << eps of a visited cell and is on its list.
// The exact per-rect operations (the compact records of rect_compact.cpp)
// give each rect's a, so the minimum and whether it is attained twice are
// exact.  scripts/grid_sim.c replays every query of a C3 frame (137 M) on
// the CPU against the reference walk: 0 differences.
//
// Face ranges (64-bit cell words): a cell entered through face f tests only
// the entries the neighbour across f -- the cell visited just before -- does
// not list.  Every entry of every visited cell's list is still tested: by
// induction, the first cell tests its whole list, and an entry of cell i that
// is skipped is on cell i-1's list, all of which was tested by then.  Testing a
// rect twice never changes (best, bk, tie) (same a, same k), so skipping the
// repeat changes nothing.
//
// A tie, a failed leaf-box check or a ray outside the Markstein guards /
// the grid runs the reference walk (the BVH traversal) instead.
#pragma once

#include "mm_trace.h"

namespace mm {

// Per-rect compact record test for the search: updates (best, bk, tie) with
// the rect's a if it is in A (every clause of ray_rect_intersect except
// a < t).  Records are rect_compact.cpp's FAST records, indexed by rect.
// With kSlow, SLOW records (rects without an exact axis-aligned form) run the
// general statement on the rect geometry (rect_test's operations).
__device__ __forceinline__ void grid_update(float a, uint32_t k, float& best, uint32_t& bk, uint32_t& tie) {
    if (a < best) {
        best = a;
        bk = k;
        tie = 0u;
    } else if (a == best && k != bk) {
        tie = 1u;
    }
}

__device__ __forceinline__ void grid_update_sel(float a, uint32_t k, float& best, uint32_t& bk, uint32_t& tie) {
    const bool lt = a < best, eq = (a == best) & (k != bk);
    tie = lt ? 0u : (tie | (eq ? 1u : 0u));
    bk = lt ? k : bk;
    best = lt ? a : best;
}

// (e: the rect's name in the search -- k, or 8 k in compact grids; rect_name)
__device__ __forceinline__ void grid_rect_general(const float4* __restrict__ geo, uint32_t k, uint32_t e,
                                                  const Ray& r, float& best, uint32_t& bk, uint32_t& tie) {
    const float4 g0 = geo[4 * k + 0], g1 = geo[4 * k + 1], g2 = geo[4 * k + 2], g3 = geo[4 * k + 3];
    const F3 o = xyz(g0), n = xyz(g1), v = xyz(g2), u = xyz(g3);
    const float lv = g0.w, lu = g1.w;
    const float nc = dot3(r.d, n);
    const float a = dot3(o - r.o, n) / nc;
    const F3 rv = (r.o - o) + a * r.d;
    const float d1 = qdiv(dot3(rv, v), lv, g2.w);
    const float d2 = qdiv(dot3(rv, u), lu, g3.w);
    if (d1 >= 0.0f && d1 <= lv && d2 >= 0.0f && d2 <= lu && nc != 0.0f && a > 0.1f) grid_update(a, e, best, bk, tie);
}

// Grid records (grid_build.cpp, 8 x u32 per rect, indexed by rect):
//   0 o_k  1 o_v  2 o_u  3 Yv_lo  4 Yv_hi  5 Yu_lo  6 Yu_hi  7 k | k_axis << 20 | kind << 30
// v = the lower of the two in-plane axes, u = the higher (so both follow from
// k_axis), and the compact record's test X_lo <= RN(Y * v_axis) <= X_hi folded
// into thresholds on Y = (ori_v - o_v) + a * d_v itself.
__device__ __forceinline__ float sel_k(bool k0, bool k2, F3 v) { return k0 ? v.x : (k2 ? v.z : v.y); }
__device__ __forceinline__ float sel_xy(bool sx, bool sy, F3 v) { return sx ? v.x : (sy ? v.y : v.z); }

// A cell list's entries (u16 rect indices).  A walk keeps its list position
// in the form the list's memory wants: in LDS the entry's byte address
// (LdsList: base + 2 i, so a rect test loads its entry with no address
// arithmetic -- ds_read_u16 straight from the position -- and steps by 2),
// in global memory the entry index (GlobalList).
struct LdsList {
    uint32_t base;  // LDS byte address of entry 0
    __device__ __forceinline__ uint32_t pos(uint32_t i) const { return base + 2u * i; }
    static constexpr uint32_t kStep = 2;
    __device__ __forceinline__ uint32_t at(uint32_t p) const {
        return *(const __attribute__((address_space(3))) uint16_t*)(uintptr_t)p;
    }
};
struct GlobalList {
    const uint16_t* p;
    __device__ __forceinline__ uint32_t pos(uint32_t i) const { return i; }
    static constexpr uint32_t kStep = 1;
    __device__ __forceinline__ uint32_t at(uint32_t i) const { return p[i]; }
};
// The grid's cell words, read the same two ways: a walk in LDS keeps the
// current cell as its word's LDS byte address (LdsCells: stepped by +-8 or +-4
// times the cell-index step, so the read carries no address arithmetic and the
// base is not reloaded per step), in global memory as the cell index.
struct LdsCells {
    uint32_t base;  // LDS byte address of cell 0's word
    template <bool kWide>
    static constexpr int kScale = kWide ? 8 : 4;
    template <bool kWide>
    __device__ __forceinline__ uint32_t pos(int ci) const { return base + (uint32_t)ci * (uint32_t)kScale<kWide>; }
    __device__ __forceinline__ uint64_t at64(uint32_t p) const {
        return *(const __attribute__((address_space(3))) uint64_t*)(uintptr_t)p;
    }
    __device__ __forceinline__ uint32_t at32(uint32_t p) const {
        return *(const __attribute__((address_space(3))) uint32_t*)(uintptr_t)p;
    }
};
struct GlobalCells {
    const char* p;
    template <bool kWide>
    static constexpr int kScale = 1;
    template <bool kWide>
    __device__ __forceinline__ uint32_t pos(int ci) const { return (uint32_t)ci; }
    __device__ __forceinline__ uint64_t at64(uint32_t i) const { return reinterpret_cast<const uint64_t*>(p)[i]; }
    __device__ __forceinline__ uint32_t at32(uint32_t i) const { return reinterpret_cast<const uint32_t*>(p)[i]; }
};

// Cell words staged into LDS (trace_kernels.hip stage_and_run): the
// first-entry field (bits 0-21) becomes the LDS byte address of that entry,
// lbase + 2 first (< 2^22), so the walk reads list ranges without address
// arithmetic (grid_search, cell_pos).  v: 16 bytes of the cells section.
template <bool kWide>
__device__ __forceinline__ uint4 grid_stage_cells(uint4 v, uint32_t lbase) {
    auto fix = [&](uint32_t w) { return (w & ~0x3FFFFFu) | (lbase + 2u * (w & 0x3FFFFFu)); };
    v.x = fix(v.x);
    v.z = fix(v.z);
    if (!kWide) {
        v.y = fix(v.y);
        v.w = fix(v.w);
    }
    return v;
}

// LDS byte address of an LDS object reached through a generic pointer.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;  // (an address-space cast)
}

// Where the grid's arrays are read from (LDS or global memory).
template <typename CellsT, typename ListT, typename RecsT, typename BoxT, typename ClsT>
struct GridView {
    CellsT cells;  // per cell: a 64-bit (wide) or 32-bit word (list range): LdsCells or GlobalCells
    ListT list;    // rect indices (u16): LdsList or GlobalList
    RecsT recs;    // 2 x uint4 per rect, or 1 (compact records)
    BoxT box;      // 3 x float2 per rect: its reference leaf's (mn, mx) per axis
    ClsT cls;      // compact records' threshold classes (float4), else unused
};
template <typename C, typename L, typename R, typename B, typename K>
__device__ __forceinline__ GridView<C, L, R, B, K> grid_view(C c, L l, R r, B b, K k) {
    return GridView<C, L, R, B, K>{c, l, r, b, k};
}

// Rect k's record: w = (o_k, o_v, o_u, meta) -- meta's axis at bit 20, kind at
// bit 30 -- and its folded thresholds (Yv_lo, Yv_hi, Yu_lo, Yu_hi).  32-B
// records hold both; compact records (kCompact, maze grids) hold w and their
// class as class << 4 (meta bits 4-9, meta & 0x3F0 = the byte offset of the
// class's 16-B entry in the class table; grid_build.cpp).
// Compact (maze) grids name a rect as e = 8 k -- the list entries, the
// global-rect indices, bk -- so that record k's byte offset 16 k = e + e is one
// pairable v_add_u32 (a shift left is single-slot on gfx950, DESIGN.md §4;
// written as asm because the compiler turns x + x into that shift).
__device__ __forceinline__ uint32_t twice(uint32_t e) {
    uint32_t r;
    asm("v_add_u32 %0, %1, %1" : "=v"(r) : "v"(e));
    return r;
}
template <bool kCompact>
__device__ __forceinline__ constexpr uint32_t rect_name(uint32_t k) { return kCompact ? 8u * k : k; }
template <bool kCompact>
__device__ __forceinline__ constexpr uint32_t rect_index(uint32_t e) { return kCompact ? e >> 3 : e; }

template <bool kCompact, typename GV>
__device__ __forceinline__ uint4 rec_words(const GV& gv, uint32_t k) {
    if constexpr (kCompact) {  // k = e = 8 x the rect index (above)
        return *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(gv.recs) + twice(k));
    } else {
        const uint4 w0 = gv.recs[2 * k + 0];
        return make_uint4(w0.x, w0.y, w0.z, gv.recs[2 * k + 1].w);
    }
}
template <bool kCompact, typename GV>
__device__ __forceinline__ float4 rec_thresholds(const GV& gv, uint32_t k, uint32_t meta) {
    if constexpr (kCompact) {
        return *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(gv.cls) + (meta & 0x3F0u));
    } else {
        const uint4 w0 = gv.recs[2 * k + 0], w1 = gv.recs[2 * k + 1];
        return make_float4(__uint_as_float(w0.w), __uint_as_float(w1.x), __uint_as_float(w1.y),
                           __uint_as_float(w1.z));
    }
}

// kXZ: every listed FAST record has its normal along x or z (the maze forms:
// grid_build.cpp checks it, the maze's y-normal floor and ceiling are global
// rects), so each select is 2-way.  kCompact: 16-B records + class table.
template <bool kSlow, bool kXZ, bool kCompact, typename GV>
__device__ __forceinline__ void grid_rect(const GV& gv, const float4* __restrict__ geo, uint32_t k, const Ray& r,
                                          float& best, uint32_t& bk, uint32_t& tie) {
    const uint4 w = rec_words<kCompact>(gv, k);
    const uint32_t meta = w.w;
    if constexpr (kSlow) {
        if ((meta >> 30) == 2u) {
            grid_rect_general(geo, rect_index<kCompact>(k), k, r, best, bk, tie);
            return;
        }
    }
    const uint32_t ak = (meta >> 20) & 3u;
    constexpr bool kTwoWay = kXZ;
    // compact (maze) records: x or z normal, y the first in-plane axis
    // (grid_build.cpp), so k0 is one compare and (v, u) = (y, the other)
    const bool k0 = kCompact ? meta < (1u << 20) : ak == 0u, k2 = kTwoWay ? !k0 : ak == 2u;
    const float ok = kTwoWay ? (k0 ? r.o.x : r.o.z) : sel_k(k0, k2, r.o);
    const float dk = kTwoWay ? (k0 ? r.d.x : r.d.z) : sel_k(k0, k2, r.d);
    const float yk = kTwoWay ? (k0 ? r.y.x : r.y.z) : sel_k(k0, k2, r.y);
    const float ov = kCompact ? r.o.y : (k0 ? r.o.y : r.o.x), dv = kCompact ? r.d.y : (k0 ? r.d.y : r.d.x);
    const float ou = kCompact ? (k0 ? r.o.z : r.o.x) : (k2 ? r.o.y : r.o.z);
    const float du = kCompact ? (k0 ? r.d.z : r.d.x) : (k2 ? r.d.y : r.d.z);
    const float4 th = rec_thresholds<kCompact>(gv, k, meta);
    const float a = qdiv(__uint_as_float(w.x) - ok, dk, yk);
    const float y1 = (ov - __uint_as_float(w.y)) + a * dv;
    const float y2 = (ou - __uint_as_float(w.z)) + a * du;
    // One branch around a select-form update (a branch-free update measured
    // 6.11 vs 5.86 ms on C3: most tests miss, and the branch skips the update
    // for the whole wave; && chains compile to one exec-mask branch per clause).
    const uint32_t hit = (uint32_t)(y1 >= th.x) & (uint32_t)(y1 <= th.y) & (uint32_t)(y2 >= th.z) &
                         (uint32_t)(y2 <= th.w) & (uint32_t)(a > 0.1f);
    if (hit) grid_update_sel(a, k, best, bk, tie);
}

// The same test for a record whose normal axis A is known (a global rect:
// its record is the same for every lane, so the caller branches on its axis
// uniformly and the per-lane axis selects go away).  v = the lower in-plane
// axis, u = the higher, as in the record; same operations as grid_rect.
template <int A>
__device__ __forceinline__ float ax(F3 v) {
    return A == 0 ? v.x : (A == 1 ? v.y : v.z);
}
template <int A, bool kCompact, typename GV>
__device__ __forceinline__ void grid_rect_axis(const GV& gv, uint32_t k, uint4 w, const Ray& r, float& best,
                                               uint32_t& bk, uint32_t& tie) {
    // (a compact z-normal record stores y first: grid_build.cpp)
    constexpr int V = A == 0 ? 1 : (A == 2 && kCompact ? 1 : 0), U = A == 2 ? (kCompact ? 0 : 1) : 2;
    const float4 th = rec_thresholds<kCompact>(gv, k, w.w);
    const float a = qdiv(__uint_as_float(w.x) - ax<A>(r.o), ax<A>(r.d), ax<A>(r.y));
    const float y1 = (ax<V>(r.o) - __uint_as_float(w.y)) + a * ax<V>(r.d);
    const float y2 = (ax<U>(r.o) - __uint_as_float(w.z)) + a * ax<U>(r.d);
    const uint32_t hit = (uint32_t)(y1 >= th.x) & (uint32_t)(y1 <= th.y) & (uint32_t)(y2 >= th.z) &
                         (uint32_t)(y2 <= th.w) & (uint32_t)(a > 0.1f);
    if (hit) grid_update_sel(a, k, best, bk, tie);
}

// A global rect (g.glob: the same k for every lane): the record's kind and
// axis are read once per wave and branched on uniformly.
template <bool kSlow, bool kCompact, typename GV>
__device__ __forceinline__ void grid_rect_uniform(const GV& gv, const float4* __restrict__ geo, uint32_t k,
                                                  const Ray& r, float& best, uint32_t& bk, uint32_t& tie) {
    const uint4 w = rec_words<kCompact>(gv, k);
    const uint32_t meta = __builtin_amdgcn_readfirstlane(w.w);
    if (kSlow && (meta >> 30) == 2u) {
        grid_rect_general(geo, rect_index<kCompact>(k), k, r, best, bk, tie);
        return;
    }
    const uint32_t ak = (meta >> 20) & 3u;
    if (ak == 0u) grid_rect_axis<0, kCompact>(gv, k, w, r, best, bk, tie);
    else if (ak == 1u) grid_rect_axis<1, kCompact>(gv, k, w, r, best, bk, tie);
    else grid_rect_axis<2, kCompact>(gv, k, w, r, best, bk, tie);
}

// (&=, not &&: see ray_fast_ok)
__device__ __forceinline__ bool grid_ray_ok(const DevGrid& g, const Ray& r) {
    bool ok = r.o.x >= g.mn[0];
    ok &= r.o.x <= g.mx[0];
    ok &= r.o.y >= g.mn[1];
    ok &= r.o.y <= g.mx[1];
    ok &= r.o.z >= g.mn[2];
    ok &= r.o.z <= g.mx[2];
    return ok;
}

__device__ __forceinline__ int grid_cell(const DevGrid& g, float o, int a) {
    const int i = (int)floorf((o - g.mn[a]) * g.inv[a]);
    return min(max(i, 0), g.nm1[a]);
}

// A kernel-argument value read at its use.  A uniform branch on a kernel
// argument inside the walk is otherwise hoisted out of the bounce loop as a
// 64-bit lane mask, which the compiler then spills to VGPR lanes (two
// single-slot v_readlane per use); through the asm the compare
// stays at the branch and the argument is reloaded (s_load) when needed.
__device__ __forceinline__ uint32_t arg_at_use(uint32_t v) {
    uint32_t r;
    asm volatile("s_mov_b32 %0, %1" : "=s"(r) : "s"(v));
    return r;
}

// DDA state per axis: the index b of the next cell boundary the ray crosses
// (boundary b lies at mn + b * cell) and the time it crosses it; the step
// direction is the sign of y = 1/d.  Going up, the current cell is b - 1
// and the walk leaves the grid past boundary n; going down, the cell is b
// and it leaves below boundary 0.
__device__ __forceinline__ float grid_time(const DevGrid& g, int a, int b, float o, float y) {
    return ((g.mn[a] + (float)b * g.cell[a]) - o) * y;
}
__device__ __forceinline__ int grid_first(const DevGrid& g, int a, float o, float y) {
    const int i = min(max((int)floorf((o - g.mn[a]) * g.inv[a]), 0), g.nm1[a]);
    return y > 0.0f ? i + 1 : i;
}

// Search + certificate.  Returns true with (t, index) = the reference's answer
// (t = kBig when nothing is hit), false when the caller must walk the BVH.
// Requires sc.fast_ok && ray_fast_ok(r) && grid_ray_ok.
// kFlat: the grid has one cell along y (g.n[1] == 1, grid_build.cpp's merged
// axis): a y step always leaves the grid, so the walk steps x or z only --
// the same cells and stop as the general walk, which breaks on the same y
// step (by leaves 0..n[1]).  These "maze forms" also need every listed record
// FAST with an x or z normal and read compact records (GridHost::flat_ok), so
// the list tests use 2-way selects and one 16-B record + a class-table entry.
template <bool kStats, bool kSlow, bool kWide, bool kFlat, typename GV>
__device__ __forceinline__ bool grid_search(const DevGrid& g, const GV& gv, const float4* __restrict__ geo,
                                            const Ray& r, float& t, uint32_t& index, Counters& c) {
    float best = kBig;
    uint32_t bk = 0xFFFFFFFFu;
    uint32_t tie = 0u;  // (a bool lives in an exec-mask register: SALU merges at every join)
    // Floor and ceiling (g.slab): a y-normal plane the ray moves away from
    // gives a = RN(num / d_y) with num = RN(Y - o_y) on the wrong side of
    // RN(0.05 d_y), so a <= 0.05 (1 + u) and a > 0.1 fails -- that rect
    // cannot change (best, bk, tie).  When every lane can skip one of the
    // two, each lane tests only the other (its record read per lane).
    bool one = false;
    uint32_t k1 = 0;
    if (arg_at_use(g.slab)) {
        const float q = 0.05f * r.d.y;
        const bool lo_dead = r.d.y > 0.0f && g.slab_y[0] - r.o.y <= q;
        const bool hi_dead = r.d.y < 0.0f && g.slab_y[1] - r.o.y >= q;
        one = __builtin_amdgcn_ballot_w64(!(lo_dead || hi_dead)) == 0;
        k1 = rect_name<kFlat>(lo_dead ? g.glob[1] : g.glob[0]);
    }
    if (one) {
        MM_LANE_STAT(kLpGlobal);
        grid_rect_axis<1, kFlat>(gv, k1, rec_words<kFlat>(gv, k1), r, best, bk, tie);
    } else {
        for (uint32_t j = 0, n = arg_at_use(g.n_glob); j < n; ++j) {
            MM_LANE_STAT(kLpGlobal);
            grid_rect_uniform<kSlow, kFlat>(gv, geo, rect_name<kFlat>(g.glob[j]), r, best, bk, tie);
        }
    }
    // The walk starts in the cell of the ray's point at t = 3/32, not at the
    // origin: a rect of A has a > 0.1, so the cells the ray occupies only for
    // t < 3/32 hold nothing it can return, and the rounding of the start
    // point (a few ulp of C) is covered by the eps-widened lists as the
    // crossing times are.  A bounce origin lies on a wall, i.e. within eps of
    // a cell face; from the origin the walk would start on the far side of
    // that face in about half the cases and test a cell the ray never enters
    // (t = 1/16: C3 3.40 -> 3.37 ms/frame, C5 scene 7.20 -> 7.05; 3/32: a
    // further 1.3 % / 1.4 %; bit-identical; profiles/r02/ab_start_cell.txt).
    // The crossing times stay those of the origin.
    const float s0 = 0.09375f;
    int bx = grid_first(g, 0, r.o.x + s0 * r.d.x, r.y.x),
        by = kFlat ? (r.y.y > 0.0f ? 1 : 0) : grid_first(g, 1, r.o.y + s0 * r.d.y, r.y.y),
        bz = grid_first(g, 2, r.o.z + s0 * r.d.z, r.y.z);
    // Crossing time of boundary b along axis a in one fma per step:
    // t = RN(b * B_a + A_a), A_a = RN(RN(mn_a - o_a) * y_a), B_a = RN(cell_a * y_a).
    // Its error along axis a, |dt| * |d_a|, is a few u (|mn_a - o_a| + b cell_a
    // + |x_a(t) - o_a|) <= ~8 u C (y_a = RN(1/d_a)); grid_time's direct form has
    // ~5 u C.  Both are far below the lists' eps = 2^-14 C = 1024 u C, which is
    // all the search's argument needs of them (header: delta + eta << eps).
    const float Ax = (g.mn[0] - r.o.x) * r.y.x, Bx = g.cell[0] * r.y.x;
    const float Az = (g.mn[2] - r.o.z) * r.y.z, Bz = g.cell[2] * r.y.z;
    const float Ay = kFlat ? 0.0f : (g.mn[1] - r.o.y) * r.y.y, By = kFlat ? 0.0f : g.cell[1] * r.y.y;
    float tx = __builtin_fmaf((float)bx, Bx, Ax), tz = __builtin_fmaf((float)bz, Bz, Az);
    float ty = kFlat ? grid_time(g, 1, by, r.o.y, r.y.y) : __builtin_fmaf((float)by, By, Ay);
    // Cell words (grid_build.cpp).  Wide (64-bit): bits 0-21 the list's first
    // entry; bit 63 set: bits 22-31 the count, the whole list for every face;
    // clear: bits 22-24 the count m <= 7, and per entry face f a 6-bit
    // (start | len << 3) at bit 25 + 6f -- the range of the list the neighbour
    // across f did not already hold.  Plain (32-bit): first | count << 22.
    // face = 6: the whole list (the first cell).  (A run-time format flag
    // cost 2 % on C3: the format is a template parameter.)
    // The current cell, stepped with the walk (index +-1 per x step, +-n0 per
    // z step (n0 n1 in 3-D), +-n0 per y step; as gv.cells' position), and the bit offset of each
    // axis's entry-face field in the wide cell word (25 + 6 f; the face
    // toward the previous cell is fixed per ray and axis), packed 8 bits per
    // axis: x, y, z.
    int ci;
    {
        const int ix = r.y.x > 0.0f ? bx - 1 : bx, iz = r.y.z > 0.0f ? bz - 1 : bz;
        const int iy = kFlat ? 0 : (r.y.y > 0.0f ? by - 1 : by);
        ci = kFlat ? iz * g.n[0] + ix : (iz * g.n[1] + iy) * g.n[0] + ix;
    }
    // the walk's cell position (gv.cells: the word's LDS byte address, or the index) and its steps
    constexpr int kCs = decltype(gv.cells)::template kScale<kWide>;
    uint32_t cp = gv.cells.template pos<kWide>(ci);
    const int dcx = r.y.x > 0.0f ? kCs : -kCs;
    const int dcz = (r.y.z > 0.0f ? kCs : -kCs) * (kFlat ? g.n[0] : g.n[0] * g.n[1]);
    const int dcy = kFlat ? 0 : (r.y.y > 0.0f ? kCs : -kCs) * g.n[0];
    const uint32_t fsh = (25u + (r.y.x > 0.0f ? 0u : 6u)) | ((37u + (r.y.y > 0.0f ? 0u : 6u)) << 8) |
                         ((49u + (r.y.z > 0.0f ? 0u : 6u)) << 16);
    // sh = 0: the whole list (the first cell)
    // The cell's list range [j, jend) in gv.list's positions: in LDS entry
    // byte addresses -- the staged cell words' first-entry fields already hold
    // them (grid_stage_cells), so the decode doubles the counts, and does it
    // without a shift left (single-slot on gfx950) --, in global
    // memory entry indices.
    uint32_t j, jend;
    auto cell_pos = [&](uint32_t sh) {
        constexpr bool kB = decltype(gv.list)::kStep == 2u;
        if constexpr (kWide && kFlat) {
            // maze forms (grid_build.cpp): no whole-list cells, and the x / z entry faces' ranges in the high
            // half at bits 5 + 6 f' (f' = 0 +x, 1 -x, 2 +z, 3 -z): sh is that shift within the high half
            const uint64_t cw = gv.cells.at64(cp);
            const uint32_t lo = (uint32_t)cw, first = lo & 0x3FFFFFu;
            if (sh == 0u) {  // the whole list (the first cell)
                j = first;
                jend = first + (kB ? (lo >> 21) & 0xEu : (lo >> 22) & 7u);
            } else {
                const uint32_t f = (uint32_t)(cw >> 32) >> sh;
                j = first + (kB ? (twice(f) & 14u) : (f & 7u));
                jend = j + (kB ? ((f >> 2) & 14u) : ((f >> 3) & 7u));
            }
        } else if constexpr (kWide) {
            const uint64_t cw = gv.cells.at64(cp);
            const uint32_t lo = (uint32_t)cw;
            const bool whole = (int32_t)(uint32_t)(cw >> 32) < 0;
            const uint32_t first = lo & 0x3FFFFFu;
            const uint32_t m = kB ? (lo >> 21) & (whole ? 0x7FEu : 0xEu) : (lo >> 22) & (whole ? 0x3FFu : 7u);
            if (sh == 0u) {  // the whole list (the first cell)
                j = first;
                jend = first + m;
            } else {
                const uint32_t f = (uint32_t)(cw >> sh);
                const uint32_t st = kB ? (twice(f) & 14u) : (f & 7u), len = kB ? ((f >> 2) & 14u) : ((f >> 3) & 7u);
                j = first + (whole ? 0u : st);
                jend = j + (whole ? m : len);
            }
        } else {
            const uint32_t cw = gv.cells.at32(cp);
            j = cw & 0x3FFFFFu;
            jend = j + (kB ? ((cw >> 21) & 0x7FEu) : (cw >> 22));
        }
    };
    cell_pos(0u);
    uint32_t cells = 1, tests = g.n_glob;
    if constexpr (kFlat) {
        // The maze forms' walk (one cell along y: the steps are x or z).  Every way
        // out of the grid is folded into one end time per ray, tend = min(ty, the
        // crossing time of the last x boundary, of the last z boundary) -- each
        // computed with the same fma as the step that would cross it, from the
        // same float boundary index, so a step reaches it exactly -- and the walk
        // continues while min(tx, tz) <= best and < tend: no per-step bounds
        // checks, no y-step test, no boundary-index conversion.  Against the 3-D
        // walk below this skips only cells entered exactly at the end time (a tie
        // of tx or tz with the exit, where that walk steps into a cell and leaves
        // the grid in the same instant): such a cell meets the ray in one point,
        // which lies on the face of the cell just tested, so the lists' eps
        // covers it (header) and the answer is unchanged.  (CPU replay of every
        // query of a C3 frame: scripts/grid_sim.c TEND=1.)
        const float sgx = r.y.x > 0.0f ? 1.0f : -1.0f, sgz = r.y.z > 0.0f ? 1.0f : -1.0f;
        float fbx = (float)bx, fbz = (float)bz;  // (exact small integers)
        const float tend = fminf(ty, fminf(__builtin_fmaf(r.y.x > 0.0f ? g.nf[0] : 0.0f, Bx, Ax),
                                           __builtin_fmaf(r.y.z > 0.0f ? g.nf[2] : 0.0f, Bz, Az)));
        // (the high-half shifts of the +x / -x / +z / -z ranges: cell_pos, grid_build.cpp)
        const uint32_t shx = kWide ? (r.y.x > 0.0f ? 5u : 11u) : 0u, shz = kWide ? (r.y.z > 0.0f ? 17u : 23u) : 0u;
        for (;;) {
            MM_LANE_STAT(kLpGridIter);
            if (j < jend) {
                do {
                    MM_LANE_STAT(kLpRectTest);
                    grid_rect<kSlow, kFlat, kFlat>(gv, geo, gv.list.at(j), r, best, bk, tie);
                    j += gv.list.kStep;
                    if (kStats) ++tests;
                } while (j < jend);
            }
            MM_LANE_STAT(kLpCellStep);
            const bool sx = tx <= tz;  // (x before z on equal times)
            const float te = sx ? tx : tz;  // (a select: fminf of selected values costs two canonicalising maxes)
            if (!(te <= best) | !(te < tend)) break;
            fbx = sx ? fbx + sgx : fbx;
            fbz = sx ? fbz : fbz + sgz;
            tx = sx ? __builtin_fmaf(fbx, Bx, Ax) : tx;
            tz = sx ? tz : __builtin_fmaf(fbz, Bz, Az);
            cp += (uint32_t)(sx ? dcx : dcz);
            cell_pos(sx ? shx : shz);
            if (kStats) ++cells;
        }
    } else {
        // Per cell: test the rects of its list, then step to the next cell (or
        // stop).  (The compiler nests the tests in a per-cell loop either way;
        // written as a do-while under one entry check, the loop carries one
        // compare per test instead of a header and a latch compare.)
        for (;;) {
            MM_LANE_STAT(kLpGridIter);
            if (j < jend) {
                do {
                    MM_LANE_STAT(kLpRectTest);
                    grid_rect<kSlow, kFlat, kFlat>(gv, geo, gv.list.at(j), r, best, bk, tie);
                    j += gv.list.kStep;
                    if (kStats) ++tests;
                } while (j < jend);
            }
            {
                MM_LANE_STAT(kLpCellStep);
                const float te = fminf(tx, fminf(ty, tz));
                if (best < te) break;
                // step the axis whose boundary comes first (x before y before z on
                // equal times) -- in selects: three exec-mask branches here cost
                // more SALU and SGPR spills than the selects cost VALU
                const bool sx = tx == te, sy = !sx && ty == te, sz = !sx && !sy;
                bx += sx ? (r.y.x > 0.0f ? 1 : -1) : 0;
                by += sy ? (r.y.y > 0.0f ? 1 : -1) : 0;
                bz += sz ? (r.y.z > 0.0f ? 1 : -1) : 0;
                if (((uint32_t)bx > (uint32_t)g.n[0]) | ((uint32_t)by > (uint32_t)g.n[1]) |
                    ((uint32_t)bz > (uint32_t)g.n[2]))
                    break;
                // grid_time of the stepped axis, the same operations on selected operands
                // (by-value selects: a select of two loads becomes a load of a
                // selected address -- of the kernel argument or a scratch copy)
                const int b = sx ? bx : (sy ? by : bz);
                const float nt = __builtin_fmaf((float)b, sel_xy(sx, sy, F3{Bx, By, Bz}),
                                                sel_xy(sx, sy, F3{Ax, Ay, Az}));
                tx = sx ? nt : tx;
                ty = sy ? nt : ty;
                tz = sz ? nt : tz;
                cp += (uint32_t)(sx ? dcx : (sy ? dcy : dcz));
                cell_pos((fsh >> (sx ? 0u : (sy ? 8u : 16u))) & 0xFFu);
                if (kStats) ++cells;
            }
        }
    }
    if (kStats) {
        c.visits += cells;
        c.rtests += tests;
    }
    if (best == kBig) {  // A is empty: the reference finds nothing either
        t = kBig;
        return !tie;
    }
    if (tie) return false;
    MM_LANE_STAT(kLpCert);
    // certificate: R*'s reference leaf box passes at every t > best
    // (compact grids: the box of rect k = e / 8 at byte 24 k = 3 e, two pairable adds)
    const float2* bp = kFlat ? reinterpret_cast<const float2*>(reinterpret_cast<const char*>(gv.box) + (bk + twice(bk)))
                             : gv.box + 3 * bk;
    bk = rect_index<kFlat>(bk);
    const float2 bxx = bp[0], byy = bp[1], bzz = bp[2];
    const float tx1 = qdiv(bxx.x - r.o.x, r.d.x, r.y.x), tx2 = qdiv(bxx.y - r.o.x, r.d.x, r.y.x);
    float tmin = fminf(tx1, tx2), tmax = fmaxf(tx1, tx2);
    const float ty1 = qdiv(byy.x - r.o.y, r.d.y, r.y.y), ty2 = qdiv(byy.y - r.o.y, r.d.y, r.y.y);
    tmin = fmaxf(tmin, fminf(ty1, ty2));
    tmax = fminf(tmax, fmaxf(ty1, ty2));
    const float tz1 = qdiv(bzz.x - r.o.z, r.d.z, r.y.z), tz2 = qdiv(bzz.y - r.o.z, r.d.z, r.y.z);
    tmin = fmaxf(tmin, fminf(tz1, tz2));
    tmax = fminf(tmax, fmaxf(tz1, tz2));
    if (!(tmax >= tmin && tmax > 0.0f && tmin <= best)) return false;
    t = best;
    index = bk;
    return true;
}

}  // namespace mm
