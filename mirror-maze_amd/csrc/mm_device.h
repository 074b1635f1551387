// mm_device.h — device-side data layout and IEEE-exact helpers shared by the
// mirror-maze HIP kernels.  Compiled only by hipcc for gfx950, with
// -ffp-contract=off: every + - * rounds separately and / and sqrtf are the
// correctly rounded expansions (hipcc's default
// -fhip-fp32-correctly-rounded-divide-sqrt), so the device arithmetic is the
// reference kernel's AIR arithmetic with IEEE intrinsics.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mm_types.h"

namespace mm {

constexpr float kBig = 1e30f;     // shaders.metal:15, 94, 149 (IR 0x46293E5940000000)
constexpr int kStackMax = 50;     // shaders.metal:123

// Diagnostics build (-DMM_LANE_STATS, scripts/lane_probe.py): per phase of the
// bounce loop, the wave-iterations that run it and the lanes active in them,
// counted in block-local LDS words and added to the wave-timeline buffer at
// exit.  Not a product build: the counting perturbs the timing.
enum LanePhase : int {
    kLpChunk, kLpBounce, kLpGlobal, kLpGridIter, kLpRectTest, kLpCellStep, kLpCert, kLpFallback,
    kLpShade, kLpDiffuse, kLpTrial, kLpMirror, kLpCount
};
constexpr uint32_t kLaneStatRecord = 49152;  // wave-timeline record (4 x u64) where the totals start
#ifdef MM_LANE_STATS
__device__ __forceinline__ uint32_t* lane_stat_words() {
    __shared__ uint32_t words[2 * kLpCount];
    return words;
}
__device__ __forceinline__ void lane_stat(int ph) {
    const uint64_t m = __ballot(1);
    if (__lane_id() == (uint32_t)(__ffsll((unsigned long long)m) - 1)) {
        atomicAdd(lane_stat_words() + 2 * ph, 1u);
        atomicAdd(lane_stat_words() + 2 * ph + 1, (uint32_t)__popcll(m));
    }
}
#define MM_LANE_STAT(ph) ::mm::lane_stat(::mm::ph)
#else
#define MM_LANE_STAT(ph) ((void)0)
#endif

// Closest-hit query methods of the wave-persistent kernel (MM_OPT_TRAVERSAL):
// BVH loop forms (mm_trace.h) and the certified grid search (mm_grid.h).
// kFormGridSlow (internal): the grid search on a scene with SLOW rect records.
// kFormGridWide / kFormGridWideSlow (internal): the same on a grid with 64-bit
// cell words (per-face list ranges; grid_build.cpp).
// kFormGridFlat (internal, + kFormGrid..kFormGridWideSlow): the same on a grid
// with one cell along y (the walk steps x / z only; mm_grid.h kFlat).
enum : int {
    kFormIfIf = 0, kFormLeafInterior = 5, kFormLean = 7,
    kFormGrid = 11, kFormGridSlow = 12, kFormGridWide = 13, kFormGridWideSlow = 14,
    kFormGridFlat = 4  // offset: 15..18
};
__host__ __device__ constexpr bool grid_form(int f) { return f >= kFormGrid && f <= kFormGridWideSlow + kFormGridFlat; }
__host__ __device__ constexpr bool grid_flat(int f) { return f > kFormGridWideSlow; }
__host__ __device__ constexpr int grid_base(int f) { return grid_flat(f) ? f - kFormGridFlat : f; }
__host__ __device__ constexpr bool grid_slow(int f) { return grid_base(f) == kFormGridSlow || grid_base(f) == kFormGridWideSlow; }
__host__ __device__ constexpr bool grid_wide(int f) { return grid_base(f) >= kFormGridWide; }

// ---- HBM layouts ------------------------------------------------------------
// Reference node (nodes_ref): 2 x float4 = the reference's 32-B bvh_node,
//   a = (mn.x, mn.y, mn.z, mx.x)   b = (mx.y, mx.z, bits(left_first), bits(count))
// Production node (nodes): a = (mn.x, mx.x, mn.y, mx.y),
//   b = (mn.z, mx.z, bits(count<<24 | left_first), 0): bounds as per-axis
//   (min, max) pairs for packed math.
// Children of an interior node are adjacent (left_first, left_first+1), so the
// pair a traversal step reads is one contiguous 64-B line.
//
// Rect geometry: 4 x float4 per rect (64 B):
//   g0 = (o.xyz, |v|)  g1 = (n.xyz, |u|)  g2 = (v.xyz, 1/|v|)  g3 = (u.xyz, 1/|u|)
// n, |v|, |u| are the per-rect subexpressions of ray_rect_intersect
// (shaders.metal:52,60,61), computed once by k_prep_rects with the same ops.
// Shade record: s0 = (color.rgb, is_mirror), s1 = emission (rgba).
// Uniform grid of the certified search (mm_grid.h, built by grid_build.cpp).
// The device image is one buffer: [cells: n_cells u64][list: u16, padded to
// 16 B][recs: 2 x uint4 per rect][box: 3 x float2 per rect]; the byte
// offsets of the sections let a kernel stage it in LDS (all of it, records
// first, or the cells + lists prefix).
struct DevGrid {
    float mn[3], mx[3];        // grid box (scene bounds widened by eps)
    float cell[3], inv[3];     // cell size per axis and its reciprocal
    int n[3];                  // cells per axis
    uint32_t n_glob;           // rects every query tests (cover > half the cells)
    uint32_t glob[4];
    const void* cells;         // per cell: list base, count (and per-face ranges when wide; mm_grid.h)
    const uint16_t* list;      // rect indices
    const uint4* recs;         // per-rect grid records (grid_build.cpp; mm_grid.h: grid_rect)
    const float2* box;         // per rect: its reference leaf's box, (mn, mx) per axis
    const uint4* image;        // the whole image (16-B units)
    uint32_t off_list, off_recs, off_box, bytes;  // section offsets in bytes
    // Compact records (maze grids, grid_build.cpp): 16 B per rect -- o_k, o_v,
    // o_u, meta = class << 4 (bits 4-9: the class's byte offset into the
    // class table) | axis << 20 | kind << 30 -- and the folded thresholds of
    // each class (Yv_lo, Yv_hi, Yu_lo, Yu_hi) in a table after the records.
    const float4* cls;
    uint32_t off_class;        // 0: 32-B records (no class table)
    uint32_t off_data;         // the data after the index: off_class (compact records), else off_recs
    // glob[0], glob[1] are y-normal FAST records in the planes y = slab_y[0] < slab_y[1] (grid_build.cpp)
    uint32_t slab;
    float slab_y[2];
    // n[a] - 1, a kernel argument of its own: the kernel reloads it where the
    // walk clamps a cell index instead of keeping a computed n - 1 live (the
    // compiler spills those to VGPR lanes: a single-slot v_readlane per use)
    int nm1[3];
    float nf[3];               // n[a] as a float (the maze forms' end time: a kernel argument, not a hoisted convert)
};

struct DevScene {
    const float4* nodes;      // 2 * n_nodes, production layout
    const float4* nodes_ref;  // 2 * n_nodes_ref, reference layout
    const float4* geo;        // 4 * n_rects
    const float4* shade;      // 2 * n_rects
    const uint32_t* idx;      // n_rects
    uint32_t n_nodes;         // production array length in nodes (breadth-first pairs)
    uint32_t n_rects;
    uint32_t root_packed;     // count<<24 | left_first of node 0
    uint32_t fast_ok;         // scene coordinates inside the Markstein guard
    const uint2* recs;        // 5 x uint2 per BVH slot: compact rect records (rect_compact.cpp)
    DevGrid grid;
};

// ---- IEEE helpers (the AIR intrinsics with their IEEE meaning) -------------
struct F3 { float x, y, z; };
__device__ __forceinline__ F3 f3(float x, float y, float z) { return F3{x, y, z}; }
__device__ __forceinline__ F3 operator+(F3 a, F3 b) { return F3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ F3 operator-(F3 a, F3 b) { return F3{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ F3 operator*(F3 a, F3 b) { return F3{a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ F3 operator*(float s, F3 a) { return F3{s * a.x, s * a.y, s * a.z}; }
// air.dot.v3f32 = (x*x' + y*y') + z*z'
__device__ __forceinline__ float dot3(F3 a, F3 b) {
    float s = a.x * b.x;
    s = s + a.y * b.y;
    return s + a.z * b.z;
}
// air.fast_rsqrt.f32 -> correctly rounded sqrt, then correctly rounded 1/x.
// For x in [2^-40, 2^40] (every normalisation on the path: |x|^2 of a unit-ish
// vector) the same two roundings come from the hardware sqrt / rcp with exact
// corrections: the sqrt is LLVM's own correctly rounded expansion without the
// denormal scaling and the zero / inf class fix-up (x is normal and finite),
// the reciprocal one fma Newton step on v_rcp_f32; bit-identical to
// 1.0f / sqrtf(x) for every x in the range (exhaustive GPU check,
// scripts/verify_fast_rsq.hip, tests/test_gpu_arith.py).  Other x take the
// IEEE expansion.
__device__ __forceinline__ float rsq_ieee(float x) { return 1.0f / sqrtf(x); }
__device__ __forceinline__ float rsq(float x) {
    if (x >= 0x1p-40f && x <= 0x1p40f) {
        float s = __builtin_amdgcn_sqrtf(x);
        const float sd = __uint_as_float(__float_as_uint(s) - 1u), su = __uint_as_float(__float_as_uint(s) + 1u);
        const float vd = __builtin_fmaf(-sd, s, x), vu = __builtin_fmaf(-su, s, x);
        s = vd <= 0.0f ? sd : s;
        s = vu > 0.0f ? su : s;
        const float y = __builtin_amdgcn_rcpf(s);
        const float e = __builtin_fmaf(-s, y, 1.0f);
        return __builtin_fmaf(e, y, y);
    }
    return rsq_ieee(x);
}
__device__ __forceinline__ F3 normalize3(F3 v) { return rsq(dot3(v, v)) * v; }
// cross(v, u) in the IR's operand order (ray_rect_intersect %22-%32)
__device__ __forceinline__ F3 cross3(F3 v, F3 u) {
    return F3{u.z * v.y - u.y * v.z, u.x * v.z - u.z * v.x, u.y * v.x - u.x * v.y};
}
__device__ __forceinline__ F3 xyz(float4 a) { return F3{a.x, a.y, a.z}; }

// (random(state) - 0.5) * 2, shaders.metal:181-186 as folded by the IR
// (%163-%174): u32 -> f32 (round to nearest) * 2^-31 - 1.
__device__ __forceinline__ float rand_pm1(uint32_t& state) {
    uint32_t s = state * 747796405u + 291336453u;
    state = s;
    uint32_t r = ((s >> ((s >> 28) + 4u)) ^ s) * 277803737u;
    r = (r >> 22) ^ r;
    // RN(RN(float(r) * 2^-31) - 1): the product is exact (a power-of-two
    // scaling of a float in [1, 2^32]), so one fma rounds the same once
    return __builtin_fmaf((float)r, 0x1p-31f, -1.0f);
}

// air.convert.u.i32.f.f32: truncation, saturating, NaN -> 0
__device__ __forceinline__ uint32_t cvt_u32_sat(float f) {
    if (!(f > 0.0f)) return 0u;
    if (f >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)f;
}

// Seed, shaders.metal:288-298 (IR %143-%161).  The sampler (repeat,
// nearest, normalized) reads texel (0,0) of noiseTexture-2.png for every
// integer gid: (128,128,128,255)/255.
__device__ __forceinline__ uint32_t seed_reference(uint32_t tx, uint32_t ty, uint32_t time) {
    const float n = 128.0f / 255.0f;
    float s = n + (float)(tx * 15823u);
    s = s + n;
    s = s + (float)(ty * 9737333u);
    s = s + (float)time;
    return cvt_u32_sat(s);
}

__device__ __forceinline__ uint32_t pcg_hash(uint32_t v) {
    uint32_t s = v * 747796405u + 2891336453u;
    uint32_t w = ((s >> ((s >> 28) + 4u)) ^ s) * 277803737u;
    return (w >> 22) ^ w;
}
// Throughput-mode seed: a function of (pixel, sample, frame) only.
__device__ __forceinline__ uint32_t seed_tile(uint32_t pixel, uint32_t sample, uint32_t frame) {
    return pcg_hash(pcg_hash(pcg_hash(frame) ^ pixel) + sample);
}

// Primary ray direction, shaders.metal:281-284 in IR order (camera centre
// cancels; quat_mult inlined as %97-%140, %190-%191).
__device__ __forceinline__ F3 primary_dir(const mm_uniform& u, uint32_t px, uint32_t py) {
    const float fx = (float)px, fy = (float)py;
    const float vx = u.cam.viewport[0], vy = u.cam.viewport[1];
    F3 p = F3{(vx * fx) / u.view_w - vx * 0.5f, (vy * fy) / u.view_h - vy * 0.5f, 0.0f - (-u.cam.focal)};
    F3 d = normalize3(p);
    const F3 q = F3{u.cam.quat[0], u.cam.quat[1], u.cam.quat[2]};
    const float qw = u.cam.quat[3];
    const F3 nq = F3{-q.x, -q.y, -q.z};
    const float s1 = -dot3(nq, d);
    const F3 c1 = F3{nq.y * d.z - nq.z * d.y, nq.z * d.x - nq.x * d.z, nq.x * d.y - nq.y * d.x};
    const F3 v1 = c1 + qw * d;
    const F3 c2 = F3{v1.y * q.z - v1.z * q.y, v1.z * q.x - v1.x * q.z, v1.x * q.y - v1.y * q.x};
    return (qw * v1 + s1 * q) + c2;
}

// beam.dir = ray_dir + (rand, rand, 0) * 0.001 (shaders.metal:303, IR %189-%192)
__device__ __forceinline__ F3 jitter(F3 d, uint32_t& seed) {
    const float j1 = rand_pm1(seed);
    const float j2 = rand_pm1(seed);
    return d + F3{j1 * 0.001f, j2 * 0.001f, 0.0f * 0.001f};
}

// Metal sign(): 1, -1, +-0 for +-0, 0 for NaN
__device__ __forceinline__ float msign(float x) {
    if (x > 0.0f) return 1.0f;
    if (x < 0.0f) return -1.0f;
    if (x != x) return 0.0f;
    return x;
}

// RGBA8Unorm store conversion: round-to-nearest-even of clamp(x,0,1)*255.
__device__ __forceinline__ uint32_t unorm8(float x) {
    x = fminf(fmaxf(x, 0.0f), 1.0f);
    return (uint32_t)rintf(x * 255.0f);
}

}  // namespace mm
