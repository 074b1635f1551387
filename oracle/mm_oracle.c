/*
 * mm_oracle.c — TEST INFRASTRUCTURE ONLY (see mm_oracle.h).
 *
 * CPU restatement of the reference kernel src/shaders.metal:245-368 and its
 * helpers, one operation per IR instruction of src/shaders.ir (disassembled
 * text; "IR %n" below names the SSA value).  Build with -O2
 * -ffp-contract=off and without fast-math: every + - * / sqrt rounds to
 * binary32 exactly where the IR rounds.  Parity status: UNPINNED against an
 * executed reference (no Metal / Rust toolchain here); pinned pieces: the
 * noise texel and the RNG (tests/golden).
 */
#include "mm_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <xmmintrin.h>

/* ---- floating-point environment (TEST INFRASTRUCTURE) -----------------------
 * The reference AIR is compiled with `air.compile.denorms_disable`
 * (src/shaders.ir metadata !47): denormal operands read as zero and denormal
 * results flush to zero.  The oracle runs IEEE binary32 (denormals kept) by
 * default, like the HIP kernels; oracle_set_fp_mode(1) runs every entry point
 * with MXCSR FTZ|DAZ (the reference's semantics) instead.  Every entry point
 * also ORs the MXCSR sticky exception flags it raised (bit 1 DE: a denormal
 * operand; bit 4 UE: a tiny inexact result) into oracle_fp_flags(), so a run
 * shows whether any denormal arose at all. */
static int g_fp_ftz = 0;
static unsigned g_fp_flags = 0;
void oracle_set_fp_mode(int ftz_daz) { g_fp_ftz = ftz_daz != 0; }
unsigned oracle_fp_flags(int reset) {
    unsigned f = __atomic_load_n(&g_fp_flags, __ATOMIC_RELAXED);
    if (reset) __atomic_store_n(&g_fp_flags, 0u, __ATOMIC_RELAXED);
    return f;
}
static unsigned fp_enter(void) {
    const unsigned saved = _mm_getcsr();
    unsigned csr = saved & ~0x3Fu;                  /* clear the sticky flags */
    if (g_fp_ftz) csr |= (1u << 15) | (1u << 6);    /* FTZ | DAZ */
    else csr &= ~((1u << 15) | (1u << 6));
    _mm_setcsr(csr);
    return saved;
}
static void fp_leave(unsigned saved) {
    __atomic_fetch_or(&g_fp_flags, _mm_getcsr() & 0x3Fu, __ATOMIC_RELAXED);
    _mm_setcsr(saved);
}

#define BIG 1e30f          /* IR 0x46293E5940000000 */
#define STACK_MAX 50       /* shaders.metal:123 */

typedef struct { float x, y, z; } v3;

static inline v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }
static inline v3 vadd(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vmul(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 vscale(float s, v3 a) { return mk(s * a.x, s * a.y, s * a.z); }
/* air.dot.v3f32 */
static inline float dot3(v3 a, v3 b) {
    float s = a.x * b.x;
    s = s + a.y * b.y;
    return s + a.z * b.z;
}
/* air.fast_rsqrt.f32 given its IEEE meaning */
static inline float rsq(float x) { return 1.0f / sqrtf(x); }
/* normalize(v) = v * rsqrt(dot(v, v)) */
static inline v3 normalize3(v3 v) { return vscale(rsq(dot3(v, v)), v); }
/* cross(v, u) as the IR spells it (ray_rect_intersect %22-%32) */
static inline v3 cross3(v3 v, v3 u) {
    return mk(u.z * v.y - u.y * v.z, u.x * v.z - u.z * v.x, u.y * v.x - u.x * v.y);
}

/* random(), shaders.metal:181-186; the kernel only ever uses
 * (random(state) - 0.5) * 2.0, which the IR folds to u32->f32 * 2^-31 - 1
 * (IR %172-%174). */
float oracle_rand_pm1(uint32_t* state) {
    uint32_t s = *state * 747796405u + 291336453u;
    *state = s;
    uint32_t r = ((s >> ((s >> 28) + 4u)) ^ s) * 277803737u;
    r = (r >> 22) ^ r;
    return (float)r * 0x1p-31f - 1.0f;
}

/* air.convert.u.i32.f.f32: truncate, saturate, NaN -> 0 */
static inline uint32_t cvt_u32_sat(float f) {
    if (!(f > 0.0f)) return 0u;
    if (f >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)f;
}

/* seed, shaders.metal:288-298; IR %143-%161.  The noise sample is texel
 * (0,0) for every thread = (128,128,128,255)/255 (tests/golden). */
uint32_t oracle_seed_reference(uint32_t tx, uint32_t ty, uint32_t time) {
    const float n = 128.0f / 255.0f;
    float s = n + (float)(tx * 15823u);    /* %157 = noise.y + f(x*15823) */
    s = s + n;                             /* %158 += noise.x             */
    s = s + (float)(ty * 9737333u);        /* %159                        */
    s = s + (float)time;                   /* %160                        */
    return cvt_u32_sat(s);
}

static inline uint32_t pcg_hash(uint32_t v) {
    uint32_t s = v * 747796405u + 2891336453u;
    uint32_t w = ((s >> ((s >> 28) + 4u)) ^ s) * 277803737u;
    return (w >> 22) ^ w;
}

/* Throughput-mode seed: keyed on (pixel, sample, frame) only, so the image is
 * independent of tiling and device count. */
uint32_t oracle_tile_seed(uint32_t pixel, uint32_t sample, uint32_t frame) {
    return pcg_hash(pcg_hash(pcg_hash(frame) ^ pixel) + sample);
}

/* Primary ray direction before jitter, shaders.metal:281-284 in IR order
 * (%50-%85 then the inlined quat_mult %97-%140, %190-%191).  The camera
 * centre cancels out of (corner + offset) - centre in the IR. */
static v3 primary_dir(const mm_uniform* u, uint32_t px, uint32_t py) {
    const mm_camera* c = &u->cam;
    float fx = (float)px, fy = (float)py;
    v3 p = mk((c->viewport[0] * fx) / u->view_w - c->viewport[0] * 0.5f,
              (c->viewport[1] * fy) / u->view_h - c->viewport[1] * 0.5f,
              0.0f - (-c->focal));
    v3 d = normalize3(p);                                   /* %85 */
    v3 q = mk(c->quat[0], c->quat[1], c->quat[2]);
    float qw = c->quat[3];
    v3 nq = mk(-q.x, -q.y, -q.z);                           /* %97 */
    float s1 = -dot3(nq, d);                                /* %99 */
    v3 c1 = mk(nq.y * d.z - nq.z * d.y, nq.z * d.x - nq.x * d.z, nq.x * d.y - nq.y * d.x);
    v3 v1 = vadd(c1, vscale(qw, d));                        /* %121 */
    v3 c2 = mk(v1.y * q.z - v1.z * q.y, v1.z * q.x - v1.x * q.z, v1.x * q.y - v1.y * q.x);
    v3 t1 = vscale(s1, q);                                  /* %139 */
    v3 t2 = vscale(qw, v1);                                 /* %140 */
    return vadd(vadd(t2, t1), c2);                          /* %190, %191 */
}

void oracle_primary_dir(const mm_uniform* u, uint32_t px, uint32_t py, float dir[3]) {
    v3 d = primary_dir(u, px, py);
    dir[0] = d.x; dir[1] = d.y; dir[2] = d.z;
}

typedef struct { v3 ori, dir; float t; uint32_t index; } ray_t;
typedef struct { uint64_t node_visits, rect_tests; int overflow; } trav_t;

/* ray_rect_intersect, shaders.metal:51-67; IR lines of @_Z18ray_rect_intersect */
static inline void ray_rect(ray_t* b, const mm_rect* r, uint32_t index) {
    v3 o = ld3(r->o), v = ld3(r->v), u = ld3(r->u);
    v3 n = normalize3(cross3(v, u));                        /* %38 */
    float nc = dot3(b->dir, n);                             /* %41 */
    float a = dot3(vsub(o, b->ori), n) / nc;                /* %49 */
    v3 rv = vadd(vsub(b->ori, o), vscale(a, b->dir));       /* %54 */
    float lv = sqrtf(dot3(v, v));                           /* %57 */
    float d1 = dot3(rv, v) / lv;                            /* %58 */
    float lu = sqrtf(dot3(u, u));                           /* %61 */
    float d2 = dot3(rv, u) / lu;                            /* %62 */
    if (d1 >= 0.0f && d1 <= lv && d2 >= 0.0f && d2 <= lu && nc != 0.0f && a > 0.1f && a < b->t) {
        b->t = a;
        b->index = index;
    }
}

/* intersect_aabb, shaders.metal:87-95 */
static inline float aabb(const ray_t* b, const float* mn, const float* mx) {
    float tx1 = (mn[0] - b->ori.x) / b->dir.x, tx2 = (mx[0] - b->ori.x) / b->dir.x;
    float tmin = fminf(tx1, tx2), tmax = fmaxf(tx1, tx2);
    float ty1 = (mn[1] - b->ori.y) / b->dir.y, ty2 = (mx[1] - b->ori.y) / b->dir.y;
    tmin = fmaxf(tmin, fminf(ty1, ty2));
    tmax = fminf(tmax, fmaxf(ty1, ty2));
    float tz1 = (mn[2] - b->ori.z) / b->dir.z, tz2 = (mx[2] - b->ori.z) / b->dir.z;
    tmin = fmaxf(tmin, fminf(tz1, tz2));
    tmax = fminf(tmax, fmaxf(tz1, tz2));
    if (tmax >= tmin && tmin < b->t && tmax > 0.0f) return tmin;
    return BIG;
}

float oracle_intersect_aabb(const float ori[3], const float dir[3], float t,
                            const float mn[3], const float mx[3]) {
    ray_t b;
    b.ori = ld3(ori); b.dir = ld3(dir); b.t = t; b.index = 0;
    return aabb(&b, mn, mx);
}

/* intersect_bvh_iterative, shaders.metal:115-156: near child first, far child
 * pushed when hit, no re-test on pop, root box never tested. */
static void intersect_bvh(ray_t* b, const oracle_scene* sc, trav_t* tr) {
    uint32_t stack[STACK_MAX];
    uint32_t head = 0, node = 0;
    for (;;) {
        const mm_node* nd = &sc->nodes[node];
        if (nd->count > 0) {
            for (uint32_t i = 0; i < nd->count; ++i) {
                uint32_t k = sc->idx[nd->left_first + i];
                ray_rect(b, &sc->rects[k], k);
            }
            tr->rect_tests += nd->count;
            if (head == 0) break;
            node = stack[--head];
            continue;
        }
        tr->node_visits++;
        uint32_t l = nd->left_first, r = nd->left_first + 1;
        float d1 = aabb(b, sc->nodes[l].mn, sc->nodes[l].mx);
        float d2 = aabb(b, sc->nodes[r].mn, sc->nodes[r].mx);
        if (d1 > d2) {
            float t = d1; d1 = d2; d2 = t;
            uint32_t x = l; l = r; r = x;
        }
        if (d1 == BIG) {
            if (head == 0) break;
            node = stack[--head];
        } else {
            node = l;
            if (d2 != BIG) {
                if (head >= STACK_MAX) { tr->overflow = 1; return; }
                stack[head++] = r;
            }
        }
    }
}

/* The closest-hit query of the path loop: the reference walk, or -- in
 * grid_cpu.c's build (the bench's same-algorithm CPU baseline, not a checker)
 * -- the product's certified grid search with this walk as its fallback. */
#ifdef ORACLE_QUERY_FN
static void ORACLE_QUERY_FN(ray_t* b, const oracle_scene* sc, trav_t* tr);
#else
#define ORACLE_QUERY_FN intersect_bvh
#endif

/* Metal sign(): 1, -1, +-0 for +-0, 0 for NaN */
static inline float msign(float x) {
    if (x > 0.0f) return 1.0f;
    if (x < 0.0f) return -1.0f;
    if (x != x) return 0.0f;
    return x;
}

/* The bounce loop, shaders.metal:302-340 in IR order (%199-%415).
 * Returns sqrt(max(L,0)) per channel (shaders.metal:344). */
static v3 trace_path(const oracle_scene* sc, v3 ori, v3 dir, uint32_t seed,
                     int bounce_limit, int mirror_limit, uint64_t* rays, trav_t* tr) {
    ray_t b;
    b.ori = ori; b.dir = dir; b.t = BIG; b.index = 0;
    v3 T = mk(1.0f, 1.0f, 1.0f), L = mk(0.0f, 0.0f, 0.0f);
    int mh = 0;
    for (int n = 0; n < bounce_limit + mh; ++n) {
        ORACLE_QUERY_FN(&b, sc, tr);
        (*rays)++;
        if (tr->overflow) break;
        if (!(b.t < BIG)) break;                               /* miss: shaders.metal:336-338 */
        const uint32_t k = b.index;
        const mm_rect* r = &sc->rects[k];
        v3 nn = normalize3(cross3(ld3(r->v), ld3(r->u)));      /* %238 */
        float sg = msign(dot3(b.dir, nn));                     /* %241 */
        float side = -sg;
        if (sc->is_mirror[k] == 0 || sg == 1.0f) {             /* matte, or mirror seen from behind */
            const float* e = &sc->emission[4 * k];
            v3 contrib = vmul(vscale(e[3], T), ld3(e));        /* %253, %254 */
            v3 newT = vmul(ld3(r->color), T);                  /* %264 */
            float rx = oracle_rand_pm1(&seed), ry = oracle_rand_pm1(&seed), rz = oracle_rand_pm1(&seed);
            v3 rd = mk(rx, ry, rz);
            float len2 = dot3(rd, rd);
            while (sqrtf(len2) > 1.0f) {                       /* %306 / %350 */
                rx = oracle_rand_pm1(&seed); ry = oracle_rand_pm1(&seed); rz = oracle_rand_pm1(&seed);
                rd = mk(rx, ry, rz);
                len2 = dot3(rd, rd);
            }
            v3 rn = vscale(rsq(len2), rd);                     /* %358 */
            b.ori = vadd(b.ori, vscale(b.t, b.dir));           /* %363 */
            v3 nd = vadd(rn, vscale(side, nn));                /* %367 */
            b.dir = vscale(rsq(dot3(nd, nd)), nd);             /* %372 */
            L = vadd(contrib, L);                              /* %409 */
            T = newT;
        } else {
            if (mh + 1 < mirror_limit) {                       /* %375: mh < 14 */
                v3 contrib = vscale(0.005f, ld3(r->color));    /* %386 */
                b.ori = vadd(b.ori, vscale(b.t, b.dir));       /* %391 */
                float dd = dot3(nn, b.dir) * 2.0f;             /* %392-%393 */
                v3 rf = vsub(b.dir, vscale(dd, nn));           /* %397 reflect */
                b.dir = vscale(rsq(dot3(rf, rf)), rf);         /* %402 */
                L = vadd(contrib, L);
                mh = mh + 1;
            } else {
                break;
            }
        }
        b.t = BIG;
    }
    return mk(sqrtf(fmaxf(L.x, 0.0f)), sqrtf(fmaxf(L.y, 0.0f)), sqrtf(fmaxf(L.z, 0.0f)));
}

static v3 jittered_dir(v3 d, uint32_t* seed) {
    float j1 = oracle_rand_pm1(seed);
    float j2 = oracle_rand_pm1(seed);
    v3 j = mk(j1 * 0.001f, j2 * 0.001f, 0.0f * 0.001f);     /* %189 */
    return vadd(d, j);                                        /* %192 */
}

static int oracle_trace_path_body(const oracle_scene* sc, const float ori[3], const float dir[3],
                      uint32_t seed, int bounce_limit, int mirror_limit,
                      float rgb_out[3], uint32_t* rays) {
    uint64_t nr = 0;
    trav_t tr = {0, 0, 0};
    v3 s = trace_path(sc, ld3(ori), ld3(dir), seed, bounce_limit, mirror_limit, &nr, &tr);
    rgb_out[0] = s.x; rgb_out[1] = s.y; rgb_out[2] = s.z;
    if (rays) *rays = (uint32_t)nr;
    return tr.overflow ? MM_ERR_STACK : MM_OK;
}

int oracle_trace_path(const oracle_scene* sc, const float ori[3], const float dir[3],
                      uint32_t seed, int bounce_limit, int mirror_limit,
                      float rgb_out[3], uint32_t* rays) {
    const unsigned saved = fp_enter();
    const int rc = oracle_trace_path_body(sc, ori, dir, seed, bounce_limit, mirror_limit, rgb_out, rays);
    fp_leave(saved);
    return rc;
}


static void add_stats(mm_stats* st, uint64_t rays, const trav_t* tr, uint64_t paths) {
    if (!st) return;
    st->rays += rays;
    st->node_visits += tr->node_visits;
    st->rect_tests += tr->rect_tests;
    st->paths += paths;
}

/* One threadgroup of compute_shader.  Threads run one at a time; the
 * threadgroup barriers of the reduction become phase boundaries. */
static int run_group(const oracle_scene* sc, const mm_uniform* u, const uint32_t* chunks,
                     uint32_t n_chunks, uint32_t tg_w, uint32_t tg_h, uint32_t gx, uint32_t gy,
                     float* fb, mm_stats* st, v3* test) {
    const uint32_t W = (uint32_t)u->view_w, H = (uint32_t)u->view_h;
    const uint32_t chunk = u->chunk_w, ppc = chunk * chunk;
    /* pixel_buffer_index, shaders.metal:266; IR %26-%31 in float */
    float pbf = ((u->view_w * 0.5f) * (float)gy) / (float)ppc + (float)gx;
    uint32_t pbi = cvt_u32_sat(pbf);
    if (pbi >= n_chunks) return MM_ERR_INVALID;
    const uint32_t cx = chunks[2 * pbi], cy = chunks[2 * pbi + 1];
    const uint32_t total = tg_w * tg_h, max_index = total / ppc;
    uint64_t rays = 0;
    trav_t tr = {0, 0, 0};
    for (uint32_t ly = 0; ly < tg_h; ++ly)
        for (uint32_t lx = 0; lx < tg_w; ++lx) {
            uint32_t flat = lx + tg_w * ly;
            uint32_t pn = flat / max_index;
            uint32_t px = cx + pn / chunk, py = cy + pn % chunk;
            uint32_t seed = oracle_seed_reference(gx * tg_w + lx, gy * tg_h + ly, u->time);
            v3 d = jittered_dir(primary_dir(u, px, py), &seed);
            v3 ori = ld3(u->cam.center);
            test[flat] = trace_path(sc, ori, d, seed, 5, 15, &rays, &tr);  /* shaders.metal:294-295 */
            if (tr.overflow) return MM_ERR_STACK;
        }
    /* tree reduction, shaders.metal:345-358 */
    for (uint32_t f = 0; f < total; f += 2) test[f] = vadd(test[f], test[f + 1]);
    for (uint32_t f = 0; f < total; f += 4) test[f] = vadd(test[f], test[f + 2]);
    for (uint32_t f = 0; f < total; f += 8) test[f] = vadd(test[f], test[f + 4]);
    for (uint32_t pn = 0; pn < total / max_index; ++pn) {
        uint32_t f = pn * max_index;
        v3 acc = test[f];
        if ((int)max_index > 15)
            for (uint32_t i = 1; i < max_index / 8; ++i) acc = vadd(acc, test[f + 8 * i]);
        float m = (float)(int)max_index;
        acc = mk(acc.x / m, acc.y / m, acc.z / m);
        uint32_t px = cx + pn / chunk, py = cy + pn % chunk;
        if (px < W && py < H) {
            float* o = fb + 4 * ((size_t)py * W + px);
            o[0] = acc.x; o[1] = acc.y; o[2] = acc.z; o[3] = 1.0f;
        }
    }
    add_stats(st, rays, &tr, total);
    return MM_OK;
}

static int check_group_shape(const mm_uniform* u, uint32_t tg_w, uint32_t tg_h) {
    const uint32_t ppc = u->chunk_w * u->chunk_w;
    if (ppc == 0 || tg_w == 0 || tg_h == 0) return MM_ERR_INVALID;
    const uint32_t total = tg_w * tg_h;
    if (total % 8 != 0 || total % ppc != 0 || total / ppc == 0 || total > 1024) return MM_ERR_INVALID;
    if (!(u->view_w >= 1.0f) || !(u->view_h >= 1.0f)) return MM_ERR_INVALID;
    return MM_OK;
}

static int oracle_trace_group_body(const oracle_scene* sc, const mm_uniform* u, const uint32_t* chunks,
                       uint32_t n_chunks, uint32_t tg_w, uint32_t tg_h, uint32_t gx, uint32_t gy,
                       float* fb, mm_stats* st) {
    int rc = check_group_shape(u, tg_w, tg_h);
    if (rc) return rc;
    v3 test[1024];
    return run_group(sc, u, chunks, n_chunks, tg_w, tg_h, gx, gy, fb, st, test);
}

int oracle_trace_group(const oracle_scene* sc, const mm_uniform* u, const uint32_t* chunks,
                       uint32_t n_chunks, uint32_t tg_w, uint32_t tg_h, uint32_t gx, uint32_t gy,
                       float* fb, mm_stats* st) {
    const unsigned saved = fp_enter();
    const int rc = oracle_trace_group_body(sc, u, chunks, n_chunks, tg_w, tg_h, gx, gy, fb, st);
    fp_leave(saved);
    return rc;
}


static int oracle_trace_chunks_body(const oracle_scene* sc, const mm_uniform* u, const uint32_t* chunks,
                        uint32_t n_chunks, uint32_t tg_w, uint32_t tg_h, float* fb, mm_stats* st) {
    int rc = check_group_shape(u, tg_w, tg_h);
    if (rc) return rc;
    const uint32_t ppc = u->chunk_w * u->chunk_w;
    /* threadgroups_per_grid, main.rs:646-650 (f32 then truncate) */
    const uint32_t gw = (uint32_t)(u->view_w / 2.0f / (float)ppc);
    const uint32_t gh = (uint32_t)(u->view_h / 2.0f / (float)ppc);
    v3 test[1024];
    for (uint32_t gy = 0; gy < gh; ++gy)
        for (uint32_t gx = 0; gx < gw; ++gx) {
            rc = run_group(sc, u, chunks, n_chunks, tg_w, tg_h, gx, gy, fb, st, test);
            if (rc) return rc;
        }
    return MM_OK;
}

int oracle_trace_chunks(const oracle_scene* sc, const mm_uniform* u, const uint32_t* chunks,
                        uint32_t n_chunks, uint32_t tg_w, uint32_t tg_h, float* fb, mm_stats* st) {
    const unsigned saved = fp_enter();
    const int rc = oracle_trace_chunks_body(sc, u, chunks, n_chunks, tg_w, tg_h, fb, st);
    fp_leave(saved);
    return rc;
}


/* Throughput mode.  Sample reduction: for spp % 8 == 0 the reference's order
 * (pairwise tree in blocks of 8, blocks summed left to right), then / spp;
 * otherwise a left-to-right sum. */
static int oracle_trace_tile_body(const oracle_scene* sc, const mm_uniform* u, const mm_ext* e,
                      uint32_t x0, uint32_t y0, uint32_t w, uint32_t h, uint32_t y_stride,
                      float* out, mm_stats* st) {
    if (!e || e->spp == 0 || e->spp > 4096 || y_stride == 0) return MM_ERR_INVALID;
    const uint32_t W = (uint32_t)u->view_w;
    v3* s = (v3*)malloc(sizeof(v3) * e->spp);
    if (!s) return MM_ERR_NOMEM;
    uint64_t rays = 0;
    trav_t tr = {0, 0, 0};
    for (uint32_t j = 0; j < h; ++j)
        for (uint32_t i = 0; i < w; ++i) {
            const uint32_t px = x0 + i, py = y0 + j * y_stride;
            const uint32_t pixel = py * W + px;
            const v3 d0 = primary_dir(u, px, py);
            for (uint32_t k = 0; k < e->spp; ++k) {
                uint32_t seed = oracle_tile_seed(pixel, k, e->frame);
                v3 d = jittered_dir(d0, &seed);
                s[k] = trace_path(sc, ld3(u->cam.center), d, seed, (int)e->bounce_limit,
                                  (int)e->mirror_limit, &rays, &tr);
                if (tr.overflow) { free(s); return MM_ERR_STACK; }
            }
            v3 acc;
            if (e->spp % 8 == 0) {
                for (uint32_t b = 0; b < e->spp; b += 8) {
                    v3 p0 = vadd(s[b + 0], s[b + 1]), p1 = vadd(s[b + 2], s[b + 3]);
                    v3 p2 = vadd(s[b + 4], s[b + 5]), p3 = vadd(s[b + 6], s[b + 7]);
                    v3 blk = vadd(vadd(p0, p1), vadd(p2, p3));
                    acc = (b == 0) ? blk : vadd(acc, blk);
                }
            } else {
                acc = s[0];
                for (uint32_t k = 1; k < e->spp; ++k) acc = vadd(acc, s[k]);
            }
            const float m = (float)e->spp;
            float* o = out + 4 * ((size_t)j * w + i);
            if (e->flags & MM_EXT_ACCUMULATE) {
                o[0] += acc.x / m; o[1] += acc.y / m; o[2] += acc.z / m; o[3] += 1.0f;
            } else {
                o[0] = acc.x / m; o[1] = acc.y / m; o[2] = acc.z / m; o[3] = 1.0f;
            }
        }
    free(s);
    add_stats(st, rays, &tr, (uint64_t)w * h * e->spp);
    return MM_OK;
}

int oracle_trace_tile(const oracle_scene* sc, const mm_uniform* u, const mm_ext* e,
                      uint32_t x0, uint32_t y0, uint32_t w, uint32_t h, uint32_t y_stride,
                      float* out, mm_stats* st) {
    const unsigned saved = fp_enter();
    const int rc = oracle_trace_tile_body(sc, u, e, x0, y0, w, h, y_stride, out, st);
    fp_leave(saved);
    return rc;
}


/* ---- display stage (TEST INFRASTRUCTURE) -------------------------------------
 * fragment_shader (src/shaders.metal:214-225) as a Jacobi step, in the
 * operation order of the compiled IR (src/shaders.ir, fragment_shader):
 *   s = ((L + R) + D) + U;  s = s * 0.5;  s = s + C;  s = s * RN(1/3)
 * texel reads c/255 (IEEE division), neighbours outside the texture read 0,
 * the write quantises with round-half-even of clamp(x,0,1)*255, alpha 255. */
static inline uint8_t q8(float x) {
    x = fminf(fmaxf(x, 0.0f), 1.0f);
    return (uint8_t)nearbyintf(x * 255.0f);
}

static inline v3 tex_rd(const uint8_t* t, int x, int y, int W, int H) {
    if (x < 0 || y < 0 || x >= W || y >= H) return mk(0.0f, 0.0f, 0.0f);
    const uint8_t* p = t + 4 * ((size_t)y * W + x);
    return mk((float)p[0] / 255.0f, (float)p[1] / 255.0f, (float)p[2] / 255.0f);
}

void oracle_present_blur(const uint8_t* in, uint8_t* out, uint32_t W, uint32_t H) {
    const float third = 0x1.555556p-2f;
    for (int y = 0; y < (int)H; ++y)
        for (int x = 0; x < (int)W; ++x) {
            const v3 c = tex_rd(in, x, y, W, H);
            const v3 r = tex_rd(in, x + 1, y, W, H), l = tex_rd(in, x - 1, y, W, H);
            const v3 d = tex_rd(in, x, y + 1, W, H), u = tex_rd(in, x, y - 1, W, H);
            v3 s = vadd(vadd(vadd(l, r), d), u);
            s = mk(s.x * 0.5f, s.y * 0.5f, s.z * 0.5f);
            s = vadd(s, c);
            s = mk(s.x * third, s.y * third, s.z * third);
            uint8_t* o = out + 4 * ((size_t)y * W + x);
            o[0] = q8(s.x); o[1] = q8(s.y); o[2] = q8(s.z); o[3] = 255;
        }
}

void oracle_quantize(const float* rgba, uint8_t* rgba8, uint64_t n_pixels) {
    for (uint64_t i = 0; i < 4 * n_pixels; ++i) rgba8[i] = q8(rgba[i]);
}
