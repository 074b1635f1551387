/*
 * grid_cpu.c -- CPU BASELINE ONLY (bench.py cpu_baseline, the "same-algorithm"
 * entry).  Not a checker and not part of the product.
 *
 * The product answers each closest-hit query with a certified uniform-grid
 * search and falls back to the reference BVH walk only when the search cannot
 * certify its answer (mirror-maze_amd/csrc/mm_grid.h).  The
 * oracle (mm_oracle.c) walks the BVH on every query -- the reference's
 * algorithm -- so the bench line's GPU / oracle ratio mixes algorithm and
 * hardware.  This file restates the grid search in scalar C inside the
 * oracle's own path loop (mm_oracle.c trace_path, through ORACLE_QUERY_FN), so the
 * same workload can be timed on the CPU with the algorithm held fixed:
 *
 *   grid     the scene box widened by eps = C * 2^-14 (C the largest
 *            |coordinate|), cells of the median rect's smaller extent
 *            (one maze cell), every rect listed in the cells its box comes
 *            within eps of; rects covering more than half the cells are
 *            tested by every query;
 *   query    those, then the cells the ray crosses from the cell of its point
 *            at t = 3/32 (crossing times as one fma, mm_grid.h), every listed
 *            rect tested with the reference's ray_rect_intersect minus its
 *            `a < t` clause, stop once the best a is below the cell's exit;
 *   certify  unique minimum and the reference leaf box of the answer passes
 *            intersect_aabb at every t > a (mm_grid.h's theorem); otherwise,
 *            or for a ray outside the grid / with a tiny direction component,
 *            the reference walk.
 *
 * It returns the reference walk's (t, index) on every query, so its images
 * equal oracle_trace_tile's bit for bit (tests/test_oracle.py).  Plain cell
 * lists (no per-face ranges: those save GPU lanes, not CPU work).  Built into
 * its own library (_build/libmm_gridcpu.so) exporting the oracle's entry
 * points plus gridcpu_build.
 */
#define ORACLE_QUERY_FN grid_query_or_walk
#include "mm_oracle.c"

#include <stdio.h>

typedef struct {
    float gmin[3], gcell[3], ginv[3], eps;
    int gn[3];
    uint32_t *cell_off, *cell_list, *glob, n_glob;
    uint32_t* leaf_of_rect;
    /* per rect: the reference's subexpressions, computed once in its operation order */
    v3 *n, *o, *v, *u;
    float *lv, *lu;
    const oracle_scene* sc;
} gridcpu_t;

static gridcpu_t G;
/* query counts since the last gridcpu_build: grid answers, walk fallbacks (ties, failed
 * certificates, rays outside the guards / grid), and queries for a scene other than the one built -- those
 * walk too, so a run that reports them is not the same-algorithm baseline */
/* Counted per thread (one 64-byte slot each, so the 16 tracing threads do not
 * share a cache line: one shared atomic counter ran the baseline 12x slower)
 * and summed by gridcpu_stats; a slot is claimed on a thread's first query
 * (past GC_SLOTS threads they are shared, hence the atomic adds). */
#define GC_SLOTS 1024
typedef struct {
    uint64_t grid, fallback, other;
    char pad[40];
} gc_slot_t;
static gc_slot_t g_slots[GC_SLOTS] __attribute__((aligned(64)));
static uint32_t g_nslots;
static __thread gc_slot_t* t_slot;
static gc_slot_t* my_slot(void) {
    if (!t_slot) t_slot = &g_slots[__atomic_fetch_add(&g_nslots, 1u, __ATOMIC_RELAXED) % GC_SLOTS];
    return t_slot;
}

static void rect_box(const mm_rect* r, double lo[3], double hi[3]) {
    for (int a = 0; a < 3; ++a) {
        double c[4] = {r->o[a], (double)r->o[a] + r->v[a], (double)r->o[a] + r->u[a],
                       (double)r->o[a] + r->v[a] + r->u[a]};
        lo[a] = hi[a] = c[0];
        for (int k = 1; k < 4; ++k) {
            if (c[k] < lo[a]) lo[a] = c[k];
            if (c[k] > hi[a]) hi[a] = c[k];
        }
    }
}

static int cmpf(const void* a, const void* b) {
    float x = *(const float*)a, y = *(const float*)b;
    return (x > y) - (x < y);
}

static void gridcpu_free(void) {
    free(G.cell_off); free(G.cell_list); free(G.glob); free(G.leaf_of_rect);
    free(G.n); free(G.o); free(G.v); free(G.u); free(G.lv); free(G.lu);
    memset(&G, 0, sizeof G);
}

/* The scene the grid was built for (NULL: none) -- one grid per process: a
 * second build replaces the first, so callers check this before tracing. */
const oracle_scene* gridcpu_scene(void) { return G.sc; }

/* out[0] grid answers, out[1] walk fallbacks, out[2] queries for another scene (walked); reset = 1 zeroes. */
void gridcpu_stats(uint64_t out[3], int reset) {
    out[0] = out[1] = out[2] = 0;
    for (int i = 0; i < GC_SLOTS; ++i) {
        gc_slot_t* q = &g_slots[i];
        out[0] += __atomic_load_n(&q->grid, __ATOMIC_RELAXED);
        out[1] += __atomic_load_n(&q->fallback, __ATOMIC_RELAXED);
        out[2] += __atomic_load_n(&q->other, __ATOMIC_RELAXED);
        if (reset) {
            __atomic_store_n(&q->grid, 0, __ATOMIC_RELAXED);
            __atomic_store_n(&q->fallback, 0, __ATOMIC_RELAXED);
            __atomic_store_n(&q->other, 0, __ATOMIC_RELAXED);
        }
    }
}

/* Builds the grid for scene sc (kept for later oracle_trace_* calls of this
 * library); returns MM_OK or MM_ERR_NOMEM / MM_ERR_INVALID.  On failure no
 * grid is left (gridcpu_scene() is NULL) and nothing leaks. */
static int gridcpu_build_body(const oracle_scene* sc, uint32_t** cnt_p, uint8_t** is_glob_p);
int gridcpu_build(const oracle_scene* sc) {
    gridcpu_free();
    uint64_t junk[3];
    gridcpu_stats(junk, 1);
    uint32_t* cnt = NULL;
    uint8_t* is_glob = NULL;
    const int rc = gridcpu_build_body(sc, &cnt, &is_glob);
    free(cnt);
    free(is_glob);
    if (rc != MM_OK) gridcpu_free();
    return rc;
}

static int gridcpu_build_body(const oracle_scene* sc, uint32_t** cnt_p, uint8_t** is_glob_p) {
    const uint32_t nr = sc->n_rects;
    if (nr == 0) return MM_ERR_INVALID;
    G.sc = sc;
    double smin[3] = {1e30, 1e30, 1e30}, smax[3] = {-1e30, -1e30, -1e30}, C = 1.0;
    float* ext = malloc(4 * (size_t)nr);
    if (!ext) return MM_ERR_NOMEM;
    uint32_t m = 0;
    for (uint32_t k = 0; k < nr; ++k) {
        double lo[3], hi[3], e1 = 0, e2 = 0;
        rect_box(&sc->rects[k], lo, hi);
        for (int a = 0; a < 3; ++a) {
            if (lo[a] < smin[a]) smin[a] = lo[a];
            if (hi[a] > smax[a]) smax[a] = hi[a];
            if (fabs(lo[a]) > C) C = fabs(lo[a]);
            if (fabs(hi[a]) > C) C = fabs(hi[a]);
            const double e = hi[a] - lo[a];
            if (e > e1) { e2 = e1; e1 = e; } else if (e > e2) e2 = e;
        }
        if (e2 > 0) ext[m++] = (float)e2;
    }
    qsort(ext, m, 4, cmpf);
    const double cell = m ? ext[m / 2] : 1.0;
    free(ext);
    G.eps = (float)(C * 0x1p-14);
    long total = 1;
    for (int a = 0; a < 3; ++a) {
        const double lo = smin[a] - G.eps, hi = smax[a] + G.eps;
        int n = (int)floor((hi - lo) / cell + 0.5);
        if (n < 1) n = 1;
        if (n > 256) n = 256;
        G.gn[a] = n;
        G.gmin[a] = (float)lo;
        G.gcell[a] = (float)((hi - lo) / n);
        G.ginv[a] = 1.0f / G.gcell[a];
        total *= n;
    }
    G.glob = malloc(4 * (size_t)nr);
    uint32_t* cnt = *cnt_p = calloc((size_t)total + 1, 4);
    uint8_t* is_glob = *is_glob_p = calloc(nr, 1);
    if (!G.glob || !cnt || !is_glob) return MM_ERR_NOMEM;
    for (int pass = 0; pass < 2; ++pass) {
        for (uint32_t k = 0; k < nr; ++k) {
            double lo[3], hi[3];
            rect_box(&sc->rects[k], lo, hi);
            int i0[3], i1[3];
            long cover = 1;
            for (int a = 0; a < 3; ++a) {
                i0[a] = (int)floor((lo[a] - G.eps - G.gmin[a]) / G.gcell[a]);
                i1[a] = (int)floor((hi[a] + G.eps - G.gmin[a]) / G.gcell[a]);
                if (i0[a] < 0) i0[a] = 0;
                if (i1[a] > G.gn[a] - 1) i1[a] = G.gn[a] - 1;
                cover *= (i1[a] - i0[a] + 1);
            }
            if (pass == 0) {
                if (cover * 2 > total) { is_glob[k] = 1; G.glob[G.n_glob++] = k; continue; }
            } else if (is_glob[k]) {
                continue;
            }
            for (int z = i0[2]; z <= i1[2]; ++z)
                for (int y = i0[1]; y <= i1[1]; ++y)
                    for (int x = i0[0]; x <= i1[0]; ++x) {
                        const long c = ((long)z * G.gn[1] + y) * G.gn[0] + x;
                        if (pass == 0) cnt[c + 1]++;
                        else G.cell_list[cnt[c]++] = k;
                    }
        }
        if (pass == 0) {
            for (long c = 0; c < total; ++c) cnt[c + 1] += cnt[c];
            G.cell_off = malloc(4 * ((size_t)total + 1));
            G.cell_list = malloc(4 * ((size_t)cnt[total] + 1));
            if (!G.cell_off || !G.cell_list) return MM_ERR_NOMEM;
            memcpy(G.cell_off, cnt, 4 * ((size_t)total + 1));
        }
    }
    G.leaf_of_rect = malloc(4 * (size_t)nr);
    G.n = malloc(sizeof(v3) * nr); G.o = malloc(sizeof(v3) * nr);
    G.v = malloc(sizeof(v3) * nr); G.u = malloc(sizeof(v3) * nr);
    G.lv = malloc(4 * (size_t)nr); G.lu = malloc(4 * (size_t)nr);
    if (!G.leaf_of_rect || !G.n || !G.o || !G.v || !G.u || !G.lv || !G.lu) return MM_ERR_NOMEM;
    for (uint32_t i = 0; i < sc->n_nodes; ++i)
        if (sc->nodes[i].count)
            for (uint32_t j = 0; j < sc->nodes[i].count; ++j) G.leaf_of_rect[sc->idx[sc->nodes[i].left_first + j]] = i;
    for (uint32_t k = 0; k < nr; ++k) {  /* ray_rect's per-rect subexpressions (mm_oracle.c ray_rect) */
        const mm_rect* r = &sc->rects[k];
        G.o[k] = ld3(r->o); G.v[k] = ld3(r->v); G.u[k] = ld3(r->u);
        G.n[k] = normalize3(cross3(G.v[k], G.u[k]));
        G.lv[k] = sqrtf(dot3(G.v[k], G.v[k]));
        G.lu[k] = sqrtf(dot3(G.u[k], G.u[k]));
    }
    return MM_OK;
}

/* ray_rect_intersect (shaders.metal:51-67) without the `a < t` clause: a or BIG */
static inline float rect_a(v3 ori, v3 dir, uint32_t k) {
    const v3 n = G.n[k];
    const float nc = dot3(dir, n);
    const float a = dot3(vsub(G.o[k], ori), n) / nc;
    const v3 rv = vadd(vsub(ori, G.o[k]), vscale(a, dir));
    const float d1 = dot3(rv, G.v[k]) / G.lv[k];
    const float d2 = dot3(rv, G.u[k]) / G.lu[k];
    if (d1 >= 0.0f && d1 <= G.lv[k] && d2 >= 0.0f && d2 <= G.lu[k] && nc != 0.0f && a > 0.1f) return a;
    return BIG;
}

static inline void consider(float a, uint32_t k, float* best, uint32_t* bk, int* tie) {
    if (a == BIG) return;
    if (a < *best) { *best = a; *bk = k; *tie = 0; }
    else if (a == *best && k != *bk) *tie = 1;
}

/* the certified search; 1 with (t, index) written, 0 when the walk must answer */
static int grid_search(const ray_t* b, float* t_out, uint32_t* i_out, uint64_t* tests) {
    const float oo[3] = {b->ori.x, b->ori.y, b->ori.z}, dd[3] = {b->dir.x, b->dir.y, b->dir.z};
    float yy[3];
    for (int a = 0; a < 3; ++a) {
        const float ad = fabsf(dd[a]);
        if (!(ad >= 0x1p-40f && ad <= 0x1p40f)) return 0;
        if (!(oo[a] >= G.gmin[a] && oo[a] <= G.gmin[a] + G.gcell[a] * G.gn[a])) return 0;
        yy[a] = 1.0f / dd[a];
    }
    float best = BIG;
    uint32_t bk = 0;
    int tie = 0;
    for (uint32_t j = 0; j < G.n_glob; ++j) consider(rect_a(b->ori, b->dir, G.glob[j]), G.glob[j], &best, &bk, &tie);
    *tests += G.n_glob;
    int ic[3], stp[3];
    float tn[3], A[3], B[3];
    for (int a = 0; a < 3; ++a) {
        const float ps = oo[a] + 0.09375f * dd[a];  /* the cell of the point at t = 3/32 (mm_grid.h) */
        int i = (int)floorf((ps - G.gmin[a]) * G.ginv[a]);
        if (i < 0) i = 0;
        if (i > G.gn[a] - 1) i = G.gn[a] - 1;
        ic[a] = i;
        stp[a] = dd[a] > 0.0f ? 1 : -1;
        A[a] = (G.gmin[a] - oo[a]) * yy[a];
        B[a] = G.gcell[a] * yy[a];
        tn[a] = fmaf((float)(i + (stp[a] > 0)), B[a], A[a]);
    }
    for (;;) {
        const long c = ((long)ic[2] * G.gn[1] + ic[1]) * G.gn[0] + ic[0];
        for (uint32_t j = G.cell_off[c]; j < G.cell_off[c + 1]; ++j) {
            const uint32_t k = G.cell_list[j];
            consider(rect_a(b->ori, b->dir, k), k, &best, &bk, &tie);
        }
        *tests += G.cell_off[c + 1] - G.cell_off[c];
        const int a = tn[0] <= tn[1] ? (tn[0] <= tn[2] ? 0 : 2) : (tn[1] <= tn[2] ? 1 : 2);
        if (best < tn[a]) break;
        ic[a] += stp[a];
        if (ic[a] < 0 || ic[a] >= G.gn[a]) break;
        tn[a] = fmaf((float)(ic[a] + (stp[a] > 0)), B[a], A[a]);
    }
    if (best == BIG) { *t_out = BIG; *i_out = 0; return 1; }
    if (tie) return 0;
    /* certificate: the answer's reference leaf box passes intersect_aabb at every t > best */
    const mm_node* L = &G.sc->nodes[G.leaf_of_rect[bk]];
    ray_t r = *b;
    r.t = BIG;
    const float tmin = aabb(&r, L->mn, L->mx);
    if (!(tmin != BIG && tmin <= best)) return 0;
    *t_out = best;
    *i_out = bk;
    return 1;
}

static void grid_query_or_walk(ray_t* b, const oracle_scene* sc, trav_t* tr) {
    float t;
    uint32_t k;
    gc_slot_t* q = my_slot();
    if (G.sc != sc) {
        __atomic_fetch_add(&q->other, 1, __ATOMIC_RELAXED);
    } else if (grid_search(b, &t, &k, &tr->rect_tests)) {
        __atomic_fetch_add(&q->grid, 1, __ATOMIC_RELAXED);
        if (t < b->t) { b->t = t; b->index = k; }
        return;
    } else {
        __atomic_fetch_add(&q->fallback, 1, __ATOMIC_RELAXED);
    }
    intersect_bvh(b, sc, tr);
}
