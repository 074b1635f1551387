/*
 * grid_sim.c — CPU experiment: closest-hit queries answered by a uniform-grid
 * search + exact verification, checked against the reference traversal
 * (oracle/mm_oracle.c's intersect_bvh) on every query of real C3 paths.
 *
 * Build: gcc -O2 -fopenmp -ffp-contract=off -o /tmp/sim/grid_sim scripts/grid_sim.c -lm
 * Run:   /tmp/sim/grid_sim /tmp/sim/scene32.bin W H spp bl ml rows_step
 *
 * The scene file holds n_rects, n_nodes, rects (48 B), nodes (32 B), idx,
 * is_mirror, emission (see the session notes in DESIGN.md).
 */
#include "../oracle/mm_oracle.c"

#include <stdio.h>
#include <float.h>

/* ---------------------------------------------------------------- scene */
static oracle_scene S;
static uint32_t* leaf_of_rect;   /* rect index -> reference leaf node */

static void load(const char* path) {
    FILE* f = fopen(path, "rb");
    if (!f) { perror(path); exit(1); }
    uint32_t nn[2];
    if (fread(nn, 4, 2, f) != 2) exit(1);
    S.n_rects = nn[0]; S.n_nodes = nn[1];
    mm_rect* r = malloc(sizeof(mm_rect) * S.n_rects);
    mm_node* n = malloc(sizeof(mm_node) * S.n_nodes);
    uint32_t* idx = malloc(4 * S.n_rects);
    uint8_t* m = malloc(S.n_rects);
    float* e = malloc(16 * S.n_rects);
    if (fread(r, sizeof(mm_rect), S.n_rects, f) != S.n_rects) exit(1);
    if (fread(n, sizeof(mm_node), S.n_nodes, f) != S.n_nodes) exit(1);
    if (fread(idx, 4, S.n_rects, f) != S.n_rects) exit(1);
    if (fread(m, 1, S.n_rects, f) != S.n_rects) exit(1);
    if (fread(e, 16, S.n_rects, f) != S.n_rects) exit(1);
    fclose(f);
    S.rects = r; S.nodes = n; S.idx = idx; S.is_mirror = m; S.emission = e;
    leaf_of_rect = malloc(4 * S.n_rects);
    for (uint32_t i = 0; i < S.n_nodes; ++i)
        if (n[i].count)
            for (uint32_t j = 0; j < n[i].count; ++j) leaf_of_rect[idx[n[i].left_first + j]] = i;
}

/* ---------------------------------------------------------------- grid */
static float gmin[3], gcell[3], ginv[3], geps;
static int gn[3];
static uint32_t* cell_off;   /* n_cells + 1 */
static uint32_t* cell_list;
static uint32_t* glob; static uint32_t n_glob;

static void rect_box(const mm_rect* r, double lo[3], double hi[3]) {
    for (int a = 0; a < 3; ++a) {
        double c[4] = {r->o[a], (double)r->o[a] + r->v[a], (double)r->o[a] + r->u[a],
                       (double)r->o[a] + r->v[a] + r->u[a]};
        lo[a] = hi[a] = c[0];
        for (int k = 1; k < 4; ++k) { if (c[k] < lo[a]) lo[a] = c[k]; if (c[k] > hi[a]) hi[a] = c[k]; }
    }
}

static int cmpf(const void* a, const void* b) {
    float x = *(const float*)a, y = *(const float*)b;
    return (x > y) - (x < y);
}

static void build_grid(double cell_target) {
    double smin[3] = {1e30, 1e30, 1e30}, smax[3] = {-1e30, -1e30, -1e30}, C = 1.0;
    for (uint32_t k = 0; k < S.n_rects; ++k) {
        double lo[3], hi[3];
        rect_box(&S.rects[k], lo, hi);
        for (int a = 0; a < 3; ++a) {
            if (lo[a] < smin[a]) smin[a] = lo[a];
            if (hi[a] > smax[a]) smax[a] = hi[a];
            if (fabs(lo[a]) > C) C = fabs(lo[a]);
            if (fabs(hi[a]) > C) C = fabs(hi[a]);
        }
    }
    geps = (float)(C * 0x1p-14);
    if (cell_target <= 0) {  /* median of the rects' smaller nonzero extent */
        float* ext = malloc(4 * S.n_rects);
        uint32_t m = 0;
        for (uint32_t k = 0; k < S.n_rects; ++k) {
            double lo[3], hi[3];
            rect_box(&S.rects[k], lo, hi);
            double e1 = 0, e2 = 0;
            for (int a = 0; a < 3; ++a) {
                double e = hi[a] - lo[a];
                if (e > e1) { e2 = e1; e1 = e; } else if (e > e2) e2 = e;
            }
            if (e2 > 0) ext[m++] = (float)e2;
        }
        qsort(ext, m, 4, cmpf);
        cell_target = ext[m / 2];
        free(ext);
    }
    long total = 1;
    for (int a = 0; a < 3; ++a) {
        double lo = smin[a] - geps, hi = smax[a] + geps;
        /* SHIFT=f: move the grid origin down by f cells (ALIGN: cells of exactly cell_target) */
        if (getenv("SHIFT")) lo -= atof(getenv("SHIFT")) * cell_target;
        int n = (int)floor((hi - lo) / cell_target + 0.5);
        if (getenv("ALIGN")) n = (int)ceil((hi - lo) / cell_target);
        if (n < 1) n = 1;
        if (n > 256) n = 256;
        /* NY=k: force k cells along y (the maze's walls span its whole height) */
        if (a == 1 && getenv("NY")) n = atoi(getenv("NY"));
        gn[a] = n;
        gmin[a] = (float)lo;
        gcell[a] = getenv("ALIGN") ? (float)cell_target : (float)((hi - lo) / n);
        ginv[a] = 1.0f / gcell[a];
        total *= n;
    }
    /* global rects: cover more than half of the cells */
    glob = malloc(4 * S.n_rects);
    uint32_t* cnt = calloc(total + 1, 4);
    uint8_t* is_glob = calloc(S.n_rects, 1);
    for (int pass = 0; pass < 2; ++pass) {
        for (uint32_t k = 0; k < S.n_rects; ++k) {
            double lo[3], hi[3];
            rect_box(&S.rects[k], lo, hi);
            int i0[3], i1[3];
            long cover = 1;
            for (int a = 0; a < 3; ++a) {
                double le = getenv("NOEPS") ? 0.0 : geps;
                i0[a] = (int)floor((lo[a] - le - gmin[a]) / gcell[a]);
                i1[a] = (int)floor((hi[a] + le - gmin[a]) / gcell[a]);
                if (i0[a] < 0) i0[a] = 0;
                if (i1[a] > gn[a] - 1) i1[a] = gn[a] - 1;
                cover *= (i1[a] - i0[a] + 1);
            }
            if (pass == 0) {
                if (cover * 2 > total) { is_glob[k] = 1; glob[n_glob++] = k; continue; }
            } else if (is_glob[k]) continue;
            for (int z = i0[2]; z <= i1[2]; ++z)
                for (int y = i0[1]; y <= i1[1]; ++y)
                    for (int x = i0[0]; x <= i1[0]; ++x) {
                        long c = ((long)z * gn[1] + y) * gn[0] + x;
                        if (pass == 0) cnt[c + 1]++;
                        else cell_list[cnt[c]++] = k;
                    }
        }
        if (pass == 0) {
            for (long c = 0; c < total; ++c) cnt[c + 1] += cnt[c];
            cell_off = malloc(4 * (total + 1));
            memcpy(cell_off, cnt, 4 * (total + 1));
            cell_list = malloc(4 * (cnt[total] + 1));
        }
    }
    fprintf(stderr, "grid %d x %d x %d, cell (%g %g %g), eps %g, %u global, %u list entries (%.2f/cell)\n",
            gn[0], gn[1], gn[2], gcell[0], gcell[1], gcell[2], geps, n_glob, cell_off[total],
            (double)cell_off[total] / total);
    free(cnt);
    free(is_glob);
}

/* face ranges: each cell's list in circular order around the cell (angle of the
   rect's box centre in the plane of the two axes with the most cells), stored
   twice over (wrap), and per entered face the shortest circular range holding
   every entry the neighbour across that face does not list */
static uint32_t *fr_off, *fr_list;
static uint8_t (*fr_s)[6], (*fr_l)[6];
static int fr_on, start_on, direct_on, tend_on;
static float start_t = 0.09375f;
static int listed_in(long c, uint32_t k) {
    for (uint32_t q = cell_off[c]; q < cell_off[c + 1]; ++q) if (cell_list[q] == k) return 1;
    return 0;
}
static void build_faces(void) {
    fr_on = getenv("FACES") != NULL;
    start_on = getenv("START") != NULL;
    direct_on = getenv("DIRECT") != NULL;
    /* TEND=1: the maze forms' walk (mm_grid.h, round 6): every exit folded into one end time per ray, the
       minimum over axes of the last boundary's crossing time (the same cell_time form), the walk stopping once
       the next crossing is not before it -- cells entered exactly at the exit instant are not visited */
    tend_on = getenv("TEND") != NULL;
    /* START=1 (or 0): the kernel's t = 3/32; START=<t>: that t */
    if (start_on) { start_t = (float)atof(getenv("START")); if (!(start_t > 0.0f) || start_t == 1.0f) start_t = 0.09375f; }
    long total = (long)gn[0] * gn[1] * gn[2];
    int ax0 = 0, ax1 = 2;  /* the plane: two axes with most cells */
    { int o[3] = {0, 1, 2};
      for (int i = 0; i < 3; ++i) for (int j = i + 1; j < 3; ++j) if (gn[o[j]] > gn[o[i]]) { int t = o[i]; o[i] = o[j]; o[j] = t; }
      ax0 = o[0]; ax1 = o[1]; }
    fr_off = malloc(8 * (total + 1)); fr_list = malloc(8 * (cell_off[total] + total + 1));
    fr_s = malloc(6 * total); fr_l = malloc(6 * total);
    uint32_t w = 0; uint64_t sum_full = 0, sum_face = 0, nf = 0;
    for (long c = 0; c < total; ++c) {
        int ic[3] = {(int)(c % gn[0]), (int)((c / gn[0]) % gn[1]), (int)(c / ((long)gn[0] * gn[1]))};
        uint32_t m = cell_off[c + 1] - cell_off[c];
        uint32_t e[64]; double ang[64];
        if (m > 64) m = 64;
        for (uint32_t i = 0; i < m; ++i) {
            e[i] = cell_list[cell_off[c] + i];
            double lo[3], hi[3]; rect_box(&S.rects[e[i]], lo, hi);
            double cc0 = gmin[ax0] + (ic[ax0] + 0.5) * gcell[ax0], cc1 = gmin[ax1] + (ic[ax1] + 0.5) * gcell[ax1];
            ang[i] = atan2(0.5 * (lo[ax1] + hi[ax1]) - cc1, 0.5 * (lo[ax0] + hi[ax0]) - cc0);
        }
        for (uint32_t i = 1; i < m; ++i) for (uint32_t j = i; j > 0 && ang[j] < ang[j - 1]; --j) {
            double ta = ang[j]; ang[j] = ang[j - 1]; ang[j - 1] = ta; uint32_t te = e[j]; e[j] = e[j - 1]; e[j - 1] = te; }
        fr_off[c] = w;
        for (uint32_t i = 0; i < m; ++i) fr_list[w++] = e[i];
        for (uint32_t i = 0; i + 1 < m; ++i) fr_list[w++] = e[i];
        for (int f = 0; f < 6; ++f) {
            int a = f >> 1, sgn = (f & 1) ? 1 : -1;  /* face f: neighbour at ic[a] + sgn */
            int nb[3] = {ic[0], ic[1], ic[2]}; nb[a] += sgn;
            int keep[64]; int nk = 0;
            for (uint32_t i = 0; i < m; ++i) {
                int in_nb = 0;
                if (nb[a] >= 0 && nb[a] < gn[a]) in_nb = listed_in(((long)nb[2] * gn[1] + nb[1]) * gn[0] + nb[0], e[i]);
                keep[i] = !in_nb; nk += keep[i];
            }
            uint32_t bs = 0, bl = m;
            if (nk == 0) { bs = 0; bl = 0; }
            else for (uint32_t st = 0; st < m; ++st) {
                if (!keep[st]) continue;
                uint32_t len = 0;
                for (uint32_t i = 0; i < m; ++i) if (keep[i]) { uint32_t d = (i + m - st) % m + 1; if (d > len) len = d; }
                if (len < bl) { bl = len; bs = st; }
            }
            fr_s[c][f] = (uint8_t)bs; fr_l[c][f] = (uint8_t)bl;
            sum_full += m; sum_face += bl; nf++;
        }
    }
    fr_off[total] = w;
    { long h[20] = {0}; for (long c = 0; c < total; ++c) { uint32_t m = cell_off[c + 1] - cell_off[c]; h[m < 19 ? m : 19]++; }
      fprintf(stderr, "list length hist:"); for (int i = 0; i < 20; ++i) if (h[i]) fprintf(stderr, " %d:%ld", i, h[i]); fprintf(stderr, "\n"); }
    fprintf(stderr, "faces: list %u -> %u entries with wrap; mean full %.3f, mean face range %.3f\n", cell_off[total], w,
            (double)sum_full / nf, (double)sum_face / nf);
}

/* ---------------------------------------------------------------- queries */
/* reference rect test without the a < t clause: a, or BIG */
static inline float rect_a(v3 ori, v3 dir, const mm_rect* r) {
    v3 o = ld3(r->o), v = ld3(r->v), u = ld3(r->u);
    v3 n = normalize3(cross3(v, u));
    float nc = dot3(dir, n);
    float a = dot3(vsub(o, ori), n) / nc;
    v3 rv = vadd(vsub(ori, o), vscale(a, dir));
    float lv = sqrtf(dot3(v, v));
    float d1 = dot3(rv, v) / lv;
    float lu = sqrtf(dot3(u, u));
    float d2 = dot3(rv, u) / lu;
    if (d1 >= 0.0f && d1 <= lv && d2 >= 0.0f && d2 <= lu && nc != 0.0f && a > 0.1f) return a;
    return BIG;
}

typedef struct {
    uint64_t tail_q, tail_tests, tail_cells, big_face, dup_prev, dup_tests, queries, cells, tests, fallback_tie, fallback_verify, fallback_guard, mismatch, miss;
    uint64_t hist_cells[64];
} gstats;

static inline void consider(float a, uint32_t k, float* best, uint32_t* bk, int* tie) {
    if (a == BIG) return;
    if (a < *best) { *best = a; *bk = k; *tie = 0; }
    else if (a == *best && k != *bk) *tie = 1;
}

/* grid search + verification; returns 1 and (t, index) when certified */
#define MAXC 128
static __thread int q_len[MAXC];   /* list lengths of the cells the last query visited */
static __thread int q_lx[MAXC];    /* ... of them x-normal (the axis-split model below) */
static uint8_t* rect_xn;           /* rect k is x-normal */
static __thread int q_n;
static __thread int q_cell0, q_oct;  /* the last query's start cell and direction octant (DUMP) */
/* crossing time of boundary b along axis a: the kernel's fma form (mm_grid.h,
 * default) or, with DIRECT=1, the direct form ((mn + b cell) - o) * y */
static float cell_time(int a, int b, float o, float y) {
    if (direct_on) return (gmin[a] + (float)b * gcell[a] - o) * y;
    const float A = (gmin[a] - o) * y, B = gcell[a] * y;
    return fmaf((float)b, B, A);
}

static int grid_query(v3 o, v3 d, float* t_out, uint32_t* i_out, gstats* st) {
    float oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z}, yy[3];
    for (int a = 0; a < 3; ++a) {
        float ad = fabsf(dd[a]);
        if (!(ad >= 0x1p-40f && ad <= 0x1p40f)) { st->fallback_guard++; return 0; }
        if (oo[a] < gmin[a] || oo[a] > gmin[a] + gcell[a] * gn[a]) { st->fallback_guard++; return 0; }
        yy[a] = 1.0f / dd[a];
    }
    float best = BIG;
    uint32_t bk = 0;
    int tie = 0;
    for (uint32_t j = 0; j < n_glob; ++j) { consider(rect_a(o, d, &S.rects[glob[j]]), glob[j], &best, &bk, &tie); st->tests++; }
    int ic[3], stp[3];
    float tn[3];
    for (int a = 0; a < 3; ++a) {
        /* the kernel starts the walk in the cell of the ray's point at t = 3/32 (mm_grid.h) */
        const float ps = start_on ? oo[a] + start_t * dd[a] : oo[a];
        int i = (int)floorf((ps - gmin[a]) * ginv[a]);
        if (i < 0) i = 0;
        if (i > gn[a] - 1) i = gn[a] - 1;
        ic[a] = i;
        stp[a] = dd[a] > 0.0f ? 1 : -1;
        tn[a] = cell_time(a, i + (stp[a] > 0), oo[a], yy[a]);
    }
    float tend = BIG;
    if (tend_on)
        for (int a = 0; a < 3; ++a) {
            const float te_a = cell_time(a, stp[a] > 0 ? gn[a] : 0, oo[a], yy[a]);
            if (te_a < tend) tend = te_a;
        }
    int ncell = 0;
    q_n = 0;
    q_cell0 = (ic[2] * gn[1] + ic[1]) * gn[0] + ic[0];
    q_oct = (dd[0] > 0.0f) | ((dd[1] > 0.0f) << 1) | ((dd[2] > 0.0f) << 2);
    uint32_t seen[256]; int n_seen = 0; long prev_c = -1; int face = -1;
    for (;;) {
        long c = ((long)ic[2] * gn[1] + ic[1]) * gn[0] + ic[0];
        uint32_t j0 = cell_off[c], j1 = cell_off[c + 1];
        const uint32_t* L = cell_list;
        if (fr_on) {
            L = fr_list; j0 = fr_off[c];
            j1 = j0 + (face < 0 ? cell_off[c + 1] - cell_off[c] : fr_l[c][face]);
            if (face >= 0 && fr_l[c][face] > 15) st->big_face++;
            if (face >= 0 && getenv("NOY") && (face >> 1) == 1) j1 = j0 + cell_off[c + 1] - cell_off[c];
            else if (face >= 0) { j0 += fr_s[c][face]; j1 += fr_s[c][face]; }
        }
        if (ncell < MAXC) {
            q_len[ncell] = (int)(j1 - j0);
            int nx = 0;
            for (uint32_t j = j0; j < j1; ++j) nx += rect_xn[L[j]];
            q_lx[ncell] = nx;
        }
        ncell++;
        q_n = ncell < MAXC ? ncell : MAXC;
        for (uint32_t j = j0; j < j1; ++j) {
            uint32_t k = L[j];
            { int dup = 0; for (int q = 0; q < n_seen; ++q) if (seen[q] == k) dup = 1;
              if (dup) st->dup_tests++; else if (n_seen < 256) seen[n_seen++] = k;
              if (prev_c >= 0) for (uint32_t q = cell_off[prev_c]; q < cell_off[prev_c + 1]; ++q) if (cell_list[q] == k) { st->dup_prev++; break; } }
            consider(rect_a(o, d, &S.rects[k]), k, &best, &bk, &tie);
            st->tests++;
        }
        int a = tn[0] <= tn[1] ? (tn[0] <= tn[2] ? 0 : 2) : (tn[1] <= tn[2] ? 1 : 2);
        prev_c = c;
        if (best < tn[a]) break;
        if (tend_on && !(tn[a] < tend)) break;
        ic[a] += stp[a];
        face = 2 * a + (stp[a] > 0 ? 0 : 1);  /* entered through the face toward the previous cell */
        if (ic[a] < 0 || ic[a] >= gn[a]) break;
        tn[a] = cell_time(a, ic[a] + (stp[a] > 0), oo[a], yy[a]);
    }
    st->cells += ncell;
    st->hist_cells[ncell < 63 ? ncell : 63]++;
    if (best == BIG) { st->miss++; *t_out = BIG; *i_out = 0; return 1; }
    if (tie) { st->fallback_tie++; return 0; }
    /* the reference leaf of bk passes at every t > best */
    const mm_node* L = &S.nodes[leaf_of_rect[bk]];
    ray_t b; b.ori = o; b.dir = d; b.t = BIG; b.index = 0;
    float tx1 = (L->mn[0] - o.x) / d.x, tx2 = (L->mx[0] - o.x) / d.x;
    float tmin = fminf(tx1, tx2), tmax = fmaxf(tx1, tx2);
    float ty1 = (L->mn[1] - o.y) / d.y, ty2 = (L->mx[1] - o.y) / d.y;
    tmin = fmaxf(tmin, fminf(ty1, ty2)); tmax = fminf(tmax, fmaxf(ty1, ty2));
    float tz1 = (L->mn[2] - o.z) / d.z, tz2 = (L->mx[2] - o.z) / d.z;
    tmin = fmaxf(tmin, fminf(tz1, tz2)); tmax = fminf(tmax, fmaxf(tz1, tz2));
    (void)b;
    if (!(tmax >= tmin && tmax > 0.0f && tmin <= best)) { st->fallback_verify++; return 0; }
    *t_out = best;
    *i_out = bk;
    return 1;
}

/* wave model: per lane, per bounce, the list lengths of the visited cells */
#define MAXB 32
static __thread int w_len[64][MAXB][16], w_lx[64][MAXB][16], w_n[64][MAXB], w_nb[64], w_lane;
/* DUMP=<file>: one 16-byte record per query, in path order, for the regrouping
   model (scripts/regroup_model.cpp): path id, bounce, start cell, octant, cells
   visited, the list length of the first 8 cells, and the rejection-sampling
   trials of the shading that follows (0: mirror bounce or path end). */
typedef struct {
    uint32_t path;
    uint16_t cell0;
    uint8_t bounce, oct, ncells, trials, lens[6];
} qrec_t;
static FILE* dump_f;
static __thread qrec_t* dump_buf;
static __thread size_t dump_n, dump_cap;
static __thread uint32_t dump_path;
static void dump_flush(void) {
    if (!dump_n) return;
#pragma omp critical(dump)
    fwrite(dump_buf, sizeof(qrec_t), dump_n, dump_f);
    dump_n = 0;
}
/* the reference path loop with every query cross-checked */
static v3 path(v3 ori, v3 dir, uint32_t seed, int bl, int ml, gstats* st, trav_t* tr, uint64_t* rays) {
    ray_t b;
    b.ori = ori; b.dir = dir; b.t = BIG; b.index = 0;
    v3 T = mk(1, 1, 1), L = mk(0, 0, 0);
    int mh = 0;
    for (int n = 0; n < bl + mh; ++n) {
        intersect_bvh(&b, &S, tr);
        (*rays)++;
        float gt; uint32_t gi;
        st->queries++;
        const uint64_t t_before = st->tests, c_before = st->cells;
        int ok_q = grid_query(b.ori, b.dir, &gt, &gi, st);
        qrec_t* qr = NULL;
        if (dump_f) {
            if (dump_n == dump_cap) { dump_cap = dump_cap ? 2 * dump_cap : 1 << 16; dump_buf = realloc(dump_buf, dump_cap * sizeof(qrec_t)); }
            qr = &dump_buf[dump_n++];
            qr->path = dump_path; qr->cell0 = (uint16_t)q_cell0; qr->bounce = (uint8_t)n; qr->oct = (uint8_t)q_oct;
            qr->ncells = (uint8_t)(q_n < 255 ? q_n : 255); qr->trials = 0;
            for (int c = 0; c < 6; ++c) qr->lens[c] = (uint8_t)(c < q_n ? (q_len[c] < 255 ? q_len[c] : 255) : 0);
        }
        if (n >= bl) { st->tail_q++; st->tail_tests += st->tests - t_before; st->tail_cells += st->cells - c_before; }
        if (n < MAXB) {
            w_n[w_lane][n] = q_n < 16 ? q_n : 16;
            for (int c = 0; c < w_n[w_lane][n]; ++c) { w_len[w_lane][n][c] = q_len[c]; w_lx[w_lane][n][c] = q_lx[c]; }
            w_nb[w_lane] = n + 1;
        }
        if (ok_q) {
            if (gt != b.t || (gt < BIG && gi != b.index)) {
                st->mismatch++;
                if (st->mismatch < 10)
                    fprintf(stderr, "MISMATCH o=(%a %a %a) d=(%a %a %a) ref t=%a k=%u grid t=%a k=%u\n", b.ori.x, b.ori.y,
                            b.ori.z, b.dir.x, b.dir.y, b.dir.z, b.t, b.index, gt, gi);
            }
        }
        if (!(b.t < BIG)) break;
        const uint32_t k = b.index;
        const mm_rect* r = &S.rects[k];
        v3 nn = normalize3(cross3(ld3(r->v), ld3(r->u)));
        float sg = msign(dot3(b.dir, nn));
        float side = -sg;
        if (S.is_mirror[k] == 0 || sg == 1.0f) {
            const float* e = &S.emission[4 * k];
            v3 contrib = vmul(vscale(e[3], T), ld3(e));
            v3 newT = vmul(ld3(r->color), T);
            float rx = oracle_rand_pm1(&seed), ry = oracle_rand_pm1(&seed), rz = oracle_rand_pm1(&seed);
            v3 rd = mk(rx, ry, rz);
            float len2 = dot3(rd, rd);
            int trials = 1;
            while (sqrtf(len2) > 1.0f) {
                rx = oracle_rand_pm1(&seed); ry = oracle_rand_pm1(&seed); rz = oracle_rand_pm1(&seed);
                rd = mk(rx, ry, rz);
                len2 = dot3(rd, rd);
                trials++;
            }
            if (qr) qr->trials = (uint8_t)(trials < 255 ? trials : 255);
            v3 rn = vscale(rsq(len2), rd);
            b.ori = vadd(b.ori, vscale(b.t, b.dir));
            v3 nd = vadd(rn, vscale(side, nn));
            b.dir = vscale(rsq(dot3(nd, nd)), nd);
            L = vadd(contrib, L);
            T = newT;
        } else {
            if (mh + 1 < ml) {
                v3 contrib = vscale(0.005f, ld3(r->color));
                b.ori = vadd(b.ori, vscale(b.t, b.dir));
                float dd = dot3(nn, b.dir) * 2.0f;
                v3 rf = vsub(b.dir, vscale(dd, nn));
                b.dir = vscale(rsq(dot3(rf, rf)), rf);
                L = vadd(contrib, L);
                mh = mh + 1;
            } else break;
        }
        b.t = BIG;
    }
    return L;
}

int main(int argc, char** argv) {
    if (argc < 8) { fprintf(stderr, "usage: grid_sim scene W H spp bl ml rowstep [cell]\n"); return 1; }
    load(argv[1]);
    int W = atoi(argv[2]), H = atoi(argv[3]), spp = atoi(argv[4]), bl = atoi(argv[5]), ml = atoi(argv[6]);
    int rs = atoi(argv[7]);
    build_grid(argc > 8 ? atof(argv[8]) : 0.0);
    if (getenv("DUMP")) dump_f = fopen(getenv("DUMP"), "wb");
    build_faces();
    rect_xn = calloc(S.n_rects, 1);
    for (uint32_t k = 0; k < S.n_rects; ++k) {
        const v3 nn = cross3(ld3(S.rects[k].v), ld3(S.rects[k].u));
        rect_xn[k] = fabsf(nn.x) > fabsf(nn.y) && fabsf(nn.x) > fabsf(nn.z);
    }
    mm_uniform u;
    /* default camera (mm_uniform_default): centre (-5,0,-45), quat from (0.1,0,1), focal 1, viewport (2W/H, 2) */
    u.cam.center[0] = -5.0f; u.cam.center[1] = 0.0f; u.cam.center[2] = -45.0f; u.cam.focal = 1.0f;
    u.cam.quat[0] = 0.0f; u.cam.quat[1] = 0.04981370270252228f; u.cam.quat[2] = 0.0f; u.cam.quat[3] = 0.9987585544586182f;
    u.cam.viewport[0] = 2.0f * (float)W / (float)H; u.cam.viewport[1] = 2.0f;
    u.view_w = (float)W; u.view_h = (float)H; u.chunk_w = 4; u.time = 0;
    gstats tot;
    memset(&tot, 0, sizeof tot);
    double wnest = 0, wflat = 0, wlane = 0, wcont[4] = {0, 0, 0, 0}, wtest = 0, wstep = 0, wshade = 0;
    double gnbmax = 0, gnbsum = 0, gnbw = 0, gact[32] = {0}, git[32] = {0};
    double gqmix = 0, gqsplit = 0, gitmix = 0, gitsplit = 0;
    uint64_t rays_tot = 0;
#pragma omp parallel
    {
        gstats st;
        memset(&st, 0, sizeof st);
        trav_t tr = {0, 0, 0};
        uint64_t rays = 0;
        double nest = 0, flat = 0, lanework = 0, ideal = 0, lockS = 0, cont[4] = {0, 0, 0, 0}, ntest = 0, nstep = 0;
        double nbmax = 0, nbsum = 0, nbw = 0, act_hist[32] = {0}, it_hist[32] = {0};
        double qmix = 0, qsplit = 0, itmix = 0, itsplit = 0;
#pragma omp for schedule(dynamic, 1)
        for (int y = 0; y < H; y += rs)
            for (int x0 = 0; x0 < W; x0 += 64 / spp) {
                for (int l = 0; l < 64; ++l) {
                    int x = x0 + l / spp, k = l % spp;
                    w_lane = l; w_nb[l] = 0;
                    if (x >= W) continue;
                    dump_path = (uint32_t)(((uint64_t)y * W + x) * spp + k);
                    v3 d0 = primary_dir(&u, x, y);
                    uint32_t seed = oracle_tile_seed(y * W + x, k, 0);
                    v3 d = jittered_dir(d0, &seed);
                    path(ld3(u.cam.center), d, seed, bl, ml, &st, &tr, &rays);
                }
                if (dump_f && dump_n > (1u << 22)) dump_flush();  /* (between chunks: a path's records stay together) */
                { int mx = 0, sum = 0, cnt = 0;
                  for (int l = 0; l < 64; ++l) if (w_nb[l] > 0) { sum += w_nb[l]; cnt++; if (w_nb[l] > mx) mx = w_nb[l]; }
                  if (cnt) { nbmax += mx; nbsum += (double)sum / cnt; nbw++;
                    /* lanes still active at bounce b, summed: lane-iterations in bounces >= 8 with <= 16 lanes */
                    for (int b = 0; b < mx; ++b) { int act = 0; for (int l = 0; l < 64; ++l) act += w_nb[l] > b; act_hist[b < 31 ? b : 31] += act; it_hist[b < 31 ? b : 31] += 1; } } }
                /* per bounce: nested (inner list loop per cell step) vs flat (one test or step per iteration) */
                for (int b = 0; b < MAXB; ++b) {
                    int any = 0, maxc = 0, maxflat = 0;
                    for (int l = 0; l < 64; ++l) if (w_nb[l] > b) {
                        any = 1;
                        int nc = w_n[l][b], fl = 0;
                        if (nc > maxc) maxc = nc;
                        for (int c = 0; c < nc; ++c) { fl += w_len[l][b][c] > 0 ? w_len[l][b][c] : 1; lanework += w_len[l][b][c] * 45.0 + 25.0; }
                        if (fl > maxflat) maxflat = fl;
                    }
                    if (!any) break;
                    for (int c = 0; c < maxc; ++c) {
                        int mx = 0, mxx = 0, mxz = 0;
                        for (int l = 0; l < 64; ++l) if (w_nb[l] > b && w_n[l][b] > c) {
                            if (w_len[l][b][c] > mx) mx = w_len[l][b][c];
                            if (w_lx[l][b][c] > mxx) mxx = w_lx[l][b][c];
                            if (w_len[l][b][c] - w_lx[l][b][c] > mxz) mxz = w_len[l][b][c] - w_lx[l][b][c];
                        }
                        nest += mx * 45.0 + 25.0;
                        ntest += mx * 45.0; nstep += 25.0;
                        /* quad-cycles: one mixed test loop (12.5 per test) vs an x loop and a z loop
                           without the axis selects (9.5 per test, 1.5 more per cell for the second loop) */
                        qmix += mx * 12.5 + 12.0; qsplit += (mxx + mxz) * 9.5 + 13.5;
                        itmix += mx; itsplit += mxx + mxz;
                    }
                    flat += maxflat * 70.0;
                    lockS += 250.0;
                }
                /* continuous (lanes run their bounces back to back) with batched shading */
                for (int K = 0; K < 4; ++K) {
                    int thr = (int[]){1, 16, 32, 64}[K];
                    int bi[64], rem[64], state[64];   /* state 0 querying, 1 waiting for shade, 2 done */
                    for (int l = 0; l < 64; ++l) {
                        bi[l] = 0; state[l] = w_nb[l] > 0 ? 0 : 2; rem[l] = 0;
                        if (state[l] == 0) { int fl = 0; for (int c = 0; c < w_n[l][0]; ++c) fl += w_len[l][0][c] > 0 ? w_len[l][0][c] : 1; rem[l] = fl; }
                    }
                    double cost = 250.0; /* first setup */
                    for (;;) {
                        int nq = 0, nw = 0;
                        for (int l = 0; l < 64; ++l) { nq += state[l] == 0; nw += state[l] == 1; }
                        if (nq == 0 && nw == 0) break;
                        if (nw >= thr || (nq == 0 && nw > 0)) {
                            cost += 250.0;
                            for (int l = 0; l < 64; ++l) if (state[l] == 1) {
                                bi[l]++;
                                if (bi[l] >= w_nb[l] || bi[l] >= MAXB) { state[l] = 2; continue; }
                                int fl = 0; for (int c = 0; c < w_n[l][bi[l]]; ++c) fl += w_len[l][bi[l]][c] > 0 ? w_len[l][bi[l]][c] : 1;
                                rem[l] = fl; state[l] = 0;
                            }
                            continue;
                        }
                        cost += 70.0;
                        for (int l = 0; l < 64; ++l) if (state[l] == 0 && --rem[l] <= 0) state[l] = 1;
                    }
                    cont[K] += cost;
                }
            }
        if (dump_f) dump_flush();
#pragma omp critical
        { gqmix += qmix; gqsplit += qsplit; gitmix += itmix; gitsplit += itsplit;
          wnest += nest + lockS; wflat += flat + lockS; wtest += ntest; wstep += nstep; wshade += lockS; wlane += lanework; for (int K = 0; K < 4; ++K) wcont[K] += cont[K];
          gnbmax += nbmax; gnbsum += nbsum; gnbw += nbw; for (int b = 0; b < 32; ++b) { gact[b] += act_hist[b]; git[b] += it_hist[b]; } }
#pragma omp critical
        {
            tot.dup_tests += st.dup_tests; tot.tail_q += st.tail_q; tot.tail_tests += st.tail_tests; tot.tail_cells += st.tail_cells; tot.dup_prev += st.dup_prev; tot.queries += st.queries; tot.cells += st.cells; tot.tests += st.tests;
            tot.fallback_tie += st.fallback_tie; tot.fallback_verify += st.fallback_verify;
            tot.fallback_guard += st.fallback_guard; tot.mismatch += st.mismatch; tot.miss += st.miss;
            for (int i = 0; i < 64; ++i) tot.hist_cells[i] += st.hist_cells[i];
            rays_tot += rays;
        }
    }
    double q = (double)tot.queries;
    printf("queries %llu  cells/query %.3f  rect tests/query %.3f  fallback tie %.5f%% verify %.5f%% guard %.5f%%  miss %llu  MISMATCH %llu\n",
           (unsigned long long)tot.queries, tot.cells / q, tot.tests / q, 100 * tot.fallback_tie / q,
           100 * tot.fallback_verify / q, 100 * tot.fallback_guard / q, (unsigned long long)tot.miss,
           (unsigned long long)tot.mismatch);
    printf("queries past the bounce limit (mirror tails): %.3f%%, tests/query %.3f, cells/query %.3f\n",
           100.0 * tot.tail_q / q, (double)tot.tail_tests / tot.tail_q, (double)tot.tail_cells / tot.tail_q);
    printf("duplicate tests (rect already tested by this query) per query %.3f, of them listed in the previous cell %.3f\n", tot.dup_tests / q, tot.dup_prev / q);
    printf("wave model (VALU slots x64 per wave): nested %.4g  flat %.4g  ideal(lane work/64) %.4g  -> util nested %.3f flat %.3f\n",
           wnest, wflat, wlane / 64, wlane / 64 / wnest, wlane / 64 / wflat);
    printf("nested split: tests %.4g  cell steps %.4g  shading %.4g\n", wtest, wstep, wshade);
    printf("axis-split model (lockstep waves): test wave-iterations mixed %.4g split %.4g (x %.3f); quad-cycles of tests + steps mixed %.4g split %.4g (x %.3f)\n",
           gitmix, gitsplit, gitsplit / gitmix, gqmix, gqsplit, gqsplit / gqmix);
    printf("with shading (250/bounce): lockstep nested %.4g flat %.4g | continuous thr1 %.4g thr16 %.4g thr32 %.4g thr64 %.4g\n",
           wnest, wflat, wcont[0], wcont[1], wcont[2], wcont[3]);
    printf("per wave: mean of max queries/lane %.3f, mean queries/lane %.3f\n", gnbmax / gnbw, gnbsum / gnbw);
    printf("bounce b: waves still running (fraction) / mean active lanes:");
    for (int b = 0; b < 24; ++b) if (git[b] > 0) printf(" %d:%.3f/%.1f", b, git[b] / gnbw, gact[b] / git[b]);
    printf("\n");
    printf("cells hist:");
    for (int i = 1; i < 40; ++i) printf(" %d:%.3f", i, tot.hist_cells[i] / q);
    printf("\n");
    return tot.mismatch ? 2 : 0;
}
