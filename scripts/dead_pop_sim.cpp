// dead_pop_sim.cpp — analysis tool (not product, not oracle): how many of the
// reference traversal's pops (intersect_bvh_iterative, shaders.metal:115-156)
// take a node whose box entry tmin -- known when it was pushed -- is already
// >= the current closest t.  For an interior node both children then miss
// (tmin is monotone from parent to child in RN arithmetic), so a kernel could
// skip that visit without changing any result; this counts the visits it
// would save per ray on a frame sample.
//
//   g++ -O2 -std=c++17 -fopenmp -ffp-contract=off scripts/dead_pop_sim.cpp -Iinclude \
//       -Lmirror-maze_amd/lib -lmirror_maze -Wl,-rpath,$PWD/mirror-maze_amd/lib -o /tmp/dead_pop_sim
//   /tmp/dead_pop_sim [maze_n W H spp bounce mirror row_step]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "mm_scene.h"

namespace {

struct V3 { float x, y, z; };
V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V3 operator*(float s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
V3 mul(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
float dot(V3 a, V3 b) { float s = a.x * b.x; s = s + a.y * b.y; return s + a.z * b.z; }
V3 ld(const float* p) { return {p[0], p[1], p[2]}; }
V3 nrm(V3 v) { return (1.0f / sqrtf(dot(v, v))) * v; }
V3 cross(V3 v, V3 u) { return {u.z * v.y - u.y * v.z, u.x * v.z - u.z * v.x, u.y * v.x - u.x * v.y}; }
float comp(V3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
constexpr float kBig = 1e30f;

float rand_pm1(uint32_t& st) {
    uint32_t s = st * 747796405u + 291336453u;
    st = s;
    uint32_t r = ((s >> ((s >> 28) + 4u)) ^ s) * 277803737u;
    r = (r >> 22) ^ r;
    return (float)r * 0x1p-31f - 1.0f;
}
uint32_t pcg(uint32_t v) {
    uint32_t s = v * 747796405u + 2891336453u;
    uint32_t w = ((s >> ((s >> 28) + 4u)) ^ s) * 277803737u;
    return (w >> 22) ^ w;
}
uint32_t seed_tile(uint32_t pixel, uint32_t sample, uint32_t frame) { return pcg(pcg(pcg(frame) ^ pixel) + sample); }

V3 primary(const mm_uniform& u, uint32_t px, uint32_t py) {
    const float vx = u.cam.viewport[0], vy = u.cam.viewport[1];
    V3 p = {(vx * (float)px) / u.view_w - vx * 0.5f, (vy * (float)py) / u.view_h - vy * 0.5f, 0.0f - (-u.cam.focal)};
    V3 d = nrm(p);
    V3 q = {u.cam.quat[0], u.cam.quat[1], u.cam.quat[2]};
    float qw = u.cam.quat[3];
    V3 nq = {-q.x, -q.y, -q.z};
    float s1 = -dot(nq, d);
    V3 c1 = {nq.y * d.z - nq.z * d.y, nq.z * d.x - nq.x * d.z, nq.x * d.y - nq.y * d.x};
    V3 v1 = c1 + qw * d;
    V3 c2 = {v1.y * q.z - v1.z * q.y, v1.z * q.x - v1.x * q.z, v1.x * q.y - v1.y * q.x};
    return (qw * v1 + s1 * q) + c2;
}

struct Scene {
    const mm_scene* s;
    std::vector<V3> n;
    std::vector<mm_node> cons;        // boxes expanded by E
    std::vector<uint32_t> slot_leaf;  // slot -> leaf node index
};

float aabb(V3 o, V3 d, float t, const float* mn, const float* mx) {
    float tx1 = (mn[0] - o.x) / d.x, tx2 = (mx[0] - o.x) / d.x;
    float tmin = fminf(tx1, tx2), tmax = fmaxf(tx1, tx2);
    float ty1 = (mn[1] - o.y) / d.y, ty2 = (mx[1] - o.y) / d.y;
    tmin = fmaxf(tmin, fminf(ty1, ty2)); tmax = fminf(tmax, fmaxf(ty1, ty2));
    float tz1 = (mn[2] - o.z) / d.z, tz2 = (mx[2] - o.z) / d.z;
    tmin = fmaxf(tmin, fminf(tz1, tz2)); tmax = fminf(tmax, fmaxf(tz1, tz2));
    return (tmax >= tmin && tmin < t && tmax > 0.0f) ? tmin : kBig;
}

// exact reference rect test; returns a if the rect is hit (ignoring a < t), else NaN
float rect_a(const Scene& sc, uint32_t k, V3 ori, V3 dir) {
    const mm_rect& r = sc.s->rects[k];
    V3 o = ld(r.o), v = ld(r.v), u = ld(r.u), n = sc.n[k];
    float nc = dot(dir, n);
    float a = dot(o - ori, n) / nc;
    V3 rv = (ori - o) + a * dir;
    float lv = sqrtf(dot(v, v)), lu = sqrtf(dot(u, u));
    float d1 = dot(rv, v) / lv, d2 = dot(rv, u) / lu;
    if (d1 >= 0 && d1 <= lv && d2 >= 0 && d2 <= lu && nc != 0 && a > 0.1f) return a;
    return NAN;
}

struct Hit { float t; uint32_t k; uint32_t visits; };

struct Dead { uint64_t visits = 0, pops = 0, dead_interior = 0, dead_leaf = 0, leaf_pops = 0; };

// intersect_bvh_iterative with the far child's tmin kept beside it on the stack;
// counts pops whose node (interior or leaf) has tmin >= the current t.
Hit reference(const Scene& sc, V3 o, V3 d, Dead& dd) {
    const mm_node* nodes = sc.s->nodes;
    uint32_t stack[64], head = 0, node = 0, visits = 0;
    float stmin[64];
    float t = kBig;
    uint32_t idx = 0;
    for (;;) {
        const mm_node& nd = nodes[node];
        if (nd.count > 0) {
            for (uint32_t i = 0; i < nd.count; ++i) {
                const uint32_t k = sc.s->idx[nd.left_first + i];
                const float a = rect_a(sc, k, o, d);
                if (a < t) { t = a; idx = k; }
            }
            if (head == 0) break;
            --head; node = stack[head];
            dd.pops++;
            if (nodes[node].count > 0) { dd.leaf_pops++; if (!(stmin[head] < t)) dd.dead_leaf++; }
            else if (!(stmin[head] < t)) dd.dead_interior++;
            continue;
        }
        visits++;
        uint32_t l = nd.left_first, r = l + 1;
        float d1 = aabb(o, d, t, nodes[l].mn, nodes[l].mx), d2 = aabb(o, d, t, nodes[r].mn, nodes[r].mx);
        if (d1 > d2) { std::swap(d1, d2); std::swap(l, r); }
        if (d1 == kBig) {
            if (head == 0) break;
            --head; node = stack[head];
            dd.pops++;
            if (nodes[node].count > 0) { dd.leaf_pops++; if (!(stmin[head] < t)) dd.dead_leaf++; }
            else if (!(stmin[head] < t)) dd.dead_interior++;
        } else {
            node = l;
            if (d2 != kBig) { stmin[head] = d2; stack[head++] = r; }
        }
    }
    dd.visits += visits;
    return Hit{t, idx, visits};
}

}  // namespace

int main(int argc, char** argv) {
    uint32_t N = argc > 1 ? atoi(argv[1]) : 32, W = argc > 2 ? atoi(argv[2]) : 1920, H = argc > 3 ? atoi(argv[3]) : 1080;
    uint32_t spp = argc > 4 ? atoi(argv[4]) : 8;
    int bl = argc > 5 ? atoi(argv[5]) : 8, ml = argc > 6 ? atoi(argv[6]) : 8;
    uint32_t row_step = argc > 7 ? atoi(argv[7]) : 16;
    const float E = argc > 8 ? (float)atof(argv[8]) : 0.01f;
    mm_scene* s = nullptr;
    if (mm_scene_build(N, 0, &s) != 0) return 1;
    Scene sc{s, {}, {}, {}};
    for (uint32_t k = 0; k < s->n_rects; ++k) sc.n.push_back(nrm(cross(ld(s->rects[k].v), ld(s->rects[k].u))));
    sc.cons.assign(s->nodes, s->nodes + s->n_nodes);
    for (auto& nd : sc.cons)
        for (int a = 0; a < 3; ++a) {
            nd.mn[a] = nextafterf((float)((double)nd.mn[a] - E), -INFINITY);
            nd.mx[a] = nextafterf((float)((double)nd.mx[a] + E), INFINITY);
        }
    sc.slot_leaf.assign(s->n_rects, 0);
    for (uint32_t i = 0; i < s->n_nodes; ++i)
        if (s->nodes[i].count > 0)
            for (uint32_t j = 0; j < s->nodes[i].count; ++j) sc.slot_leaf[s->nodes[i].left_first + j] = i;
    mm_uniform u;
    mm_uniform_default((float)W, (float)H, 0, &u);
    const V3 cam = {u.cam.center[0], u.cam.center[1], u.cam.center[2]};
    struct Stats { uint64_t rays = 0; };
    Stats tot;
    Dead dtot;
    std::vector<uint32_t> rows;
    for (uint32_t y = 0; y < H; y += row_step) rows.push_back(y);
    const uint32_t frame = getenv("FRAME") ? atoi(getenv("FRAME")) : 0;
#pragma omp parallel
    {
        Stats st;
        Dead dd;
#pragma omp for schedule(dynamic, 1)
        for (size_t ri = 0; ri < rows.size(); ++ri) {
            const uint32_t py = rows[ri];
            for (uint32_t px = 0; px < W; ++px)
                for (uint32_t smp = 0; smp < spp; ++smp) {
                    uint32_t seed = seed_tile(py * W + px, smp, frame);
                    V3 dir = primary(u, px, py);
                    float j1 = rand_pm1(seed), j2 = rand_pm1(seed);
                    dir = dir + V3{j1 * 0.001f, j2 * 0.001f, 0.0f * 0.001f};
                    V3 ori = cam, T = {1, 1, 1};
                    int mh = 0;
                    for (int n = 0; n < bl + mh; ++n) {
                        const Hit ref = reference(sc, ori, dir, dd);
                        st.rays++;
                        const float t = ref.t;
                        const uint32_t k = ref.k;
                        if (!(t < kBig)) break;
                        const mm_rect& r = s->rects[k];
                        V3 nn = sc.n[k];
                        float dd = dot(dir, nn);
                        float sg = dd > 0 ? 1.0f : (dd < 0 ? -1.0f : dd);
                        if (s->is_mirror[k] == 0 || sg == 1.0f) {
                            T = mul(ld(r.color), T);
                            V3 rd;
                            do { float a = rand_pm1(seed), b = rand_pm1(seed), cc = rand_pm1(seed); rd = {a, b, cc}; }
                            while (sqrtf(dot(rd, rd)) > 1.0f);
                            V3 rn = (1.0f / sqrtf(dot(rd, rd))) * rd;
                            ori = ori + t * dir;
                            dir = nrm(rn + (-sg) * nn);
                        } else {
                            if (!(mh + 1 < ml)) break;
                            ori = ori + t * dir;
                            float q = dot(nn, dir) * 2.0f;
                            dir = nrm(dir - q * nn);
                            mh++;
                        }
                    }
                }
        }
#pragma omp critical
        {
            tot.rays += st.rays;
            dtot.visits += dd.visits; dtot.pops += dd.pops; dtot.dead_interior += dd.dead_interior;
            dtot.dead_leaf += dd.dead_leaf; dtot.leaf_pops += dd.leaf_pops;
        }
    }
    printf("# maze %u %ux%u spp %u limits %d/%d rows every %u\n", N, W, H, spp, bl, ml, row_step);
    printf("rays %llu  interior visits/ray %.3f  pops/ray %.3f  (leaf pops %.3f)\n", (unsigned long long)tot.rays,
           (double)dtot.visits / tot.rays, (double)dtot.pops / tot.rays, (double)dtot.leaf_pops / tot.rays);
    printf("dead pops (popped node's tmin >= current t): interior %.3f/ray (%.1f%% of interior visits), leaf %.3f/ray\n",
           (double)dtot.dead_interior / tot.rays, 100.0 * dtot.dead_interior / dtot.visits,
           (double)dtot.dead_leaf / tot.rays);
    mm_scene_free(s);
    return 0;
}
