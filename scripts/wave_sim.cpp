// wave_sim.cpp — analysis tool (not product, not oracle): a CPU model of how
// the throughput megakernel's waves spend their issue slots.
//
// Traces a row sample of a throughput frame with a plain float statement of
// the path loop (same algorithm as the kernels: shaders.metal:115-156,
// 302-340), records for every ray its traversal step sequence (interior step /
// leaf with k rects), then replays the 64-lane lockstep execution of the
// wave-persistent kernel under several scheduling policies and reports wave
// iterations, lane utilisation and a VALU estimate per policy.
//
//   g++ -O2 -std=c++17 -fopenmp scripts/wave_sim.cpp -Iinclude \
//       -Lmirror-maze_amd/lib -lmirror_maze -Wl,-rpath,$PWD/mirror-maze_amd/lib -o /tmp/wave_sim
//   /tmp/wave_sim [maze_n W H spp bounce mirror row_step]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "mm_scene.h"

namespace {

uint32_t g_frame = 0;

struct V3 { float x, y, z; };
V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V3 operator*(float s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
V3 mul(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
float dot(V3 a, V3 b) { float s = a.x * b.x; s = s + a.y * b.y; return s + a.z * b.z; }
V3 ld(const float* p) { return {p[0], p[1], p[2]}; }
V3 nrm(V3 v) { return (1.0f / sqrtf(dot(v, v))) * v; }
V3 cross(V3 v, V3 u) { return {u.z * v.y - u.y * v.z, u.x * v.z - u.z * v.x, u.y * v.x - u.x * v.y}; }
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
};

float aabb(V3 o, V3 d, float t, const mm_node& nd) {
    float tx1 = (nd.mn[0] - o.x) / d.x, tx2 = (nd.mx[0] - o.x) / d.x;
    float tmin = fminf(tx1, tx2), tmax = fmaxf(tx1, tx2);
    float ty1 = (nd.mn[1] - o.y) / d.y, ty2 = (nd.mx[1] - o.y) / d.y;
    tmin = fmaxf(tmin, fminf(ty1, ty2)); tmax = fminf(tmax, fmaxf(ty1, ty2));
    float tz1 = (nd.mn[2] - o.z) / d.z, tz2 = (nd.mx[2] - o.z) / d.z;
    tmin = fmaxf(tmin, fminf(tz1, tz2)); tmax = fminf(tmax, fmaxf(tz1, tz2));
    return (tmax >= tmin && tmin < t && tmax > 0.0f) ? tmin : kBig;
}

void rect(const Scene& sc, uint32_t k, V3 ori, V3 dir, float& t, uint32_t& idx) {
    const mm_rect& r = sc.s->rects[k];
    V3 o = ld(r.o), v = ld(r.v), u = ld(r.u), n = sc.n[k];
    float nc = dot(dir, n);
    float a = dot(o - ori, n) / nc;
    V3 rv = (ori - o) + a * dir;
    float lv = sqrtf(dot(v, v)), lu = sqrtf(dot(u, u));
    float d1 = dot(rv, v) / lv, d2 = dot(rv, u) / lu;
    if (d1 >= 0 && d1 <= lv && d2 >= 0 && d2 <= lu && nc != 0 && a > 0.1f && a < t) { t = a; idx = k; }
}

// One closest-hit query; appends its step codes (0 interior, k leaf of k rects)
// and a terminator 0xFF.
void query(const Scene& sc, V3 o, V3 d, float& t, uint32_t& idx, std::vector<uint8_t>& steps) {
    const mm_node* nodes = sc.s->nodes;
    uint32_t stack[64], head = 0, node = 0;
    for (;;) {
        const mm_node& nd = nodes[node];
        if (nd.count > 0) {
            steps.push_back((uint8_t)nd.count);
            for (uint32_t i = 0; i < nd.count; ++i) rect(sc, sc.s->idx[nd.left_first + i], o, d, t, idx);
            if (head == 0) break;
            node = stack[--head];
            continue;
        }
        steps.push_back(0);
        uint32_t l = nd.left_first, r = l + 1;
        float d1 = aabb(o, d, t, nodes[l]), d2 = aabb(o, d, t, nodes[r]);
        if (d1 > d2) { std::swap(d1, d2); std::swap(l, r); }
        if (d1 == kBig) {
            if (head == 0) break;
            node = stack[--head];
        } else {
            node = l;
            if (d2 != kBig) stack[head++] = r;
        }
    }
    steps.push_back(0xFF);
}

struct Ray { uint32_t off; };      // offset of the ray's step codes in the chunk's buffer
struct PathRec { std::vector<uint32_t> rays; uint8_t dir_oct[32]; };

// Trace one path, recording its rays.
void trace(const Scene& sc, V3 ori, V3 dir, uint32_t seed, int bl, int ml, std::vector<uint8_t>& buf,
           std::vector<uint32_t>& rays, std::vector<uint32_t>& keys) {
    V3 T = {1, 1, 1}, L = {0, 0, 0};
    int mh = 0;
    for (int n = 0; n < bl + mh; ++n) {
        float t = kBig; uint32_t k = 0;
        rays.push_back((uint32_t)buf.size());
        // sort key: origin cell (10 units) and direction octant
        int cx = (int)floorf(ori.x / 10.0f) & 255, cz = (int)floorf(ori.z / 10.0f) & 255;
        keys.push_back(((uint32_t)cx << 16 | (uint32_t)cz << 8) << 3 | (dir.x > 0) | (dir.y > 0) << 1 | (dir.z > 0) << 2);
        query(sc, ori, dir, t, k, buf);
        if (!(t < kBig)) break;
        const mm_rect& r = sc.s->rects[k];
        V3 nn = sc.n[k];
        float dd = dot(dir, nn);
        float sg = dd > 0 ? 1.0f : (dd < 0 ? -1.0f : dd);
        if (sc.s->is_mirror[k] == 0 || sg == 1.0f) {
            const float* e = &sc.s->emission[4 * k];
            L = mul(e[3] * T, ld(e)) + L;
            T = mul(ld(r.color), T);
            V3 rd;
            do { float a = rand_pm1(seed), b = rand_pm1(seed), c = rand_pm1(seed); rd = {a, b, c}; } while (sqrtf(dot(rd, rd)) > 1.0f);
            V3 rn = (1.0f / sqrtf(dot(rd, rd))) * rd;
            ori = ori + t * dir;
            V3 nd = rn + (-sg) * nn;
            dir = nrm(nd);
        } else {
            if (!(mh + 1 < ml)) break;
            ori = ori + t * dir;
            float q = dot(nn, dir) * 2.0f;
            dir = nrm(dir - q * nn);
            mh++;
        }
    }
}

// ---- cost model (VALU wave-instructions) -----------------------------------
struct Cost {
    double interior = 85, leaf = 45, loop = 12, shade = 160, setup = 120;
};
struct Tally {
    double iters = 0, int_iters = 0, leaf_iters = 0, leaf_rect_iters = 0, bounce_iters = 0;
    double lane_int = 0, lane_leaf = 0, lane_slots = 0;  // useful lane-steps, 64 x iterations
    double valu = 0;
    void add(const Tally& o) {
        iters += o.iters; int_iters += o.int_iters; leaf_iters += o.leaf_iters; leaf_rect_iters += o.leaf_rect_iters;
        bounce_iters += o.bounce_iters; lane_int += o.lane_int; lane_leaf += o.lane_leaf; lane_slots += o.lane_slots;
        valu += o.valu;
    }
};

// Lockstep traversal of one ray per lane (nullptr = inactive lane).
// mode 0: if-if (each iteration: interior block if any lane interior, leaf
//         block if any lane at a leaf);  mode k>=2: leaves are tested only
//         every k-th iteration (or when no lane has interior work).
//         mode 1: leaf-then-interior in the same iteration.
void lockstep(const std::vector<const uint8_t*>& lanes, int mode, const Cost& c, Tally& t) {
    std::vector<const uint8_t*> p = lanes;
    uint64_t it = 0;
    for (;;) {
        bool any = false, any_int = false, any_leaf = false;
        int max_cnt = 0, n_int = 0, n_leaf = 0;
        for (auto& q : p) {
            if (!q || *q == 0xFF) continue;
            any = true;
            if (*q == 0) { any_int = true; n_int++; }
            else { any_leaf = true; n_leaf++; max_cnt = std::max(max_cnt, (int)*q); }
        }
        if (!any) break;
        bool do_leaf = any_leaf;
        if (mode >= 2) do_leaf = any_leaf && ((it % mode) == 0 || !any_int);
        t.iters++; it++;
        t.valu += c.loop;
        if (mode == 1) {
            // leaf lanes test and pop, then every lane at an interior node steps
            if (any_leaf) { t.leaf_iters++; t.leaf_rect_iters += max_cnt; t.valu += c.leaf * max_cnt; t.lane_leaf += n_leaf; }
            bool any_int2 = false; int n2 = 0;
            for (auto& q : p) {
                if (!q || *q == 0xFF) continue;
                if (*q != 0) { ++q; if (*q == 0) { any_int2 = true; n2++; ++q; } continue; }
                any_int2 = true; n2++; ++q;
            }
            if (any_int2) { t.int_iters++; t.valu += c.interior; t.lane_int += n2; }
            t.lane_slots += 64;
            continue;
        }
        if (any_int) { t.int_iters++; t.valu += c.interior; t.lane_int += n_int; }
        if (do_leaf) { t.leaf_iters++; t.leaf_rect_iters += max_cnt; t.valu += c.leaf * max_cnt; t.lane_leaf += n_leaf; }
        t.lane_slots += 64;
        for (auto& q : p) {
            if (!q || *q == 0xFF) continue;
            if (*q == 0 || do_leaf) ++q;
        }
    }
}

}  // namespace

// Path -> lane mappings of a 64-path chunk over a band of 8 rows (spp = 8):
// 0 current (8 consecutive pixels of a row x 8 samples), 1 2x4 pixel tile x 8
// samples, 2 4x2 tile x 8, 3 8x8 pixel tile x 1 sample (sample s of the tile
// in chunk s), 4 64 consecutive pixels of a row x 1 sample.
int map_mode(const Scene& sc, const mm_uniform& u, V3 cam, uint32_t W, uint32_t H, uint32_t spp, int bl, int ml,
             uint32_t band_step) {
    if (spp != 8) { fprintf(stderr, "mapping study needs spp 8\n"); return 1; }
    const int NM = 5;
    const char* names[NM] = {"8 px (row) x 8 spp  [current]", "2x4 px tile x 8 spp", "4x2 px tile x 8 spp",
                             "8x8 px tile x 1 spp", "64 px (row) x 1 spp"};
    std::vector<double> valu(NM, 0.0), iters(NM, 0.0);
    std::vector<uint32_t> bands;
    for (uint32_t y = 0; y + 8 <= H; y += band_step) bands.push_back(y);
    Cost c;
#pragma omp parallel for schedule(dynamic, 1)
    for (size_t bi = 0; bi < bands.size(); ++bi) {
        const uint32_t y0 = bands[bi];
        std::vector<uint8_t> buf;
        std::vector<std::vector<uint32_t>> prays((size_t)8 * W * spp);
        auto pid = [&](uint32_t px, uint32_t dy, uint32_t s) { return ((size_t)dy * W + px) * spp + s; };
        for (uint32_t dy = 0; dy < 8; ++dy)
            for (uint32_t px = 0; px < W; ++px)
                for (uint32_t s = 0; s < spp; ++s) {
                    const uint32_t y = y0 + dy;
                    uint32_t seed = seed_tile(y * W + px, s, g_frame);
                    V3 d = primary(u, px, y);
                    float j1 = rand_pm1(seed), j2 = rand_pm1(seed);
                    d = d + V3{j1 * 0.001f, j2 * 0.001f, 0.0f * 0.001f};
                    std::vector<uint32_t> keys;
                    trace(sc, cam, d, seed, bl, ml, buf, prays[pid(px, dy, s)], keys);
                }
        std::vector<double> lv(NM, 0.0), li(NM, 0.0);
        for (int m = 0; m < NM; ++m) {
            std::vector<std::vector<size_t>> chunks;
            if (m == 0) {
                for (uint32_t dy = 0; dy < 8; ++dy)
                    for (uint32_t px = 0; px < W; px += 8) {
                        std::vector<size_t> ch;
                        for (uint32_t k = 0; k < 8; ++k) for (uint32_t s = 0; s < 8; ++s) ch.push_back(pid(px + k, dy, s));
                        chunks.push_back(ch);
                    }
            } else if (m == 1 || m == 2) {
                const uint32_t tw = m == 1 ? 4 : 2, th = m == 1 ? 2 : 4;
                for (uint32_t dy = 0; dy < 8; dy += th)
                    for (uint32_t px = 0; px < W; px += tw) {
                        std::vector<size_t> ch;
                        for (uint32_t j = 0; j < th; ++j) for (uint32_t i = 0; i < tw; ++i)
                            for (uint32_t s = 0; s < 8; ++s) ch.push_back(pid(px + i, dy + j, s));
                        chunks.push_back(ch);
                    }
            } else if (m == 3) {
                for (uint32_t px = 0; px < W; px += 8)
                    for (uint32_t s = 0; s < 8; ++s) {
                        std::vector<size_t> ch;
                        for (uint32_t j = 0; j < 8; ++j) for (uint32_t i = 0; i < 8; ++i) ch.push_back(pid(px + i, j, s));
                        chunks.push_back(ch);
                    }
            } else {
                for (uint32_t dy = 0; dy < 8; ++dy)
                    for (uint32_t px = 0; px < W; px += 64)
                        for (uint32_t s = 0; s < 8; ++s) {
                            std::vector<size_t> ch;
                            for (uint32_t i = 0; i < 64 && px + i < W; ++i) ch.push_back(pid(px + i, dy, s));
                            chunks.push_back(ch);
                        }
            }
            Tally t;
            for (auto& ch : chunks) {
                size_t maxb = 0;
                for (size_t q : ch) maxb = std::max(maxb, prays[q].size());
                for (size_t b = 0; b < maxb; ++b) {
                    std::vector<const uint8_t*> lanes(64, nullptr);
                    for (size_t l = 0; l < ch.size(); ++l)
                        if (b < prays[ch[l]].size()) lanes[l] = &buf[prays[ch[l]][b]];
                    t.valu += c.shade;
                    lockstep(lanes, 1, c, t);
                }
                t.valu += c.setup;
            }
            lv[m] = t.valu;
            li[m] = t.iters;
        }
#pragma omp critical
        for (int m = 0; m < NM; ++m) { valu[m] += lv[m]; iters[m] += li[m]; }
    }
    printf("# path->lane mappings, loop form 5 lockstep model, %zu bands of 8 rows (every %u rows)\n", bands.size(),
           band_step);
    for (int m = 0; m < NM; ++m)
        printf("%-34s iters %10.0f  VALU(model) %12.4g  rel %.3f\n", names[m], iters[m], valu[m], valu[m] / valu[0]);
    return 0;
}

int main(int argc, char** argv) {
    uint32_t N = argc > 1 ? atoi(argv[1]) : 32, W = argc > 2 ? atoi(argv[2]) : 1920, H = argc > 3 ? atoi(argv[3]) : 1080;
    uint32_t spp = argc > 4 ? atoi(argv[4]) : 8;
    int bl = argc > 5 ? atoi(argv[5]) : 8, ml = argc > 6 ? atoi(argv[6]) : 8;
    uint32_t row_step = argc > 7 ? atoi(argv[7]) : 8;
    mm_scene* s = nullptr;
    if (mm_scene_build(N, 0, &s) != 0) { fprintf(stderr, "scene build failed\n"); return 1; }
    Scene sc{s, {}};
    for (uint32_t k = 0; k < s->n_rects; ++k) sc.n.push_back(nrm(cross(ld(s->rects[k].v), ld(s->rects[k].u))));
    mm_uniform u;
    mm_uniform_default((float)W, (float)H, 0, &u);
    const V3 cam = {u.cam.center[0], u.cam.center[1], u.cam.center[2]};
    if (getenv("MAPS")) return map_mode(sc, u, cam, W, H, spp, bl, ml, row_step);

    // rows sampled: y = 0, row_step, ...; a "chunk" is 64 consecutive paths of
    // one row (path = pixel*spp + sample, as the kernel numbers them)
    std::vector<uint32_t> rows;
    for (uint32_t y = 0; y < H; y += row_step) rows.push_back(y);
    const uint32_t paths_per_row = W * spp, chunks_per_row = (paths_per_row + 63) / 64;
    const int NK = 6, NR = 4, NP = 5 + NK + NR + 1;
    const int kThresholds[NR] = {0, 8, 16, 32};  // policies
    const char* names[NP] = {"if-if (current)", "leaf+interior same iter", "leaves every 2nd iter",
                             "leaves every 3rd iter", "bounce-boundary refill (1024-path stream)",
                             "block-sync bounce, compaction only", "block-sync, sort by octant",
                             "block-sync, sort by cell+octant", "block-sync, sort by cell",
                             "block-sync, sort by exact length (bound)", "block-sync, sort by octant,cell",
                             "per-ray refill, th 0", "per-ray refill, th 8", "per-ray refill, th 16",
                             "per-ray refill, th 32", "ideal (no divergence)"};
    std::vector<Tally> tot(NP);
    double rays_total = 0, steps_int = 0, steps_leaf = 0, rects_total = 0;
    Cost c;
    if (getenv("FRAME")) g_frame = (uint32_t)atoi(getenv("FRAME"));
    std::vector<double> chunk_cost(rows.size() * chunks_per_row, 0.0);

#pragma omp parallel for schedule(dynamic, 1) reduction(+ : rays_total, steps_int, steps_leaf, rects_total)
    for (size_t ri = 0; ri < rows.size(); ++ri) {
        const uint32_t y = rows[ri];
        std::vector<Tally> loc(NP);
        // process the row in blocks of 16 chunks (1024 paths)
        for (uint32_t cb = 0; cb < chunks_per_row; cb += 16) {
            const uint32_t nch = std::min(16u, chunks_per_row - cb);
            std::vector<uint8_t> buf;
            std::vector<std::vector<uint32_t>> prays(nch * 64), pkeys(nch * 64);
            for (uint32_t l = 0; l < nch * 64; ++l) {
                const uint32_t path = (cb * 64) + l;
                if (path >= paths_per_row) continue;
                const uint32_t px = path / spp, smp = path % spp;
                uint32_t seed = seed_tile(y * W + px, smp, g_frame);
                V3 d = primary(u, px, y);
                float j1 = rand_pm1(seed), j2 = rand_pm1(seed);
                d = d + V3{j1 * 0.001f, j2 * 0.001f, 0.0f * 0.001f};
                trace(sc, cam, d, seed, bl, ml, buf, prays[l], pkeys[l]);
            }
            for (uint32_t l = 0; l < nch * 64; ++l) {
                rays_total += prays[l].size();
                for (uint32_t off : prays[l])
                    for (const uint8_t* q = &buf[off]; *q != 0xFF; ++q) {
                        if (*q == 0) steps_int++; else { steps_leaf++; rects_total += *q; }
                    }
            }
            // policies 0-3: per chunk, bounce-synchronous lockstep
            for (int pol = 0; pol < 4; ++pol) {
                const int mode = pol == 0 ? 0 : (pol == 1 ? 1 : pol);
                for (uint32_t ch = 0; ch < nch; ++ch) {
                    const double v0 = loc[pol].valu;
                    size_t maxb = 0;
                    for (uint32_t l = 0; l < 64; ++l) maxb = std::max(maxb, prays[ch * 64 + l].size());
                    for (size_t b = 0; b < maxb; ++b) {
                        std::vector<const uint8_t*> lanes(64, nullptr);
                        for (uint32_t l = 0; l < 64; ++l)
                            if (b < prays[ch * 64 + l].size()) lanes[l] = &buf[prays[ch * 64 + l][b]];
                        loc[pol].bounce_iters++;
                        loc[pol].valu += c.shade;
                        lockstep(lanes, mode, c, loc[pol]);
                    }
                    loc[pol].valu += c.setup;
                    if (pol == 0) chunk_cost[ri * chunks_per_row + cb + ch] = loc[pol].valu - v0;
                }
            }
            // policy 4: bounce-boundary refill within the wave's stream of paths
            {
                std::vector<uint32_t> queue;
                for (uint32_t l = 0; l < nch * 64; ++l) queue.push_back(l);
                size_t next = 0;
                std::vector<int> lane_path(64, -1);
                std::vector<size_t> lane_b(64, 0);
                for (;;) {
                    for (int l = 0; l < 64; ++l)
                        if (lane_path[l] < 0 && next < queue.size()) { lane_path[l] = (int)queue[next++]; lane_b[l] = 0; loc[4].valu += 0; }
                    bool any = false;
                    std::vector<const uint8_t*> lanes(64, nullptr);
                    for (int l = 0; l < 64; ++l)
                        if (lane_path[l] >= 0) { any = true; lanes[l] = &buf[prays[lane_path[l]][lane_b[l]]]; }
                    if (!any) break;
                    loc[4].bounce_iters++;
                    loc[4].valu += c.shade + c.setup / 4;
                    lockstep(lanes, 0, c, loc[4]);
                    for (int l = 0; l < 64; ++l)
                        if (lane_path[l] >= 0 && ++lane_b[l] >= prays[lane_path[l]].size()) lane_path[l] = -1;
                }
            }
            // per-ray lane refill (k_trace_persist's state machine): a wave
            // steps traversals while more than `th` lanes traverse, then
            // shades the finished lanes and refills idle ones from its stream
            for (int ti = 0; ti < NR; ++ti) {
                const int th = kThresholds[ti];
                Tally& tl = loc[5 + NK + ti];
                size_t next = 0;
                std::vector<int> lp(64, -1);
                std::vector<size_t> lb(64, 0);
                std::vector<const uint8_t*> q(64, nullptr);
                std::vector<uint8_t> st(64, 0);  // 0 idle, 1 trav, 2 finished query
                for (;;) {
                    // shade finished queries
                    bool any_sh = false, any_ref = false;
                    for (int l = 0; l < 64; ++l)
                        if (st[l] == 2) {
                            any_sh = true;
                            if (++lb[l] >= prays[lp[l]].size()) { st[l] = 0; lp[l] = -1; }
                            else { st[l] = 1; q[l] = &buf[prays[lp[l]][lb[l]]]; }
                        }
                    if (any_sh) tl.valu += c.shade;
                    for (int l = 0; l < 64; ++l)
                        if (st[l] == 0 && next < (size_t)nch * 64) {
                            any_ref = true; lp[l] = (int)next++; lb[l] = 0; st[l] = 1; q[l] = &buf[prays[lp[l]][0]];
                        }
                    if (any_ref) tl.valu += c.setup;
                    int ntr = 0;
                    for (int l = 0; l < 64; ++l) ntr += st[l] == 1;
                    if (ntr == 0) break;
                    tl.bounce_iters++;
                    for (;;) {
                        int nt = 0, nwait = 0;
                        for (int l = 0; l < 64; ++l) { nt += st[l] == 1; nwait += st[l] == 2 || (st[l] == 0 && next < (size_t)nch * 64); }
                        if (nt == 0 || (nt <= th && nwait > 0)) break;
                        bool any_int = false, any_leaf = false; int mc = 0, ni = 0, nl = 0;
                        for (int l = 0; l < 64; ++l) if (st[l] == 1) {
                            if (*q[l] == 0) { any_int = true; ni++; } else { any_leaf = true; nl++; mc = std::max(mc, (int)*q[l]); }
                        }
                        tl.iters++; tl.valu += c.loop + 8;  // + state-machine control
                        if (any_int) { tl.int_iters++; tl.valu += c.interior; tl.lane_int += ni; }
                        if (any_leaf) { tl.leaf_iters++; tl.valu += c.leaf * mc; tl.lane_leaf += nl; }
                        tl.lane_slots += 64;
                        for (int l = 0; l < 64; ++l) if (st[l] == 1) { ++q[l]; if (*q[l] == 0xFF) st[l] = 2; }
                    }
                }
            }
            // policies 5..: bounce-synchronous over the 1024-path block, the
            // live rays of each bounce compacted (and optionally sorted by a
            // key) and packed into waves
            for (int kp = 0; kp < NK; ++kp) {
                Tally& tl = loc[5 + kp];
                size_t maxb = 0;
                for (auto& v : prays) maxb = std::max(maxb, v.size());
                for (size_t b = 0; b < maxb; ++b) {
                    std::vector<std::pair<uint64_t, uint32_t>> live;
                    for (uint32_t l = 0; l < nch * 64; ++l)
                        if (b < prays[l].size()) {
                            const uint32_t k = pkeys[l][b];
                            const uint8_t* q = &buf[prays[l][b]];
                            uint32_t len = 0;
                            while (q[len] != 0xFF) ++len;
                            uint64_t key = 0;
                            switch (kp) {
                                case 0: key = l; break;                      // compaction only
                                case 1: key = k & 7u; break;                 // octant
                                case 2: key = k; break;                      // cell + octant
                                case 3: key = (k >> 3) & 0xFFFF; break;      // cell
                                case 4: key = len; break;                    // exact length (oracle bound)
                                case 5: key = ((uint64_t)(k & 7u) << 32) | ((k >> 3) & 0xFFFF); break;  // octant, then cell
                            }
                            live.push_back({key << 16 | l, prays[l][b]});
                        }
                    std::stable_sort(live.begin(), live.end());
                    for (size_t w = 0; w < live.size(); w += 64) {
                        std::vector<const uint8_t*> lanes(64, nullptr);
                        for (size_t l = 0; l < 64 && w + l < live.size(); ++l) lanes[l] = &buf[live[w + l].second];
                        tl.bounce_iters++;
                        tl.valu += c.shade + 60;  // + state exchange through LDS
                        lockstep(lanes, 0, c, tl);
                    }
                }
                for (uint32_t ch = 0; ch < nch; ++ch) tl.valu += c.setup;
            }
        }
        // policy 6: ideal = useful work only (filled below from totals)
#pragma omp critical
        for (int p = 0; p < NP; ++p) tot[p].add(loc[p]);
    }
    if (getenv("CHUNK_DUMP")) {
        FILE* f = fopen(getenv("CHUNK_DUMP"), "wb");
        fwrite(chunk_cost.data(), sizeof(double), chunk_cost.size(), f);
        fclose(f);
    }
    const double scale = (double)H / rows.size();
    printf("# maze %u, %ux%u, %u spp, limits %d/%d; rows sampled %zu (every %u)\n", N, W, H, spp, bl, ml,
           rows.size(), row_step);
    printf("# per frame (scaled): rays %.1f M, interior steps/ray %.2f, leaf visits/ray %.2f, rect tests/ray %.2f\n",
           rays_total * scale / 1e6, steps_int / rays_total, steps_leaf / rays_total, rects_total / rays_total);
    tot[NP - 1].valu = (steps_int * c.interior + rects_total * c.leaf + (steps_int + steps_leaf) * c.loop) / 64.0 +
                  rays_total * c.shade / 64.0;
    printf("%-40s %10s %9s %9s %9s %8s %10s %7s\n", "policy", "iters(M)", "int-it%", "leaf-it%", "lane-util", "rays/it",
           "VALU(G)", "rel");
    for (int p = 0; p < NP; ++p) {
        const Tally& t = tot[p];
        const double util = t.lane_slots > 0 ? (t.lane_int + t.lane_leaf) / t.lane_slots : 1.0;
        printf("%-40s %10.2f %9.1f %9.1f %9.3f %8.2f %10.3f %7.3f\n", names[p], t.iters * scale / 1e6,
               t.iters ? 100 * t.int_iters / t.iters : 0, t.iters ? 100 * t.leaf_iters / t.iters : 0, util,
               t.bounce_iters ? rays_total / t.bounce_iters : 0, t.valu * scale / 1e9, t.valu / tot[0].valu);
    }
    mm_scene_free(s);
    return 0;
}
