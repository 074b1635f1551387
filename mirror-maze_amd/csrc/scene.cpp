// scene.cpp — host-side restatement of the reference's scene plumbing
// (src/main.rs, src/maths.rs) in C++17 behind the C ABI of include/mm_scene.h.
//
// Float semantics: built with -ffp-contract=off and no fast-math, so every
// expression rounds exactly where the Rust f32 code rounds (Rust never
// contracts to FMA and evaluates left to right).
#include "mm_scene.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <new>
#include <utility>
#include <vector>

namespace {

// ---------------------------------------------------------------------------
// ChaCha block function (D. J. Bernstein; RFC 8439 §2.3 for the 20-round
// known answer).  Word layout of the djb variant used by rand_chacha 0.3.1:
// 4 constants, 8 key words, 64-bit block counter (words 12,13), 64-bit stream
// id (words 14,15).
// ---------------------------------------------------------------------------
inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

inline void quarter(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
    a += b; d ^= a; d = rotl32(d, 16);
    c += d; b ^= c; b = rotl32(b, 12);
    a += b; d ^= a; d = rotl32(d, 8);
    c += d; b ^= c; b = rotl32(b, 7);
}

void chacha_block(const uint32_t key[8], uint64_t counter, uint64_t stream, int rounds,
                  uint32_t out[16]) {
    uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                      key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7],
                      (uint32_t)counter, (uint32_t)(counter >> 32),
                      (uint32_t)stream, (uint32_t)(stream >> 32)};
    uint32_t x[16];
    std::memcpy(x, s, sizeof(x));
    for (int i = 0; i < rounds; i += 2) {
        quarter(x[0], x[4], x[8], x[12]);
        quarter(x[1], x[5], x[9], x[13]);
        quarter(x[2], x[6], x[10], x[14]);
        quarter(x[3], x[7], x[11], x[15]);
        quarter(x[0], x[5], x[10], x[15]);
        quarter(x[1], x[6], x[11], x[12]);
        quarter(x[2], x[7], x[8], x[13]);
        quarter(x[3], x[4], x[9], x[14]);
    }
    for (int i = 0; i < 16; ++i) out[i] = x[i] + s[i];
}

// rand_chacha 0.3.1 keeps a 4-block (64-word) results buffer; words are
// consumed in keystream order and the block counter advances by 4 per refill.
void rng_refill(mm_rng* r) {
    for (int b = 0; b < 4; ++b) chacha_block(r->key, r->counter + (uint64_t)b, 0, 12, r->buf + 16 * b);
    r->counter += 4;
    r->pos = 0;
}

// ---------------------------------------------------------------------------
// f32 helpers mirroring src/maths.rs
// ---------------------------------------------------------------------------
struct F3 { float x, y, z; };
inline F3 f3(float x, float y, float z) { return F3{x, y, z}; }
inline F3 add3(F3 a, F3 b) { return F3{a.x + b.x, a.y + b.y, a.z + b.z}; }        // float3_add
inline F3 sub3(F3 a, F3 b) { return F3{a.x - b.x, a.y - b.y, a.z - b.z}; }        // float3_subtract
inline F3 scale3(F3 v, float f) { return F3{v.x * f, v.y * f, v.z * f}; }        // scale3
// Index<usize> for Float3 (maths.rs:37-48): out-of-range indices read .0
inline float idx3(F3 v, int i) { return i == 1 ? v.y : (i == 2 ? v.z : v.x); }
inline F3 from_arr(const float* a) { return F3{a[0], a[1], a[2]}; }

// Plane::get_center (main.rs:69-71): origin + (u + v) * 0.5
inline F3 plane_center(const mm_rect& p) {
    return add3(from_arr(p.o), scale3(add3(from_arr(p.u), from_arr(p.v)), 0.5f));
}

// aabb (main.rs:214-236).  Rust f32::min/max ignore a NaN operand, as fminf.
struct Box {
    F3 mn{1e30f, 1e30f, 1e30f};
    F3 mx{-1e30f, -1e30f, -1e30f};
    void grow(F3 p) {
        mn = F3{std::fmin(mn.x, p.x), std::fmin(mn.y, p.y), std::fmin(mn.z, p.z)};
        mx = F3{std::fmax(mx.x, p.x), std::fmax(mx.y, p.y), std::fmax(mx.z, p.z)};
    }
    void grow_plane(const mm_rect& p) {  // main.rs:95-97, 195-197
        F3 o = from_arr(p.o);
        grow(o);
        grow(add3(o, from_arr(p.u)));
        grow(add3(o, from_arr(p.v)));
    }
    float area() const {  // main.rs:233-236, left to right
        F3 e = sub3(mx, mn);
        float a = e.x * e.y;
        a = a + e.y * e.z;
        a = a + e.z * e.x;
        return a;
    }
};

// ---------------------------------------------------------------------------
// SAH BVH builder (main.rs:82-263).  Node allocation order, tie breaking
// (`cost <= best_cost`, last candidate wins) and the partition loop follow
// the reference exactly, so the node array is identical.
// ---------------------------------------------------------------------------
struct BvhBuilder {
    const mm_rect* planes;
    std::vector<F3> centers;
    std::vector<uint32_t> idx;
    std::vector<mm_node> nodes;
    bool exhaustive = false;  // the reference's O(n^2) candidate loop (MM_BVH_EXHAUSTIVE)

    static mm_node new_node(uint32_t lf, uint32_t count) {
        mm_node n;
        n.mn[0] = n.mn[1] = n.mn[2] = 1e30f;
        n.mx[0] = n.mx[1] = n.mx[2] = -1e30f;
        n.left_first = lf;
        n.count = count;
        return n;
    }
    void update_bounds(mm_node& n) const {  // main.rs:91-101
        Box b;
        for (uint32_t i = n.left_first; i < n.left_first + n.count; ++i) b.grow_plane(planes[idx[i]]);
        n.mn[0] = b.mn.x; n.mn[1] = b.mn.y; n.mn[2] = b.mn.z;
        n.mx[0] = b.mx.x; n.mx[1] = b.mx.y; n.mx[2] = b.mx.z;
    }
    float eval_sah(const mm_node& n, int axis, float pos) const {  // main.rs:180-211
        Box lb, rb;
        int lc = 0, rc = 0;
        for (uint32_t i = n.left_first; i < n.left_first + n.count; ++i) {
            const mm_rect& p = planes[idx[i]];
            if (idx3(plane_center(p), axis) < pos) { ++lc; lb.grow_plane(p); }
            else { ++rc; rb.grow_plane(p); }
        }
        float cost = (float)lc * lb.area();
        cost = cost + (float)rc * rb.area();
        return cost > 0.0f ? cost : 1e30f;  // NaN (0*inf) also maps to 1e30
    }
    // The same candidate loop in O(n log n) per node.  eval_sah's left set for
    // candidate c on `axis` is {p : center_p[axis] < c}: a prefix of the
    // primitives sorted by center.  Growing a box is min/max, so the prefix
    // (suffix) box over the sorted order has the bounds eval_sah accumulates in
    // index order — up to the sign of a zero bound, which cannot change the
    // value of a cost — and the cost expression is evaluated with eval_sah's
    // operations on the same counts.  Candidates are visited in eval order with
    // the same `<=`, so the chosen (axis, pos) is identical.  Returns false
    // (caller runs the exhaustive loop) if a center is NaN.
    bool sweep_split(const mm_node& self, int& best_axis, float& best_pos, float& best_cost) const {
        const uint32_t n = self.count, lf = self.left_first;
        std::vector<Box> pbox(n);
        for (uint32_t i = 0; i < n; ++i) pbox[i].grow_plane(planes[idx[lf + i]]);
        std::vector<uint32_t> ord(n);
        std::vector<float> keys(n), lterm(n + 1), rterm(n + 1);
        for (int axis = 0; axis <= 2; ++axis) {
            for (uint32_t i = 0; i < n; ++i) {
                keys[i] = idx3(centers[idx[lf + i]], axis);
                if (std::isnan(keys[i])) return false;
                ord[i] = i;
            }
            std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return keys[a] < keys[b]; });
            Box acc;
            lterm[0] = 0.0f * acc.area();
            for (uint32_t k = 1; k <= n; ++k) {
                const Box& b = pbox[ord[k - 1]];
                acc.mn = F3{std::fmin(acc.mn.x, b.mn.x), std::fmin(acc.mn.y, b.mn.y), std::fmin(acc.mn.z, b.mn.z)};
                acc.mx = F3{std::fmax(acc.mx.x, b.mx.x), std::fmax(acc.mx.y, b.mx.y), std::fmax(acc.mx.z, b.mx.z)};
                lterm[k] = (float)k * acc.area();
            }
            acc = Box();
            rterm[n] = 0.0f * acc.area();
            for (uint32_t k = n; k-- > 0;) {
                const Box& b = pbox[ord[k]];
                acc.mn = F3{std::fmin(acc.mn.x, b.mn.x), std::fmin(acc.mn.y, b.mn.y), std::fmin(acc.mn.z, b.mn.z)};
                acc.mx = F3{std::fmax(acc.mx.x, b.mx.x), std::fmax(acc.mx.y, b.mx.y), std::fmax(acc.mx.z, b.mx.z)};
                rterm[k] = (float)(n - k) * acc.area();
            }
            std::vector<float> sorted(n);
            for (uint32_t k = 0; k < n; ++k) sorted[k] = keys[ord[k]];
            for (uint32_t i = 0; i < n; ++i) {
                const float cand = keys[i];
                const uint32_t lc = (uint32_t)(std::lower_bound(sorted.begin(), sorted.end(), cand) - sorted.begin());
                float cost = lterm[lc];
                cost = cost + rterm[lc];
                cost = cost > 0.0f ? cost : 1e30f;
                if (cost <= best_cost) { best_cost = cost; best_pos = cand; best_axis = axis; }
            }
        }
        return true;
    }
    // subdivide (main.rs:102-179).  `self` is the node value held by the
    // caller; children are pushed, recursed, then written back.
    void subdivide(mm_node& self) {
        if (self.count == 1) return;
        float best_pos = 0.0f, best_cost = 1e30f;
        int best_axis = 6;
        if (exhaustive || !sweep_split(self, best_axis, best_pos, best_cost)) {
            for (int axis = 0; axis <= 2; ++axis) {
                for (uint32_t i = self.left_first; i < self.left_first + self.count; ++i) {
                    float cand = idx3(plane_center(planes[idx[i]]), axis);
                    float cost = eval_sah(self, axis, cand);
                    if (cost <= best_cost) { best_cost = cost; best_pos = cand; best_axis = axis; }
                }
            }
        }
        F3 diag = sub3(F3{self.mx[0], self.mx[1], self.mx[2]}, F3{self.mn[0], self.mn[1], self.mn[2]});
        float area = diag.x * diag.y;
        area = area + diag.y * diag.z;
        area = area + diag.z * diag.x;
        float parent_cost = (float)self.count * area;
        if (best_cost > parent_cost) return;
        const int axis = best_axis;
        const float split = best_pos;
        int i = (int)self.left_first;
        int j = i + (int)self.count - 1;
        while (i <= j) {
            float ap = idx3(centers[idx[i]], axis);  // axis 6 never reaches here unless all costs NaN
            if (ap < split) ++i;
            else { std::swap(idx[i], idx[j]); --j; }
        }
        uint32_t left_count = (uint32_t)i - self.left_first;
        if (left_count == 0 || left_count == self.count) return;
        mm_node left = new_node(self.left_first, left_count);
        update_bounds(left);
        self.left_first = (uint32_t)nodes.size();
        nodes.push_back(left);
        mm_node right = new_node((uint32_t)i, self.count - left_count);
        update_bounds(right);
        nodes.push_back(right);
        subdivide(left);
        subdivide(right);
        nodes[self.left_first] = left;
        nodes[self.left_first + 1] = right;
        self.count = 0;
    }
};

uint32_t depth_of(const mm_node* nodes, uint32_t n_nodes, uint32_t node, uint32_t d) {
    const mm_node& nd = nodes[node];
    if (nd.count > 0 || nd.left_first + 1 >= n_nodes) return d;
    uint32_t a = depth_of(nodes, n_nodes, nd.left_first, d + 1);
    uint32_t b = depth_of(nodes, n_nodes, nd.left_first + 1, d + 1);
    return a > b ? a : b;
}

// Kruskal union-find of main.rs:328-352: connect() hangs the CHILD's root
// under the parent node itself (not under the parent's root).
struct TreeBuilder {
    std::vector<int64_t> parent;  // -1 = None
    size_t root(size_t i) const {
        while (parent[i] >= 0) i = (size_t)parent[i];
        return i;
    }
    bool connected(size_t a, size_t b) const { return root(a) == root(b); }
    void connect(size_t p, size_t child) { parent[root(child)] = (int64_t)p; }
};

struct Wall { float a, b, len; };  // (x|y, start, length) as f32, main.rs:409,431

void push_plane(std::vector<mm_rect>& out, F3 o, F3 v, F3 u, F3 c) {
    mm_rect r;
    r.o[0] = o.x; r.o[1] = o.y; r.o[2] = o.z;
    r.v[0] = v.x; r.v[1] = v.y; r.v[2] = v.z;
    r.u[0] = u.x; r.u[1] = u.y; r.u[2] = u.z;
    r.color[0] = c.x; r.color[1] = c.y; r.color[2] = c.z;
    out.push_back(r);
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

void mm_chacha_block(const uint32_t key[8], uint64_t counter, uint64_t stream, int rounds,
                     uint32_t out[16]) {
    chacha_block(key, counter, stream, rounds, out);
}

void mm_rng_from_seed(mm_rng* r, const uint8_t seed[32]) {
    for (int i = 0; i < 8; ++i)
        r->key[i] = (uint32_t)seed[4 * i] | ((uint32_t)seed[4 * i + 1] << 8) |
                    ((uint32_t)seed[4 * i + 2] << 16) | ((uint32_t)seed[4 * i + 3] << 24);
    r->counter = 0;
    r->pos = 64;
    std::memset(r->buf, 0, sizeof(r->buf));
}

// rand_core 0.6.4 SeedableRng::seed_from_u64: PCG32 fills the 32-byte seed.
void mm_rng_seed_from_u64(mm_rng* r, uint64_t state) {
    const uint64_t MUL = 6364136223846793005ull, INC = 11634580027462260723ull;
    uint8_t seed[32];
    for (int c = 0; c < 8; ++c) {
        state = state * MUL + INC;
        uint32_t xorshifted = (uint32_t)(((state >> 18) ^ state) >> 27);
        uint32_t rot = (uint32_t)(state >> 59);
        uint32_t x = (xorshifted >> rot) | (xorshifted << ((32 - rot) & 31));
        seed[4 * c + 0] = (uint8_t)x;
        seed[4 * c + 1] = (uint8_t)(x >> 8);
        seed[4 * c + 2] = (uint8_t)(x >> 16);
        seed[4 * c + 3] = (uint8_t)(x >> 24);
    }
    mm_rng_from_seed(r, seed);
}

uint32_t mm_rng_next_u32(mm_rng* r) {
    if (r->pos >= 64) rng_refill(r);
    return r->buf[r->pos++];
}

// rand_core BlockRng::next_u64, including the buffer-straddling case.
uint64_t mm_rng_next_u64(mm_rng* r) {
    if (r->pos < 63) {
        uint64_t lo = r->buf[r->pos], hi = r->buf[r->pos + 1];
        r->pos += 2;
        return (hi << 32) | lo;
    }
    if (r->pos >= 64) {
        rng_refill(r);
        r->pos = 2;
        return ((uint64_t)r->buf[1] << 32) | r->buf[0];
    }
    uint64_t lo = r->buf[63];
    rng_refill(r);
    r->pos = 1;
    return ((uint64_t)r->buf[0] << 32) | lo;
}

// rand 0.8.5 Standard for f32: 24 high bits scaled by 2^-24.
float mm_rng_gen_f32(mm_rng* r) {
    uint32_t v = mm_rng_next_u32(r) >> 8;
    return (1.0f / (float)(1u << 24)) * (float)v;
}

// rand 0.8.5 UniformInt<u32>::sample_single (Lemire widening multiply with the
// "conservative zone" rejection).
uint32_t mm_rng_gen_range_u32(mm_rng* r, uint32_t lo, uint32_t hi) {
    uint32_t range = (hi - 1) - lo + 1;
    if (range == 0) return mm_rng_next_u32(r);
    uint32_t lz = (uint32_t)__builtin_clz(range);
    uint32_t zone = (range << lz) - 1u;
    for (;;) {
        uint64_t m = (uint64_t)mm_rng_next_u32(r) * (uint64_t)range;
        if ((uint32_t)m <= zone) return lo + (uint32_t)(m >> 32);
    }
}

int mm_bvh_build(const mm_rect* rects, uint32_t n, mm_node* nodes_out, uint32_t* n_nodes,
                 uint32_t* idx_out) {
    return mm_bvh_build_ex(rects, n, nodes_out, n_nodes, idx_out, MM_BVH_SWEEP);
}

int mm_bvh_build_ex(const mm_rect* rects, uint32_t n, mm_node* nodes_out, uint32_t* n_nodes,
                    uint32_t* idx_out, int method) {
    if (!rects || !nodes_out || !n_nodes || !idx_out || n == 0) return MM_ERR_INVALID;
    if (method != MM_BVH_SWEEP && method != MM_BVH_EXHAUSTIVE) return MM_ERR_INVALID;
    try {
        BvhBuilder b;
        b.planes = rects;
        b.exhaustive = method == MM_BVH_EXHAUSTIVE;
        b.nodes.reserve(2 * (size_t)n - 1);
        b.centers.resize(n);
        b.idx.resize(n);
        for (uint32_t i = 0; i < n; ++i) { b.centers[i] = plane_center(rects[i]); b.idx[i] = i; }
        mm_node root = BvhBuilder::new_node(0, n);
        b.update_bounds(root);
        b.nodes.push_back(root);
        b.subdivide(root);
        b.nodes[0] = root;
        std::memcpy(nodes_out, b.nodes.data(), b.nodes.size() * sizeof(mm_node));
        std::memcpy(idx_out, b.idx.data(), n * sizeof(uint32_t));
        *n_nodes = (uint32_t)b.nodes.size();
    } catch (const std::bad_alloc&) {
        return MM_ERR_NOMEM;
    }
    return MM_OK;
}

uint32_t mm_bvh_depth(const mm_node* nodes, uint32_t n_nodes) {
    if (!nodes || n_nodes == 0) return 0;
    return depth_of(nodes, n_nodes, 0, 0);
}

int mm_scene_build(uint32_t N, uint64_t seed, mm_scene** out) {
    if (!out || N < 2 || N > 4096) return MM_ERR_INVALID;
    *out = nullptr;
    try {
        const size_t W = N, H = N;  // main.rs:362-363
        TreeBuilder builder;
        std::vector<uint8_t> grid(W * H, 0);
        struct Edge { uint32_t x, y; bool up; };
        std::vector<Edge> edges;
        for (size_t y = 0; y < H; ++y)
            for (size_t x = 0; x < W; ++x) {
                if (y != 0) edges.push_back(Edge{(uint32_t)x, (uint32_t)y, true});
                if (x != 0) edges.push_back(Edge{(uint32_t)x, (uint32_t)y, false});
                builder.parent.push_back(-1);  // sets[y][x] = y*W + x
            }
        mm_rng rng;
        mm_rng_seed_from_u64(&rng, seed);  // main.rs:381
        // SliceRandom::shuffle (rand 0.8.5): for i in (1..len).rev() swap(i, gen_index(i+1))
        for (size_t i = edges.size(); i-- > 1;) {
            uint32_t j = mm_rng_gen_range_u32(&rng, 0, (uint32_t)(i + 1));
            std::swap(edges[i], edges[j]);
        }
        for (const Edge& e : edges) {  // main.rs:384-396
            size_t nx = e.up ? e.x : e.x - 1, ny = e.up ? e.y - 1 : e.y;
            size_t a = e.y * W + e.x, b = ny * W + nx;
            if (!builder.connected(a, b)) {
                builder.connect(a, b);
                if (e.up) { grid[e.y * W + e.x] |= 1; grid[ny * W + nx] |= 2; }
                else      { grid[e.y * W + e.x] |= 4; grid[ny * W + nx] |= 8; }
            }
        }
        // wall runs (main.rs:397-438); the trailing push keeps zero-length runs
        std::vector<Wall> vert, hori;
        for (size_t x = 0; x < W; ++x) {
            size_t start = 0, h = 0;
            for (size_t y = 0; y < H; ++y) {
                if (x == 0) { ++h; continue; }
                if ((grid[y * W + x] & 4) == 0 && (grid[y * W + x - 1] & 8) == 0) ++h;
                else {
                    if (h > 0) vert.push_back(Wall{(float)x, (float)start, (float)h});
                    h = 0;
                    start = y + 1;
                }
            }
            vert.push_back(Wall{(float)x, (float)start, (float)h});
        }
        for (size_t y = 0; y < H; ++y) {
            size_t start = 0, l = 0;
            for (size_t x = 0; x < W; ++x) {
                if (y == 0) { ++l; continue; }
                if ((grid[y * W + x] & 1) == 0 && (grid[(y - 1) * W + x] & 2) == 0) ++l;
                else {
                    if (l > 0) hori.push_back(Wall{(float)y, (float)start, (float)l});
                    l = 0;
                    start = x + 1;
                }
            }
            hori.push_back(Wall{(float)y, (float)start, (float)l});
        }
        // planes (main.rs:443-586)
        std::vector<mm_rect> planes;
        std::vector<uint8_t> mats;
        std::vector<float> emis;
        auto push_emi = [&](float a, float b, float c, float d) {
            emis.push_back(a); emis.push_back(b); emis.push_back(c); emis.push_back(d);
        };
        const F3 wall_color = f3(0.3f, 0.35f, 0.4f);
        const float half = (float)H / 2.0f;
        const float base = -10.0f * half;  // -10.0 * (height as f32 / 2.0)
        for (const Wall& w : vert) {
            push_plane(planes, f3(base + w.a * 10.0f, 2.0f, base + w.b * 10.0f),
                       f3(0.0f, 0.0f, w.len * 10.0f), f3(0.0f, -10.0f, 0.0f), wall_color);
            mats.push_back(mm_rng_gen_f32(&rng) < 0.85f ? 0 : 1);
            push_emi(1.0f, 0.0f, 0.0f, 0.0f);
            if (w.len <= 2.0f && mm_rng_gen_f32(&rng) < 0.3f) {
                push_plane(planes, f3((base + w.a * 10.0f) + 0.1f, 2.0f, base + w.b * 10.0f),
                           f3(0.0f, 0.0f, 9.9f), f3(0.0f, -6.0f, 0.0f), wall_color);
                mats.push_back(0);
                push_emi(1.0f, 0.8f, 0.3f, 2.0f);
            }
        }
        for (const Wall& w : hori) {
            push_plane(planes, f3(base + w.b * 10.0f, 2.0f, base + w.a * 10.0f),
                       f3(w.len * 10.0f, 0.0f, 0.0f), f3(0.0f, -10.0f, 0.0f), wall_color);
            mats.push_back(mm_rng_gen_f32(&rng) < 0.90f ? 0 : 1);
            push_emi(1.0f, 0.0f, 0.0f, 0.0f);
            if (w.len <= 2.0f && mm_rng_gen_f32(&rng) < 0.3f) {
                push_plane(planes, f3(base + w.b * 10.0f, 2.0f, (base + w.a * 10.0f) + 0.1f),
                           f3(9.9f, 0.0f, 0.0f), f3(0.0f, -6.0f, 0.0f), wall_color);
                mats.push_back(0);
                push_emi(1.0f, 0.8f, 0.3f, 2.0f);
            }
        }
        // boundary, floor, spawn light, roof — the reference's +-50 / 100 are
        // 5N / 10N (identical for N = 10)
        const float B = 5.0f * (float)N, L = 10.0f * (float)N;
        push_plane(planes, f3(-B, 2.0f, -B), f3(0.0f, -20.0f, 0.0f), f3(L, 0.0f, 0.0f), wall_color);
        mats.push_back(0); push_emi(1.0f, 1.0f, 1.0f, 0.0f);
        push_plane(planes, f3(-B, 2.0f, B), f3(L, 0.0f, 0.0f), f3(0.0f, -20.0f, 0.0f), wall_color);
        mats.push_back(0); push_emi(1.0f, 1.0f, 1.0f, 0.0f);
        push_plane(planes, f3(-B, 2.0f, -B), f3(0.0f, 0.0f, L), f3(0.0f, -20.0f, 0.0f), wall_color);
        mats.push_back(0); push_emi(1.0f, 1.0f, 1.0f, 0.0f);
        push_plane(planes, f3(B, 2.0f, -B), f3(0.0f, -20.0f, 0.0f), f3(0.0f, 0.0f, L), wall_color);
        mats.push_back(0); push_emi(1.0f, 1.0f, 1.0f, 0.0f);
        push_plane(planes, f3(-B, 2.0f, B), f3(0.0f, 0.0f, -L), f3(L, 0.0f, 0.0f), f3(0.4f, 0.45f, 0.3f));
        mats.push_back(0); push_emi(1.0f, 1.0f, 1.0f, 0.0f);
        push_plane(planes, f3(-5.0f, 2.0f, -49.9f), f3(10.0f, 0.0f, 0.0f), f3(0.0f, -6.0f, 0.0f), f3(0.0f, 0.0f, 0.0f));
        mats.push_back(0); push_emi(1.0f, 0.8f, 0.3f, 2.0f);
        push_plane(planes, f3(-B, -8.0f, B), f3(0.0f, 0.0f, -L), f3(L, 0.0f, 0.0f), f3(0.0f, 0.0f, 0.0f));
        mats.push_back(0); push_emi(1.0f, 0.8f, 0.3f, 0.02f);

        const uint32_t n = (uint32_t)planes.size();
        mm_scene* s = (mm_scene*)std::calloc(1, sizeof(mm_scene));
        if (!s) return MM_ERR_NOMEM;
        s->maze_n = N;
        s->n_rects = n;
        s->rects = (mm_rect*)std::malloc(n * sizeof(mm_rect));
        s->is_mirror = (uint8_t*)std::malloc(n);
        s->emission = (float*)std::malloc(n * 4 * sizeof(float));
        s->nodes = (mm_node*)std::malloc((2 * (size_t)n - 1) * sizeof(mm_node));
        s->idx = (uint32_t*)std::malloc(n * sizeof(uint32_t));
        s->grid = (uint8_t*)std::malloc(W * H);
        if (!s->rects || !s->is_mirror || !s->emission || !s->nodes || !s->idx || !s->grid) {
            mm_scene_free(s);
            return MM_ERR_NOMEM;
        }
        std::memcpy(s->rects, planes.data(), n * sizeof(mm_rect));
        std::memcpy(s->is_mirror, mats.data(), n);
        std::memcpy(s->emission, emis.data(), n * 4 * sizeof(float));
        std::memcpy(s->grid, grid.data(), W * H);
        s->n_vert_walls = (uint32_t)vert.size();
        s->n_hori_walls = (uint32_t)hori.size();
        int rc = mm_bvh_build(s->rects, n, s->nodes, &s->n_nodes, s->idx);  // main.rs:588
        if (rc != MM_OK) { mm_scene_free(s); return rc; }
        s->bvh_depth = mm_bvh_depth(s->nodes, s->n_nodes);
        *out = s;
    } catch (const std::bad_alloc&) {
        return MM_ERR_NOMEM;
    }
    return MM_OK;
}

void mm_scene_free(mm_scene* s) {
    if (!s) return;
    std::free(s->rects);
    std::free(s->is_mirror);
    std::free(s->emission);
    std::free(s->nodes);
    std::free(s->idx);
    std::free(s->grid);
    std::free(s);
}

// calculate_quaternion (maths.rs:139-156).  magnitude() = sqrt(x^2 + y^2 + z^2)
// left to right (powf(x, 2.0) is x*x); normalized() divides by it.
void mm_calculate_quaternion(const float dir[3], float q[4]) {
    auto mag = [](F3 v) {
        float s = v.x * v.x;
        s = s + v.y * v.y;
        s = s + v.z * v.z;
        return std::sqrt(s);
    };
    auto normed = [&](F3 v) {
        float m = mag(v);
        return F3{v.x / m, v.y / m, v.z / m};
    };
    const F3 def = f3(0.0f, 0.0f, 1.0f);
    const F3 cam = normed(f3(dir[0], dir[1], dir[2]));
    // cross_product (maths.rs:130-136)
    const F3 axis = f3(def.y * cam.z - def.z * cam.y, def.z * cam.x - def.x * cam.z,
                       def.x * cam.y - def.y * cam.x);
    const F3 an = normed(axis);
    const float half_theta = (float)std::asin((double)mag(axis)) / 2.0f;
    const float s = (float)std::sin((double)half_theta);
    const float c = (float)std::cos((double)half_theta);
    q[0] = an.x * s;
    q[1] = an.y * s;
    q[2] = an.z * s;
    q[3] = c;
}

void mm_uniform_default(float view_w, float view_h, uint32_t time, mm_uniform* u) {
    std::memset(u, 0, sizeof(*u));
    const float vh = 2.0f;
    const float vw = vh * (view_w / view_h);  // main.rs:732-733
    u->cam.center[0] = -5.0f;
    u->cam.center[1] = 0.0f;
    u->cam.center[2] = -45.0f;
    u->cam.focal = 1.0f;
    const float d[3] = {0.1f, 0.0f, 1.0f};
    mm_calculate_quaternion(d, u->cam.quat);
    u->cam.viewport[0] = vw;
    u->cam.viewport[1] = vh;
    u->view_w = view_w;
    u->view_h = view_h;
    u->chunk_w = 4;  // main.rs:602
    u->time = time;
}

// ---- chunk scheduler ------------------------------------------------------
struct mm_chunk_sched {
    std::vector<uint32_t> original;  // xy pairs, shuffled once (gen_pixels)
    std::vector<uint32_t> pixels;    // working stack (pop from back)
};

int mm_chunks_create(float view_w, float view_h, uint32_t chunk_w, uint64_t seed,
                     mm_chunk_sched** out) {
    if (!out || chunk_w == 0 || !(view_w >= 1.0f) || !(view_h >= 1.0f)) return MM_ERR_INVALID;
    try {
        auto* s = new mm_chunk_sched();
        const uint32_t w = (uint32_t)view_w / chunk_w, h = (uint32_t)view_h / chunk_w;
        for (uint32_t i = 0; i < w; ++i)       // main.rs:298-302 (x outer, y inner)
            for (uint32_t j = 0; j < h; ++j) {
                s->original.push_back(chunk_w * i);
                s->original.push_back(chunk_w * j);
            }
        mm_rng rng;
        mm_rng_seed_from_u64(&rng, seed);
        const size_t n = s->original.size() / 2;
        for (size_t i = n; i-- > 1;) {
            uint32_t j = mm_rng_gen_range_u32(&rng, 0, (uint32_t)(i + 1));
            std::swap(s->original[2 * i], s->original[2 * j]);
            std::swap(s->original[2 * i + 1], s->original[2 * j + 1]);
        }
        s->pixels = s->original;
        *out = s;
    } catch (const std::bad_alloc&) {
        return MM_ERR_NOMEM;
    }
    return MM_OK;
}

uint32_t mm_chunks_total(const mm_chunk_sched* s) { return s ? (uint32_t)(s->original.size() / 2) : 0; }

int mm_chunks_next(mm_chunk_sched* s, uint32_t n, uint32_t* out_xy) {  // main.rs:309-326
    if (!s || (!out_xy && n) || s->original.empty()) return MM_ERR_INVALID;
    for (uint32_t k = 0; k < n; ++k) {
        if (s->pixels.empty()) s->pixels = s->original;
        out_xy[2 * k + 1] = s->pixels.back(); s->pixels.pop_back();
        out_xy[2 * k + 0] = s->pixels.back(); s->pixels.pop_back();
    }
    return MM_OK;
}

void mm_chunks_free(mm_chunk_sched* s) { delete s; }

}  // extern "C"
