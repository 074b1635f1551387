// grid_build.cpp — host construction of the uniform grid the certified search
// walks (mm_grid.h; the proof of the search is there).
//
// Geometry: the box of every rect corner, widened by eps = C * 2^-14 (C = the
// largest |coordinate|, at least 1), cut into n[a] cells per axis with
// n[a] = round(extent / s) for a cell size s = the median over the scene's
// non-degenerate rects of their second-largest extent (the maze's wall
// height: one cell per maze cell), clamped to 1..256 per axis; s grows by
// 1.25x until the cells and lists fit the LDS budget the caller gives.
// Lists: a rect goes on the list of every cell its box comes within eps of;
// rects that would sit on more than half of the cells (the maze floor) go on
// the global list every query tests instead (at most 4); zero-length rects
// (SKIP records: never hit) go nowhere.  Rects that are not axis-aligned
// with exact unit normals (SLOW records) are listed too; the kernel runs the
// general ray_rect_intersect on them (grid_rect<kSlow>).
// Per rect the image also holds its grid record (mm_grid.h: grid_rect; made
// from rect_compact.cpp's record, built with identity slots) and the box of
// the reference BVH leaf holding it -- the box the certificate tests.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "grid_build.h"
#include "mm_types.h"

namespace mm {

size_t build_compact_rects(const mm_rect* rects, uint32_t n_rects, const uint32_t* idx, std::vector<uint32_t>& out,
                           size_t* n_slow);

namespace {

void rect_box(const mm_rect& r, double lo[3], double hi[3]) {
    for (int a = 0; a < 3; ++a) {
        const double c[4] = {r.o[a], (double)r.o[a] + r.v[a], (double)r.o[a] + r.u[a],
                             (double)r.o[a] + r.v[a] + r.u[a]};
        lo[a] = *std::min_element(c, c + 4);
        hi[a] = *std::max_element(c, c + 4);
    }
}

inline uint32_t align16(uint32_t x) { return (x + 15u) & ~15u; }

inline uint32_t f2u(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
inline float u2f(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
inline int64_t fkey(float f) {  // monotone integer key of a non-NaN float (+-0 -> 0)
    const uint32_t u = f2u(f);
    return (u & 0x80000000u) ? -(int64_t)(u & 0x7FFFFFFFu) : (int64_t)u;
}
inline float from_key(int64_t k) { return k >= 0 ? u2f((uint32_t)k) : u2f(0x80000000u | (uint32_t)(-k)); }
inline float mul_rn(float x, float s) {
    volatile float a = x, b = s;
    return a * b;
}

// {Y : xlo <= RN(Y * s) <= xhi} for the compact record's X thresholds.  Y ->
// RN(Y * s) is monotone, so the set is an interval of floats; it holds 0
// (xlo <= 0 <= xhi, checked) and not +-inf (finite thresholds), and its ends
// are found by bisection over the float order.  The kernel's test
// ylo <= Y <= yhi is then the same predicate, bit for bit, for every Y
// (NaN fails both forms).
bool fold_thresholds(float s, float xlo, float xhi, float& ylo, float& yhi) {
    auto P = [&](float y) { const float p = mul_rn(y, s); return p >= xlo && p <= xhi; };
    if (!std::isfinite(s) || s == 0.0f || !std::isfinite(xlo) || !std::isfinite(xhi) || !P(0.0f) || P(INFINITY) ||
        P(-INFINITY))
        return false;
    int64_t lo = fkey(0.0f), hi = fkey(INFINITY);  // P(lo) true, P(hi) false
    while (hi - lo > 1) {
        const int64_t mid = lo + (hi - lo) / 2;
        if (P(from_key(mid))) lo = mid; else hi = mid;
    }
    yhi = from_key(lo);
    lo = fkey(-INFINITY); hi = fkey(0.0f);  // P(lo) false, P(hi) true
    while (hi - lo > 1) {
        const int64_t mid = lo + (hi - lo) / 2;
        if (P(from_key(mid))) hi = mid; else lo = mid;
    }
    ylo = from_key(hi);
    return true;
}

// rect_compact.cpp's 10-word record of each rect -> the 8-word grid record
// (mm_grid.h).  A record whose thresholds do not fold becomes SLOW.
uint32_t grid_records(const std::vector<uint32_t>& rc, uint32_t n_rects, std::vector<uint32_t>& out) {
    out.assign(8 * (size_t)n_rects, 0);
    uint32_t n_slow = 0;
    for (uint32_t k = 0; k < n_rects; ++k) {
        const uint32_t* w = &rc[10 * (size_t)k];
        uint32_t* g = &out[8 * (size_t)k];
        uint32_t kind = w[9] >> 30;
        const uint32_t ak = (w[9] >> 20) & 3u, av = (w[9] >> 22) & 3u, au = (w[9] >> 24) & 3u;
        if (kind == 0u) {
            float y1lo, y1hi, y2lo, y2hi;
            if (fold_thresholds(u2f(w[3]), u2f(w[5]), u2f(w[6]), y1lo, y1hi) &&
                fold_thresholds(u2f(w[4]), u2f(w[7]), u2f(w[8]), y2lo, y2hi)) {
                const bool swap = av > au;  // the lower axis first
                g[0] = w[0];
                g[1] = swap ? w[2] : w[1];
                g[2] = swap ? w[1] : w[2];
                g[3] = f2u(swap ? y2lo : y1lo);
                g[4] = f2u(swap ? y2hi : y1hi);
                g[5] = f2u(swap ? y1lo : y2lo);
                g[6] = f2u(swap ? y1hi : y2hi);
            } else {
                kind = 2u;
            }
        }
        if (kind == 1u) {  // never hits (not listed either)
            g[3] = g[5] = f2u(INFINITY);
            g[4] = g[6] = f2u(-INFINITY);
        }
        g[7] = k | ((kind == 0u ? ak : 0u) << 20) | (kind << 30);
        n_slow += kind == 2u;
    }
    return n_slow;
}

// Cells of size ~s over the scene box widened by eps = C * 2^-14, their lists
// and the image layout (recs and boxes are filled by the caller).
bool build_lists(const mm_rect* rects, uint32_t n_rects, const std::vector<uint32_t>& recs, const double smin[3],
                 const double smax[3], double C, double s, bool wide, bool merge_axes, GridHost& g,
                 std::string& why) {
    g.wide = wide;
    g.n_glob = 0;
    const double eps = C * 0x1p-14;
    long total = 1;
    auto set_axis = [&](int a, int n) {
        const float lo = std::nextafter((float)(smin[a] - eps), -INFINITY);
        const float hi = std::nextafter((float)(smax[a] + eps), INFINITY);
        g.n[a] = n;
        g.mn[a] = lo;
        g.mx[a] = hi;
        g.cell[a] = (float)(((double)hi - lo) / n);
        g.inv[a] = 1.0f / g.cell[a];
    };
    for (int a = 0; a < 3; ++a) {
        const double ext = (double)std::nextafter((float)(smax[a] + eps), INFINITY) -
                           std::nextafter((float)(smin[a] - eps), -INFINITY);
        set_axis(a, std::max(1, std::min(256, (int)std::floor(ext / s + 0.5))));
        total *= g.n[a];
    }
    if (total > (1l << 20)) { why = "more than 2^20 cells"; return false; }
    // the kernels' ray guard takes |o| <= 2^60 from the box (mm_trace.h ray_fast_ok_boxed)
    for (int a = 0; a < 3; ++a)
        if (!(std::fabs(g.mn[a]) <= 0x1p60f && std::fabs(g.mx[a]) <= 0x1p60f)) {
            why = "grid box past 2^60";
            return false;
        }
    // cell ranges of every rect (widened by eps), global rects
    struct Span { int i0[3], i1[3]; long cover; };
    std::vector<Span> span(n_rects);
    std::vector<uint8_t> skip(n_rects, 0), glob(n_rects, 0);
    auto spans = [&]() {
        for (uint32_t k = 0; k < n_rects; ++k) {
            skip[k] = (recs[10 * (size_t)k + 9] >> 30) == 1u;
            double lo[3], hi[3];
            rect_box(rects[k], lo, hi);
            Span& sp = span[k];
            sp.cover = 1;
            for (int a = 0; a < 3; ++a) {
                sp.i0[a] = std::max(0, (int)std::floor((lo[a] - eps - g.mn[a]) / g.cell[a]));
                sp.i1[a] = std::min(g.n[a] - 1, (int)std::floor((hi[a] + eps - g.mn[a]) / g.cell[a]));
                sp.cover *= std::max(0, sp.i1[a] - sp.i0[a] + 1);
            }
        }
    };
    spans();
    // An axis whose cells do not shorten the lists gets one cell: when the
    // listed rects span (nearly) all of its cells -- the maze's walls span its
    // whole height -- splitting it only adds cell steps (C3: 2.13 -> 1.91 cell
    // steps per query at the same 4.4 rect tests, scripts/grid_sim.c NY=1;
    // the search and its proof are the same for any cell counts).
    // Criterion: merging the axis does not lengthen the longest list among the
    // cells it merges (summed over the merged cells, within 10 %) -- the
    // maze's lower y cell is the space below the floor and lists a subset of
    // the walls above it, which a ray enters only to find that the floor hit
    // just below the boundary was its answer.
    for (int a = 0; merge_axes && a < 3; ++a) {
        if (g.n[a] == 1) continue;
        std::vector<uint32_t> split(total, 0), merged(total / g.n[a], 0);
        for (uint32_t k = 0; k < n_rects; ++k) {
            const Span& sp = span[k];
            if (skip[k] || sp.cover * 2 > total) continue;  // (the global rects are tested by every query)
            for (int z = sp.i0[2]; z <= sp.i1[2]; ++z)
                for (int y = sp.i0[1]; y <= sp.i1[1]; ++y)
                    for (int x = sp.i0[0]; x <= sp.i1[0]; ++x) {
                        split[((long)z * g.n[1] + y) * g.n[0] + x]++;
                        const int q[3] = {x, y, z};
                        if (q[a] != sp.i0[a]) continue;  // once per merged cell
                        int m[3] = {x, y, z};
                        m[a] = 0;
                        int nm[3] = {g.n[0], g.n[1], g.n[2]};
                        nm[a] = 1;
                        merged[((long)m[2] * nm[1] + m[1]) * nm[0] + m[0]]++;
                    }
        }
        double longest = 0.0, union_len = 0.0;
        for (long c = 0; c < total; ++c) {
            const int q[3] = {(int)(c % g.n[0]), (int)((c / g.n[0]) % g.n[1]), (int)(c / ((long)g.n[0] * g.n[1]))};
            if (q[a] != 0) continue;
            int step[3] = {1, g.n[0], g.n[0] * g.n[1]};
            uint32_t mx = 0;
            for (int i = 0; i < g.n[a]; ++i) mx = std::max(mx, split[c + (long)i * step[a]]);
            longest += mx;
            int m[3] = {q[0], q[1], q[2]};
            int nm[3] = {g.n[0], g.n[1], g.n[2]};
            nm[a] = 1;
            union_len += merged[((long)m[2] * nm[1] + m[1]) * nm[0] + m[0]];
        }
        if (union_len <= 1.1 * longest) {
            total /= g.n[a];
            set_axis(a, 1);
            spans();
        }
    }
    std::vector<std::pair<long, uint32_t>> big;
    for (uint32_t k = 0; k < n_rects; ++k)
        if (!skip[k] && span[k].cover * 2 > total) big.push_back({span[k].cover, k});
    std::sort(big.begin(), big.end(), [](auto& x, auto& y) { return x.first > y.first; });
    for (size_t i = 0; i < big.size() && i < 4; ++i) {
        glob[big[i].second] = 1;
        g.glob[g.n_glob++] = big[i].second;
    }
    // counting sort of (cell, rect)
    std::vector<uint32_t> cnt(total + 1, 0);
    std::vector<uint16_t> flat;
    for (int pass = 0; pass < 2; ++pass) {
        std::vector<uint32_t> cur(pass ? cnt : std::vector<uint32_t>());
        for (uint32_t k = 0; k < n_rects; ++k) {
            if (skip[k] || glob[k]) continue;
            const Span& sp = span[k];
            for (int z = sp.i0[2]; z <= sp.i1[2]; ++z)
                for (int y = sp.i0[1]; y <= sp.i1[1]; ++y)
                    for (int x = sp.i0[0]; x <= sp.i1[0]; ++x) {
                        const long c = ((long)z * g.n[1] + y) * g.n[0] + x;
                        if (pass == 0) cnt[c + 1]++;
                        else flat[cur[c]++] = (uint16_t)k;
                    }
        }
        if (pass == 0) {
            for (long c = 0; c < total; ++c) {
                if (cnt[c + 1] >= 1024u) { why = "a cell lists 1024 or more rects"; return false; }
                cnt[c + 1] += cnt[c];
            }
            flat.assign(cnt[total], 0);
        }
    }
    if (!wide) {  // plain 32-bit cell words: first entry | count << 22
        if (cnt[total] >= (1u << 22)) { why = "more than 2^22 list entries"; return false; }
        g.n_list = cnt[total];
        g.off_list = align16(4u * (uint32_t)total);
        g.off_recs = align16(g.off_list + 2u * g.n_list);
        g.off_box = align16(g.off_recs + 32u * n_rects);
        g.bytes = align16(g.off_box + 24u * n_rects);
        g.image.assign(g.bytes, 0);
        for (long c = 0; c < total; ++c) {
            const uint32_t w = cnt[c] | ((cnt[c + 1] - cnt[c]) << 22);
            std::memcpy(&g.image[4 * (size_t)c], &w, 4);
        }
        if (!flat.empty()) std::memcpy(&g.image[g.off_list], flat.data(), 2 * flat.size());
        return true;
    }
    // Face ranges.  A query that steps into cell c through face f has tested
    // every entry of the previous cell's list (by induction: the first cell's
    // whole list, then each cell's range plus what the cell before it listed),
    // so it need only test the entries of c that the neighbour across f does
    // not list.  Each list is put in circular order around the cell (angle of
    // the rect's box centre in the plane of the two axes with the most cells:
    // in a maze the entries a neighbour shares are then adjacent) and stored
    // with its first m - 1 entries repeated, so the entries to test form one
    // range [start, start + len) for every face.  Face f = 2a + (0 when the
    // query moved +a, 1 when it moved -a); the neighbour is on the -a / +a side.
    int pl[3] = {0, 1, 2};
    std::stable_sort(pl, pl + 3, [&](int x, int y) { return g.n[x] > g.n[y]; });
    const int p0 = pl[0], p1 = pl[1];
    std::vector<uint16_t> ext;
    std::vector<uint64_t> words(total);
    auto listed = [&](long c, uint16_t k) {
        for (uint32_t q = cnt[c]; q < cnt[c + 1]; ++q)
            if (flat[q] == k) return true;
        return false;
    };
    for (long c = 0; c < total; ++c) {
        const int ic[3] = {(int)(c % g.n[0]), (int)((c / g.n[0]) % g.n[1]), (int)(c / ((long)g.n[0] * g.n[1]))};
        const uint32_t m = cnt[c + 1] - cnt[c];
        const uint64_t base = ext.size();
        if (base + 2 * (uint64_t)m >= (1u << 22)) { why = "more than 2^22 list entries"; return false; }
        if (m > 7) {  // whole list for every face
            for (uint32_t q = cnt[c]; q < cnt[c + 1]; ++q) ext.push_back(flat[q]);
            words[c] = (1ull << 63) | ((uint64_t)m << 22) | base;
            continue;
        }
        std::vector<std::pair<double, uint16_t>> e;
        for (uint32_t q = cnt[c]; q < cnt[c + 1]; ++q) {
            double lo[3], hi[3];
            rect_box(rects[flat[q]], lo, hi);
            const double c0 = g.mn[p0] + (ic[p0] + 0.5) * (double)g.cell[p0];
            const double c1 = g.mn[p1] + (ic[p1] + 0.5) * (double)g.cell[p1];
            e.push_back({std::atan2(0.5 * (lo[p1] + hi[p1]) - c1, 0.5 * (lo[p0] + hi[p0]) - c0), flat[q]});
        }
        std::stable_sort(e.begin(), e.end(), [](auto& x, auto& y) { return x.first < y.first; });
        for (uint32_t i = 0; i < m; ++i) ext.push_back(e[i].second);
        for (uint32_t i = 0; i + 1 < m; ++i) ext.push_back(e[i].second);
        uint64_t w = base | ((uint64_t)m << 22);
        for (int f = 0; f < 6; ++f) {
            const int ax = f >> 1;
            int nb[3] = {ic[0], ic[1], ic[2]};
            nb[ax] += (f & 1) ? 1 : -1;
            const bool inside = nb[ax] >= 0 && nb[ax] < g.n[ax];
            const long cn = ((long)nb[2] * g.n[1] + nb[1]) * g.n[0] + nb[0];
            bool keep[8];
            uint32_t nk = 0;
            for (uint32_t i = 0; i < m; ++i) nk += keep[i] = !(inside && listed(cn, e[i].second));
            uint32_t bs = 0, bl = nk ? m : 0;
            for (uint32_t st = 0; st < m && nk; ++st) {
                if (!keep[st]) continue;
                uint32_t len = 0;
                for (uint32_t i = 0; i < m; ++i)
                    if (keep[i]) len = std::max(len, (i + m - st) % m + 1);
                if (len < bl) { bl = len; bs = st; }
            }
            w |= (uint64_t)(bs | (bl << 3)) << (25 + 6 * f);
        }
        words[c] = w;
    }
    g.n_list = (uint32_t)ext.size();
    g.off_list = align16(8u * (uint32_t)total);
    g.off_recs = align16(g.off_list + 2u * g.n_list);
    g.off_box = align16(g.off_recs + 32u * n_rects);
    g.bytes = align16(g.off_box + 24u * n_rects);
    g.image.assign(g.bytes, 0);
    std::memcpy(&g.image[0], words.data(), 8 * (size_t)total);
    if (!ext.empty()) std::memcpy(&g.image[g.off_list], ext.data(), 2 * ext.size());
    return true;
}

}  // namespace

// Returns false (with a reason) when the scene does not suit the search (too
// many rects or cells).  The cell size starts at the scene's typical rect
// extent and grows by 1.25x until the cells + lists (the part the kernel keeps
// in LDS) fit index_budget bytes.
bool build_grid(const mm_rect* rects, uint32_t n_rects, const mm_node* nodes, uint32_t n_nodes,
                const uint32_t* idx, size_t index_budget, GridHost& g, std::string& why, bool merge_axes,
                double cell_scale, bool wide) {
    if (n_rects == 0 || n_rects > 65535) { why = "rect count outside 1..65535"; return false; }
    std::vector<uint32_t> ident(n_rects), recs;
    for (uint32_t k = 0; k < n_rects; ++k) ident[k] = k;
    size_t n_slow = 0;
    build_compact_rects(rects, n_rects, ident.data(), recs, &n_slow);
    // scene box, C, eps, cell size
    double smin[3] = {INFINITY, INFINITY, INFINITY}, smax[3] = {-INFINITY, -INFINITY, -INFINITY}, C = 1.0;
    std::vector<double> ext2;
    for (uint32_t k = 0; k < n_rects; ++k) {
        double lo[3], hi[3];
        rect_box(rects[k], lo, hi);
        double e[3];
        for (int a = 0; a < 3; ++a) {
            if (!std::isfinite(lo[a]) || !std::isfinite(hi[a])) { why = "non-finite rect"; return false; }
            smin[a] = std::min(smin[a], lo[a]);
            smax[a] = std::max(smax[a], hi[a]);
            C = std::max(C, std::max(std::fabs(lo[a]), std::fabs(hi[a])));
            e[a] = hi[a] - lo[a];
        }
        std::sort(e, e + 3);
        if (e[1] > 0.0) ext2.push_back(e[1]);
    }
    if (ext2.empty()) { why = "no rect with area"; return false; }
    std::nth_element(ext2.begin(), ext2.begin() + ext2.size() / 2, ext2.end());
    // grid records and their threshold classes do not depend on the cells
    std::vector<uint32_t> grecs;
    const uint32_t n_slow_g = grid_records(recs, n_rects, grecs);
    std::vector<uint32_t> cls;  // 4 words per class
    std::vector<uint32_t> cls_of(n_rects, 0);
    bool classes_ok = n_slow_g == 0;
    // compact (maze) records keep y as the first in-plane axis: a z-normal
    // record's (v, u) = (x, y) is stored as (y, x) -- its o_v / o_u and its
    // threshold pairs swapped -- so the kernel reads y for the first in-plane
    // axis of every listed record without a select (mm_grid.h grid_rect)
    auto y_first = [&](uint32_t k) { return ((grecs[8 * (size_t)k + 7] >> 20) & 3u) == 2u; };
    for (uint32_t k = 0; k < n_rects && classes_ok; ++k) {
        const uint32_t* g8 = &grecs[8 * (size_t)k + 3];
        uint32_t t[4] = {g8[0], g8[1], g8[2], g8[3]};
        if (y_first(k)) { std::swap(t[0], t[2]); std::swap(t[1], t[3]); }
        uint32_t c = 0;
        while (c < cls.size() / 4 && !std::equal(t, t + 4, &cls[4 * c])) ++c;
        if (c == cls.size() / 4) {
            if (c == kMaxClasses) { classes_ok = false; break; }
            cls.insert(cls.end(), t, t + 4);
        }
        cls_of[k] = c;
    }
    // Maze forms: one y cell, no SLOW record, every listed (non-global) record
    // normal to x or z, and few distinct folded threshold tuples (C3: 22,
    // N=64: 26 -- the walls come in a handful of lengths and heights)
    auto maze_form = [&](const GridHost& gg) {
        // (the lists name rect k as 8 k in u16 entries: mm_grid.h rec_words)
        if (gg.n[1] != 1 || !classes_ok || n_rects > 8191u) return false;
        for (uint32_t k = 0; k < n_rects; ++k) {
            const uint32_t meta = grecs[8 * (size_t)k + 7];
            const bool global = std::find(gg.glob, gg.glob + gg.n_glob, k) != gg.glob + gg.n_glob;
            if (!global && (meta >> 30) == 0u && ((meta >> 20) & 3u) == 1u) return false;
        }
        return true;
    };
    // compact records: the class table (kMaxClasses x 16 B), then per rect o_k, o_v, o_u (y first, above),
    // class << 4 | axis << 20 | kind << 30 (the rect index, implied by the record's position, is dropped;
    // the class's byte offset in the table is meta & 0x3F0, and a listed record's axis is x iff meta <
    // 2^20); then the leaf boxes.  The table comes first so that, staged at LDS address 0, it and the
    // records sit at compile-time offsets (mm_grid.h, trace_kernels.hip stage_and_run).
    auto compact_layout = [&](GridHost& gg) {
        gg.off_class = gg.off_data = align16(gg.off_list + 2u * gg.n_list);
        gg.off_recs = gg.off_class + kGridClassBytes;
        gg.off_box = align16(gg.off_recs + 16u * n_rects);
        gg.bytes = align16(gg.off_box + 24u * n_rects);
    };
    double s = ext2[ext2.size() / 2] * cell_scale;
    for (int attempt = 0; attempt < 24; ++attempt, s *= 1.25) {
        // 64-bit cell words with face ranges where the whole image fits the
        // budget, else plain 32-bit words at the same cell size, before
        // coarser cells (the kernel variant for wide words stages all of it)
        if (wide && build_lists(rects, n_rects, recs, smin, smax, C, s, true, merge_axes, g, why)) {
            const bool mf = maze_form(g);
            if (mf) compact_layout(g);
            // the maze forms' walk decodes face ranges only (no whole-list cells, mm_grid.h): a maze grid
            // with a cell of more than 7 entries takes plain words
            bool whole = false;
            for (size_t c = 0; mf && c < (size_t)g.n[0] * g.n[1] * g.n[2]; ++c)
                whole |= (g.image[8 * c + 7] & 0x80u) != 0;
            if (g.bytes <= index_budget && !whole) break;
        }
        if (build_lists(rects, n_rects, recs, smin, smax, C, s, false, merge_axes, g, why) &&
            g.off_recs <= index_budget)
            break;
        if (attempt == 23) { why = "no grid index fits the LDS budget"; return false; }
    }
    g.n_slow = n_slow_g;
    g.flat_ok = maze_form(g);
    if (g.wide && g.flat_ok) {
        // The maze forms never step y, so their x-entry faces' ranges move into the y faces' slots:
        // +x -> bits 37-42, -x -> 43-48, beside +z / -z at 49-54 / 55-60 -- every range the walk reads
        // is then in the word's high half (one 32-bit shift, mm_grid.h grid_search)
        for (size_t c = 0; c < (size_t)g.n[0] * g.n[1] * g.n[2]; ++c) {
            uint64_t w;
            std::memcpy(&w, &g.image[8 * c], 8);
            const uint64_t xf = (w >> 25) & 0xFFFull;
            w = (w & ~(0xFFFull << 37)) | (xf << 37);
            std::memcpy(&g.image[8 * c], &w, 8);
        }
    }
    g.slab = false;
    if (g.n_glob == 2) {
        const uint32_t m0 = grecs[8 * (size_t)g.glob[0] + 7], m1 = grecs[8 * (size_t)g.glob[1] + 7];
        const bool y_fast = (m0 >> 30) == 0u && (m1 >> 30) == 0u && ((m0 >> 20) & 3u) == 1u && ((m1 >> 20) & 3u) == 1u;
        float y0, y1;
        std::memcpy(&y0, &grecs[8 * (size_t)g.glob[0]], 4);
        std::memcpy(&y1, &grecs[8 * (size_t)g.glob[1]], 4);
        if (y_fast && y0 != y1 && std::isfinite(y0) && std::isfinite(y1)) {
            if (y1 < y0) { std::swap(g.glob[0], g.glob[1]); std::swap(y0, y1); }
            g.slab = true;
            g.slab_y[0] = y0;
            g.slab_y[1] = y1;
        }
    }
    if (g.flat_ok) {
        g.n_class = (uint32_t)cls.size() / 4;
        compact_layout(g);
        g.image.resize(g.bytes);
        std::memset(&g.image[g.off_recs], 0, g.bytes - g.off_recs);
        for (uint32_t k = 0; k < n_rects; ++k) {
            const uint32_t* w = &grecs[8 * (size_t)k];
            const uint32_t meta = (w[7] & (3u << 20)) | (cls_of[k] << 4) | (w[7] & (3u << 30));
            const uint32_t r[4] = {w[0], y_first(k) ? w[2] : w[1], y_first(k) ? w[1] : w[2], meta};
            std::memcpy(&g.image[g.off_recs + 16u * k], r, 16);
        }
        std::memcpy(&g.image[g.off_class], cls.data(), 4 * cls.size());
        // list entries name rect k as 8 k (record k's byte offset 16 k is then one pairable add)
        for (uint32_t i = 0; i < g.n_list; ++i) {
            uint16_t e;
            std::memcpy(&e, &g.image[g.off_list + 2u * i], 2);
            e = (uint16_t)(8u * e);
            std::memcpy(&g.image[g.off_list + 2u * i], &e, 2);
        }
    } else {
        g.off_class = 0;
        g.off_data = g.off_recs;
        g.off_box = align16(g.off_recs + 32u * n_rects);
        g.bytes = align16(g.off_box + 24u * n_rects);
        g.image.resize(g.bytes);
        std::memcpy(&g.image[g.off_recs], grecs.data(), 32u * (size_t)n_rects);
    }
    // the reference leaf box of every rect; a rect in no leaf gets an empty
    // box, so a certificate for it always fails (the reference never tests it)
    std::vector<float> box(6 * (size_t)n_rects);
    for (uint32_t k = 0; k < n_rects; ++k) {
        const float e[6] = {INFINITY, -INFINITY, INFINITY, -INFINITY, INFINITY, -INFINITY};
        std::memcpy(&box[6 * (size_t)k], e, sizeof e);
    }
    for (uint32_t i = 0; i < n_nodes; ++i) {
        const mm_node& nd = nodes[i];
        if (nd.count == 0) continue;
        for (uint32_t j = 0; j < nd.count; ++j) {
            const uint32_t k = idx[nd.left_first + j];
            const float b[6] = {nd.mn[0], nd.mx[0], nd.mn[1], nd.mx[1], nd.mn[2], nd.mx[2]};
            std::memcpy(&box[6 * (size_t)k], b, sizeof b);
        }
    }
    std::memcpy(&g.image[g.off_box], box.data(), 24u * (size_t)n_rects);
    return true;
}

}  // namespace mm
