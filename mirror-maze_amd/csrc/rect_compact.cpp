// rect_compact.cpp — host construction of the compact, leaf-ordered rect
// records the LDS-resident traversal tests (mm_trace.h: rect_test_compact).
//
// For an axis-aligned rect whose side v lies on axis iv, side u on axis iu and
// whose reference normal n = normalize(cross(v, u)) (shaders.metal:52) is
// EXACTLY +-1 on the third axis k and +-0 elsewhere, ray_rect_intersect
// (shaders.metal:51-67) reduces, operation for operation, to
//     a  = (o_k - ori_k) / d_k                    (n_k = +-1: the signs cancel)
//     X1 = ((ori_iv - o_iv) + a*d_iv) * v_iv      (= dot(rect_vect, v) up to the
//     X2 = ((ori_iu - o_iu) + a*d_iu) * u_iu       sign of a zero)
//     hit  <=>  0 <= RN(X1/|v|) <= |v|  &&  0 <= RN(X2/|u|) <= |u|
//               && d_k != 0 && a > 0.1 && a < t
// and because x -> RN(x/|v|) is monotone, 0 <= RN(X1/|v|) <= |v| is exactly
// X1lo <= X1 <= X1hi for two per-rect floats found here by bisection over the
// float ordering with IEEE division (the device's division is the same IEEE
// operation, so the thresholds are exact).  |v| = sqrt(dot(v, v)) and n are
// computed with the kernel's own operation order.  Rects that do not meet the
// conditions are marked SLOW (the kernel runs the general test on them);
// zero-length rects (n = NaN, never hit, shaders.metal:63) are marked SKIP.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "mm_types.h"

namespace mm {

namespace {

inline uint32_t f2u(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
inline float u2f(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
// monotone integer key of a non-NaN float (-0 and +0 both map to 0)
inline int64_t fkey(float f) {
    const uint32_t u = f2u(f);
    return (u & 0x80000000u) ? -(int64_t)(u & 0x7FFFFFFFu) : (int64_t)u;
}
inline float from_key(int64_t k) { return k >= 0 ? u2f((uint32_t)k) : u2f(0x80000000u | (uint32_t)(-k)); }
inline float div_rn(float x, float l) {
    volatile float a = x, b = l;
    return a / b;
}

struct V3 { float x, y, z; };
inline float dot3(V3 a, V3 b) {
    float s = a.x * b.x;
    s = s + a.y * b.y;
    return s + a.z * b.z;
}
inline float comp(V3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }

// largest x with RN(x/l) <= l
float x_hi(float l) {
    int64_t lo = fkey(0.0f), hi = fkey(INFINITY);  // P(lo) true, P(hi) false
    while (hi - lo > 1) {
        const int64_t mid = lo + (hi - lo) / 2;
        if (div_rn(from_key(mid), l) <= l) lo = mid; else hi = mid;
    }
    return from_key(lo);
}
// smallest x with RN(x/l) >= 0 (a -0 quotient counts as >= 0)
float x_lo(float l) {
    int64_t lo = fkey(-INFINITY), hi = fkey(-0.0f);  // Q(lo) false, Q(hi) true
    while (hi - lo > 1) {
        const int64_t mid = lo + (hi - lo) / 2;
        if (div_rn(from_key(mid), l) >= 0.0f) hi = mid; else lo = mid;
    }
    return from_key(hi);
}

int single_axis(V3 v) {
    const int nz = (v.x != 0.0f) + (v.y != 0.0f) + (v.z != 0.0f);
    if (nz != 1) return -1;
    return v.x != 0.0f ? 0 : (v.y != 0.0f ? 1 : 2);
}

}  // namespace

// Record layout (10 x u32 per slot, slot = position in the BVH index array):
//   0 o_k  1 o_iv  2 o_iu  3 v_iv  4 u_iu  5 X1lo  6 X1hi  7 X2lo  8 X2hi
//   9 k | k_axis << 20 | iv << 22 | iu << 24 | kind << 30
// kind: 0 FAST, 1 SKIP (zero-length: never hits), 2 SLOW (general test).
constexpr uint32_t kRecWords = 10;

size_t build_compact_rects(const mm_rect* rects, uint32_t n_rects, const uint32_t* idx, std::vector<uint32_t>& out,
                           size_t* n_slow) {
    std::vector<uint32_t> per(kRecWords * (size_t)n_rects, 0);
    size_t n_fast = 0, slow = 0;
    for (uint32_t k = 0; k < n_rects; ++k) {
        const mm_rect& r = rects[k];
        const V3 o{r.o[0], r.o[1], r.o[2]}, v{r.v[0], r.v[1], r.v[2]}, u{r.u[0], r.u[1], r.u[2]};
        uint32_t* w = &per[kRecWords * (size_t)k];
        uint32_t kind = 2, ak = 0, av = 0, au = 0;
        // n = normalize(cross(v, u)) in the kernel's order
        const V3 c{u.z * v.y - u.y * v.z, u.x * v.z - u.z * v.x, u.y * v.x - u.x * v.y};
        const float rs = 1.0f / std::sqrt(dot3(c, c));
        const V3 n{rs * c.x, rs * c.y, rs * c.z};
        const float lv = std::sqrt(dot3(v, v)), lu = std::sqrt(dot3(u, u));
        if (std::isnan(n.x) || std::isnan(n.y) || std::isnan(n.z)) {
            kind = 1;  // zero-length wall: nc is NaN, `nc != 0` true but a = NaN fails a > 0.1
            // Also a valid FAST record that can never hit (thresholds lo = +inf,
            // hi = -inf fail for every x1, NaN included), for the branch-free
            // leaf test of scenes without SLOW records (rect_test_compact_lean).
            const float never[9] = {0.0f, 0.0f, 0.0f, 1.0f, 1.0f, INFINITY, -INFINITY, INFINITY, -INFINITY};
            for (int j = 0; j < 9; ++j) w[j] = f2u(never[j]);
            ak = 0; av = 1; au = 2;
        } else {
            const int iv = single_axis(v), iu = single_axis(u);
            if (iv >= 0 && iu >= 0 && iv != iu) {
                const int kk = 3 - iv - iu;
                const float nk = comp(n, kk);
                bool ok = (nk == 1.0f || nk == -1.0f);
                for (int a = 0; a < 3; ++a)
                    if (a != kk && comp(n, a) != 0.0f) ok = false;
                ok = ok && std::isfinite(lv) && std::isfinite(lu) && lv > 0.0f && lu > 0.0f;
                if (ok) {
                    kind = 0;
                    ak = (uint32_t)kk; av = (uint32_t)iv; au = (uint32_t)iu;
                    const float vals[9] = {comp(o, kk), comp(o, iv), comp(o, iu), comp(v, iv), comp(u, iu),
                                           x_lo(lv), x_hi(lv), x_lo(lu), x_hi(lu)};
                    for (int j = 0; j < 9; ++j) w[j] = f2u(vals[j]);
                }
            }
        }
        if (kind == 0) ++n_fast;
        if (kind == 2) ++slow;
        w[9] = (k & 0xFFFFFu) | (ak << 20) | (av << 22) | (au << 24) | (kind << 30);
    }
    out.assign(kRecWords * (size_t)n_rects, 0);
    for (uint32_t s = 0; s < n_rects; ++s)
        std::memcpy(&out[kRecWords * (size_t)s], &per[kRecWords * (size_t)idx[s]], kRecWords * 4);
    if (n_slow) *n_slow = slow;
    return n_fast;
}

}  // namespace mm
