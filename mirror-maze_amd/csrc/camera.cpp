// camera.cpp — the reference's interactive camera and player collision
// (SURVEY.md §8f item 4), restated in C++ behind the C ABI of mm_scene.h so an
// offline sequence (a fly-through) or a front end can drive the camera the way
// the reference's event loop does:
//
//   quat_mult          src/maths.rs:165-178   v' = q^-1 (v, 0) q  (quat_dot twice)
//   update_quat_angle  src/maths.rs:159-162   keep the axis, set the half angle
//   aabb::intersect    src/main.rs:237-245    closed-interval box overlap
//   check_collision    src/main.rs:265-291    recursive BVH walk, first leaf hit
//   player step        src/main.rs:786-842    WASD moves of 5/fps along the
//                                             rotated axes, undone on collision;
//                                             mouse deltaX turns half_theta
//                                             (main.rs:922-924)
//
// f32 arithmetic in the reference's operation order (-ffp-contract=off);
// sin/acos are evaluated in double and rounded once, as mm_calculate_quaternion
// does (Rust's f32 sin/acos go to the platform libm, which is not correctly
// rounded everywhere), so results are platform independent.
#include <cmath>
#include <cstdint>
#include <vector>

#include "mm_scene.h"

namespace {

struct V3 { float x, y, z; };
struct Q4 { float x, y, z, w; };

V3 add(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
V3 sub(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
V3 scale(V3 v, float f) { return V3{v.x * f, v.y * f, v.z * f}; }
float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }  // maths.rs:105-108, left to right
V3 cross(V3 a, V3 b) {                                                // maths.rs:130-136
    return V3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

// quat_dot (maths.rs:169-173): s = w1 w2 - v1.v2; v = v1 x v2 + (v2 w1 + v1 w2)
Q4 quat_dot(Q4 a, Q4 b) {
    const V3 va{a.x, a.y, a.z}, vb{b.x, b.y, b.z};
    const float s = a.w * b.w - dot(va, vb);
    const V3 v = add(cross(va, vb), add(scale(vb, a.w), scale(va, b.w)));
    return Q4{v.x, v.y, v.z, s};
}

V3 quat_mult(V3 v, Q4 q) {
    const Q4 inv{-q.x, -q.y, -q.z, q.w};
    const Q4 r = quat_dot(quat_dot(inv, Q4{v.x, v.y, v.z, 0.0f}), q);
    return V3{r.x, r.y, r.z};
}

bool overlap(const float amn[3], const float amx[3], const float bmn[3], const float bmx[3]) {
    return amn[0] <= bmx[0] && amx[0] >= bmn[0] && amn[1] <= bmx[1] && amx[1] >= bmn[1] && amn[2] <= bmx[2] &&
           amx[2] >= bmn[2];
}

// check_collision: a node with exactly one plane is a leaf; any other node is
// walked into left_first and left_first + 1, as the reference does.  The
// reference indexes out of bounds (a panic) for a leaf of >= 2 planes whose
// left_first + 1 is past the array; here that is an error (-2).
int collide(const mm_node* nodes, uint32_t n_nodes, const float mn[3], const float mx[3], uint32_t i,
            uint32_t depth) {
    if (i >= n_nodes || depth > 4096) return -2;
    const mm_node& nd = nodes[i];
    if (nd.count == 1) return overlap(mn, mx, nd.mn, nd.mx) ? (int)i : -1;
    if (!overlap(mn, mx, nd.mn, nd.mx)) return -1;
    const int l = collide(nodes, n_nodes, mn, mx, nd.left_first, depth + 1);
    if (l != -1) return l;
    return collide(nodes, n_nodes, mn, mx, nd.left_first + 1, depth + 1);
}

}  // namespace

extern "C" {

void mm_quat_mult(const float v[3], const float q[4], float out[3]) {
    const V3 r = quat_mult(V3{v[0], v[1], v[2]}, Q4{q[0], q[1], q[2], q[3]});
    out[0] = r.x;
    out[1] = r.y;
    out[2] = r.z;
}

void mm_update_quat_angle(const float q[4], float theta, float out[4]) {
    const float ratio = (float)std::sin((double)theta) / (float)std::sin((double)(float)std::acos((double)q[3]));
    out[0] = q[0] * ratio;
    out[1] = q[1] * ratio;
    out[2] = q[2] * ratio;
    out[3] = (float)std::cos((double)theta);
}

int mm_check_collision(const mm_node* nodes, uint32_t n_nodes, const float bmin[3], const float bmax[3]) {
    if (!nodes || n_nodes == 0 || !bmin || !bmax) return -2;
    return collide(nodes, n_nodes, bmin, bmax, 0, 0);
}

int mm_player_init(const float quat[4], mm_player* p) {
    if (!quat || !p) return MM_ERR_INVALID;
    p->center[0] = -5.0f;  // main.rs:732-733
    p->center[1] = 0.0f;
    p->center[2] = -45.0f;
    for (int i = 0; i < 4; ++i) p->quat[i] = quat[i];
    p->half_theta = (float)std::acos((double)quat[3]);  // main.rs:741
    p->fps = 60.0f;                                      // main.rs:760
    return MM_OK;
}

int mm_player_step(mm_player* p, const uint16_t* keys, uint32_t n_keys, const float* mouse_dx, uint32_t n_mouse,
                   const mm_node* nodes, uint32_t n_nodes, uint32_t* flags) {
    if (!p || (n_keys && !keys) || (n_mouse && !mouse_dx) || !nodes || n_nodes == 0) return MM_ERR_INVALID;
    uint32_t f = 0;
    // The reference's frame: move by the held keys with the current rotation,
    // undo the move on collision, then apply the rotation the previous frame's
    // MouseMoved events set up (main.rs:786-838; events 922-924 run after the
    // frame is encoded, so callers pass the previous frame's deltaX values).
    const V3 prev{p->center[0], p->center[1], p->center[2]};
    V3 c = prev;
    const Q4 q{p->quat[0], p->quat[1], p->quat[2], p->quat[3]};
    const float step = 5.0f / p->fps;
    for (uint32_t i = 0; i < n_keys; ++i) {  // main.rs:787-813, in keys_pressed order
        switch (keys[i]) {
            case 0: c = sub(c, quat_mult(V3{step, 0.0f, 0.0f}, q)); break;   // A
            case 1: c = sub(c, quat_mult(V3{0.0f, 0.0f, step}, q)); break;   // S
            case 2: c = add(c, quat_mult(V3{step, 0.0f, 0.0f}, q)); break;   // D
            case 13: c = add(c, quat_mult(V3{0.0f, 0.0f, step}, q)); break;  // W
            default: break;
        }
    }
    const V3 diag{0.5f, 0.2f, 0.5f};  // player_diag, main.rs:738
    const V3 mn = sub(c, diag), mx = add(c, diag);
    const float bmn[3] = {mn.x, mn.y, mn.z}, bmx[3] = {mx.x, mx.y, mx.z};
    const int hit = collide(nodes, n_nodes, bmn, bmx, 0, 0);
    if (hit == -2) return MM_ERR_INVALID;
    if (hit >= 0) {  // main.rs:816-825
        c = prev;
        f |= MM_PLAYER_COLLIDED;
    }
    p->center[0] = c.x;
    p->center[1] = c.y;
    p->center[2] = c.z;
    if (n_mouse) {
        const float pi = 3.14159265358979323846f;  // std::f32::consts::PI
        float h = p->half_theta;
        for (uint32_t i = 0; i < n_mouse; ++i) {  // (h - dx / 512).rem_euclid(PI), one event at a time
            const float x = h - mouse_dx[i] / 512.0f;
            float r = std::fmod(x, pi);  // exact, like Rust's %
            if (r < 0.0f) r = r + pi;
            h = r;
        }
        p->half_theta = h;
        float nq[4];
        mm_update_quat_angle(p->quat, h, nq);
        if (std::isnan(nq[0]) || std::isnan(nq[1]) || std::isnan(nq[2]) || std::isnan(nq[3])) {
            f |= MM_PLAYER_NAN_QUAT;  // the reference prints "Help!" and keeps the old quaternion
        } else {
            for (int i = 0; i < 4; ++i) p->quat[i] = nq[i];
            f |= MM_PLAYER_ROTATED;
        }
    }
    if (flags) *flags = f;
    return MM_OK;
}

int mm_player_uniform(const mm_player* p, float view_w, float view_h, uint32_t time, mm_uniform* u) {
    if (!p || !u) return MM_ERR_INVALID;
    mm_uniform_default(view_w, view_h, time, u);
    for (int i = 0; i < 3; ++i) u->cam.center[i] = p->center[i];
    for (int i = 0; i < 4; ++i) u->cam.quat[i] = p->quat[i];
    return MM_OK;
}

}  // extern "C"
