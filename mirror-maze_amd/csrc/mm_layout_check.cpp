// mm_layout_check.cpp — compile-time proof that the C ABI structs are
// byte-identical to the reference's #[repr(C)] types / Metal structs.
#include <cstddef>

#include "mm_types.h"

// Plane (src/main.rs:51-58) / rect (src/shaders.metal:19-24): 4 x packed_float3
static_assert(sizeof(mm_rect) == 48, "Plane is 48 B");
static_assert(offsetof(mm_rect, v) == 12 && offsetof(mm_rect, u) == 24 && offsetof(mm_rect, color) == 36,
              "Plane field offsets");
// BVHNode (src/main.rs:74-81) / bvh_node (src/shaders.metal:30-35)
static_assert(sizeof(mm_node) == 32, "BVHNode is 32 B");
static_assert(offsetof(mm_node, mx) == 12 && offsetof(mm_node, left_first) == 24 && offsetof(mm_node, count) == 28,
              "BVHNode field offsets");
// Camera (src/main.rs:32-39) / camera (src/shaders.metal:37-42)
static_assert(sizeof(mm_camera) == 40, "Camera is 40 B");
static_assert(offsetof(mm_camera, focal) == 12 && offsetof(mm_camera, quat) == 16 && offsetof(mm_camera, viewport) == 32,
              "Camera field offsets");
// Uniform (src/main.rs:41-49) / uni (src/shaders.metal:237-243)
static_assert(sizeof(mm_uniform) == 56, "Uniform is 56 B");
static_assert(offsetof(mm_uniform, view_w) == 40 && offsetof(mm_uniform, view_h) == 44 &&
                  offsetof(mm_uniform, chunk_w) == 48 && offsetof(mm_uniform, time) == 52,
              "Uniform field offsets");
static_assert(sizeof(mm_ext) == 24, "mm_ext is 24 B");
static_assert(sizeof(mm_stats) == 32, "mm_stats is 32 B");

extern "C" int mm_layout_ok(void) { return 1; }
