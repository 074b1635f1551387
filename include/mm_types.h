/*
 * mm_types.h — plain-old-data types shared by the HIP path (mm_api.h) and the
 * host scene builder (mm_scene.h).
 *
 * Every struct is byte-identical to the reference's `#[repr(C)]` Rust type and
 * to the Metal struct the kernel reads, so a Rust host could pass its own
 * `Vec<Plane>` / `Vec<BVHNode>` / `Uniform` straight through an `extern "C"`
 * block.  Sizes and offsets are pinned by static asserts in
 * mirror-maze_amd/csrc/mm_layout_check.cpp and by tests/test_layout.py.
 */
#ifndef MM_TYPES_H
#define MM_TYPES_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* == Plane   (src/main.rs:51-58)   == rect     (src/shaders.metal:19-24)
 *    origin, side v, side u, albedo; packed_float3 x 4 = 48 B               */
typedef struct mm_rect {
    float o[3];
    float v[3];
    float u[3];
    float color[3];
} mm_rect;

/* == BVHNode (src/main.rs:74-81)   == bvh_node (src/shaders.metal:30-35)
 *    count > 0: leaf covering idx[left_first .. left_first+count)
 *    count = 0: interior node, children at left_first and left_first+1       */
typedef struct mm_node {
    float mn[3];
    float mx[3];
    uint32_t left_first;
    uint32_t count;
} mm_node;

/* == Camera  (src/main.rs:32-39)   == camera   (src/shaders.metal:37-42)
 *    quat is (x, y, z, w)                                                    */
typedef struct mm_camera {
    float center[3];
    float focal;
    float quat[4];
    float viewport[2];
} mm_camera;

/* == Uniform (src/main.rs:41-49)   == uni      (src/shaders.metal:237-243)  */
typedef struct mm_uniform {
    mm_camera cam;
    float view_w;
    float view_h;
    uint32_t chunk_w;
    uint32_t time;
} mm_uniform;

/* Throughput-mode extension.  The reference hard-codes these inside the
 * kernel (src/shaders.metal:293-296, "TODO: uniform this"); the offline
 * renderer lifts them into a uniform.                                        */
typedef struct mm_ext {
    uint32_t spp;           /* samples per pixel (reference: 64)              */
    uint32_t bounce_limit;  /* reference: 5   (shaders.metal:294)             */
    uint32_t mirror_limit;  /* reference: 15  (shaders.metal:295)             */
    uint32_t frame;         /* RNG key; plays the role of uni.time            */
    uint32_t flags;         /* MM_EXT_* bits                                   */
    uint32_t reserved;
} mm_ext;

/* mm_ext.flags */
#define MM_EXT_COUNT_STATS   0x1u  /* fill mm_stats (costs a few %)            */
#define MM_EXT_ACCUMULATE    0x2u  /* out += frame value instead of out = ...  */
#define MM_EXT_RGBA8         0x4u  /* out holds RGBA8 (4 B per pixel: the texture-write
                                      conversion of mm_quantize_rgba8, alpha 255)
                                      instead of float4; not with ACCUMULATE    */

/* Work counters.  A "ray" is one closest-hit BVH query, i.e. one execution
 * of src/shaders.metal:307.                                  */
typedef struct mm_stats {
    uint64_t rays;          /* intersect_bvh_iterative calls                  */
    uint64_t node_visits;   /* interior nodes expanded (2 AABB tests each)    */
    uint64_t rect_tests;    /* ray_rect_intersect calls                       */
    uint64_t paths;         /* samples traced                                 */
} mm_stats;

/* Return codes (0 = success; never panics or throws across the ABI). */
#define MM_OK               0
#define MM_ERR_INVALID     -1  /* bad argument / shape                        */
#define MM_ERR_HIP         -2  /* HIP runtime error (message in last_error)   */
#define MM_ERR_NOMEM       -3
#define MM_ERR_NO_SCENE    -4  /* trace before upload                          */
#define MM_ERR_STACK       -5  /* BVH deeper than the 50-entry stack           */
#define MM_ERR_UNSUPPORTED -6  /* geometry the kernel does not implement       */

#ifdef __cplusplus
}
#endif
#endif /* MM_TYPES_H */
