/*
 * mm_scene.h — host-side restatement (C++17 behind a C ABI) of the reference's
 * scene plumbing that feeds the kernel.  The reference's host is Rust; there
 * is no Rust toolchain in this image, so this is the "host side above the
 * C-ABI in C++" (see DESIGN.md §Boundary).
 *
 *   mm_rng_*          rand 0.8.5 StdRng (= rand_chacha 0.3.1 ChaCha12Rng),
 *                     seed_from_u64 (rand_core 0.6.4), gen::<f32>, gen_range,
 *                     SliceRandom::shuffle — used at src/main.rs:18,381-382,
 *                     460,467,494,501,303-305
 *   mm_maze_build     Kruskal maze + wall runs + planes   src/main.rs:356-586
 *   mm_bvh_build      SAH BVH                              src/main.rs:74-263
 *   mm_bvh_build_ex   same, explicit split-search method   src/main.rs:102-211
 *   mm_camera_default camera + calculate_quaternion        src/main.rs:732-755,
 *                                                          src/maths.rs:139-156
 *   mm_chunks_*       chunk scheduler gen_pixels/random_pixels
 *                                                          src/main.rs:293-326
 *   mm_player_*, mm_check_collision, mm_quat_mult, mm_update_quat_angle
 *                     interactive camera + collision       src/main.rs:265-291,
 *                                                          738-842, 922-924;
 *                                                          src/maths.rs:159-178
 */
#ifndef MM_SCENE_H
#define MM_SCENE_H

#include "mm_types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- rand 0.8.5 StdRng ---------------------------------------------------*/
typedef struct mm_rng {
    uint32_t key[8];        /* ChaCha key (the 32-byte seed, LE words)        */
    uint64_t counter;       /* next 4-block refill starts at this block       */
    uint32_t buf[64];       /* 4 ChaCha12 blocks, consumed word by word       */
    uint32_t pos;           /* next unread word in buf (64 = empty)           */
} mm_rng;

void     mm_rng_seed_from_u64(mm_rng* r, uint64_t seed);   /* SeedableRng::seed_from_u64 */
void     mm_rng_from_seed(mm_rng* r, const uint8_t seed[32]);
uint32_t mm_rng_next_u32(mm_rng* r);
uint64_t mm_rng_next_u64(mm_rng* r);
float    mm_rng_gen_f32(mm_rng* r);                         /* rng.gen::<f32>()           */
uint32_t mm_rng_gen_range_u32(mm_rng* r, uint32_t lo, uint32_t hi); /* lo..hi, hi excl.  */
/* ChaCha block function with a configurable round count (20 for the RFC 8439
 * known-answer test, 12 for StdRng).  out = 16 LE words. */
void     mm_chacha_block(const uint32_t key[8], uint64_t counter, uint64_t stream,
                         int rounds, uint32_t out[16]);

/* ---- scene ----------------------------------------------------------------*/
typedef struct mm_scene {
    uint32_t  maze_n;       /* maze is maze_n x maze_n cells                  */
    uint32_t  n_rects;
    mm_rect*  rects;        /* buffer 1                                        */
    uint8_t*  is_mirror;    /* buffer 5                                        */
    float*    emission;     /* buffer 6, n_rects x 4                          */
    uint32_t  n_nodes;
    mm_node*  nodes;        /* buffer 2                                        */
    uint32_t* idx;          /* buffer 3                                        */
    uint8_t*  grid;         /* maze_n*maze_n cell bitmasks (1 up, 2 down, 4 left, 8 right) */
    uint32_t  n_vert_walls, n_hori_walls;
    uint32_t  bvh_depth;    /* max root-to-leaf depth (stack bound)           */
} mm_scene;

/* Maze + planes (+ BVH).  maze_n = 10 and seed = 0 reproduce the reference
 * (src/main.rs:362-363, 381).  For maze_n != 10 the hard-coded +-50 boundary,
 * floor and roof (src/main.rs:517-585) scale to +-5*maze_n; the spawn light and
 * the camera stay where the reference puts them.  Returns MM_OK or an error. */
int  mm_scene_build(uint32_t maze_n, uint64_t seed, mm_scene** out);
void mm_scene_free(mm_scene* s);

/* SAH BVH over n rects (src/main.rs:247-263).  nodes_out must hold 2n-1
 * nodes, idx_out n entries.  *n_nodes receives the number used.  The split
 * search is the sorted sweep (MM_BVH_SWEEP): same tree as the reference. */
int  mm_bvh_build(const mm_rect* rects, uint32_t n, mm_node* nodes_out,
                  uint32_t* n_nodes, uint32_t* idx_out);
/* Split-search methods; both produce the reference's node array bit for bit.
 *   MM_BVH_SWEEP       sort each axis once per node, prefix/suffix boxes:
 *                      O(n log n) per node (N=64 maze: milliseconds)
 *   MM_BVH_EXHAUSTIVE  the reference's loop, every candidate re-scans the node
 *                      (src/main.rs:110-125, 180-211): O(n^2) per node */
#define MM_BVH_SWEEP      0
#define MM_BVH_EXHAUSTIVE 1
int  mm_bvh_build_ex(const mm_rect* rects, uint32_t n, mm_node* nodes_out,
                     uint32_t* n_nodes, uint32_t* idx_out, int method);
/* Max depth of the tree (root = 0) — the traversal stack never holds more. */
uint32_t mm_bvh_depth(const mm_node* nodes, uint32_t n_nodes);

/* calculate_quaternion (src/maths.rs:139-156).  Transcendentals are evaluated
 * in double and rounded once (correctly rounded in practice), so the result is
 * platform independent. */
void mm_calculate_quaternion(const float dir[3], float q_out[4]);
/* Camera + Uniform of src/main.rs:732-755: center (-5,0,-45), focal 1,
 * quaternion of (0.1,0,1), viewport (2*W/H, 2); chunk_w 4; time as given. */
void mm_uniform_default(float view_w, float view_h, uint32_t time, mm_uniform* out);

/* ---- chunk scheduler (src/main.rs:293-326) ---------------------------------
 * gen_pixels shuffles all 4x4 chunk origins; the reference uses the unseeded
 * thread_rng, here an explicitly seeded StdRng makes runs reproducible.
 * random_pixels pops n origins from the back, refilling from the original
 * list when empty. */
typedef struct mm_chunk_sched mm_chunk_sched;
int  mm_chunks_create(float view_w, float view_h, uint32_t chunk_w, uint64_t seed,
                      mm_chunk_sched** out);
uint32_t mm_chunks_total(const mm_chunk_sched* s);
int  mm_chunks_next(mm_chunk_sched* s, uint32_t n, uint32_t* out_xy /* n*2 */);
void mm_chunks_free(mm_chunk_sched* s);

/* ---- interactive camera and player collision (src/main.rs:265-291, 738-842,
 * 922-924; src/maths.rs:159-178) -- SURVEY.md §8f item 4.  Drives the camera of
 * an offline sequence (or a front end) exactly as the reference's event loop.  */
typedef struct mm_player {
    float center[3];        /* camera_center, starts at (-5, 0, -45)          */
    float quat[4];          /* rotation (x, y, z, w)                           */
    float half_theta;       /* mouse-driven half angle, acos(quat.w) at start  */
    float fps;              /* 60 (main.rs:760): a key moves 5/fps per frame   */
} mm_player;
#define MM_PLAYER_COLLIDED  0x1u   /* the move was undone (check_collision hit)   */
#define MM_PLAYER_ROTATED   0x2u   /* quat changed: the reference regenerates its chunk list */
#define MM_PLAYER_NAN_QUAT  0x4u   /* rotation rejected (reference prints "Help!") */
/* v' = q^-1 (v, 0) q  (quat_mult, maths.rs:175-178) */
void mm_quat_mult(const float v[3], const float q[4], float out[3]);
/* same axis, half angle theta (update_quat_angle, maths.rs:159-162) */
void mm_update_quat_angle(const float q[4], float theta, float out[4]);
/* first leaf (node index) whose box overlaps [bmin, bmax] in the reference's
 * recursive order (check_collision, main.rs:265-291); -1 none, -2 bad tree */
int  mm_check_collision(const mm_node* nodes, uint32_t n_nodes, const float bmin[3], const float bmax[3]);
int  mm_player_init(const float quat[4], mm_player* p);
/* One frame: keys (macOS key codes 0 A, 1 S, 2 D, 13 W, in pressed order) move
 * the camera, a collision with the player box (+-0.5, 0.2, 0.5) undoes the
 * move, then the previous frame's mouse deltaX values turn half_theta and the
 * quaternion.  *flags receives MM_PLAYER_* bits. */
int  mm_player_step(mm_player* p, const uint16_t* keys, uint32_t n_keys, const float* mouse_dx, uint32_t n_mouse,
                    const mm_node* nodes, uint32_t n_nodes, uint32_t* flags);
/* mm_uniform_default with the player's camera centre and rotation. */
int  mm_player_uniform(const mm_player* p, float view_w, float view_h, uint32_t time, mm_uniform* u);

#ifdef __cplusplus
}
#endif
#endif /* MM_SCENE_H */
