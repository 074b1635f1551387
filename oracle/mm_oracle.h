/*
 * mm_oracle.h — TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference
 * kernel `compute_shader` (src/shaders.metal:245-368) used as the parity
 * checker.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it; the product (mirror-maze_amd/) never links or calls it.
 *
 * PARITY UNPINNED against an executed reference: the reference is Rust +
 * Metal Shading Language and neither toolchain exists in this image (see
 * DESIGN.md §Oracle).  The arithmetic follows the operation order of the
 * reference's compiled AIR (src/shaders.ir, read as disassembled text), with
 * IEEE-754 binary32 semantics for every operation and the AIR intrinsics
 * given their IEEE meaning (dot = (x*x'+y*y')+z*z', fast_rsqrt = 1/sqrt,
 * fast_sqrt = sqrt, fast_fmin/fmax = fminf/fmaxf).
 */
#ifndef MM_ORACLE_H
#define MM_ORACLE_H

#include "../include/mm_types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_scene {
    const mm_rect*  rects;
    uint32_t        n_rects;
    const mm_node*  nodes;
    uint32_t        n_nodes;
    const uint32_t* idx;
    const uint8_t*  is_mirror;
    const float*    emission;   /* n_rects x 4 */
} oracle_scene;

/* Reference dispatch: (view_w/2/ppc) x (view_h/2/ppc) threadgroups of
 * tg_w x tg_h threads (the reference runs 32 x 32).  Writes RGBA floats
 * (alpha 1) into fb (view_w x view_h x 4), leaving other texels untouched.
 * Returns 0, or MM_ERR_* (stack overflow, bad shape). */
int oracle_trace_chunks(const oracle_scene* sc, const mm_uniform* uni,
                        const uint32_t* chunks, uint32_t n_chunks,
                        uint32_t tg_w, uint32_t tg_h, float* fb, mm_stats* stats);

/* One reference threadgroup (tgid_x, tgid_y) only — for sampled checks. */
int oracle_trace_group(const oracle_scene* sc, const mm_uniform* uni,
                       const uint32_t* chunks, uint32_t n_chunks,
                       uint32_t tg_w, uint32_t tg_h, uint32_t tgid_x, uint32_t tgid_y,
                       float* fb, mm_stats* stats);

/* Throughput-mode definition (the offline renderer's generalisation):
 * pixels (x0+i, y0+j*y_stride), ext->spp samples, bounce/mirror limits from
 * ext, RNG seed = mm_tile_seed(pixel, sample, frame).  out: w*h*4 floats. */
int oracle_trace_tile(const oracle_scene* sc, const mm_uniform* uni, const mm_ext* ext,
                      uint32_t x0, uint32_t y0, uint32_t w, uint32_t h, uint32_t y_stride,
                      float* out, mm_stats* stats);

/* Single path, for diagnosis: returns the per-sample value sqrt(max(L,0))
 * in rgb_out and the number of BVH queries in *rays. */
int oracle_trace_path(const oracle_scene* sc, const float ori[3], const float dir[3],
                      uint32_t seed, int bounce_limit, int mirror_limit,
                      float rgb_out[3], uint32_t* rays);

/* Display stage: fragment_shader blur as a Jacobi step (RGBA8 in -> out,
 * W x H, in != out) and the RGBA8 store conversion. */
void oracle_present_blur(const uint8_t* in, uint8_t* out, uint32_t W, uint32_t H);
void oracle_quantize(const float* rgba, uint8_t* rgba8, uint64_t n_pixels);

/* Floating-point environment of the trace entry points: 0 IEEE binary32
 * with denormals (default, the HIP kernels' semantics), 1 MXCSR FTZ|DAZ (the
 * reference's `air.compile.denorms_disable`, src/shaders.ir !47).  The MXCSR
 * sticky flags the entry points raised (bit 1 DE denormal operand, bit 4 UE
 * underflow) accumulate in oracle_fp_flags (reset = 1 clears them). */
void     oracle_set_fp_mode(int ftz_daz);
unsigned oracle_fp_flags(int reset);

/* Pieces exported for unit tests. */
float    oracle_rand_pm1(uint32_t* state);          /* (random(state)-0.5)*2 */
uint32_t oracle_seed_reference(uint32_t tx, uint32_t ty, uint32_t time);
uint32_t oracle_tile_seed(uint32_t pixel, uint32_t sample, uint32_t frame);
void     oracle_primary_dir(const mm_uniform* uni, uint32_t px, uint32_t py, float dir[3]);
float    oracle_intersect_aabb(const float ori[3], const float dir[3], float t,
                               const float mn[3], const float mx[3]);

#ifdef __cplusplus
}
#endif
#endif
