/*
 * mm_api.h — the drop-in boundary: a C ABI over the MI355X (gfx950) HIP
 * implementation of mirror-maze's per-pixel ray-trace loop.
 *
 * Reference interface replaced (all paths relative to the reference repo):
 *   - the Metal compute dispatch of `compute_shader`
 *       kernel signature        src/shaders.metal:245-259
 *       argument table binding  src/main.rs:870-883  (set_buffer 0..6,
 *                               set_bytes(4, Uniform), set_texture 0/1)
 *       dispatch                src/main.rs:884-885  (32x24 groups of 32x32)
 *   - the Metal buffer plumbing  src/utils.rs:86-102 (make_buf/copy_to_buf)
 *   - device/queue creation      src/main.rs:616-626, 638-640
 *   - the render pass's blur     src/main.rs:888-891, src/shaders.metal:214-225
 *                                (mm_present)
 *
 * Conventions: 0 on success, a negative MM_ERR_* code otherwise (message via
 * mm_last_error); no exceptions or aborts cross the ABI; host memory is owned
 * by the caller and copied; device memory is owned by the context unless a
 * function says it writes into a caller-provided device pointer.  A context is
 * bound to one GPU and is not thread-safe (the reference drives Metal from one
 * main thread too, src/main.rs:591).  All work is enqueued on the context's
 * stream; mm_sync waits for it (the reference never waits, src/main.rs:894).
 */
#ifndef MM_API_H
#define MM_API_H

#include "mm_types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mm_ctx mm_ctx;

/* Library version, e.g. "mirror-maze-amd 0.1 gfx950". */
const char* mm_version(void);

/* Replaces Device::system_default() + new_command_queue (main.rs:616-623).
 * device: HIP ordinal.  The context owns a non-blocking stream. */
int  mm_create(int device, mm_ctx** out);
void mm_destroy(mm_ctx* ctx);
const char* mm_last_error(const mm_ctx* ctx);

/* Enqueue on a caller stream (hipStream_t passed as void*), e.g. torch's
 * current stream.  NULL is HIP's default (null) stream, as in HIP itself;
 * MM_OWN_STREAM restores the context's own non-blocking stream. */
#define MM_OWN_STREAM ((void*)(intptr_t)-1)
int  mm_set_stream(mm_ctx* ctx, void* hip_stream);
/* The stream work is enqueued on (after mm_set_stream; initially the
 * context's own stream), e.g. to wrap it for torch.cuda.ExternalStream. */
int  mm_get_stream(const mm_ctx* ctx, void** hip_stream);

/* Replaces make_buf for buffers 1,2,3,5,6 (main.rs:725-730):
 *   rects      buffer 1  mirrors      n_rects x 48 B
 *   nodes      buffer 2  nodes        n_nodes x 32 B
 *   idx        buffer 3  indices      n_rects x u32
 *   is_mirror  buffer 5  materials    n_rects x 1 B (bool)
 *   emission   buffer 6  emissions    n_rects x float4
 * Copies the data; validates the tree (indices in range, stack depth <= 50). */
int  mm_upload_scene(mm_ctx* ctx,
                     const mm_rect* rects, uint32_t n_rects,
                     const mm_node* nodes, uint32_t n_nodes,
                     const uint32_t* idx,
                     const uint8_t* is_mirror,
                     const float* emission);

/* ---- parity mode: the reference dispatch, bit for bit --------------------
 * Replaces copy_to_buf(chunks) + dispatch_thread_groups (main.rs:778-885).
 * Launches (view_w/2/ppc) x (view_h/2/ppc) reference threadgroups of 32x32
 * threads (ppc = chunk_w^2 = 16, 64 samples per pixel); threadgroup g reads
 * chunk origin chunks[g] (uint2, buffer 0) and writes 16 texels of the
 * context's framebuffer (the `texout` texture, RGBA; never cleared, like the
 * reference's Private screen texture).  n_chunks must cover the grid. */
int  mm_trace_chunks(mm_ctx* ctx, const mm_uniform* uni,
                     const uint32_t* chunks, uint32_t n_chunks);

/* Download the framebuffer (view_w x view_h, row-major, y down).
 * rgba_f32: 4 floats/texel before unorm quantisation (alpha = 1), or NULL;
 * rgba8:    RGBA8Unorm as the texture stores it (round-to-nearest-even of
 *           clamp(x,0,1)*255), or NULL. */
int  mm_read_framebuffer(mm_ctx* ctx, float* rgba_f32, uint8_t* rgba8);

/* One presentation step: the render pass's fragment_shader 5-tap blur of the
 * RGBA8 texture (src/main.rs:888-891, src/shaders.metal:214-225), as a Jacobi
 * step — every texel reads the previous texture, neighbours outside it read 0,
 * alpha is written as 1 — so the frame sequence is deterministic (the
 * reference blurs in place from concurrent fragments).  Operation order of
 * the compiled IR: c = (((L+R)+D)+U)*0.5 + C, then c * RN(1/3).  Acts on the
 * RGBA8 texture only (the float framebuffer keeps the traced values). */
int  mm_present(mm_ctx* ctx);

/* The per-pixel packets of the last mm_trace_chunks, in the layout of the
 * shaders.air revision's extra `device float4* pixel_data` output (the
 * streaming-tile format): packets[(c*16 + pn)*4 ..] = (r, g, b,
 * bitcast<float>(x << 16 | y)) for pixel pn = 0..15 of chunk c, x = chunk.x +
 * pn/4, y = chunk.y + pn%4; rgb is the 64-sample mean before quantisation.
 * packets: host buffer of n_chunks*16*4 floats; n_chunks <= the last dispatch's. */
int  mm_read_packets(mm_ctx* ctx, float* packets, uint32_t n_chunks);

/* Device-side RGBA8 quantisation of a float RGBA image (e.g. an mm_trace_tile
 * output) with the texture-write conversion (round-to-nearest-even of
 * clamp(x,0,1)*255, all four channels).  Queued on the context's stream. */
int  mm_quantize_rgba8(mm_ctx* ctx, const float* rgba_dev, uint8_t* rgba8_dev, uint64_t n_pixels);

/* ---- throughput mode: offline renderer ------------------------------------
 * Renders pixels (x0 + i, y0 + j*y_stride), 0<=i<w, 0<=j<h, of the frame
 * uni->view_w x uni->view_h with ext->spp samples each (1..4096),
 * ext->bounce_limit / ext->mirror_limit (0..32767; MM_ERR_INVALID otherwise),
 * RNG keyed on (pixel, sample, ext->frame) so any tiling
 * over any number of GPUs reproduces the 1-GPU image bit for bit.
 * out_dev: caller DEVICE pointer to w*h float4 (row-major over (j,i));
 * alpha = 1 (or, with MM_EXT_ACCUMULATE, += the frame value, alpha += 1).
 * With MM_EXT_RGBA8 out_dev holds w*h 4-byte RGBA8 pixels instead: the
 * texture-write conversion of that float4 (mm_quantize_rgba8's, alpha 255),
 * written by the trace's own resolve (the reference's output texture format,
 * src/main.rs:702-709, without a float frame in between); not with
 * MM_EXT_ACCUMULATE.
 * stats: optional host pointer; filled after an implicit sync when
 * MM_EXT_COUNT_STATS is set.  rays and paths are exact; node_visits and
 * rect_tests count the work of the query method that ran (BVH: interior
 * nodes expanded and rect tests; grid search: cells visited and rect tests,
 * plus the BVH walk's counts for the queries that fell back to it). */
int  mm_trace_tile(mm_ctx* ctx, const mm_uniform* uni, const mm_ext* ext,
                   uint32_t x0, uint32_t y0, uint32_t w, uint32_t h,
                   uint32_t y_stride, float* out_dev, mm_stats* stats);

/* Several consecutive frames of the same tile in ONE launch: frame f (0 <=
 * f < n_frames) is traced with RNG frame ext->frame + f into out_dev + f*w*h*4
 * (out_dev: n_frames*w*h float4, frame-major; 4-byte pixels with
 * MM_EXT_RGBA8); each frame is bit-identical to
 * mm_trace_tile(..., frame = ext->frame + f).  The frames share the launch's
 * work queue, so the ~0.4 ms tail in which the last waves finish their last
 * chunks is paid once per launch instead of once per frame (throughput mode
 * for frame sequences; a frame's result is only complete when the launch is).
 * Needs the wave-persistent kernel with the fused resolve (64 % spp == 0) or
 * with the mirror-tail deferral (any spp: samples staged per frame and
 * resolved in one pass, at most 2^29 staged paths = 6 GiB per launch; over
 * that a fusable launch runs without deferral, others get MM_ERR_INVALID);
 * MM_EXT_ACCUMULATE is rejected (frames of one launch run concurrently). */
int  mm_trace_tile_frames(mm_ctx* ctx, const mm_uniform* uni, const mm_ext* ext, uint32_t n_frames,
                          uint32_t x0, uint32_t y0, uint32_t w, uint32_t h,
                          uint32_t y_stride, float* out_dev, mm_stats* stats);

/* Pipeline selection for mm_trace_tile (MM_PIPE_AUTO picks the fastest). */
#define MM_PIPE_AUTO       0
#define MM_PIPE_MEGAKERNEL 1   /* bounce loop in-kernel (MM_OPT_PERSIST picks the kernel) */
#define MM_PIPE_WAVEFRONT  2   /* the wave-persistent kernel with the mirror-tail deferral always on
                                  (MM_OPT_DEFER, 32 lanes unless set): a wave's divergent tail is parked
                                  in its block's ring and resumed 64 paths at a time, densely.  The round-1
                                  fully flattened pipeline
                                  (SoA state in HBM, one extend/shade launch pair per bounce) measured
                                  ~45 ms vs 5.7 ms per C3 frame and was retired (DESIGN.md §4,
                                  profiles/r02/wavefront_pmc.txt) */
#define MM_PIPE_REFERENCE  3   /* straight statement of the reference kernel, one thread per path
                                  (IEEE division everywhere); A/B baseline  */
int  mm_set_pipeline(mm_ctx* ctx, int pipe);

/* Tuning knobs (results never change; only speed does).  Every value is
 * bit-identical to the reference; the defaults are the measured fastest
 * (DESIGN.md §4).  Options removed after round 1 (measured slower or
 * neutral: 4, 5, 6, 10, 11, 13-17) return MM_ERR_INVALID. */
#define MM_OPT_LDS_NODES   1   /* 1: stage scene data (BVH or grid) in LDS where it fits (default), 0: read
                                  everything through L1/L2 */
#define MM_OPT_BLOCK       2   /* threads per workgroup of MM_PIPE_REFERENCE's one-thread-per-path kernel
                                  (64..1024, x64) */
#define MM_OPT_PERSIST     3   /* 2: wave-persistent kernel, 64-path chunks, pixels resolved in the wave
                                  (default, the only one); 0 (one thread per path) was removed in round 6:
                                  MM_ERR_UNSUPPORTED */
#define MM_OPT_TRAVERSAL   7   /* closest-hit query of the wave-persistent kernel:
                                  -1 auto (default): 11 when the scene allows it, else 7 when every rect has a
                                     compact record, else 5;
                                  11 certified grid search (mm_grid.h): same answer as the reference's BVH walk,
                                     which runs instead on ties / failed certificates / rays outside the grid;
                                  0 (the reference's BVH loop form) was removed in round 6: MM_ERR_UNSUPPORTED
                                    (the parity-mode kernel, mm_trace_chunks, still walks it);
                                  5 BVH, leaf tests and the next interior step in one iteration;
                                  7 form 5 with branch-free compact leaf tests (scenes without SLOW records) */
#define MM_OPT_LDS_RECTS   8   /* BVH forms: 1 compact rect records in LDS beside the nodes when both fit (default) */
#define MM_OPT_LDS_SPLIT   9   /* removed in round 6 (the top-of-tree node cache measured slower): 0 / 1 are
                                  accepted and select nothing, > 1 returns MM_ERR_UNSUPPORTED */
#define MM_OPT_FUSE_RESOLVE 12 /* wave-persistent kernel: 1 reduce each pixel's samples inside the wave
                                  that traced them when 64 % spp == 0 (default), 0 separate k_resolve */
#define MM_OPT_RESERVE_CUS 19 /* wave-persistent kernel: launch that many CUs' worth of resident blocks
                                  fewer (0..128), so kernels of other streams -- a collective moving the
                                  previous frames -- find free CUs while it runs; 0 default */
#define MM_OPT_DICT_NODES 20  /* removed in round 6 (dictionary-coded BVH nodes measured slower): 0 / 1 are
                                  accepted and select nothing, 2 returns MM_ERR_UNSUPPORTED */
#define MM_OPT_DEFER      21  /* wave-persistent kernel: once at most this many lanes of a wave still trace
                                  (past bounce_limit only mirror-hit paths run on), those paths' states go to
                                  their block's tail ring (512 entries) and the block's waves take 64 of them at
                                  a time as a chunk of their own; samples are then staged per path and resolved
                                  by k_resolve (same order).  0 off, 1..64; default: 32 when the search
                                  structure sits whole in LDS (the maze grid with its leaf boxes, or BVH nodes +
                                  compact records) and bounce_limit >= 8 (C3, 20 frames per launch: 2.64 ms/frame
                                  on vs 2.74 off; C4 20.97 vs 21.80), or 64 % spp != 0 (samples staged anyway),
                                  else off (the N=64 scene, leaf boxes via L1/L2: 5.23 on vs 4.90 off) --
                                  profiles/r03/ab_defer_claims.txt.  Built for the grid search and the lean BVH
                                  form with records in LDS; other forms ignore it */
#define MM_OPT_DEFER_MIN  22  /* MM_OPT_DEFER applies to launches of at least this many paths (w*h*spp*frames;
                                  default 2^24: a single C3 frame (16.6 M paths) runs without the rings; rank
                                  0 of an 8-way C3 split, 20 frames = 41 M paths per launch, 0.356 ms/frame
                                  with them vs 0.362 without -- profiles/r03/emulated_scaling/); 0: always */
#define MM_OPT_GRID_MERGE 24  /* grid search: 1 (default) an axis whose cells would not shorten the lists
                                  gets one cell (the maze: one cell along y -- its walls span the height, the
                                  lower cell is the space below the floor); 0 cells per axis by the typical
                                  rect size only.  Read by mm_upload_scene */
#define MM_OPT_GRID_CELL  25  /* grid search: the first cell size tried, in percent of the median rect extent
                                  (25..400, default 100; coarser cells follow until the index fits the LDS
                                  budget).  Read by mm_upload_scene */
#define MM_OPT_GRID_WIDE  26  /* grid search: 1 (default) 64-bit cell words with per-face list ranges where the
                                  image fits the LDS budget; 0 plain 32-bit words (whole list per cell).  Read
                                  by mm_upload_scene */
#define MM_OPT_FAULT_INJECT 23 /* tests of the error path (results are then invalid): 0 off (default); 1 every
                                  wave-persistent launch raises an injected fault (error bit 3); 2 the tail
                                  rings' protocol waits give up at once (bit 2 when a wait was needed; a
                                  writer that gives up leaves NaN in its sample, mm_last_error names the
                                  first timed-out wait); 3 the trace call fails with MM_ERR_HIP after
                                  taking its first launch's status slot, before the launch is enqueued;
                                  4 the launch's first deferred path is lost (its ring entry is reserved,
                                  never written): its reader times out after the normal bound and every
                                  later protocol wait of the launch gives up within 256 polls */
/* The library holds the kernels MM_PIPE_AUTO can select; the values that chose
 * the variants removed in round 6 (MM_OPT_PERSIST 0, MM_OPT_TRAVERSAL 0,
 * MM_OPT_LDS_SPLIT > 1, MM_OPT_DICT_NODES 2, BVH form 7 without nodes +
 * records in LDS) return MM_ERR_UNSUPPORTED. */
int  mm_set_option(mm_ctx* ctx, int key, int value);

/* Facts about the uploaded scene's search structures (double-valued):
 *   MM_INFO_GRID_OK          1 if the certified grid search is available
 *   MM_INFO_GRID_CELLS_X/Y/Z grid cells per axis
 *   MM_INFO_GRID_GLOBAL      rects every query tests (e.g. the maze floor)
 *   MM_INFO_GRID_BYTES       the grid image (cells, lists, records, leaf boxes)
 *   MM_INFO_GRID_INDEX_BYTES its cells + lists part
 *   MM_INFO_LEAN             1 if every rect has a compact record
 *   MM_INFO_DEPTH            BVH depth (max traversal stack entries)
 *   MM_INFO_DICT_OK          0 (dictionary-coded nodes were removed in round 6; the key is kept)
 *   MM_INFO_LAST_FORM        query method of the last wave-persistent launch (MM_OPT_TRAVERSAL value)
 *   MM_INFO_LAST_LDS_MODE    its LDS mode (trace_kernels.hip: 0, 1, 3 BVH; 11-14 grid)
 *   MM_INFO_GRID_FACES       1 if the grid cells carry per-face list ranges (64-bit cell words)
 *   MM_INFO_LAST_DEFER       1 if the last mm_trace_tile* call ran the mirror-tail rings
 *   MM_INFO_LAST_VGPRS       VGPRs per lane of the last wave-persistent kernel (code-object metadata)
 *   MM_INFO_LAST_SCRATCH     its private (scratch) bytes per lane: VGPR spills + traversal stack
 *   MM_INFO_LAST_STATIC_LDS  its static LDS bytes per block (the tail ring's words)
 *   MM_INFO_GRID_LDS_CAP     bytes the grid placements 11 / 14 stage into (their static LDS array without
 *                            tail rings; the grid builder's budget: no grid image is built larger) */
#define MM_INFO_GRID_OK          1
#define MM_INFO_GRID_CELLS_X     2
#define MM_INFO_GRID_CELLS_Y     3
#define MM_INFO_GRID_CELLS_Z     4
#define MM_INFO_GRID_GLOBAL      5
#define MM_INFO_GRID_BYTES       6
#define MM_INFO_GRID_INDEX_BYTES 7
#define MM_INFO_LEAN             8
#define MM_INFO_DEPTH            9
#define MM_INFO_DICT_OK          10
#define MM_INFO_LAST_FORM        11
#define MM_INFO_LAST_LDS_MODE    12
#define MM_INFO_GRID_FACES       13
#define MM_INFO_LAST_DEFER       14
#define MM_INFO_LAST_VGPRS       15
#define MM_INFO_LAST_SCRATCH     16
#define MM_INFO_LAST_STATIC_LDS  17
#define MM_INFO_GRID_LDS_CAP     18
int  mm_scene_info(const mm_ctx* ctx, int key, double* value);

/* Diagnostics: record, for every wave of the wave-persistent kernel, four u64
 * into the device buffer `dev_buf` (n_waves x 4): entry time, LDS staging
 * done, exit time (wall_clock64 ticks, 100 MHz) and the number of 64-path
 * chunks it traced.  NULL turns it off (default).  scripts/timeline_probe.py */
int  mm_set_wave_timeline(mm_ctx* ctx, unsigned long long* dev_buf, uint32_t n_waves);

/* Wait for all work queued by this context; returns the error of the oldest
 * mm_trace_tile* call that failed on the GPU and was not reported yet. */
int  mm_sync(mm_ctx* ctx);

/* Asynchronous errors.  mm_trace_tile / mm_trace_tile_frames return before
 * the GPU runs them; each such call is numbered (1, 2, ...) and its launches
 * publish their error flags (traversal stack overflow, a tail-ring protocol
 * timeout, an injected fault) into host-mapped status words when they end.
 * A call that failed is reported -- its return code, and mm_last_error naming
 * "call #N (what it traced)" -- by the first of: the next mm_trace_tile* call
 * on the context (which is then not enqueued), mm_sync, or mm_call_status(N).
 * It is never attributed to a later call's own work.  (The reference has no
 * error path: a Metal command buffer fails silently, src/main.rs:893-894.) */
#define MM_PENDING 1
int  mm_last_call(const mm_ctx* ctx, uint64_t* call_id);
/* Without waiting: MM_OK (finished clean), MM_PENDING (still running) or the
 * call's error code (message in mm_last_error). */
int  mm_call_status(mm_ctx* ctx, uint64_t call_id);

/* Per-kernel timing of the dominant (ray-trace) kernel: when enabled, every
 * trace-kernel launch is bracketed by HIP events on the context's stream.
 * mm_kernel_timing syncs, returns the summed ms and the launch count since the
 * last reset, and optionally resets. */
int  mm_set_profiling(mm_ctx* ctx, int enable);
int  mm_kernel_timing(mm_ctx* ctx, float* total_ms, uint32_t* launches, int reset);

/* Device-side timing of the last mm_trace_tile / mm_trace_chunks call,
 * measured with HIP events on the context's stream (ms), and the number of
 * kernel launches it made. */
int  mm_last_timing(mm_ctx* ctx, float* ms, uint32_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* MM_API_H */
