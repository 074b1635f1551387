/*
 * mm_comm.h — the multi-GPU frame path of the C ABI: RCCL communicators over
 * the contexts' GPUs and the frame-end gather of interleaved row tiles
 * (north star: "tiles of the framebuffer shard one-per-GPU across the
 * 8xMI355X node with a single RCCL gather over xGMI at frame end").
 *
 * Reference interface replaced (paths relative to the reference repo):
 *   - the single Metal device          src/main.rs:616 (Device::system_default)
 *   - the frame-end dispatch + commit  src/main.rs:884-894 (the texture the
 *     compute pass wrote is handed to the render pass; here rank 0 receives
 *     every rank's rows of the frame)
 * The reference renders on one device and has no collective; these entry
 * points are what its Rust host would bind to drive N GPUs.
 *
 * Row split (mm_row_shard): rank r of N renders the frame rows r, r+N, r+2N,
 * ... into a tile of rows_max = ceil(H/N) rows (its last row unused when H %
 * N <= r), so each rank gets the same share of the very uneven per-row cost
 * with no scheduling, and -- the RNG being keyed on (pixel, sample, frame) --
 * the assembled frame is bit-identical to the 1-GPU frame.
 *
 * Two ways to build the communicators, both RCCL (over xGMI between the
 * node's GPUs):
 *   - one process per GPU: rank 0 calls mm_comm_unique_id, the host's own
 *     rendezvous hands the 128 bytes to every rank, each calls
 *     mm_comm_init_rank (collective: blocks until all N have joined);
 *   - one process driving N GPUs (one context each): mm_comm_init_all, then
 *     mm_gather_rows_all issues every rank's part in one RCCL group.
 * Conventions as in mm_api.h: 0 or a negative MM_ERR_* code, message in the
 * context's mm_last_error; work is enqueued on the context's stream.
 */
#ifndef MM_COMM_H
#define MM_COMM_H

#include "mm_api.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mm_comm mm_comm;

#define MM_COMM_ID_BYTES 128

/* RCCL's unique id for a new communicator (ncclGetUniqueId), to be created
 * once (rank 0) and shared with every rank by the caller. */
int mm_comm_unique_id(mm_ctx* ctx, uint8_t id[MM_COMM_ID_BYTES]);

/* Join communicator `id` as `rank` of `n_ranks` on ctx's GPU (collective). */
int mm_comm_init_rank(mm_ctx* ctx, int n_ranks, int rank, const uint8_t id[MM_COMM_ID_BYTES], mm_comm** out);

/* One process, n contexts on n distinct GPUs: out[i] is rank i on ctxs[i]'s
 * GPU (ncclCommInitAll).  Errors go to ctxs[0]. */
int mm_comm_init_all(int n, mm_ctx* const* ctxs, mm_comm** out);

/* rank, n_ranks and HIP device of a communicator (any pointer may be NULL). */
int mm_comm_info(const mm_comm* comm, int* rank, int* n_ranks, int* device);

/* The RCCL version the library runs against (ncclGetVersion, e.g. 22606: in a
 * process that already mapped an RCCL -- torch's -- the loader reuses it by
 * soname), and the version of the rccl.h it was compiled with (e.g. 22707).
 * mm_comm_init_rank / mm_comm_init_all refuse (MM_ERR_UNSUPPORTED, both
 * versions named) a runtime of another major version or older than 2.18: the
 * calls used here (unique id, init rank / all, send / recv in groups, version
 * and error strings, destroy) keep their ABI across NCCL 2.18+. */
int mm_comm_rccl_version(void);
int mm_comm_rccl_header_version(void);

void mm_comm_destroy(mm_comm* comm);

/* The interleaved row set of `rank`: first row y0, row stride (= n_ranks),
 * its row count, and the tile height every rank uses (ceil(height/n_ranks)). */
int mm_row_shard(uint32_t height, uint32_t n_ranks, uint32_t rank, uint32_t* y0, uint32_t* y_stride,
                 uint32_t* rows, uint32_t* rows_max);

/* Frame-end gather to rank 0.  tile_dev (this rank's GPU): n_frames tiles of
 * rows_max x width pixels of bytes_per_px bytes (4: the reference's RGBA8
 * texture, 16: float RGBA), frame-major, row i of a tile = frame row
 * rank + i * n_ranks.  Every rank calls it with the same n_frames, width,
 * height and bytes_per_px.  On rank 0 frame_dev receives n_frames frames of
 * height x width pixels (frame-major, rows in order); other ranks pass NULL.
 * Non-root ranks send their tiles (ncclSend); rank 0 receives them into a
 * staging buffer of the context (ncclRecv, one RCCL group) and one kernel
 * writes every row to its place in the frames -- its own rows straight from
 * tile_dev.  Enqueued on ctx's stream (the tiles must be complete in stream
 * order).  flags: MM_GATHER_SELF_VIA_RCCL also routes rank 0's own tile
 * through an RCCL send/recv to itself (exercises the transport at one rank;
 * one extra copy of 1/N of the frame). */
#define MM_GATHER_SELF_VIA_RCCL 1u
int mm_gather_rows(mm_ctx* ctx, mm_comm* comm, const void* tile_dev, uint32_t n_frames, uint32_t width,
                   uint32_t height, uint32_t bytes_per_px, void* frame_dev, uint32_t flags);

/* mm_gather_rows for all n ranks of one process (communicators from
 * mm_comm_init_all): comms[i] / tiles_dev[i] on ctxs[i]'s GPU; frame_dev on
 * the GPU of the context whose communicator is rank 0.  One RCCL group. */
int mm_gather_rows_all(int n, mm_ctx* const* ctxs, mm_comm* const* comms, const void* const* tiles_dev,
                       uint32_t n_frames, uint32_t width, uint32_t height, uint32_t bytes_per_px, void* frame_dev,
                       uint32_t flags);

/* The de-interleave alone, for a host with its own transport: tiles_dev holds
 * n_ranks ranks' tiles back to back on ctx's GPU (rank-major, then as
 * tile_dev above); frame_dev receives the n_frames frames.  Enqueued on
 * ctx's stream. */
int mm_assemble_rows(mm_ctx* ctx, const void* tiles_dev, uint32_t n_ranks, uint32_t n_frames, uint32_t width,
                     uint32_t height, uint32_t bytes_per_px, void* frame_dev);

#ifdef __cplusplus
}
#endif
#endif /* MM_COMM_H */
