// mm_launch.h — host-callable launchers for the kernels in trace_*.hip.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>

#include "mm_device.h"

namespace mm {

// Per-rect derived data for the scene (n, |v|, |u|, kind) from raw rects.
hipError_t launch_prep_rects(const mm_rect* rects_dev, uint32_t n, float4* geo_dev, hipStream_t s);

// Parity mode: the reference dispatch (grid_w x grid_h groups of 32x32).
hipError_t launch_trace_chunks(const DevScene& sc, const mm_uniform& u, const uint32_t* chunks_dev,
                               uint32_t grid_w, uint32_t grid_h, float4* fb, uint32_t* fb8,
                               unsigned long long* stats_dev, uint32_t* err, bool count_stats, hipStream_t s);

// A staged sample: the path's value sqrt(max(L, 0)) (shaders.metal:342-344),
// 12 B -- the resolve reads these back (round 6: 16-B float4 slots before, a
// quarter of the staged traffic unused).
using Sample = F3;
static_assert(sizeof(Sample) == 12, "three floats, no padding");

// Deferred path states (mirror-tail deferral): one 64-byte record per entry
// (rec[4*i .. 4*i+3] = ori.xyz dir.x | dir.yz T.xy | T.z L.xyz | seed,
// (n - mh) | mh << 15 | bank << 30, sample slot, s1 -- one base pointer; 16 SoA field arrays would
// hold 15 addresses in SGPRs across the bounce loop), `cap` records; resident
// block b owns the kTailRing records from b * kTailRing (its tail ring, at most
// 2 blocks per CU).
constexpr uint32_t kTailRing = 512;

struct TailQueue {
    uint4* rec = nullptr;
    uint32_t cap = 0;
};

struct TileJob {
    mm_uniform u;
    mm_ext e;
    uint32_t x0, y0, w, h, y_stride;
    uint32_t view_w;     // (uint32_t)u.view_w — pixel index stride
    // Fused resolve (wave-persistent kernel, 64 % spp == 0): each wave reduces
    // its chunk's whole pixels in registers and writes out[pixel] itself, in
    // k_resolve's order; no per-sample staging buffer, no resolve launch.
    void* out = nullptr;  // float4 per pixel, or RGBA8 (4 B) with MM_EXT_RGBA8 (mm_wave_util.h store_pixel)
    uint32_t fuse = 0;
    // Diagnostics (mm_set_wave_timeline): per wave of the wave-persistent
    // kernel, 4 x u64 = (entry, LDS staged, exit, chunks) in wall_clock64()
    // ticks (100 MHz).  Null = off.
    unsigned long long* wave_ts = nullptr;
    uint32_t wave_ts_cap = 0;
    // Multi-frame launch (mm_trace_tile_frames; wave-persistent kernel, fused
    // resolve): the queue holds n_frames frames' chunks back to back; frame f
    // uses RNG frame e.frame + f and writes out + f * w * h.
    uint32_t n_frames = 1;
    // CUs' worth of blocks the wave-persistent grid leaves free (MM_OPT_RESERVE_CUS)
    uint32_t reserve_cus = 0;
    // Mirror-tail deferral (MM_OPT_DEFER; wave-persistent kernel, samples
    // staged per path, no fused resolve): a wave whose paths are at bounce
    // >= defer_from with at most defer_lanes lanes still running queues those
    // paths' state in its block's tail ring (ballot + prefix compaction, one
    // LDS atomic per wave) and moves on; the block's waves take 64 queued tails
    // at a time as a chunk.  Sample slot of a path: fr * (w*h*spp) + path.
    // defer_from >= 2^30: off.
    uint32_t defer_from = 1u << 30, defer_lanes = 0;
    TailQueue tail;
    // 1: the rings' records in LDS (the kRing = 2 kernel, where the grid image leaves room); 0: in `tail`
    uint32_t ring_lds = 0;
    // Per-launch status word (host-mapped pinned memory, mm_runtime.hip): the
    // last wave of the launch moves the error flag into it, | kStatusDone, so
    // the host attributes an error to the call that launched it without a
    // sync.  Null: the error flag stays sticky (parity mode reads it itself).
    uint32_t* status = nullptr;
    // Polls a tail-ring protocol wait may take before it gives up (error bit
    // 2; ~50 ms; a wait lasts at most a few bounces).  The round-3 trip of the
    // 64-lane deferral test was a livelock ending at the 32-bit entry
    // counters' wrap, not a slow wait (trace_kernels.hip).
    // MM_OPT_FAULT_INJECT 2 sets 0.
    uint32_t ring_spin = 1u << 20;
    // The launch's first timed-out ring wait writes 16 words here
    // (host-mapped; trace_kernels.hip ring_timeout); launch_id goes into it.
    uint32_t* ring_diag = nullptr;
    uint32_t launch_id = 0;
    // MM_OPT_FAULT_INJECT 1: the launch raises error bit 3; 4: its first
    // deferred path is lost (bit 4, and the reader's ring timeout) -- tests of
    // the error path.
    uint32_t fault = 0;
};

// Error flag bits (aux word 4, and the status word's low bits).
constexpr uint32_t kErrStack = 1u, kErrRing = 2u, kErrInjected = 8u, kErrLost = 16u, kErrPublish = 32u;
constexpr uint32_t kStatusDone = 0x80000000u;

// One-thread kernel that publishes a non-persistent launch's error flag into
// its status word (the persistent kernel's last wave does this itself).
hipError_t launch_publish_status(uint32_t* err, uint32_t* status, hipStream_t s);

struct MegaOpts {
    bool reference = false;   // traverse_reference (IEEE division): MM_PIPE_REFERENCE, the only form built
    uint32_t block = 256;     // threads per workgroup
};

// MM_PIPE_REFERENCE: one thread per (pixel, sample) path; writes
// the per-sample value sqrt(max(L,0)) to samples[path] (path = pixel*spp+s).
hipError_t launch_trace_mega(const DevScene& sc, const TileJob& job, Sample* samples,
                             unsigned long long* stats_dev, uint32_t* err, bool count_stats,
                             const MegaOpts& o, hipStream_t s);

// Throughput mode, wave-persistent megakernel: resident 1024-thread blocks,
// waves pull 64-path chunks from work[0]; work[0..1] must be zero at launch
// and are left zero by the kernel itself (the last wave re-zeroes them).
// lds_mode / form: trace_kernels.hip (k_trace_wavepersist); returns
// hipErrorInvalidValue for a pair that is not instantiated.
hipError_t launch_trace_wavepersist(const DevScene& sc, const TileJob& job, Sample* samples,
                                    unsigned long long* stats, uint32_t* err, uint32_t* work, bool count_stats,
                                    int lds_mode, int form, hipStream_t s);
size_t wavepersist_lds_bytes(const DevScene& sc, int lds_mode);
// LDS modes 11 / 14 stage the grid image into a static array of this many bytes (ring: 0 none, 1 global
// records, 2 records in LDS); other modes use dynamic LDS beside the kernel's static words.
uint32_t wavepersist_grid_cap(int ring);
// Whether the tail-deferral variant / any variant exists for this (LDS mode, form).
bool wavepersist_defer_built(int lds_mode, int form);
bool wavepersist_built(int lds_mode, int form);
// Register / scratch / LDS use of the (kStats = false) instance.
// ring: 0 no tail deferral, 1 rings with global records, 2 rings with records in LDS.
hipError_t wavepersist_attributes(int lds_mode, int form, int ring, hipFuncAttributes* a);
// Display stage (display.hip).
hipError_t launch_present_blur(const uint32_t* in, uint32_t* out, uint32_t W, uint32_t H, hipStream_t s);
hipError_t launch_chunk_packets(const float4* fb, const uint32_t* chunks, uint32_t n_chunks, uint32_t W, uint32_t H,
                                float4* out, hipStream_t s);
hipError_t launch_quantize(const float4* in, uint32_t* out, size_t n, hipStream_t s);

// Per-pixel reduction of spp samples in the reference's order, then / spp.
hipError_t launch_resolve(const TileJob& job, const Sample* samples, void* out, hipStream_t s);

}  // namespace mm
