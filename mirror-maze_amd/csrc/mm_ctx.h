// mm_ctx.h — the context behind the C ABI's opaque mm_ctx (include/mm_api.h),
// shared by the runtime (mm_runtime.hip) and the multi-GPU frame path
// (mm_comm.hip).  Private to the library.
#pragma once

#include <hip/hip_runtime.h>

#include <deque>
#include <string>
#include <vector>

#include "mm_api.h"
#include "mm_launch.h"

using mm::DevGrid;

struct mm_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    // scene (buffers 1,2,3,5,6 of compute_shader)
    mm_rect* d_rects = nullptr;
    float4* d_nodes = nullptr;      // production layout (packed child words)
    float4* d_nodes_ref = nullptr;  // reference layout
    uint32_t root_packed = 0;
    bool fast_ok = false;
    uint32_t depth = 0;         // tree depth = max traversal stack entries
    float4* d_geo = nullptr;
    float4* d_shade = nullptr;
    uint2* d_recs = nullptr;    // compact leaf-ordered rect records
    size_t n_fast_recs = 0;
    bool lean_ok = false;       // no SLOW rect records (loop form 7, grid search)
    uint8_t* d_grid = nullptr;  // certified grid search (grid_build.cpp, mm_grid.h)
    DevGrid grid{};
    bool grid_ok = false;
    bool grid_slow = false;  // the grid has SLOW records (general rect test)
    bool grid_wide = false;  // 64-bit cell words with per-face list ranges
    bool grid_flat = false;  // the flat forms apply (grid_build.h GridHost::flat_ok)
    std::string grid_why;
    uint32_t* d_idx = nullptr;
    uint32_t n_rects = 0, n_nodes = 0;
    bool has_scene = false;
    // texout (parity mode)
    float4* d_fb = nullptr;
    uint32_t* d_fb8 = nullptr;
    uint32_t* d_fb8_alt = nullptr;  // presentation blur target (swapped with d_fb8)
    uint32_t last_chunks = 0;       // chunk count of the last mm_trace_chunks
    float4* d_packets = nullptr;
    size_t packets_cap = 0;
    uint32_t fb_w = 0, fb_h = 0;
    // chunk list (buffer 0)
    uint32_t* d_chunks = nullptr;
    size_t chunks_cap = 0;
    // per-sample staging (throughput mode)
    mm::Sample* d_samples = nullptr;
    size_t samples_cap = 0;
    // mirror-tail rings' records (MM_OPT_DEFER)
    void* d_tail = nullptr;
    uint32_t tail_cap = 0;
    // aux: stats[4] (u64) + error flag (u32)
    unsigned long long* d_aux = nullptr;
    uint32_t* d_work = nullptr;  // the wave-persistent kernel's self-cleaning queue heads + waves-done word (4 KB)
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    float last_ms = 0.0f;
    uint32_t last_launches = 0;
    int pipe = MM_PIPE_AUTO;
    // options (include/mm_api.h MM_OPT_*); defaults = the measured fastest
    bool opt_lds = true;            // stage scene data in LDS where it fits
    uint32_t opt_block = 0;         // k_trace_mega block size (0 = auto)
    int opt_persist = 2;            // 0 one thread per path (k_trace_mega), 2 wave-persistent
    int opt_ww = -1;                // loop form: -1 auto, 0, 5, 7 (BVH), 11 (grid search)
    int opt_lds_rects = 1;          // compact rect records in LDS beside the nodes when they fit
    bool opt_fuse = true;           // resolve fused into the wave when 64 % spp == 0
    uint32_t opt_reserve_cus = 0;   // MM_OPT_RESERVE_CUS
    int opt_defer = -1;             // MM_OPT_DEFER: defer a wave's paths once <= this many lanes run (0 off, -1 auto)
    uint32_t opt_defer_min = 1u << 24;  // MM_OPT_DEFER_MIN: ... in launches of at least this many paths
    int last_form = -1, last_mode = -1;  // of the last wave-persistent launch (mm_scene_info)
    unsigned long long* d_wave_ts = nullptr;  // diagnostics (mm_set_wave_timeline)
    uint32_t wave_ts_cap = 0;
    // per-kernel profiling of the trace kernel (mm_set_profiling)
    bool prof = false;
    std::vector<hipEvent_t> prof_ev;   // pairs (start, stop)
    size_t prof_used = 0;              // events recorded since last reset
    // Per-launch status words (host-mapped pinned memory): launch L of the
    // context writes slot L % kStatusSlots when it ends (error bits |
    // kStatusDone).  Each mm_trace_tile* call is a numbered "call" owning a
    // run of launches; a call whose launches raised an error is reported,
    // naming the call, by the next call on the context, mm_sync or
    // mm_call_status -- never blamed on a later call's work.
    uint32_t* h_status = nullptr;
    uint32_t* d_status = nullptr;
    std::vector<uint64_t> slot_owner;  // launch id + 1 holding each slot, 0 = free
    uint64_t launch_seq = 0, call_seq = 0;
    struct Call { uint64_t id, first, n; std::string what; uint32_t bits; };
    struct Failed { uint64_t id; uint32_t bits; std::string what; bool reported; };
    std::deque<Call> pending;
    std::deque<Failed> failed;  // the last kFailedKept failed calls
    uint64_t failed_dropped = 0;  // highest call id dropped from `failed` (older ids: status no longer kept)
    int opt_fault = 0;           // MM_OPT_FAULT_INJECT
    bool opt_grid_merge = true;  // MM_OPT_GRID_MERGE (read by mm_upload_scene)
    int opt_grid_cell = 100;     // MM_OPT_GRID_CELL (read by mm_upload_scene)
    bool opt_grid_wide = true;   // MM_OPT_GRID_WIDE (read by mm_upload_scene)
    bool last_defer = false;     // the last trace call ran the tail rings
    int last_kern_mode = -1, last_kern_form = -1;  // for MM_INFO_LAST_VGPRS / _SCRATCH
    int last_kern_ring = 0;      // its tail-ring kind (wavepersist_attributes: 0 none, 1 global, 2 LDS records)
    // frame-end gather (mm_comm.hip): the root's receive staging, one slab per rank
    uint8_t* d_gather = nullptr;
    size_t gather_cap = 0;
    // the last gather that used d_gather: its assembly is done at this event (recorded on the stream the gather
    // ran on); a gather on another stream waits for it before reusing the staging, and a regrow waits before
    // freeing it (two gathers on different streams raced on the one staging buffer)
    hipEvent_t gather_done = nullptr;
    bool gather_pending = false;
};

namespace mm {
// Record `msg` as the context's last error and return `code`.
inline int ctx_fail(mm_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}
}  // namespace mm
