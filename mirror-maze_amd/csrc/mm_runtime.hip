// mm_runtime.hip — the C ABI of include/mm_api.h over the HIP runtime.
//
// Replaces the reference's Metal plumbing: device/queue creation
// (src/main.rs:616-626), buffer creation and updates (src/utils.rs:86-102,
// src/main.rs:723-730, 784) and the compute dispatch (src/main.rs:867-886).
// No exception or abort crosses the ABI; every HIP error becomes
// MM_ERR_HIP with the runtime's message in mm_last_error().
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <deque>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "grid_build.h"
#include "mm_api.h"
#include "mm_ctx.h"
#include "mm_launch.h"

using namespace mm;

namespace mm {
size_t build_compact_rects(const mm_rect* rects, uint32_t n_rects, const uint32_t* idx, std::vector<uint32_t>& out,
                           size_t* n_slow);
}

constexpr uint32_t kStatusSlots = 1024;
constexpr uint32_t kRingDiagWords = 16;  // after the status words: the first timed-out ring wait's record
constexpr size_t kFailedKept = 64;
// Staged samples (tail deferral / no fused resolve) per launch: whole rows up
// to this many paths (12 B each: 6 GiB).  A multi-frame launch over the cap
// runs without deferral (fused resolve) or is refused.
constexpr uint64_t kStagePathsMax = 1ull << 29;

namespace {

int fail(mm_ctx* c, int code, const std::string& msg) { return ctx_fail(c, code, msg); }

#define HIPC(ctx, expr)                                                                           \
    do {                                                                                          \
        hipError_t _e = (expr);                                                                   \
        if (_e != hipSuccess)                                                                     \
            return fail((ctx), MM_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

template <typename T>
int ensure(mm_ctx* c, T*& ptr, size_t& cap, size_t n) {
    if (n <= cap && ptr) return MM_OK;
    if (ptr) { (void)hipFree(ptr); ptr = nullptr; cap = 0; }
    HIPC(c, hipMalloc((void**)&ptr, std::max<size_t>(n, 1) * sizeof(T)));
    cap = n;
    return MM_OK;
}

DevScene dev_scene(const mm_ctx* c) {
    DevScene s;
    s.nodes = c->d_nodes;
    s.nodes_ref = c->d_nodes_ref;
    s.root_packed = c->root_packed;
    s.fast_ok = c->fast_ok ? 1u : 0u;
    s.geo = c->d_geo;
    s.recs = c->d_recs;
    s.grid = c->grid;
    s.shade = c->d_shade;
    s.idx = c->d_idx;
    s.n_nodes = c->n_nodes;
    s.n_rects = c->n_rects;
    return s;
}

void free_scene(mm_ctx* c) {
    (void)hipFree(c->d_rects); (void)hipFree(c->d_nodes); (void)hipFree(c->d_nodes_ref); (void)hipFree(c->d_geo);
    (void)hipFree(c->d_shade); (void)hipFree(c->d_idx); (void)hipFree(c->d_recs);
    (void)hipFree(c->d_grid);
    c->d_grid = nullptr; c->grid = DevGrid{}; c->grid_ok = false; c->grid_slow = false; c->grid_wide = false;
    c->grid_flat = false;
    c->d_rects = nullptr; c->d_nodes = nullptr; c->d_nodes_ref = nullptr; c->d_geo = nullptr; c->d_recs = nullptr; c->d_shade = nullptr; c->d_idx = nullptr;
    c->has_scene = false;
}

// Stack depth the near-first traversal can reach: at most one pending far
// child per level, so the tree depth bounds it.
int check_tree(const mm_node* nodes, uint32_t n_nodes, const uint32_t* idx, uint32_t n_rects, std::string& why,
               uint32_t* depth_out) {
    for (uint32_t i = 0; i < n_rects; ++i)
        if (idx[i] >= n_rects) { why = "idx out of range"; return MM_ERR_INVALID; }
    std::vector<std::pair<uint32_t, uint32_t>> todo{{0u, 0u}};
    std::vector<uint8_t> seen(n_nodes, 0);
    uint32_t maxd = 0;
    while (!todo.empty()) {
        auto [n, d] = todo.back();
        todo.pop_back();
        if (n >= n_nodes || seen[n]) { why = "node graph is not a tree"; return MM_ERR_INVALID; }
        seen[n] = 1;
        maxd = std::max(maxd, d);
        const mm_node& nd = nodes[n];
        if (nd.count > 0) {
            if ((uint64_t)nd.left_first + nd.count > n_rects) { why = "leaf range out of bounds"; return MM_ERR_INVALID; }
        } else {
            if ((uint64_t)nd.left_first + 1 >= n_nodes) { why = "child index out of range"; return MM_ERR_INVALID; }
            todo.push_back({nd.left_first, d + 1});
            todo.push_back({nd.left_first + 1, d + 1});
        }
    }
    if (maxd > (uint32_t)kStackMax) { why = "BVH deeper than the 50-entry traversal stack"; return MM_ERR_STACK; }
    *depth_out = maxd;
    return MM_OK;
}

// Coordinates inside the Markstein-quotient guard (mm_trace.h): 0 or
// |x| in [2^-30, 2^60]; rect extents 0 or |x| in [2^-10, 2^60].
bool coord_ok(float x) {
    const float a = std::fabs(x);
    return a == 0.0f || (a >= 0x1p-30f && a <= 0x1p60f);
}
bool extent_ok(float x) {
    const float a = std::fabs(x);
    return a == 0.0f || (a >= 0x1p-10f && a <= 0x1p60f);
}

// The tail rings' records (mm_launch.h TailQueue): kTailRing per resident
// block, at most 2 blocks per CU.
int tail_queue(mm_ctx* c, TailQueue& q) {
    int cus = 0;
    HIPC(c, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
    const uint32_t cap = 2u * (uint32_t)cus * kTailRing;
    if (c->tail_cap < cap || !c->d_tail) {
        (void)hipFree(c->d_tail);
        c->d_tail = nullptr;
        c->tail_cap = 0;
        HIPC(c, hipMalloc(&c->d_tail, (size_t)cap * 64));
        c->tail_cap = cap;
    }
    q.rec = reinterpret_cast<uint4*>(c->d_tail);
    q.cap = c->tail_cap;
    return MM_OK;
}

int begin_timing(mm_ctx* c) {
    HIPC(c, hipEventRecord(c->ev0, c->stream));
    return MM_OK;
}
int end_timing(mm_ctx* c, uint32_t launches) {
    HIPC(c, hipEventRecord(c->ev1, c->stream));
    c->last_launches = launches;
    c->last_ms = -1.0f;  // resolved lazily in mm_last_timing
    return MM_OK;
}

// Bracket one trace-kernel launch with events when profiling is on.
int prof_mark(mm_ctx* c) {
    if (!c->prof) return MM_OK;
    if (c->prof_used == c->prof_ev.size()) {
        hipEvent_t e;
        HIPC(c, hipEventCreate(&e));
        c->prof_ev.push_back(e);
    }
    HIPC(c, hipEventRecord(c->prof_ev[c->prof_used++], c->stream));
    return MM_OK;
}

int read_aux(mm_ctx* c, mm_stats* st) {
    unsigned long long h[5];
    HIPC(c, hipMemcpyAsync(h, c->d_aux, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    if (st) { st->rays = h[0]; st->node_visits = h[1]; st->rect_tests = h[2]; st->paths = h[3]; }
    if ((uint32_t)h[4] != 0) {
        HIPC(c, hipMemsetAsync(c->d_aux + 4, 0, sizeof(unsigned long long), c->stream));
        if (h[4] & 2u) return fail(c, MM_ERR_HIP, "tail ring wait timed out (kernel protocol error)");
        return fail(c, MM_ERR_STACK, "traversal stack overflow (depth > 50)");
    }
    return MM_OK;
}

// ---- per-call status (see mm_ctx::h_status) -------------------------------
uint32_t status_load(const mm_ctx* c, uint64_t launch) {
    return __atomic_load_n(c->h_status + launch % kStatusSlots, __ATOMIC_ACQUIRE);
}

// Device address of the status word for the next launch.  A slot still held
// by a launch kStatusSlots earlier that has not finished is waited for.
int next_status(mm_ctx* c, uint32_t*& dev_word) {
    const uint64_t id = c->launch_seq;
    const uint32_t s = (uint32_t)(id % kStatusSlots);
    if (c->slot_owner[s] && !(status_load(c, c->slot_owner[s] - 1) & kStatusDone)) {
        HIPC(c, hipStreamSynchronize(c->stream));
        if (!(status_load(c, c->slot_owner[s] - 1) & kStatusDone)) HIPC(c, hipDeviceSynchronize());
        if (!(status_load(c, c->slot_owner[s] - 1) & kStatusDone))
            return fail(c, MM_ERR_HIP, "status word of an earlier launch never completed");
    }
    if (c->slot_owner[s]) {  // fold the finished occupant's bits into its call, if still pending
        const uint64_t prev = c->slot_owner[s] - 1;
        for (auto& k : c->pending)
            if (prev >= k.first && prev < k.first + k.n) k.bits |= status_load(c, prev) & ~kStatusDone;
    }
    __atomic_store_n(c->h_status + s, 0u, __ATOMIC_RELEASE);
    c->slot_owner[s] = id + 1;
    c->launch_seq = id + 1;
    dev_word = c->d_status + s;
    return MM_OK;
}

// The record a timed-out ring wait left (trace_kernels.hip ring_timeout), as
// text, when it belongs to one of the launches [first, first + n) of the call
// being reported; consumed then (the device writes a new record only into a
// consumed one).  A record of an older launch than the call's is stale (its
// call was reported without it) and is dropped; a newer one is left for its
// own call.
std::string ring_diag_text(mm_ctx* c, uint64_t first, uint64_t n) {
    uint32_t* d = c->h_status + kStatusSlots;
    if (__atomic_load_n(d, __ATOMIC_ACQUIRE) != 1u) return "";  // none, or being written (2)
    uint32_t w[kRingDiagWords];
    for (uint32_t i = 0; i < kRingDiagWords; ++i) w[i] = __atomic_load_n(d + i, __ATOMIC_RELAXED);
    const uint32_t rel = w[15] - (uint32_t)first;  // launch ids are the context's launch numbers, mod 2^32
    if (rel >= (uint32_t)n) {
        if ((int32_t)rel < 0) __atomic_store_n(d, 0u, __ATOMIC_RELEASE);  // stale: free the record
        return "";
    }
    const uint64_t t1 = w[12] | (uint64_t)w[13] << 32;
    char b[320];
    snprintf(b, sizeof(b),
             " [first timed-out wait (launch %u): %s of entry %u (slot %u, lap %u) in block %u wave %u lane %u "
             "wanted turn %u, saw %u; reserved %u, claimed %u; gave up after %u polls at device clock %llu]",
             w[15], w[1] == 1 ? "reader" : "writer", w[2], w[2] % kTailRing, w[2] / kTailRing, w[7], w[8], w[9],
             w[3], w[4], w[5], w[6], w[14], (unsigned long long)t1);
    __atomic_store_n(d, 0u, __ATOMIC_RELEASE);
    return b;
}

std::string error_text(mm_ctx* c, uint32_t bits, uint64_t first, uint64_t n) {
    std::string s;
    auto add = [&](const std::string& m) { s += s.empty() ? m : std::string("; ") + m; };
    if (bits & kErrStack) add("traversal stack overflow (depth > 50)");
    if (bits & kErrRing) add("tail ring wait timed out (kernel protocol error)" + ring_diag_text(c, first, n));
    if (bits & kErrInjected) add("injected fault (MM_OPT_FAULT_INJECT)");
    if (bits & kErrLost) add("injected lost tail-ring entry (MM_OPT_FAULT_INJECT 4)");
    if (bits & kErrPublish) add("the launch's status could not be published (its error flag was read after a sync)");
    return s.empty() ? "unknown error" : s;
}
int error_code(uint32_t bits) { return (bits & ~kErrStack) ? MM_ERR_HIP : MM_ERR_STACK; }

// Fold finished calls' status words into the failed list (non-blocking).
void poll_calls(mm_ctx* c) {
    for (auto it = c->pending.begin(); it != c->pending.end();) {
        uint32_t bits = it->bits;
        bool done = true;
        for (uint64_t l = it->first; l < it->first + it->n && done; ++l) {
            // a slot reused by a later launch: this launch finished, its bits are in it->bits
            if (c->slot_owner[l % kStatusSlots] != l + 1) continue;
            const uint32_t w = status_load(c, l);
            done = (w & kStatusDone) != 0;
            bits |= w & ~kStatusDone;
        }
        if (!done) { ++it; continue; }
        if (bits) {
            c->failed.push_back({it->id, bits, it->what + " -- " + error_text(c, bits, it->first, it->n), false});
            if (c->failed.size() > kFailedKept) {
                c->failed_dropped = std::max(c->failed_dropped, c->failed.front().id);
                c->failed.pop_front();
            }
        }
        it = c->pending.erase(it);
    }
}

// "call #N (what) failed on the GPU: why" (Failed::what holds "what -- why").
std::string failed_text(const mm_ctx::Failed& f) {
    const size_t k = f.what.find(" -- ");
    return "call #" + std::to_string(f.id) + " (" + f.what.substr(0, k) + ") failed on the GPU: " +
           (k == std::string::npos ? std::string("unknown error") : f.what.substr(k + 4));
}

// The oldest unreported failed call, as this call's return code.
int report_failure(mm_ctx* c, const char* suffix) {
    poll_calls(c);
    for (auto& f : c->failed)
        if (!f.reported) {
            f.reported = true;
            return fail(c, error_code(f.bits), failed_text(f) + suffix);
        }
    return MM_OK;
}

}  // namespace

extern "C" {

const char* mm_version(void) {
    return "mirror-maze-amd 0.4 gfx950";
}

int mm_create(int device, mm_ctx** out) {
    if (!out) return MM_ERR_INVALID;
    *out = nullptr;
    mm_ctx* c = new (std::nothrow) mm_ctx();
    if (!c) return MM_ERR_NOMEM;
    c->device = device;
    int rc = MM_OK;
    auto chk = [&](hipError_t e, const char* what) {
        if (e != hipSuccess && rc == MM_OK) rc = fail(c, MM_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
    };
    int n = 0;
    chk(hipGetDeviceCount(&n), "hipGetDeviceCount");
    if (rc == MM_OK && (device < 0 || device >= n)) rc = fail(c, MM_ERR_INVALID, "no such HIP device");
    if (rc == MM_OK) chk(hipSetDevice(device), "hipSetDevice");
    if (rc == MM_OK) chk(hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking), "hipStreamCreate");
    if (rc == MM_OK) chk(hipEventCreate(&c->ev0), "hipEventCreate");
    if (rc == MM_OK) chk(hipEventCreate(&c->ev1), "hipEventCreate");
    if (rc == MM_OK) chk(hipMalloc((void**)&c->d_aux, 8 * sizeof(unsigned long long)), "hipMalloc(aux)");
    if (rc == MM_OK) chk(hipMemset(c->d_aux, 0, 8 * sizeof(unsigned long long)), "hipMemset(aux)");
    if (rc == MM_OK) chk(hipMalloc((void**)&c->d_work, 4096), "hipMalloc(work)");
    if (rc == MM_OK) chk(hipMemset(c->d_work, 0, 4096), "hipMemset(work)");
    if (rc == MM_OK)
        chk(hipHostMalloc((void**)&c->h_status, (kStatusSlots + kRingDiagWords) * sizeof(uint32_t),
                          hipHostMallocMapped | hipHostMallocCoherent),
            "hipHostMalloc(status)");
    if (rc == MM_OK) chk(hipHostGetDevicePointer((void**)&c->d_status, c->h_status, 0), "hipHostGetDevicePointer");
    if (rc == MM_OK) {
        std::memset(c->h_status, 0, (kStatusSlots + kRingDiagWords) * sizeof(uint32_t));
        c->slot_owner.assign(kStatusSlots, 0);
    }
    if (rc != MM_OK) {
        fprintf(stderr, "mm_create: %s\n", c->err.c_str());
        mm_destroy(c);
        return rc;
    }
    c->stream = c->own_stream;
    *out = c;
    return MM_OK;
}

void mm_destroy(mm_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    free_scene(c);
    (void)hipFree(c->d_fb); (void)hipFree(c->d_fb8); (void)hipFree(c->d_chunks);
    (void)hipFree(c->d_fb8_alt); (void)hipFree(c->d_packets);
    (void)hipFree(c->d_samples); (void)hipFree(c->d_aux); (void)hipFree(c->d_tail); (void)hipFree(c->d_work);
    (void)hipFree(c->d_gather);
    if (c->gather_done) (void)hipEventDestroy(c->gather_done);
    if (c->h_status) (void)hipHostFree(c->h_status);
    for (hipEvent_t e : c->prof_ev) (void)hipEventDestroy(e);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
}

const char* mm_last_error(const mm_ctx* c) { return c ? c->err.c_str() : "null context"; }

int mm_set_stream(mm_ctx* c, void* s) {
    if (!c) return MM_ERR_INVALID;
    c->stream = (s == MM_OWN_STREAM) ? c->own_stream : (hipStream_t)s;
    return MM_OK;
}

int mm_set_wave_timeline(mm_ctx* c, unsigned long long* buf, uint32_t n_waves) {
    if (!c) return MM_ERR_INVALID;
    c->d_wave_ts = n_waves ? buf : nullptr;
    c->wave_ts_cap = buf ? n_waves : 0;
    return MM_OK;
}

int mm_get_stream(const mm_ctx* c, void** s) {
    if (!c || !s) return MM_ERR_INVALID;
    *s = (void*)c->stream;
    return MM_OK;
}

int mm_set_pipeline(mm_ctx* c, int pipe) {
    if (!c) return MM_ERR_INVALID;
    if (pipe < MM_PIPE_AUTO || pipe > MM_PIPE_REFERENCE) return fail(c, MM_ERR_INVALID, "unknown pipeline");
    c->pipe = pipe;
    return MM_OK;
}

// Kernel variants removed in round 6: every one measured slower than what
// MM_PIPE_AUTO selects; the options that chose them are refused by name.
static const char* const kRemoved =
    "this kernel variant (one thread per path over the production BVH forms, loop form 0, the split node "
    "cache, dictionary-coded nodes) measured slower and was removed (DESIGN.md §4)";

int mm_set_option(mm_ctx* c, int key, int value) {
    if (!c) return MM_ERR_INVALID;
    switch (key) {
        case MM_OPT_LDS_NODES: c->opt_lds = value != 0; return MM_OK;
        case MM_OPT_BLOCK:
            if (value < 64 || value > 1024 || value % 64) return fail(c, MM_ERR_INVALID, "block must be 64..1024, x64");
            c->opt_block = (uint32_t)value;
            return MM_OK;
        case MM_OPT_PERSIST:
            if (value != 0 && value != 2) return fail(c, MM_ERR_INVALID, "persist must be 0 or 2");
            if (value == 0) return fail(c, MM_ERR_UNSUPPORTED, kRemoved);
            c->opt_persist = value;
            return MM_OK;
        case MM_OPT_TRAVERSAL:
            if (value != -1 && value != 0 && value != 5 && value != 7 && value != 11)
                return fail(c, MM_ERR_INVALID, "traversal must be -1 (auto), 0, 5, 7 or 11 (grid search)");
            if (value == 0) return fail(c, MM_ERR_UNSUPPORTED, kRemoved);
            c->opt_ww = value;
            return MM_OK;
        case MM_OPT_LDS_RECTS: c->opt_lds_rects = value != 0; return MM_OK;
        case MM_OPT_LDS_SPLIT:
            if (value < 0) return fail(c, MM_ERR_INVALID, "split cache size must be >= 0 (0 off, 1 auto, else KB)");
            if (value > 1) return fail(c, MM_ERR_UNSUPPORTED, kRemoved);
            return MM_OK;  // 0 / 1: accepted, nothing to select (no split cache is built)
        case MM_OPT_FUSE_RESOLVE: c->opt_fuse = value != 0; return MM_OK;
        case MM_OPT_RESERVE_CUS:
            if (value < 0 || value > 128) return fail(c, MM_ERR_INVALID, "reserved CUs must be 0..128");
            c->opt_reserve_cus = (uint32_t)value;
            return MM_OK;
        case MM_OPT_DEFER:
            if (value < 0 || value > 64) return fail(c, MM_ERR_INVALID, "defer lanes must be 0..64");
            c->opt_defer = value;
            return MM_OK;
        case MM_OPT_DEFER_MIN:
            if (value < 0) return fail(c, MM_ERR_INVALID, "defer min paths must be >= 0");
            c->opt_defer_min = (uint32_t)value;
            return MM_OK;
        case MM_OPT_DICT_NODES:
            if (value < 0 || value > 2) return fail(c, MM_ERR_INVALID, "dict nodes must be 0, 1 or 2");
            if (value == 2) return fail(c, MM_ERR_UNSUPPORTED, kRemoved);
            return MM_OK;  // 0 / 1: accepted, nothing to select (no dictionary is built)
        case MM_OPT_GRID_MERGE: c->opt_grid_merge = value != 0; return MM_OK;
        case MM_OPT_GRID_WIDE: c->opt_grid_wide = value != 0; return MM_OK;
        case MM_OPT_GRID_CELL:
            if (value < 25 || value > 400) return fail(c, MM_ERR_INVALID, "grid cell scale must be 25..400 (%)");
            c->opt_grid_cell = value;
            return MM_OK;
        case MM_OPT_FAULT_INJECT:
            if (value < 0 || value > 4) return fail(c, MM_ERR_INVALID, "fault inject must be 0..4");
            c->opt_fault = value;
            return MM_OK;
        default: return fail(c, MM_ERR_INVALID, "unknown option");
    }
}

int mm_scene_info(const mm_ctx* c, int key, double* value) {
    if (!c || !value) return MM_ERR_INVALID;
    if (!c->has_scene) return MM_ERR_NO_SCENE;
    const DevGrid& g = c->grid;
    switch (key) {
        case MM_INFO_GRID_OK: *value = c->grid_ok ? 1.0 : 0.0; return MM_OK;
        case MM_INFO_GRID_CELLS_X: *value = g.n[0]; return MM_OK;
        case MM_INFO_GRID_CELLS_Y: *value = g.n[1]; return MM_OK;
        case MM_INFO_GRID_CELLS_Z: *value = g.n[2]; return MM_OK;
        case MM_INFO_GRID_GLOBAL: *value = g.n_glob; return MM_OK;
        case MM_INFO_GRID_BYTES: *value = g.bytes; return MM_OK;
        case MM_INFO_GRID_INDEX_BYTES: *value = g.off_data; return MM_OK;
        case MM_INFO_LEAN: *value = c->lean_ok ? 1.0 : 0.0; return MM_OK;
        case MM_INFO_DEPTH: *value = c->depth; return MM_OK;
        case MM_INFO_DICT_OK: *value = 0.0; return MM_OK;  // (dictionary-coded nodes removed in round 6)
        case MM_INFO_LAST_FORM: *value = c->last_form; return MM_OK;
        case MM_INFO_LAST_LDS_MODE: *value = c->last_mode; return MM_OK;
        case MM_INFO_GRID_FACES: *value = c->grid_ok && c->grid_wide ? 1.0 : 0.0; return MM_OK;
        case MM_INFO_LAST_DEFER: *value = c->last_defer ? 1.0 : 0.0; return MM_OK;
        case MM_INFO_GRID_LDS_CAP: *value = wavepersist_grid_cap(0); return MM_OK;
        case MM_INFO_LAST_VGPRS:
        case MM_INFO_LAST_SCRATCH:
        case MM_INFO_LAST_STATIC_LDS: {
            if (c->last_kern_mode < 0) return MM_ERR_INVALID;
            hipFuncAttributes a{};
            if (wavepersist_attributes(c->last_kern_mode, c->last_kern_form, c->last_kern_ring, &a) != hipSuccess)
                return MM_ERR_HIP;
            *value = key == MM_INFO_LAST_VGPRS ? a.numRegs
                     : key == MM_INFO_LAST_SCRATCH ? (double)a.localSizeBytes : (double)a.sharedSizeBytes;
            return MM_OK;
        }
        default: return MM_ERR_INVALID;
    }
}

int mm_upload_scene(mm_ctx* c, const mm_rect* rects, uint32_t n_rects, const mm_node* nodes, uint32_t n_nodes,
                    const uint32_t* idx, const uint8_t* is_mirror, const float* emission) {
    if (!c) return MM_ERR_INVALID;
    if (!rects || !nodes || !idx || !is_mirror || !emission || n_rects == 0 || n_nodes == 0)
        return fail(c, MM_ERR_INVALID, "mm_upload_scene: null array or empty scene");
    if (n_nodes > 2 * n_rects) return fail(c, MM_ERR_INVALID, "mm_upload_scene: more than 2n-1 nodes");
    std::string why;
    uint32_t depth = 0;
    int rc = check_tree(nodes, n_nodes, idx, n_rects, why, &depth);
    if (rc != MM_OK) return fail(c, rc, "mm_upload_scene: " + why);
    // Production node layout: a = (mn.x, mx.x, mn.y, mx.y), b = (mn.z, mx.z, packed, 0),
    // packed = count << 24 | left_first.  Child pairs are renumbered
    // breadth-first from the root's pair, which lands at node 2 (nodes 0-1 are
    // never read: the root is not tested, shaders.metal:123-125), so every pair
    // is one aligned 64-B line and a prefix of the array is the top of the tree
    // (the split LDS cache of mm_trace.h).  Only traversal order matters to the
    // result, and it depends on distances, not on indices.
    for (uint32_t i = 0; i < n_nodes; ++i)
        if (nodes[i].count >= 256u || nodes[i].left_first >= (1u << 24))
            return fail(c, MM_ERR_UNSUPPORTED, "mm_upload_scene: leaf with >= 256 planes or index >= 2^24");
    std::vector<uint32_t> pair_old;  // old index of each pair's left node, breadth-first
    if (nodes[0].count == 0) pair_old.push_back(nodes[0].left_first);
    for (size_t q = 0; q < pair_old.size(); ++q)
        for (uint32_t k = 0; k < 2; ++k) {
            const mm_node& nd = nodes[pair_old[q] + k];
            if (nd.count == 0) pair_old.push_back(nd.left_first);
        }
    std::vector<uint32_t> pair_new(n_nodes, 0);  // old left index -> new left index
    for (size_t q = 0; q < pair_old.size(); ++q) pair_new[pair_old[q]] = 2 + 2 * (uint32_t)q;
    if (2 + 2 * pair_old.size() >= (1u << 24))
        return fail(c, MM_ERR_UNSUPPORTED, "mm_upload_scene: node index >= 2^24");
    auto pack = [&](const mm_node& nd) {
        return nd.count > 0 ? (nd.count << 24) | nd.left_first : pair_new[nd.left_first];
    };
    const uint32_t n_prod = 2 + 2 * (uint32_t)pair_old.size();
    std::vector<float4> packed(2 * (size_t)n_prod, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    for (size_t q = 0; q < pair_old.size(); ++q)
        for (uint32_t k = 0; k < 2; ++k) {
            const mm_node& nd = nodes[pair_old[q] + k];
            const uint32_t pk = pack(nd);
            float pkf;
            std::memcpy(&pkf, &pk, 4);
            const size_t i = 2 + 2 * q + k;
            packed[2 * i] = make_float4(nd.mn[0], nd.mx[0], nd.mn[1], nd.mx[1]);
            packed[2 * i + 1] = make_float4(nd.mn[2], nd.mx[2], pkf, 0.0f);
        }
    bool fast = true;
    for (uint32_t i = 0; i < n_nodes && fast; ++i)
        for (int a = 0; a < 3; ++a) fast = fast && coord_ok(nodes[i].mn[a]) && coord_ok(nodes[i].mx[a]);
    for (uint32_t k = 0; k < n_rects && fast; ++k)
        for (int a = 0; a < 3; ++a)
            fast = fast && coord_ok(rects[k].o[a]) && extent_ok(rects[k].v[a]) && extent_ok(rects[k].u[a]);
    HIPC(c, hipSetDevice(c->device));
    free_scene(c);
    std::vector<float4> shade(2 * (size_t)n_rects);
    for (uint32_t k = 0; k < n_rects; ++k) {
        shade[2 * k] = make_float4(rects[k].color[0], rects[k].color[1], rects[k].color[2], is_mirror[k] ? 1.0f : 0.0f);
        shade[2 * k + 1] = make_float4(emission[4 * k], emission[4 * k + 1], emission[4 * k + 2], emission[4 * k + 3]);
    }
    HIPC(c, hipMalloc((void**)&c->d_rects, n_rects * sizeof(mm_rect)));
    HIPC(c, hipMalloc((void**)&c->d_nodes, packed.size() * sizeof(float4)));
    HIPC(c, hipMalloc((void**)&c->d_nodes_ref, n_nodes * sizeof(mm_node)));
    HIPC(c, hipMalloc((void**)&c->d_geo, 4 * (size_t)n_rects * sizeof(float4)));
    HIPC(c, hipMalloc((void**)&c->d_shade, 2 * (size_t)n_rects * sizeof(float4)));
    HIPC(c, hipMalloc((void**)&c->d_idx, n_rects * sizeof(uint32_t)));
    std::vector<uint32_t> recs;
    size_t n_slow = n_rects;
    c->n_fast_recs = n_rects < (1u << 20) ? build_compact_rects(rects, n_rects, idx, recs, &n_slow) : 0;
    if (n_rects >= (1u << 20)) recs.assign(10 * (size_t)n_rects, 2u << 30);  // all SLOW (index does not fit)
    HIPC(c, hipMalloc((void**)&c->d_recs, recs.size() * sizeof(uint32_t)));
    HIPC(c, hipMemcpyAsync(c->d_recs, recs.data(), recs.size() * sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
    HIPC(c, hipMemcpyAsync(c->d_rects, rects, n_rects * sizeof(mm_rect), hipMemcpyHostToDevice, c->stream));
    // mm_node is exactly two float4: (mn.xyz, mx.x) (mx.yz, left_first, count)
    HIPC(c, hipMemcpyAsync(c->d_nodes_ref, nodes, n_nodes * sizeof(mm_node), hipMemcpyHostToDevice, c->stream));
    HIPC(c, hipMemcpyAsync(c->d_nodes, packed.data(), packed.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
    // certified grid search (mm_grid.h): needs the Markstein guards and axis-aligned rects
    GridHost gh;
    std::string gwhy;
    // the budget: what the static grid array of modes 11 / 14 holds beside the kernel's other static LDS
    // (wavepersist_grid_cap(0), 80 KB -- the LDS of one of the two 1024-thread blocks per CU -- less its
    // claimed-range words; ADVICE r05: an image between that and 80 KB failed the launch)
    const bool grid_ok = fast && build_grid(rects, n_rects, nodes, n_nodes, idx, wavepersist_grid_cap(0), gh, gwhy,
                                            c->opt_grid_merge, c->opt_grid_cell / 100.0, c->opt_grid_wide);
    if (!fast) gwhy = "scene coordinates outside the exact-division guards";
    DevGrid dg{};
    if (grid_ok) {
        HIPC(c, hipMalloc((void**)&c->d_grid, gh.bytes));
        HIPC(c, hipMemcpyAsync(c->d_grid, gh.image.data(), gh.bytes, hipMemcpyHostToDevice, c->stream));
        for (int a = 0; a < 3; ++a) {
            dg.mn[a] = gh.mn[a]; dg.mx[a] = gh.mx[a]; dg.cell[a] = gh.cell[a]; dg.inv[a] = gh.inv[a];
            dg.n[a] = gh.n[a];
        }
        dg.n_glob = gh.n_glob;
        dg.slab = gh.slab ? 1u : 0u;
        dg.slab_y[0] = gh.slab_y[0];
        dg.slab_y[1] = gh.slab_y[1];
        for (int a = 0; a < 3; ++a) {
            dg.nm1[a] = gh.n[a] - 1;
            dg.nf[a] = (float)gh.n[a];
        }
        for (int i = 0; i < 4; ++i) dg.glob[i] = gh.glob[i];
        dg.cells = c->d_grid;
        dg.list = reinterpret_cast<const uint16_t*>(c->d_grid + gh.off_list);
        dg.recs = reinterpret_cast<const uint4*>(c->d_grid + gh.off_recs);
        dg.box = reinterpret_cast<const float2*>(c->d_grid + gh.off_box);
        dg.image = reinterpret_cast<const uint4*>(c->d_grid);
        dg.off_list = gh.off_list; dg.off_recs = gh.off_recs; dg.off_box = gh.off_box; dg.bytes = gh.bytes;
        dg.off_class = gh.off_class;  // 0: 32-byte records, no class table
        dg.off_data = gh.off_data;
        dg.cls = gh.off_class ? reinterpret_cast<const float4*>(c->d_grid + gh.off_class) : nullptr;
        c->grid_slow = gh.n_slow > 0;
        c->grid_wide = gh.wide;
        c->grid_flat = gh.flat_ok;
    }
    HIPC(c, hipMemcpyAsync(c->d_shade, shade.data(), shade.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
    HIPC(c, hipMemcpyAsync(c->d_idx, idx, n_rects * sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
    HIPC(c, launch_prep_rects(c->d_rects, n_rects, c->d_geo, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));  // host arrays may be freed on return
    c->n_rects = n_rects;
    c->n_nodes = n_prod;
    c->root_packed = pack(nodes[0]);
    c->depth = depth;
    c->fast_ok = fast;
    c->lean_ok = n_slow == 0;
    c->grid = dg;
    c->grid_ok = grid_ok;
    c->grid_why = grid_ok ? std::string() : gwhy;
    c->has_scene = true;
    return MM_OK;
}

int mm_trace_chunks(mm_ctx* c, const mm_uniform* u, const uint32_t* chunks, uint32_t n_chunks) {
    if (!c) return MM_ERR_INVALID;
    if (!c->has_scene) return fail(c, MM_ERR_NO_SCENE, "mm_trace_chunks: no scene uploaded");
    if (!u || !chunks) return fail(c, MM_ERR_INVALID, "mm_trace_chunks: null argument");
    if (!(u->view_w >= 1.0f && u->view_w <= 65536.0f && u->view_h >= 1.0f && u->view_h <= 65536.0f))
        return fail(c, MM_ERR_INVALID, "mm_trace_chunks: bad view size");
    // The kernel maps one wave64 to one pixel's samples: 32x32 threads / ppc
    // must be 64, i.e. chunk_w = 4 as in the reference (main.rs:602).
    if (u->chunk_w != 4) return fail(c, MM_ERR_UNSUPPORTED, "mm_trace_chunks: chunk_w must be 4 (64 samples/pixel)");
    const uint32_t ppc = 16;
    const uint32_t gw = (uint32_t)(u->view_w / 2.0f / (float)ppc), gh = (uint32_t)(u->view_h / 2.0f / (float)ppc);
    if (gw == 0 || gh == 0) return fail(c, MM_ERR_INVALID, "mm_trace_chunks: view too small for one group");
    // every pixel_buffer_index the groups compute (in float, IR %26-%31) must be in range
    uint32_t max_pbi = 0;
    for (uint32_t gy = 0; gy < gh; ++gy) {
        float f = ((u->view_w * 0.5f) * (float)gy) / (float)ppc + (float)(gw - 1);
        max_pbi = std::max(max_pbi, (uint32_t)f);
    }
    if (max_pbi >= n_chunks) return fail(c, MM_ERR_INVALID, "mm_trace_chunks: chunk list shorter than the grid");
    const uint32_t W = (uint32_t)u->view_w, H = (uint32_t)u->view_h;
    HIPC(c, hipSetDevice(c->device));
    if (W != c->fb_w || H != c->fb_h) {
        (void)hipFree(c->d_fb); (void)hipFree(c->d_fb8); (void)hipFree(c->d_fb8_alt);
        c->d_fb = nullptr; c->d_fb8 = nullptr; c->d_fb8_alt = nullptr;
        c->fb_w = c->fb_h = 0;
        HIPC(c, hipMalloc((void**)&c->d_fb, (size_t)W * H * sizeof(float4)));
        HIPC(c, hipMalloc((void**)&c->d_fb8, (size_t)W * H * sizeof(uint32_t)));
        HIPC(c, hipMalloc((void**)&c->d_fb8_alt, (size_t)W * H * sizeof(uint32_t)));
        HIPC(c, hipMemsetAsync(c->d_fb, 0, (size_t)W * H * sizeof(float4), c->stream));
        HIPC(c, hipMemsetAsync(c->d_fb8, 0, (size_t)W * H * sizeof(uint32_t), c->stream));
        c->fb_w = W; c->fb_h = H;
    }
    int rc = ensure(c, c->d_chunks, c->chunks_cap, 2 * (size_t)n_chunks);
    if (rc) return rc;
    HIPC(c, hipMemcpyAsync(c->d_chunks, chunks, 2 * (size_t)n_chunks * sizeof(uint32_t), hipMemcpyHostToDevice,
                           c->stream));
    HIPC(c, hipMemsetAsync(c->d_aux, 0, 5 * sizeof(unsigned long long), c->stream));  // stats, error flag
    if ((rc = begin_timing(c))) return rc;
    HIPC(c, launch_trace_chunks(dev_scene(c), *u, c->d_chunks, gw, gh, c->d_fb, c->d_fb8, c->d_aux,
                                reinterpret_cast<uint32_t*>(c->d_aux + 4), false, c->stream));
    if ((rc = end_timing(c, 1))) return rc;
    c->last_chunks = n_chunks;
    return read_aux(c, nullptr);
}

int mm_present(mm_ctx* c) {
    if (!c) return MM_ERR_INVALID;
    if (!c->d_fb8) return fail(c, MM_ERR_INVALID, "mm_present: nothing rendered yet");
    HIPC(c, hipSetDevice(c->device));
    HIPC(c, launch_present_blur(c->d_fb8, c->d_fb8_alt, c->fb_w, c->fb_h, c->stream));
    std::swap(c->d_fb8, c->d_fb8_alt);
    return MM_OK;
}

int mm_read_packets(mm_ctx* c, float* packets, uint32_t n_chunks) {
    if (!c) return MM_ERR_INVALID;
    if (!packets) return fail(c, MM_ERR_INVALID, "mm_read_packets: null output");
    if (!c->d_fb || c->last_chunks == 0) return fail(c, MM_ERR_INVALID, "mm_read_packets: no mm_trace_chunks yet");
    if (n_chunks > c->last_chunks)
        return fail(c, MM_ERR_INVALID, "mm_read_packets: more chunks than the last dispatch used");
    if (n_chunks == 0) return MM_OK;
    HIPC(c, hipSetDevice(c->device));
    int rc = ensure(c, c->d_packets, c->packets_cap, 16 * (size_t)n_chunks);
    if (rc) return rc;
    HIPC(c, launch_chunk_packets(c->d_fb, c->d_chunks, n_chunks, c->fb_w, c->fb_h, c->d_packets, c->stream));
    HIPC(c, hipMemcpyAsync(packets, c->d_packets, 16 * (size_t)n_chunks * sizeof(float4), hipMemcpyDeviceToHost,
                           c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    return MM_OK;
}

int mm_quantize_rgba8(mm_ctx* c, const float* rgba_dev, uint8_t* rgba8_dev, uint64_t n_pixels) {
    if (!c) return MM_ERR_INVALID;
    if ((!rgba_dev || !rgba8_dev) && n_pixels) return fail(c, MM_ERR_INVALID, "mm_quantize_rgba8: null buffer");
    if (n_pixels == 0) return MM_OK;
    if (reinterpret_cast<uintptr_t>(rgba_dev) % 16 || reinterpret_cast<uintptr_t>(rgba8_dev) % 4)
        return fail(c, MM_ERR_INVALID, "mm_quantize_rgba8: misaligned buffer");
    HIPC(c, hipSetDevice(c->device));
    HIPC(c, launch_quantize(reinterpret_cast<const float4*>(rgba_dev), reinterpret_cast<uint32_t*>(rgba8_dev),
                            (size_t)n_pixels, c->stream));
    return MM_OK;
}

int mm_read_framebuffer(mm_ctx* c, float* rgba, uint8_t* rgba8) {
    if (!c) return MM_ERR_INVALID;
    if (!c->d_fb) return fail(c, MM_ERR_INVALID, "mm_read_framebuffer: nothing rendered yet");
    const size_t n = (size_t)c->fb_w * c->fb_h;
    HIPC(c, hipSetDevice(c->device));
    if (rgba) HIPC(c, hipMemcpyAsync(rgba, c->d_fb, n * sizeof(float4), hipMemcpyDeviceToHost, c->stream));
    if (rgba8) HIPC(c, hipMemcpyAsync(rgba8, c->d_fb8, n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPC(c, hipStreamSynchronize(c->stream));
    return MM_OK;
}

namespace {

// Loop form and LDS mode of the wave-persistent kernel (trace_kernels.hip).
// 1024-thread blocks at 8 waves per SIMD -> two blocks per CU -> 80 KB of LDS
// each.  Auto (MM_OPT_TRAVERSAL -1): the certified grid search when the scene
// allows it (C3 ...), else the lean BVH loop (form 7) when every rect has a
// compact record and the nodes + records fit LDS, else form 5 with the nodes
// in LDS when they fit, else through L1/L2.  MM_OPT_LDS_NODES 0 stages nothing.
int choose_wavepersist(mm_ctx* c, DevScene& sc, int& form, int& mode) {
    const size_t budget = 80 * 1024;
    const bool auto_form = c->opt_ww < 0;
    form = auto_form ? (c->grid_ok ? kFormGrid : (c->lean_ok ? kFormLean : kFormLeafInterior)) : c->opt_ww;
    if (form == kFormGrid) {
        if (!c->grid_ok)
            return fail(c, MM_ERR_UNSUPPORTED, "grid search unavailable for this scene: " + c->grid_why);
        if (!c->lean_ok || c->grid_slow) form = kFormGridSlow;  // general rect tests for the SLOW records
        // maze grids (one cell along y, compact records): only the maze forms read them
        auto flat = [&](int m) {
            if (c->grid_flat) {
                if (form != kFormGrid && form != kFormGridWide)
                    return fail(c, MM_ERR_UNSUPPORTED, "maze grid with SLOW records");
                form += kFormGridFlat;
            }
            if (!wavepersist_built(m, form))
                return fail(c, MM_ERR_UNSUPPORTED,
                            "grid form " + std::to_string(form) + " not built for LDS mode " + std::to_string(m));
            mode = m;
            return MM_OK;
        };
        // modes 11 / 14 stage into the kernel's static grid array: their images must fit its capacity
        const size_t cap = wavepersist_grid_cap(0);
        if (c->grid_wide) {  // built only when the whole image fits that capacity (grid_build.cpp)
            form += kFormGridWide - kFormGrid;
            return flat(c->opt_lds && c->grid.bytes <= cap ? 11 : 13);
        }
        if (c->opt_lds && c->grid.bytes <= cap) return flat(11);
        // compact records + class table + index (N=64: ~77 KB), leaf boxes global
        if (c->opt_lds && c->grid_flat && c->grid.off_box <= cap) return flat(14);
        if (c->opt_lds && c->grid.off_data <= budget) return flat(12);
        if (!auto_form || !c->opt_lds) return flat(13);
        // the index does not fit LDS: auto takes the BVH (nodes in LDS or cached), which is not
        // measured against the all-global grid
        form = c->lean_ok ? kFormLean : kFormLeafInterior;
    }
    if (form == kFormLean && !c->lean_ok) {
        if (!auto_form) return fail(c, MM_ERR_UNSUPPORTED, "loop form 7 needs compact records for every rect");
        form = kFormLeafInterior;
    }
    const size_t nodes_b = 2 * (size_t)c->n_nodes * sizeof(float4);
    const size_t recs_b = 40 * (size_t)c->n_rects;
    // nodes + records in LDS (lean form 7 or form 5), nodes only (form 5), or nothing
    if (c->opt_lds && c->opt_lds_rects && nodes_b + recs_b <= budget) {
        mode = 3;
    } else {
        if (form == kFormLean && !auto_form)
            return fail(c, MM_ERR_UNSUPPORTED,
                        "loop form 7 needs the BVH nodes + compact records in LDS (its other placements "
                        "measured slower and were removed, DESIGN.md §4)");
        form = kFormLeafInterior;
        mode = (c->opt_lds && nodes_b <= budget) ? 1 : 0;
    }
    return MM_OK;
}

int trace_tile_impl(mm_ctx* c, const mm_uniform* u, const mm_ext* e, uint32_t n_frames, uint32_t x0, uint32_t y0,
                    uint32_t w, uint32_t h, uint32_t y_stride, float* out_dev, mm_stats* stats) {
    if (!c) return MM_ERR_INVALID;
    // an earlier call that failed on the GPU is reported first, by name; this call is then not enqueued
    if (int rc0 = report_failure(c, "; this call was not enqueued")) return rc0;
    if (!c->has_scene) return fail(c, MM_ERR_NO_SCENE, "mm_trace_tile: no scene uploaded");
    if (!u || !e || !out_dev) return fail(c, MM_ERR_INVALID, "mm_trace_tile: null argument");
    if (!(u->view_w >= 1.0f && u->view_w <= 65536.0f && u->view_h >= 1.0f && u->view_h <= 65536.0f))
        return fail(c, MM_ERR_INVALID, "mm_trace_tile: bad view size");
    const uint32_t W = (uint32_t)u->view_w, H = (uint32_t)u->view_h;
    if (w == 0 || h == 0 || y_stride == 0 || e->spp == 0 || e->spp > 4096)
        return fail(c, MM_ERR_INVALID, "mm_trace_tile: empty tile or bad spp");
    // the tail records pack bounces | mirror hits << 16 (trace_kernels.hip tail_store)
    if (e->bounce_limit > 32767 || e->mirror_limit > 32767)
        return fail(c, MM_ERR_INVALID, "mm_trace_tile: bounce or mirror limit above 32767");
    if ((uint64_t)x0 + w > W || (uint64_t)y0 + (uint64_t)(h - 1) * y_stride >= H)
        return fail(c, MM_ERR_INVALID, "mm_trace_tile: tile outside the frame");
    if (n_frames == 0) return fail(c, MM_ERR_INVALID, "mm_trace_tile_frames: no frames");
    // MM_EXT_RGBA8: 4-byte RGBA8 pixels (the fused texture-write conversion) instead of float4
    const bool rgba8 = (e->flags & MM_EXT_RGBA8) != 0;
    if (rgba8 && (e->flags & MM_EXT_ACCUMULATE))
        return fail(c, MM_ERR_INVALID, "mm_trace_tile: MM_EXT_RGBA8 frames cannot accumulate");
    const size_t out_bpp = rgba8 ? 4 : 16;
    // the stores are out_bpp wide (a float4 per pixel, or one RGBA8 word): the output must be aligned to that
    if (reinterpret_cast<uintptr_t>(out_dev) % out_bpp)
        return fail(c, MM_ERR_INVALID, std::string("mm_trace_tile: output not ") + std::to_string(out_bpp) +
                                           "-byte aligned");
    HIPC(c, hipSetDevice(c->device));
    const bool want_stats = (e->flags & MM_EXT_COUNT_STATS) != 0;
    const uint64_t row_paths = (uint64_t)w * e->spp;
    const uint64_t tile_paths = row_paths * h;
    // MM_PIPE_WAVEFRONT: the wave-persistent kernel with mirror-tail deferral (compaction) always on
    const bool wave = c->pipe == MM_PIPE_WAVEFRONT;
    const bool persist = c->pipe != MM_PIPE_REFERENCE && (wave || c->opt_persist == 2);
    if (!persist && c->pipe != MM_PIPE_REFERENCE) return fail(c, MM_ERR_UNSUPPORTED, kRemoved);
    int form = 0, mode = 0;
    DevScene sc = dev_scene(c);
    if (persist) {
        int rc0 = choose_wavepersist(c, sc, form, mode);
        if (rc0) return rc0;
    }
    // mirror-tail deferral (MM_OPT_DEFER): samples staged per path, tails run from block-local rings; built for
    // the grid search and the lean BVH form with records in LDS (other forms run without it).  Auto: with the
    // whole search structure in LDS (the maze grid with its leaf boxes, or BVH nodes + compact records) and paths
    // of >= 8 bounces, on launches of >= MM_OPT_DEFER_MIN paths (C3 20 frames per launch 2.64 vs 2.74 ms/frame,
    // C4 20.97 vs 21.80, profiles/r03/ab_defer_claims.txt; rank 0 of an 8-way C3 split, 41 M paths per launch,
    // 0.356 vs 0.362, profiles/r03/emulated_scaling/; the N=64 scene, leaf boxes via L1/L2: 5.23 vs 4.90 without),
    // or where the samples are staged anyway (64 % spp != 0)
    const bool defer_on =
        c->opt_defer > 0 ||
        (c->opt_defer < 0 && (((mode == 11 || mode == 3) && e->bounce_limit >= 8u) ||
                              ((mode == 11 || mode == 3 || mode == 14) && 64 % e->spp != 0)));
    const bool defer_built = persist && wavepersist_defer_built(mode, form);
    if (wave && !defer_built)
        return fail(c, MM_ERR_UNSUPPORTED, "MM_PIPE_WAVEFRONT: no tail-deferral kernel for this scene's query "
                                           "method / LDS placement (grid search, or BVH form 7 with nodes + "
                                           "records in LDS)");
    bool defer = defer_built && (defer_on || wave) && (wave || tile_paths * n_frames >= c->opt_defer_min);
    // the deferral kernel's static LDS (tail ring, claimed queue ranges, and with ring kind 2 the rings'
    // 32 KB of records) must leave two 1024-thread blocks per CU: the records go to LDS where the
    // image leaves room (C3: 44 KB + 34 KB), else to global memory; a grid image without room even for the
    // ring words runs without the rings
    int ring = 0;
    if (defer) {
        const size_t img = wavepersist_lds_bytes(sc, mode);
        const bool static_grid = mode == 11 || mode == 14;  // the image goes into the kernel's static array
        for (int kind : {2, 1}) {
            hipFuncAttributes dattr{};
            if (wavepersist_attributes(mode, form, kind, &dattr) == hipSuccess &&
                (static_grid ? img <= wavepersist_grid_cap(kind) : img + dattr.sharedSizeBytes <= 80 * 1024)) {
                ring = kind;
                break;
            }
        }
        if (!ring) {
            if (wave)
                return fail(c, MM_ERR_UNSUPPORTED, "MM_PIPE_WAVEFRONT: grid image + tail ring exceed the LDS budget");
            defer = false;
        }
    }
    const bool fusable = persist && c->opt_fuse && 64 % e->spp == 0;
    // staging bound: a multi-frame launch stages all its frames at once; past kStagePathsMax it runs without
    // the rings (fused resolve) if it can
    if (defer && n_frames > 1 && tile_paths * n_frames > kStagePathsMax && fusable && !wave) defer = false;
    // wave-persistent kernel with whole pixels per 64-path chunk: resolve fused
    const bool fuse = fusable && !defer;
    // Rows per launch: the fused resolve needs no staging (one launch covers up to 2^31 paths, a whole C5
    // frame); staged samples (tail deferral, or no fused resolve) are bounded by kStagePathsMax per launch
    // (64 Mi paths without deferral, where the non-persistent kernels' short launches lose nothing)
    const uint64_t batch_paths = fuse ? (1ull << 31) : defer ? kStagePathsMax : (64ull << 20);
    const uint32_t rows_per_batch = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(h, batch_paths / row_paths));
    if (row_paths * rows_per_batch > 0xFFFFFFFFull) return fail(c, MM_ERR_INVALID, "mm_trace_tile: row too large");
    if (n_frames > 1) {
        // several frames in one launch: the wave-persistent kernel's queue, with the fused resolve or
        // (tail deferral) samples staged per frame
        if (!fuse && !defer)
            return fail(c, MM_ERR_UNSUPPORTED, "mm_trace_tile_frames: needs the wave-persistent kernel with the "
                                               "fused resolve (64 % spp == 0) or tail deferral");
        if (e->flags & MM_EXT_ACCUMULATE)
            return fail(c, MM_ERR_INVALID, "mm_trace_tile_frames: frames of one launch cannot accumulate into "
                                           "one image");
        const uint64_t queue = ((tile_paths + 63) / 64) * 64 * n_frames;
        if (queue + (1ull << 24) > 0xFFFFFFFFull)
            return fail(c, MM_ERR_INVALID, "mm_trace_tile_frames: more paths than one launch holds (2^32)");
        if (defer && tile_paths * n_frames > kStagePathsMax)
            return fail(c, MM_ERR_INVALID, "mm_trace_tile_frames: the frames' staged samples exceed 6 GiB "
                                           "(2^29 paths) per launch; use fewer frames per launch");
        if (rows_per_batch < h) return fail(c, MM_ERR_INVALID, "mm_trace_tile_frames: tile too large for one launch");
    }
    int rc = fuse ? MM_OK : ensure(c, c->d_samples, c->samples_cap,
                                   (size_t)(row_paths * rows_per_batch) * (defer ? n_frames : 1));
    if (rc) return rc;
    TailQueue tq;
    if (defer && ring == 1 && (rc = tail_queue(c, tq))) return rc;  // (records in LDS: no global ring)
    // aux: [0..3] stats (zeroed only when counted), [4] error flag (moved into the launch's status word by
    // the launch itself).  d_work: the wave-persistent kernel's queue head(s) and waves-done word
    // (self-cleaning).  No fill kernel on the default path: see k_trace_wavepersist.
    if (want_stats) HIPC(c, hipMemsetAsync(c->d_aux, 0, 4 * sizeof(unsigned long long), c->stream));
    if ((rc = begin_timing(c))) return rc;
    uint32_t* err_dev = reinterpret_cast<uint32_t*>(c->d_aux + 4);
    const uint64_t call_id = ++c->call_seq, first_launch = c->launch_seq;
    uint32_t launches = 0;
    for (uint32_t j0 = 0; j0 < h; j0 += rows_per_batch) {
        TileJob job;
        job.u = *u;
        job.e = *e;
        job.x0 = x0;
        job.y0 = y0 + j0 * y_stride;
        job.w = w;
        job.h = std::min(rows_per_batch, h - j0);
        job.y_stride = y_stride;
        job.view_w = W;
        job.fuse = fuse ? 1u : 0u;
        job.wave_ts = c->d_wave_ts;
        job.wave_ts_cap = c->wave_ts_cap;
        job.out = reinterpret_cast<char*>(out_dev) + (size_t)j0 * w * out_bpp;
        job.n_frames = n_frames;
        job.reserve_cus = c->opt_reserve_cus;
        job.fault = (c->opt_fault == 1 || c->opt_fault == 4) ? (uint32_t)c->opt_fault : 0u;
        if (c->opt_fault == 2) job.ring_spin = 0;
        if (defer) {
            job.defer_from = 1;
            job.defer_lanes = c->opt_defer > 0 ? (uint32_t)c->opt_defer : 32u;
            job.tail = tq;
            job.ring_lds = ring == 2 ? 1u : 0u;
        }
        // The launch's status slot is taken first (its device address is a kernel argument); if the
        // launch then fails to enqueue, the slot is released as finished-clean (a slot left
        // owned by a launch that never runs would fail every later call on the context), and the call
        // is still tracked below for the launches it did enqueue.
        if ((rc = next_status(c, job.status))) break;
        job.ring_diag = c->d_status + kStatusSlots;
        job.launch_id = (uint32_t)(c->launch_seq - 1);
        bool enqueued = false;
        rc = [&]() -> int {
            if (int r = prof_mark(c)) return r;
            if (c->opt_fault == 3) return fail(c, MM_ERR_HIP, "injected enqueue failure (MM_OPT_FAULT_INJECT 3)");
            if (persist) {
                c->last_form = form >= kFormGrid ? kFormGrid : form;
                c->last_mode = mode;
                c->last_kern_mode = mode;
                c->last_kern_form = form;
                c->last_kern_ring = defer ? ring : 0;
                HIPC(c, launch_trace_wavepersist(sc, job, c->d_samples, c->d_aux, err_dev,
                                                 c->d_work, want_stats, mode, form,
                                                 c->stream));
            } else {
                MegaOpts mo;
                mo.reference = c->pipe == MM_PIPE_REFERENCE;
                mo.block = c->opt_block ? c->opt_block : 256u;
                HIPC(c, launch_trace_mega(dev_scene(c), job, c->d_samples, c->d_aux, err_dev, want_stats, mo,
                                          c->stream));
                enqueued = true;  // the kernel runs: its slot is written by the publish below or here
                const hipError_t pe = launch_publish_status(err_dev, job.status, c->stream);
                if (pe != hipSuccess) {
                    // fold the kernel's error flag into THIS launch's slot (after a sync), so it is
                    // never published by -- and blamed on -- a later call's launch
                    uint32_t bits = 0;
                    (void)hipStreamSynchronize(c->stream);
                    (void)hipMemcpy(&bits, err_dev, sizeof(bits), hipMemcpyDeviceToHost);
                    (void)hipMemset(err_dev, 0, sizeof(bits));
                    __atomic_store_n(c->h_status + (c->launch_seq - 1) % kStatusSlots,
                                     bits | kErrPublish | kStatusDone, __ATOMIC_RELEASE);
                    return fail(c, MM_ERR_HIP, std::string("launch_publish_status: ") + hipGetErrorString(pe));
                }
            }
            enqueued = true;
            return prof_mark(c);
        }();
        if (!enqueued) {
            c->h_status[(c->launch_seq - 1) % kStatusSlots] = kStatusDone;  // nothing will write this slot
            break;
        }
        launches += fuse ? 1 : 2;
        if (rc) break;
        if (fuse) continue;
        // the frames' staged samples and output slices are contiguous (a multi-frame launch is one
        // row batch), so one resolve over h x n_frames rows covers them all
        TileJob rj = job;
        if (defer) rj.h = job.h * n_frames;
        const hipError_t re = launch_resolve(rj, c->d_samples, job.out, c->stream);
        if (re != hipSuccess) {
            rc = fail(c, MM_ERR_HIP, std::string("launch_resolve: ") + hipGetErrorString(re));
            break;
        }
    }
    c->last_defer = defer;
    if (c->launch_seq > first_launch) {  // the launches this call enqueued (all of them unless rc)
        char what[160];
        snprintf(what, sizeof(what), "%s, frames %u..%u, tile (%u, %u) %ux%u / %u, %u spp", n_frames > 1 ?
                 "mm_trace_tile_frames" : "mm_trace_tile", e->frame, e->frame + n_frames - 1, x0, y0, w, h,
                 y_stride, e->spp);
        c->pending.push_back({call_id, first_launch, c->launch_seq - first_launch, what, 0u});
    }
    if (rc) return rc;
    if ((rc = end_timing(c, launches))) return rc;
    if (want_stats) {
        if ((rc = read_aux(c, stats))) return rc;
        return report_failure(c, "");  // (synced: this call's own error, if any)
    }
    return MM_OK;
}

}  // namespace

int mm_trace_tile(mm_ctx* c, const mm_uniform* u, const mm_ext* e, uint32_t x0, uint32_t y0, uint32_t w,
                  uint32_t h, uint32_t y_stride, float* out_dev, mm_stats* stats) {
    return trace_tile_impl(c, u, e, 1, x0, y0, w, h, y_stride, out_dev, stats);
}

int mm_trace_tile_frames(mm_ctx* c, const mm_uniform* u, const mm_ext* e, uint32_t n_frames, uint32_t x0,
                         uint32_t y0, uint32_t w, uint32_t h, uint32_t y_stride, float* out_dev, mm_stats* stats) {
    return trace_tile_impl(c, u, e, n_frames, x0, y0, w, h, y_stride, out_dev, stats);
}

int mm_sync(mm_ctx* c) {
    if (!c) return MM_ERR_INVALID;
    HIPC(c, hipSetDevice(c->device));
    HIPC(c, hipStreamSynchronize(c->stream));
    if (int rc = read_aux(c, nullptr)) return rc;
    return report_failure(c, "");
}

int mm_last_call(const mm_ctx* c, uint64_t* call_id) {
    if (!c || !call_id) return MM_ERR_INVALID;
    *call_id = c->call_seq;
    return MM_OK;
}

int mm_call_status(mm_ctx* c, uint64_t call_id) {
    if (!c) return MM_ERR_INVALID;
    if (call_id == 0 || call_id > c->call_seq) return fail(c, MM_ERR_INVALID, "mm_call_status: no such call");
    poll_calls(c);
    for (const auto& k : c->pending)
        if (k.id == call_id) return MM_PENDING;
    for (auto& f : c->failed)
        if (f.id == call_id) {
            f.reported = true;
            return fail(c, error_code(f.bits), failed_text(f));
        }
    // a finished call not in the failed list: clean -- unless failed calls as old as it were dropped from the list
    if (call_id <= c->failed_dropped)
        return fail(c, MM_ERR_INVALID, "mm_call_status: status of call #" + std::to_string(call_id) +
                                           " no longer kept (older than the last " + std::to_string(kFailedKept) +
                                           " failed calls)");
    return MM_OK;
}

int mm_set_profiling(mm_ctx* c, int enable) {
    if (!c) return MM_ERR_INVALID;
    c->prof = enable != 0;
    return MM_OK;
}

int mm_kernel_timing(mm_ctx* c, float* total_ms, uint32_t* launches, int reset) {
    if (!c) return MM_ERR_INVALID;
    HIPC(c, hipSetDevice(c->device));
    float sum = 0.0f;
    for (size_t i = 0; i + 1 < c->prof_used; i += 2) {
        float ms = 0.0f;
        HIPC(c, hipEventSynchronize(c->prof_ev[i + 1]));
        HIPC(c, hipEventElapsedTime(&ms, c->prof_ev[i], c->prof_ev[i + 1]));
        sum += ms;
    }
    if (total_ms) *total_ms = sum;
    if (launches) *launches = (uint32_t)(c->prof_used / 2);
    if (reset) c->prof_used = 0;
    return MM_OK;
}

int mm_last_timing(mm_ctx* c, float* ms, uint32_t* launches) {
    if (!c) return MM_ERR_INVALID;
    if (c->last_ms < 0.0f) {
        HIPC(c, hipEventSynchronize(c->ev1));
        HIPC(c, hipEventElapsedTime(&c->last_ms, c->ev0, c->ev1));
    }
    if (ms) *ms = c->last_ms;
    if (launches) *launches = c->last_launches;
    return MM_OK;
}

}  // extern "C"
