// mm_comm.hip — the multi-GPU frame path of the C ABI (include/mm_comm.h):
// RCCL communicators over the contexts' GPUs, the frame-end gather of
// interleaved row tiles to rank 0, and the de-interleave kernel.
//
// Replaces the reference's single Metal device (src/main.rs:616) and its
// frame-end commit (src/main.rs:884-894) with N GPUs and one collective per
// gather.  The transfer is RCCL point-to-point (ncclSend / ncclRecv in one
// group: each rank's tile goes over its own xGMI link to rank 0, the links in
// parallel); the tiles are contiguous so RCCL moves them without packing, and
// rank 0 puts rows in frame order with one HBM-bound copy kernel.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <new>
#include <string>
#include <vector>

#include "mm_comm.h"
#include "mm_ctx.h"

using namespace mm;

struct mm_comm {
    ncclComm_t comm = nullptr;
    int rank = 0, n = 1, device = 0;
};

namespace {

#define HIPC(ctx, expr)                                                                                   \
    do {                                                                                                  \
        hipError_t _e = (expr);                                                                           \
        if (_e != hipSuccess) return ctx_fail((ctx), MM_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

#define NCCLC(ctx, comm, expr)                                                                            \
    do {                                                                                                  \
        ncclResult_t _r = (expr);                                                                         \
        if (_r != ncclSuccess) {                                                                          \
            const char* _l = (comm) ? ncclGetLastError(comm) : nullptr;                                   \
            return ctx_fail((ctx), MM_ERR_HIP, std::string(#expr) + ": " + ncclGetErrorString(_r) +      \
                                                   (_l && *_l ? std::string(" (") + _l + ")" : std::string())); \
        }                                                                                                 \
    } while (0)

// One block per (frame row y, frame f): row i = y / N of rank r = y % N's tile
// for frame f -- from `self` for rank 0 when given, else from the rank's slab of
// `staging` (rank-major, then frame, then row) -- to frame f's row y.  W: the
// widest word the row length and the pointers allow (16 B for any RGBA row of
// 4-pixel multiples).  HBM-bound: one read and one write of each byte.
template <typename W>
__global__ __launch_bounds__(256) void k_assemble_rows(const uint8_t* __restrict__ staging,
                                                       const uint8_t* __restrict__ self, uint8_t* __restrict__ frame,
                                                       uint32_t n_ranks, uint32_t n_frames, uint32_t rows_max,
                                                       uint32_t height, uint32_t row_words) {
    const uint32_t y = blockIdx.x, f = blockIdx.y;
    const uint32_t r = y % n_ranks, i = y / n_ranks;
    const size_t rb = (size_t)row_words * sizeof(W);
    const uint8_t* s = (r == 0 && self) ? self + ((size_t)f * rows_max + i) * rb
                                        : staging + (((size_t)r * n_frames + f) * rows_max + i) * rb;
    const W* src = reinterpret_cast<const W*>(s);
    W* dst = reinterpret_cast<W*>(frame + ((size_t)f * height + y) * rb);
    for (uint32_t k = threadIdx.x; k < row_words; k += blockDim.x) dst[k] = src[k];
}

bool aligned(const void* p, size_t a) { return reinterpret_cast<uintptr_t>(p) % a == 0; }

// the library is compiled against /opt/rocm's rccl.h but, in a
// process that mapped another librccl.so first (torch's), runs against that
// one.  The entry points used here are NCCL 2.x's stable ABI from 2.18 on;
// another major version, or an older runtime, is refused by name.
constexpr int kRcclMinVersion = 21800;
int check_rccl_runtime(mm_ctx* c, const char* who) {
    int v = 0;
    if (ncclGetVersion(&v) != ncclSuccess) return ctx_fail(c, MM_ERR_HIP, std::string(who) + ": ncclGetVersion failed");
    if (v / 10000 != NCCL_VERSION_CODE / 10000 || v < kRcclMinVersion)
        return ctx_fail(c, MM_ERR_UNSUPPORTED,
                        std::string(who) + ": RCCL runtime " + std::to_string(v) + " is not ABI-compatible with the "
                        "rccl.h " + std::to_string(NCCL_VERSION_CODE) + " the library was built with (needs major " +
                        std::to_string(NCCL_VERSION_CODE / 10000) + ", >= " + std::to_string(kRcclMinVersion) + ")");
    return MM_OK;
}

int launch_assemble(mm_ctx* c, const uint8_t* staging, const uint8_t* self, uint8_t* frame, uint32_t n_ranks,
                    uint32_t n_frames, uint32_t rows_max, uint32_t height, size_t row_bytes) {
    const dim3 grid(height, n_frames), block(256);
    const bool a16 = row_bytes % 16 == 0 && aligned(staging, 16) && (!self || aligned(self, 16)) && aligned(frame, 16);
    const bool a4 = row_bytes % 4 == 0 && aligned(staging, 4) && (!self || aligned(self, 4)) && aligned(frame, 4);
    if (a16)
        hipLaunchKernelGGL(k_assemble_rows<uint4>, grid, block, 0, c->stream, staging, self, frame, n_ranks, n_frames,
                           rows_max, height, (uint32_t)(row_bytes / 16));
    else if (a4)
        hipLaunchKernelGGL(k_assemble_rows<uint32_t>, grid, block, 0, c->stream, staging, self, frame, n_ranks,
                           n_frames, rows_max, height, (uint32_t)(row_bytes / 4));
    else
        hipLaunchKernelGGL(k_assemble_rows<uint8_t>, grid, block, 0, c->stream, staging, self, frame, n_ranks,
                           n_frames, rows_max, height, (uint32_t)row_bytes);
    HIPC(c, hipGetLastError());
    return MM_OK;
}

// Shape checks shared by the gathers: returns the tile's row bytes and rows.
int check_shape(mm_ctx* c, const char* who, uint32_t n_ranks, uint32_t n_frames, uint32_t width, uint32_t height,
                uint32_t bpp, size_t& row_bytes, uint32_t& rows_max) {
    if (n_ranks == 0 || n_frames == 0 || width == 0 || height == 0 || bpp == 0)
        return ctx_fail(c, MM_ERR_INVALID, std::string(who) + ": empty shape");
    if (n_frames > 65535 || height > (1u << 20) || bpp > 64)
        return ctx_fail(c, MM_ERR_INVALID, std::string(who) + ": more than 65535 frames, 2^20 rows or 64 B/px");
    if (n_ranks > height) return ctx_fail(c, MM_ERR_INVALID, std::string(who) + ": more ranks than rows");
    row_bytes = (size_t)width * bpp;
    rows_max = (height + n_ranks - 1) / n_ranks;
    return MM_OK;
}

// Rank 0's receive staging: n_ranks slabs of one tile set each, used by one
// gather at a time: the stream of this gather waits for the previous gather's
// assembly (it may have run on another stream), and a regrow frees the old
// buffer only once that assembly is done.
int ensure_staging(mm_ctx* c, size_t bytes) {
    if (!c->gather_done) HIPC(c, hipEventCreateWithFlags(&c->gather_done, hipEventDisableTiming));
    if (c->gather_pending) HIPC(c, hipStreamWaitEvent(c->stream, c->gather_done, 0));
    if (c->d_gather && c->gather_cap >= bytes) return MM_OK;
    if (c->gather_pending) HIPC(c, hipEventSynchronize(c->gather_done));
    (void)hipFree(c->d_gather);
    c->d_gather = nullptr;
    c->gather_cap = 0;
    HIPC(c, hipMalloc((void**)&c->d_gather, std::max<size_t>(bytes, 16)));
    c->gather_cap = bytes;
    return MM_OK;
}

// After a gather's assembly: mark the staging busy until this point of the
// gather's stream (only when the gather used it).
int staging_released(mm_ctx* c, bool used) {
    if (!used) return MM_OK;
    HIPC(c, hipEventRecord(c->gather_done, c->stream));
    c->gather_pending = true;
    return MM_OK;
}

// Rank r's part of the gather inside an open RCCL group.
int gather_part(mm_ctx* c, mm_comm* m, const void* tile, size_t slab, uint32_t flags) {
    if (m->rank != 0) {
        NCCLC(c, m->comm, ncclSend(tile, slab, ncclUint8, 0, m->comm, c->stream));
        return MM_OK;
    }
    for (int r = 1; r < m->n; ++r)
        NCCLC(c, m->comm, ncclRecv(c->d_gather + (size_t)r * slab, slab, ncclUint8, r, m->comm, c->stream));
    if (flags & MM_GATHER_SELF_VIA_RCCL) {
        NCCLC(c, m->comm, ncclSend(tile, slab, ncclUint8, 0, m->comm, c->stream));
        NCCLC(c, m->comm, ncclRecv(c->d_gather, slab, ncclUint8, 0, m->comm, c->stream));
    }
    return MM_OK;
}

}  // namespace

extern "C" {

int mm_comm_unique_id(mm_ctx* c, uint8_t id[MM_COMM_ID_BYTES]) {
    if (!c || !id) return MM_ERR_INVALID;
    static_assert(sizeof(ncclUniqueId) == MM_COMM_ID_BYTES, "RCCL unique id size");
    HIPC(c, hipSetDevice(c->device));
    ncclUniqueId u;
    NCCLC(c, nullptr, ncclGetUniqueId(&u));
    std::copy(u.internal, u.internal + MM_COMM_ID_BYTES, reinterpret_cast<char*>(id));
    return MM_OK;
}

int mm_comm_init_rank(mm_ctx* c, int n_ranks, int rank, const uint8_t id[MM_COMM_ID_BYTES], mm_comm** out) {
    if (!c || !id || !out) return MM_ERR_INVALID;
    *out = nullptr;
    if (n_ranks < 1 || rank < 0 || rank >= n_ranks) return ctx_fail(c, MM_ERR_INVALID, "mm_comm_init_rank: bad rank");
    if (int rc = check_rccl_runtime(c, "mm_comm_init_rank")) return rc;
    HIPC(c, hipSetDevice(c->device));
    ncclUniqueId u;
    std::copy(id, id + MM_COMM_ID_BYTES, reinterpret_cast<uint8_t*>(u.internal));
    mm_comm* m = new (std::nothrow) mm_comm();
    if (!m) return MM_ERR_NOMEM;
    const ncclResult_t r = ncclCommInitRank(&m->comm, n_ranks, u, rank);
    if (r != ncclSuccess) {
        delete m;
        return ctx_fail(c, MM_ERR_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    }
    m->rank = rank;
    m->n = n_ranks;
    m->device = c->device;
    *out = m;
    return MM_OK;
}

int mm_comm_init_all(int n, mm_ctx* const* ctxs, mm_comm** out) {
    if (n < 1 || !ctxs || !out || !ctxs[0]) return MM_ERR_INVALID;
    mm_ctx* c0 = ctxs[0];
    std::vector<int> devs(n);
    for (int i = 0; i < n; ++i) {
        if (!ctxs[i]) return ctx_fail(c0, MM_ERR_INVALID, "mm_comm_init_all: null context");
        devs[i] = ctxs[i]->device;
        for (int j = 0; j < i; ++j)
            if (devs[j] == devs[i]) return ctx_fail(c0, MM_ERR_INVALID, "mm_comm_init_all: two contexts on one GPU");
        out[i] = nullptr;
    }
    if (int rc = check_rccl_runtime(c0, "mm_comm_init_all")) return rc;
    std::vector<ncclComm_t> comms(n);
    NCCLC(c0, nullptr, ncclCommInitAll(comms.data(), n, devs.data()));
    for (int i = 0; i < n; ++i) {
        mm_comm* m = new (std::nothrow) mm_comm();
        if (!m) {
            for (int j = 0; j < n; ++j) {
                if (j < i) { delete out[j]; out[j] = nullptr; }
                (void)ncclCommDestroy(comms[j]);
            }
            return MM_ERR_NOMEM;
        }
        m->comm = comms[i];
        m->rank = i;
        m->n = n;
        m->device = devs[i];
        out[i] = m;
    }
    return MM_OK;
}

int mm_comm_info(const mm_comm* m, int* rank, int* n_ranks, int* device) {
    if (!m) return MM_ERR_INVALID;
    if (rank) *rank = m->rank;
    if (n_ranks) *n_ranks = m->n;
    if (device) *device = m->device;
    return MM_OK;
}

int mm_comm_rccl_version(void) {
    int v = 0;
    return ncclGetVersion(&v) == ncclSuccess ? v : 0;
}

int mm_comm_rccl_header_version(void) { return NCCL_VERSION_CODE; }

void mm_comm_destroy(mm_comm* m) {
    if (!m) return;
    if (m->comm) {
        (void)hipSetDevice(m->device);
        (void)ncclCommDestroy(m->comm);
    }
    delete m;
}

int mm_row_shard(uint32_t height, uint32_t n_ranks, uint32_t rank, uint32_t* y0, uint32_t* y_stride, uint32_t* rows,
                 uint32_t* rows_max) {
    if (n_ranks == 0 || rank >= n_ranks || height == 0) return MM_ERR_INVALID;
    if (y0) *y0 = rank;
    if (y_stride) *y_stride = n_ranks;
    if (rows) *rows = rank < height ? (height - rank + n_ranks - 1) / n_ranks : 0;
    if (rows_max) *rows_max = (height + n_ranks - 1) / n_ranks;
    return MM_OK;
}

int mm_gather_rows(mm_ctx* c, mm_comm* m, const void* tile, uint32_t n_frames, uint32_t width, uint32_t height,
                   uint32_t bpp, void* frame, uint32_t flags) {
    if (!c) return MM_ERR_INVALID;
    if (!m || !tile) return ctx_fail(c, MM_ERR_INVALID, "mm_gather_rows: null communicator or tile");
    if (m->device != c->device) return ctx_fail(c, MM_ERR_INVALID, "mm_gather_rows: communicator of another GPU");
    size_t rb = 0;
    uint32_t rows_max = 0;
    if (int rc = check_shape(c, "mm_gather_rows", (uint32_t)m->n, n_frames, width, height, bpp, rb, rows_max)) return rc;
    if (m->rank == 0 && !frame) return ctx_fail(c, MM_ERR_INVALID, "mm_gather_rows: rank 0 needs frame_dev");
    const size_t slab = (size_t)n_frames * rows_max * rb;
    HIPC(c, hipSetDevice(c->device));
    const bool via = (flags & MM_GATHER_SELF_VIA_RCCL) != 0;
    if (m->rank == 0 && (m->n > 1 || via))
        if (int rc = ensure_staging(c, (size_t)m->n * slab)) return rc;
    if (m->n > 1 || via) {
        NCCLC(c, m->comm, ncclGroupStart());
        const int rc = gather_part(c, m, tile, slab, flags);
        const ncclResult_t ge = ncclGroupEnd();
        if (rc) return rc;
        if (ge != ncclSuccess) return ctx_fail(c, MM_ERR_HIP, std::string("ncclGroupEnd: ") + ncclGetErrorString(ge));
    }
    if (m->rank != 0) return MM_OK;
    if (int rc = launch_assemble(c, c->d_gather, via ? nullptr : static_cast<const uint8_t*>(tile),
                                 static_cast<uint8_t*>(frame), (uint32_t)m->n, n_frames, rows_max, height, rb))
        return rc;
    return staging_released(c, m->n > 1 || via);
}

int mm_gather_rows_all(int n, mm_ctx* const* ctxs, mm_comm* const* comms, const void* const* tiles, uint32_t n_frames,
                       uint32_t width, uint32_t height, uint32_t bpp, void* frame, uint32_t flags) {
    if (n < 1 || !ctxs || !comms || !tiles || !ctxs[0]) return MM_ERR_INVALID;
    mm_ctx* c0 = ctxs[0];
    int root = -1;
    for (int i = 0; i < n; ++i) {
        if (!ctxs[i] || !comms[i] || !tiles[i]) return ctx_fail(c0, MM_ERR_INVALID, "mm_gather_rows_all: null entry");
        if (comms[i]->n != n || comms[i]->device != ctxs[i]->device)
            return ctx_fail(c0, MM_ERR_INVALID, "mm_gather_rows_all: communicators do not match the contexts");
        if (comms[i]->rank == 0) root = i;
    }
    if (root < 0) return ctx_fail(c0, MM_ERR_INVALID, "mm_gather_rows_all: no rank 0");
    mm_ctx* cr = ctxs[root];
    size_t rb = 0;
    uint32_t rows_max = 0;
    if (int rc = check_shape(cr, "mm_gather_rows_all", (uint32_t)n, n_frames, width, height, bpp, rb, rows_max)) return rc;
    if (!frame) return ctx_fail(cr, MM_ERR_INVALID, "mm_gather_rows_all: null frame_dev");
    const size_t slab = (size_t)n_frames * rows_max * rb;
    const bool via = (flags & MM_GATHER_SELF_VIA_RCCL) != 0;
    HIPC(cr, hipSetDevice(cr->device));
    if (n > 1 || via)
        if (int rc = ensure_staging(cr, (size_t)n * slab)) return rc;
    if (n > 1 || via) {
        // one thread drives every GPU: the ranks' parts must be one group (RCCL's rule for several devices
        // per thread), each on its own context's stream
        NCCLC(cr, comms[root]->comm, ncclGroupStart());
        int rc = MM_OK;
        for (int i = 0; i < n && rc == MM_OK; ++i) {
            if (hipSetDevice(ctxs[i]->device) != hipSuccess) {
                rc = ctx_fail(cr, MM_ERR_HIP, "mm_gather_rows_all: hipSetDevice");
                break;
            }
            rc = gather_part(ctxs[i], comms[i], tiles[i], slab, flags);
            if (rc && ctxs[i] != cr) ctx_fail(cr, rc, ctxs[i]->err);
        }
        const ncclResult_t ge = ncclGroupEnd();
        if (rc) return rc;
        if (ge != ncclSuccess) return ctx_fail(cr, MM_ERR_HIP, std::string("ncclGroupEnd: ") + ncclGetErrorString(ge));
        HIPC(cr, hipSetDevice(cr->device));
    }
    if (int rc = launch_assemble(cr, cr->d_gather, via ? nullptr : static_cast<const uint8_t*>(tiles[root]),
                                 static_cast<uint8_t*>(frame), (uint32_t)n, n_frames, rows_max, height, rb))
        return rc;
    return staging_released(cr, n > 1 || via);
}

int mm_assemble_rows(mm_ctx* c, const void* tiles, uint32_t n_ranks, uint32_t n_frames, uint32_t width,
                     uint32_t height, uint32_t bpp, void* frame) {
    if (!c) return MM_ERR_INVALID;
    if (!tiles || !frame) return ctx_fail(c, MM_ERR_INVALID, "mm_assemble_rows: null buffer");
    size_t rb = 0;
    uint32_t rows_max = 0;
    if (int rc = check_shape(c, "mm_assemble_rows", n_ranks, n_frames, width, height, bpp, rb, rows_max)) return rc;
    HIPC(c, hipSetDevice(c->device));
    return launch_assemble(c, static_cast<const uint8_t*>(tiles), nullptr, static_cast<uint8_t*>(frame), n_ranks,
                           n_frames, rows_max, height, rb);
}

}  // extern "C"
