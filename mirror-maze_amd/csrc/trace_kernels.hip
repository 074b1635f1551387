// trace_kernels.hip — gfx950 kernels for mirror-maze's per-pixel ray-trace loop.
//
//   k_prep_rects         per-rect subexpressions of ray_rect_intersect
//   k_trace_chunks       parity mode: the reference dispatch (shaders.metal:245-368)
//   k_trace_mega         MM_PIPE_REFERENCE: one thread per (pixel, sample) path,
//                        the straight statement (IEEE division everywhere)
//   k_trace_wavepersist  throughput mode, the production kernel: resident
//                        blocks, waves pull 64-path chunks, pixels resolved in
//                        the wave
//   k_resolve            per-pixel sample reduction in the reference's order
#include <hip/hip_runtime.h>

#include "grid_build.h"
#include "mm_launch.h"
#include "mm_path.h"
#include "mm_wave_util.h"

namespace mm {

// ---------------------------------------------------------------------------
__global__ void k_prep_rects(const mm_rect* __restrict__ rects, uint32_t n, float4* __restrict__ geo) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const mm_rect r = rects[k];
    const F3 o = F3{r.o[0], r.o[1], r.o[2]};
    const F3 v = F3{r.v[0], r.v[1], r.v[2]};
    const F3 u = F3{r.u[0], r.u[1], r.u[2]};
    const F3 nn = normalize3(cross3(v, u));       // shaders.metal:52 (and :309)
    const float lv = sqrtf(dot3(v, v));           // length(mirror.v), :60
    const float lu = sqrtf(dot3(u, u));           // length(mirror.u), :61
    geo[4 * k + 0] = make_float4(o.x, o.y, o.z, lv);
    geo[4 * k + 1] = make_float4(nn.x, nn.y, nn.z, lu);
    geo[4 * k + 2] = make_float4(v.x, v.y, v.z, 1.0f / lv);
    geo[4 * k + 3] = make_float4(u.x, u.y, u.z, 1.0f / lu);
}

hipError_t launch_prep_rects(const mm_rect* rects, uint32_t n, float4* geo_dev, hipStream_t s) {
    hipLaunchKernelGGL(k_prep_rects, dim3((n + 255) / 256), dim3(256), 0, s, rects, n, geo_dev);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Parity mode.  One workgroup = one reference threadgroup of 32x32 threads;
// flat = gid.x + 32*gid.y, so each wave64 holds exactly the 64 samples of one
// pixel (pixel_number = flat/64, shaders.metal:271-275) and the reference's
// threadgroup-memory tree reduction (shaders.metal:342-367) becomes a
// shuffle reduction inside the wave with the same pairing and order.
template <bool kStats>
__global__ __launch_bounds__(1024) void k_trace_chunks(DevScene sc, mm_uniform u,
                                                       const uint32_t* __restrict__ chunks, float4* __restrict__ fb,
                                                       uint32_t* __restrict__ fb8, unsigned long long* stats,
                                                       uint32_t* err) {
    const uint32_t W = (uint32_t)u.view_w, H = (uint32_t)u.view_h;
    const uint32_t chunk = u.chunk_w, ppc = chunk * chunk;  // 4, 16
    const uint32_t gx = blockIdx.x, gy = blockIdx.y;
    // pixel_buffer_index in float, IR %26-%31
    const uint32_t pbi = cvt_u32_sat(((u.view_w * 0.5f) * (float)gy) / (float)ppc + (float)gx);
    const uint32_t cx = chunks[2 * pbi], cy = chunks[2 * pbi + 1];
    const uint32_t flat = threadIdx.x;          // 0..1023
    const uint32_t lx = flat & 31, ly = flat >> 5;
    const uint32_t pn = flat >> 6;              // flat / (1024 / 16)
    const uint32_t px = cx + pn / chunk, py = cy + pn % chunk;
    uint32_t seed = seed_reference(gx * 32 + lx, gy * 32 + ly, u.time);
    const F3 d = jitter(primary_dir(u, px, py), seed);
    const F3 ori = F3{u.cam.center[0], u.cam.center[1], u.cam.center[2]};
    ScratchStack stack;
    Counters c;
    bool overflow = false;
    const BvhQuery<kStats, kFormIfIf, NodeView<const float4*>> q{sc, view(sc.nodes)};
    F3 s = trace_path<kStats>(sc, q, ori, d, seed, 5, 15, stack, c, overflow);  // shaders.metal:294-295
    if (overflow) atomicOr(err, 1u);
    // level 1..3: test[f] += test[f+1], += test[f+2], += test[f+4]
    s = s + F3{__shfl_xor(s.x, 1), __shfl_xor(s.y, 1), __shfl_xor(s.z, 1)};
    s = s + F3{__shfl_xor(s.x, 2), __shfl_xor(s.y, 2), __shfl_xor(s.z, 2)};
    s = s + F3{__shfl_xor(s.x, 4), __shfl_xor(s.y, 4), __shfl_xor(s.z, 4)};
    // first thread of the pixel: acc = blk0 + blk1 + ... + blk7, then / 64
    F3 acc = s;
#pragma unroll
    for (int i = 1; i < 8; ++i) acc = acc + F3{__shfl(s.x, 8 * i), __shfl(s.y, 8 * i), __shfl(s.z, 8 * i)};
    if (kStats) flush_stats(stats, c, 64);
    if ((flat & 63) == 0 && px < W && py < H) {
        const float m = 64.0f;
        const F3 o = F3{acc.x / m, acc.y / m, acc.z / m};
        fb[(size_t)py * W + px] = make_float4(o.x, o.y, o.z, 1.0f);
        fb8[(size_t)py * W + px] = unorm8(o.x) | (unorm8(o.y) << 8) | (unorm8(o.z) << 16) | (255u << 24);
    }
}

hipError_t launch_trace_chunks(const DevScene& sc, const mm_uniform& u, const uint32_t* chunks_dev,
                               uint32_t grid_w, uint32_t grid_h, float4* fb, uint32_t* fb8,
                               unsigned long long* stats_dev, uint32_t* err, bool count_stats, hipStream_t s) {
    if (count_stats)
        hipLaunchKernelGGL(k_trace_chunks<true>, dim3(grid_w, grid_h), dim3(1024), 0, s, sc, u, chunks_dev, fb, fb8,
                           stats_dev, err);
    else
        hipLaunchKernelGGL(k_trace_chunks<false>, dim3(grid_w, grid_h), dim3(1024), 0, s, sc, u, chunks_dev, fb, fb8,
                           stats_dev, err);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// MM_PIPE_REFERENCE, one thread per path: path = pixel*spp + sample, the
// straight statement of the reference walk (traverse_reference, IEEE division
// everywhere).  (The round-1 one-thread-per-path kernels over the production
// BVH loop forms measured slower than the wave-persistent kernel and were
// removed in round 6)
template <bool kStats, typename Q>
__device__ __forceinline__ void mega_body(const DevScene& sc, const Q& q, const TileJob& job,
                                          Sample* __restrict__ samples, unsigned long long* stats, uint32_t* err) {
    const uint32_t spp = job.e.spp;
    const uint32_t n_paths = job.w * job.h * spp;
    const uint32_t path = blockIdx.x * blockDim.x + threadIdx.x;
    Counters c;
    if (path < n_paths) {
        const uint32_t pix = path / spp, smp = path - pix * spp;
        const uint32_t j = pix / job.w, i = pix - j * job.w;
        const uint32_t px = job.x0 + i, py = job.y0 + j * job.y_stride;
        uint32_t seed = seed_tile(py * job.view_w + px, smp, job.e.frame);
        const F3 d = jitter(primary_dir(job.u, px, py), seed);
        const F3 ori = F3{job.u.cam.center[0], job.u.cam.center[1], job.u.cam.center[2]};
        ScratchStack stack;
        bool overflow = false;
        const F3 s = trace_path<kStats>(sc, q, ori, d, seed, (int)job.e.bounce_limit, (int)job.e.mirror_limit, stack,
                                        c, overflow);
        if (overflow) atomicOr(err, 1u);
        samples[path] = s;
    }
    if (kStats) flush_stats(stats, c, path < n_paths ? 1u : 0u);
}

template <bool kStats>
__global__ __launch_bounds__(1024) void k_trace_mega(DevScene sc, TileJob job, Sample* __restrict__ samples,
                                                     unsigned long long* stats, uint32_t* err) {
    mega_body<kStats>(sc, RefQuery<kStats>{sc}, job, samples, stats, err);
}

// ---------------------------------------------------------------------------
// Wave-persistent megakernel: resident 1024-thread blocks (two per CU at
// <= 64 VGPRs, 8 waves per SIMD) fill LDS once; each wave takes 64
// consecutive paths at a time from a global counter and traces them, so no
// block waits for its slowest wave before the CU can take more work.  With
// 64 % spp == 0 the wave's 64 paths are whole pixels and it resolves them
// itself (job.fuse).  A multi-frame launch queues frame 0's chunks, then frame
// 1's, ...; a chunk's frame picks its RNG frame and output slice.
//
// Mirror-tail deferral (job.defer_from < 2^30): once at most defer_lanes of a
// wave's 64 lanes still run -- past bounce_limit only paths that hit mirrors
// continue (shaders.metal:306, `n < bounce_limit + mirror_hits`) -- those
// lanes queue their path state in their block's tail ring and the wave takes
// a new chunk; the block's waves take 64 queued tails at a time as a chunk of
// their own.  On C3 a wave otherwise spends ~27 % of its bounce iterations on
// <= 12 live lanes (scripts/grid_sim.c).  Samples are then staged per path and
// resolved by k_resolve (the same operations in the same order as the fused
// resolve).

// A deferred path's state (64 B: ori.xyz dir.x | dir.yz T.xy | T.z L.xyz |
// seed, (n - mh) | mh << 15 | bank << 30, sample slot, s1) into / out of slot s of its block's tail
// ring.  kLdsPay (the deferral kernel with kRing = 2, chosen where the grid
// image leaves room -- C3: 44 KB image + 34 KB static LDS per block, two
// blocks per CU): the payload lives in the block's LDS beside the turn words,
// word group j of slot s at ring_pay()[j * kTailRing + s] (a wave's
// consecutive entries are consecutive 16-B words: no bank conflicts), 32 KB
// per block.  Otherwise (kRing = 1): the queue's global records
// blockIdx.x * kTailRing + s (mm_launch.h TailQueue).
__device__ __forceinline__ uint4* ring_pay() {
    __shared__ uint4 pay[4 * kTailRing];
    return pay;
}

template <bool kLdsPay>
__device__ __forceinline__ void tail_store(const TailQueue& q, uint32_t s, const PathState& p, uint32_t slot) {
    const uint4 w0 = make_uint4(__float_as_uint(p.ori.x), __float_as_uint(p.ori.y), __float_as_uint(p.ori.z),
                                __float_as_uint(p.dir.x));
    const uint4 w1 = make_uint4(__float_as_uint(p.dir.y), __float_as_uint(p.dir.z), __float_as_uint(p.T.x),
                                __float_as_uint(p.T.y));
    const uint4 w2 = make_uint4(__float_as_uint(p.T.z), __float_as_uint(p.L.x), __float_as_uint(p.L.y),
                                __float_as_uint(p.L.z));
    // (mh <= n and n - mh < bounce_limit <= 32767, mh < mirror_limit <= 32767: mm_runtime.hip checks the limits)
    const uint32_t nmb = (uint32_t)(p.n - p.mh) | ((uint32_t)p.mh << 15) | (p.bank << 30);
    const uint4 w3 = make_uint4(p.seed, nmb, slot, p.s1);
    if constexpr (kLdsPay) {
        uint4* r = ring_pay() + s;
        r[0] = w0; r[kTailRing] = w1; r[2 * kTailRing] = w2; r[3 * kTailRing] = w3;
    } else {
        uint4* r = q.rec + 4u * ((size_t)blockIdx.x * kTailRing + s);
        r[0] = w0; r[1] = w1; r[2] = w2; r[3] = w3;
    }
}

template <bool kLdsPay>
__device__ __forceinline__ uint32_t tail_load(const TailQueue& q, uint32_t s, PathState& p) {
    uint4 a, b, c, d;
    if constexpr (kLdsPay) {
        const uint4* r = ring_pay() + s;
        a = r[0]; b = r[kTailRing]; c = r[2 * kTailRing]; d = r[3 * kTailRing];
    } else {
        const uint4* r = q.rec + 4u * ((size_t)blockIdx.x * kTailRing + s);
        a = r[0]; b = r[1]; c = r[2]; d = r[3];
    }
    p.ori = F3{__uint_as_float(a.x), __uint_as_float(a.y), __uint_as_float(a.z)};
    p.dir = F3{__uint_as_float(a.w), __uint_as_float(b.x), __uint_as_float(b.y)};
    p.T = F3{__uint_as_float(b.z), __uint_as_float(b.w), __uint_as_float(c.x)};
    p.L = F3{__uint_as_float(c.y), __uint_as_float(c.z), __uint_as_float(c.w)};
    p.seed = d.x;
    p.mh = (int)((d.y >> 15) & 0x7FFFu);
    p.n = (int)(d.y & 0x7FFFu) + p.mh;
    p.bank = d.y >> 30;
    p.s1 = d.w;
    return d.z;
}

__device__ __forceinline__ F3 path_value(const PathState& p) {
    return F3{sqrtf(fmaxf(p.L.x, 0.0f)), sqrtf(fmaxf(p.L.y, 0.0f)), sqrtf(fmaxf(p.L.z, 0.0f))};
}

// Block-local tail ring (kDefer): kTailRing entries per
// block, payload in the queue's records blockIdx.x * kTailRing + slot.  LDS
// words (static, at constant addresses -- every word of the ring's state that
// lives in an SGPR across the bounce loop pushes a grid-search value into a
// spill): ctl[0] = entries reserved, ctl[1] = entries claimed, ctl[2..3]
// unused, then one turn word per slot.  Entry n lives in slot
// n % kTailRing; its writer waits for turn == 2 * lap (the previous lap's
// reader is done), writes the payload, sets 2 * lap + 1; its reader waits for
// that, loads, sets 2 * lap + 2 (turn values modulo 2^24, ring_turn_value).  A
// writer reserves only entries whose previous-lap entry is claimed and a
// reader claims only reserved entries, so every wait is on an operation of a
// smaller entry number that is already under way -- no cycle (and no cycle
// through the SIMT rule either: a reader's 64 entries and a writer's <= 64
// are within 127 of each other, a lap is 512).  Progress: every claim of
// tails runs at least one bounce (wavepersist_ring_body).  Only waves of one
// block (one CU) touch a ring: workgroup-scope release / acquire order the
// payload, no L2 writeback or invalidate.  Protocol model:
// tests/ring_model/ring_model.cpp (tests/test_ring_model.py).
//
// Memory ordering of the payload.  Payload in LDS
// (kRing = 2): payload and turn word are both LDS operations of the same
// wave, and the workgroup-scope release / acquire put s_waitcnt lgkmcnt(0)
// between them.  Payload in global memory: the release of a turn word is a
// plain ds_write_b32 with no s_waitcnt vmcnt before it -- the writer's four
// global_store_dwordx4 and the reader's four global_load_dwordx4 are still in
// flight when it issues (DESIGN.md s4 quotes the ISA).  That is LLVM's AMDGPU
// memory model for a workgroup-scope release on gfx94x/gfx950 outside
// threadgroup-split mode (.amdhsa_tg_split 0 here): all waves of a work-group
// use the same vector L1, which serves a CU's vector memory requests in
// order, so a later load by a block-mate that has seen the turn word cannot
// pass the earlier stores; no wait is needed.
__device__ __forceinline__ uint32_t* ring_ctl() {
    __shared__ uint32_t words[4 + kTailRing];
    return words;
}
__device__ __forceinline__ uint32_t* ring_turn(uint32_t seq) { return ring_ctl() + 4 + (seq % kTailRing); }
__device__ __forceinline__ uint32_t ring_lap(uint32_t seq) { return seq / kTailRing; }
// 2 * lap + c modulo 2^24: the entry counters are 32-bit, so lap wraps from
// 2^32 / kTailRing - 1 = 2^23 - 1 to 0 and 2 * lap + 2 = 2^24 must read as the
// next lap's 0 (without the mask the first writer after the wrap waits for 0
// while its slot holds 2^24: the round-3 timeout, tests/test_ring_model.py).
static_assert(kTailRing == 512, "turn values are taken modulo 2 * 2^32 / kTailRing");
__device__ __forceinline__ uint32_t ring_turn_value(uint32_t seq, uint32_t c) {
    return (2u * ring_lap(seq) + c) & 0xFFFFFFu;
}

__device__ __forceinline__ uint32_t lds_ld(uint32_t* a) {
    return __hip_atomic_load(a, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The executing lanes reserve consecutive entries: ONE compare-and-swap by the
// leader, no retry loop (a loop nested in the bounce loop costs SGPRs the grid
// search then spills).  It fails if the ring lacks room for them or another
// wave of the block reserved in between; then no lane defers and the wave
// tries again at its next bounce.  Exact: `reserved - claimed` never passes
// kTailRing.
__device__ __forceinline__ bool ring_reserve(uint32_t& seq) {
    uint32_t* ctl = ring_ctl();
    const uint64_t m = __ballot(1);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t leader = (uint32_t)__ffsll((unsigned long long)m) - 1u;
    const uint32_t cnt = (uint32_t)__popcll(m);
    uint32_t base = 0xFFFFFFFFu;
    if (lane == leader) {
        const uint32_t claimed = lds_ld(ctl + 1);
        uint32_t reserved = lds_ld(ctl + 0);  // read after claimed: reserved >= claimed
        if (reserved + cnt - claimed <= kTailRing &&
            __hip_atomic_compare_exchange_strong(ctl + 0, &reserved, reserved + cnt, __ATOMIC_ACQ_REL,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
            base = reserved;
    }
    base = __shfl(base, (int)leader);
    if (base == 0xFFFFFFFFu) return false;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    seq = base + (uint32_t)__popcll(m & lt);
    return true;
}

// Leader lane: claim min(available, 64) entries if at least `need` are
// reserved and not yet claimed; returns the count (0: none), first in `first`.
__device__ __forceinline__ uint32_t ring_claim(uint32_t need, uint32_t& first) {
    uint32_t* ctl = ring_ctl();
    uint32_t claimed = lds_ld(ctl + 1);
    const uint32_t reserved = lds_ld(ctl + 0);  // read after claimed: reserved >= claimed
    const uint32_t avail = reserved - claimed;
    if (avail < need) return 0;
    const uint32_t k = min(avail, 64u);
    if (!__hip_atomic_compare_exchange_strong(ctl + 1, &claimed, claimed + k, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE,
                                              __HIP_MEMORY_SCOPE_WORKGROUP))
        return 0;
    first = claimed;
    return k;
}

// A protocol wait -- a reader for the writer of its entry, a writer for the
// previous lap's reader -- waits on a step already under way, so it is
// bounded (job.ring_spin polls, ~50 ms): a protocol bug ends the launch with
// error bit 2 rather than a grid that never drains, and the launch's first
// timed-out wait leaves a record of itself (ring_timeout).  Returns false on
// timeout; the caller then skips its load / store.
//
// The record (TileJob::ring_diag, host-mapped, 16 words; mm_last_error prints
// it): [0] 1 = written, [1] role (1 reader, 2 writer), [2] entry seq, [3]
// wanted turn value, [4] the turn value last seen, [5] reserved, [6] claimed,
// [7] block, [8] wave, [9] lane, [10..11] unused, [12..13] wall clock at the
// timeout (100 MHz), [14] polls, [15] launch id.  (No clock at the wait's
// start: a 64-bit value live across the wait loop cost the deferral kernel
// 10 more scratch operations in its chunk loop; the polls give the length.)
// [0] is taken by a compare-and-swap 0 -> 2 before the fields are written and
// set to 1 after: a record the host has not read yet (1) is never overwritten
// by a later launch's timeout, and the host reads only 1.
__device__ __forceinline__ void ring_timeout(const TileJob& job, uint32_t* err, uint32_t role, uint32_t seq,
                                             uint32_t want, uint32_t seen, uint32_t polls) {
    if (atomicOr(err, kErrRing) & kErrRing) return;  // not the launch's first timeout
    uint32_t* d = job.ring_diag;
    if (!d) return;
    uint32_t free_word = 0u;
    if (!__hip_atomic_compare_exchange_strong(d, &free_word, 2u, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_SYSTEM))
        return;  // an earlier launch's record is still unread
    const uint64_t t1 = wall_clock64();
    d[1] = role; d[2] = seq; d[3] = want; d[4] = seen;
    d[5] = lds_ld(ring_ctl() + 0); d[6] = lds_ld(ring_ctl() + 1);
    d[7] = blockIdx.x; d[8] = threadIdx.x >> 6; d[9] = threadIdx.x & 63u;
    d[12] = (uint32_t)t1; d[13] = (uint32_t)(t1 >> 32);  // ([10..11] unwritten: two zero registers
    // held for them across the kernel were spilled around every chunk's bounce loop -- 1 KB of scratch per chunk)
    d[14] = polls; d[15] = job.launch_id;
    __threadfence_system();
    __hip_atomic_store(d, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ bool ring_wait(uint32_t seq, uint32_t c, uint32_t role, const TileJob& job, uint32_t* err) {
    uint32_t* turn = ring_turn(seq);
    const uint32_t want = ring_turn_value(seq, c);
    for (uint32_t i = 0;; ++i) {
        const uint32_t seen = lds_ld(turn);
        if (seen == want) return true;
        if (i >= job.ring_spin) {
            ring_timeout(job, err, role, seq, want, seen, i);
            return false;
        }
        // Once a wait of this launch has timed out (error bit 2) the turn words no longer
        // describe the ring: a reader that gave up never releases its slot's next lap, a
        // writer that gave up never releases its entry.  Every later wait gives up within
        // 256 polls instead of spinning the whole bound, so one protocol slip ends the
        // launch in milliseconds, not in (waits x 50 ms) -- ADVICE r04.
        if ((i & 255u) == 255u &&
            (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & kErrRing))
            return false;
        __builtin_amdgcn_s_sleep(1);
    }
}

__device__ __forceinline__ void poison(Sample* samples, uint32_t slot, uint32_t n_slots) {
    if (slot < n_slots) samples[slot] = Sample{__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf("")};
}

#ifndef MM_CLAIM_CHUNKS
#define MM_CLAIM_CHUNKS 4
#endif
constexpr uint32_t kClaimChunks = MM_CLAIM_CHUNKS;  // chunks per dequeue (A/B: -DMM_CLAIM_CHUNKS=k)
#ifndef MM_CLAIM_TAIL
#define MM_CLAIM_TAIL 1
#endif
constexpr uint32_t kClaimTail = MM_CLAIM_TAIL;  // single claims for the last kClaimTail x (waves x big) paths

// The next 64-path chunk of the global queue for this wave (its first path;
// >= n_queue: the queue is out).  Claims of kClaimChunks chunks per returning
// device-scope atomicAdd while every wave of the grid could still take one more
// such claim, then one chunk at a time: one counter word saturates at ~88
// dequeues per us (MI355X_MICROARCH.md, "dequeue"), C3's chunk rate at one
// chunk per claim (259,200 chunks in 2.95 ms; profiles/r03/ab_claim_chunks.txt).
// The wave's claimed range [next, end) lives in LDS, not in registers held
// across the bounce loop (SGPR pressure there spills into VGPR lanes).
#ifdef MM_TAIL_CLOCKS
constexpr uint32_t kClaimWords = 16;
#else
constexpr uint32_t kClaimWords = 2;
#endif
__device__ __forceinline__ uint32_t* claim_words() {
    // (next, end) per wave of a <= 1024-thread block; diagnostics build MM_TAIL_CLOCKS: then the wall clock
    // at the start of the wave's current chunk (lo, hi), its longest chunk so far (10 ns units), its chunks
    // over 100 us, the clock when it saw the global queue out (lo, hi)
    __shared__ uint32_t w[kClaimWords * 16];
    return w + kClaimWords * (threadIdx.x >> 6);
}
// Diagnostics build -DMM_TAIL_CLOCKS (mm_set_wave_timeline), for the launch-tail probe
// (scripts/timeline_probe.py --tail): chunk start times and durations per wave.  kind: 0 new, 1 tail.
__device__ __forceinline__ void mark_chunk_start(const TileJob& job, uint32_t kind) {
#ifndef MM_TAIL_CLOCKS
    (void)job; (void)kind;
#else
    if (job.wave_ts && (threadIdx.x & 63u) == 0) {
        uint32_t* cw = claim_words();
        const uint64_t t = wall_clock64();
        const uint64_t prev = cw[4] | (uint64_t)(cw[5] & 0x7FFFFFFFu) << 32;
        if (prev) {
            const uint32_t d = (uint32_t)min<uint64_t>(t - prev, 0xFFFFFFFFull);
            const uint32_t pk = cw[5] >> 31;  // the previous chunk's kind
            cw[6] = max(cw[6], d);
            cw[7] += d > 10000u ? 1u : 0u;
            cw[10 + 2 * pk] += d;  // per kind (new / tail): summed duration, count, longest
            cw[11 + 2 * pk] += 1u;
            cw[14 + pk] = max(cw[14 + pk], d);
        }
        cw[4] = (uint32_t)t;
        cw[5] = (uint32_t)(t >> 32) | (kind << 31);
    }
#endif
}
__device__ __forceinline__ void mark_queue_out(const TileJob& job) {
#ifndef MM_TAIL_CLOCKS
    (void)job;
#else
    if (job.wave_ts && (threadIdx.x & 63u) == 0 && !claim_words()[9]) {
        const uint64_t t = wall_clock64();
        claim_words()[8] = (uint32_t)t;
        claim_words()[9] = (uint32_t)(t >> 32);
    }
#endif
}
__device__ __forceinline__ void claim_reset() {
    if ((threadIdx.x & 63u) == 0) {
        for (uint32_t i = 0; i < kClaimWords; ++i) claim_words()[i] = 0u;
    }
}
constexpr uint32_t kDoneWord = 1;  // work[0] = next path, work[1] = waves done
__device__ __forceinline__ uint32_t dequeue(uint32_t* work, uint32_t n_queue) {
    uint32_t* cw = claim_words();
    uint32_t next = __builtin_amdgcn_readfirstlane(cw[0]), end = __builtin_amdgcn_readfirstlane(cw[1]);
    if (next >= end) {
        const uint32_t big = kClaimChunks * 64u;
        const uint32_t tail = kClaimTail * gridDim.x * (blockDim.x >> 6) * big;  // below: single claims
        const uint32_t k = (n_queue > tail && next < n_queue - tail) ? big : 64u;
        uint32_t b = 0;
        if ((threadIdx.x & 63u) == 0) b = atomicAdd(work, k);
        next = __builtin_amdgcn_readfirstlane(b);
        end = min(next + k, n_queue);
    }
    if ((threadIdx.x & 63u) == 0) { cw[0] = next + 64u; cw[1] = end; }
    return next;
}

template <bool kStats, typename Q>
__device__ __forceinline__ uint32_t wavepersist_body(const DevScene& sc, const Q& q, const TileJob& job,
                                                     Sample* __restrict__ samples, unsigned long long* stats,
                                                     uint32_t* err, uint32_t* work) {
    const uint32_t spp = job.e.spp;
    const uint32_t n_paths = job.w * job.h * spp;         // per frame
    const uint32_t cpf = (n_paths + 63u) / 64u;           // 64-path chunks per frame
    const uint32_t n_queue = cpf * 64u * job.n_frames;    // the queue, in paths (chunks padded to 64)
    const uint32_t lane = threadIdx.x & 63u;
    const F3 ori = F3{job.u.cam.center[0], job.u.cam.center[1], job.u.cam.center[2]};
    Counters c;
    ScratchStack stack;
    uint32_t paths = 0, chunks = 0;
    claim_reset();
    for (;;) {
        const uint32_t base = dequeue(work, n_queue);
        if (base >= n_queue) {
            mark_queue_out(job);
            break;
        }
        ++chunks;
        mark_chunk_start(job, 0u);
        const uint32_t qc = base >> 6;
        const uint32_t fr = job.n_frames > 1 ? qc / cpf : 0u;
        const uint32_t path = (qc - fr * cpf) * 64u + lane;
        const bool valid = path < n_paths;
        F3 s = F3{0.0f, 0.0f, 0.0f};
        if (valid) {
            const uint32_t pix = path / spp, smp = path - pix * spp;
            const uint32_t j = pix / job.w, i = pix - j * job.w;
            const uint32_t px = job.x0 + i, py = job.y0 + j * job.y_stride;
            PathState p;
            p.seed = seed_tile(py * job.view_w + px, smp, job.e.frame + fr);
            p.dir = jitter(primary_dir(job.u, px, py), p.seed);
            p.ori = ori;
            p.T = F3{1.0f, 1.0f, 1.0f};
            p.L = F3{0.0f, 0.0f, 0.0f};
            p.n = 0;
            p.mh = 0;
            p.bank = 0u;
            p.s1 = 0u;
            bool overflow = false;
            bounce_loop<kStats>(sc, q, p, (int)job.e.bounce_limit, (int)job.e.mirror_limit, stack, c, overflow);
            if (overflow) atomicOr(err, kErrStack);
            s = path_value(p);
            if (!job.fuse) samples[fr * n_paths + path] = s;
            paths++;
        }
        if (job.fuse) resolve_in_wave(job, s, path, valid, job.out, (size_t)fr * job.w * job.h);
    }
#ifdef MM_PHASE_CLOCKS
    {  // the wave's time in queries / shading: the max over its lanes (some lane runs every iteration)
        uint64_t qc = c.q_cyc, sc2 = c.s_cyc;
        for (int o = 32; o > 0; o >>= 1) {
            qc = max(qc, (uint64_t)__shfl_xor((unsigned long long)qc, o));
            sc2 = max(sc2, (uint64_t)__shfl_xor((unsigned long long)sc2, o));
        }
        if (job.wave_ts && lane == 0) {
            const uint32_t wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
            if (wid < job.wave_ts_cap) {
                job.wave_ts[4 * wid + 1] = qc;
                job.wave_ts[4 * wid + 3] = sc2;
            }
        }
    }
#endif
    if (kStats) flush_stats(stats, c, paths);
    return chunks;
}

// With tail deferral (kDefer): a wave's next chunk is 64 queued
// tails from its block's ring when there are that many, else 64 new paths
// from the global queue; once that is out, whatever the ring still holds
// (deferral off), and the wave exits as soon as its block's ring is empty.
// No wave waits for its block-mates: a wave defers tails only before it has
// seen the global queue out, and after it has seen that it claims from the
// ring until the ring is empty -- so every tail is claimed by the wave that
// parked it if by no other (a drain wait for block-mates' last chunks, which
// last up to bounce_limit + mirror_limit iterations, would need a bound that a
// valid 32767-bounce chunk outlasts).  A tail chunk runs the same bounce loop
// as a new one (and may defer again) -- one copy of the loop in the kernel.
template <bool kStats, bool kLdsPay, typename Q>
__device__ __forceinline__ uint32_t wavepersist_ring_body(const DevScene& sc, const Q& q, const TileJob& job,
                                              Sample* __restrict__ samples, unsigned long long* stats, uint32_t* err,
                                              uint32_t* work) {
    const uint32_t spp = job.e.spp;
    const uint32_t n_paths = job.w * job.h * spp;
    const uint32_t cpf = (n_paths + 63u) / 64u;
    const uint32_t n_queue = cpf * 64u * job.n_frames;
    const uint32_t lane = threadIdx.x & 63u;
    const F3 ori = F3{job.u.cam.center[0], job.u.cam.center[1], job.u.cam.center[2]};
    const TailQueue& tq = job.tail;
    const uint32_t n_slots = n_paths * job.n_frames;
    Counters c;
    ScratchStack stack;
    uint32_t paths = 0, chunks = 0;
    int defer_from = (int)job.defer_from;  // 2^30 (off) once the global queue is out
    claim_reset();
#ifdef MM_RING_CLOCKS  // diagnostics: per wave (main chunks, tail chunks, claim retries) wall clock
    uint64_t rc_main = 0, rc_tail = 0, rc_idle = 0;
    uint64_t rc_t0 = 0;
#endif
    for (;;) {
#ifdef MM_RING_CLOCKS
        rc_t0 = wall_clock64();
#endif
        uint32_t first = 0, k = 0, b = 0;
        if (lane == 0) k = ring_claim(defer_from == (1 << 30) ? 1u : 64u, first);
        k = __builtin_amdgcn_readfirstlane(k);
        if (!k) {
            if (defer_from == (1 << 30)) {
                // the claim failed: the ring is empty (exit) or a block-mate's claim won the race (retry)
                uint32_t left = 0;
                if (lane == 0) {
                    const uint32_t claimed = lds_ld(ring_ctl() + 1);
                    left = lds_ld(ring_ctl() + 0) - claimed;  // (read after claimed)
                }
                if (!__builtin_amdgcn_readfirstlane(left)) break;
#ifdef MM_RING_CLOCKS
                rc_idle += wall_clock64() - rc_t0;
#endif
                continue;
            }
            b = dequeue(work, n_queue);
            if (b >= n_queue) {
                defer_from = 1 << 30;
                mark_queue_out(job);
                continue;
            }
        }
        ++chunks;
        mark_chunk_start(job, k ? 1u : 0u);
        PathState p{};
        uint32_t slot = 0;
        bool live;
        if (k) {  // queued tails
            live = lane < k;
            if (live) {
                const uint32_t seq = __builtin_amdgcn_readfirstlane(first) + lane;
                if (ring_wait(seq, 1u, 1u, job, err)) {
                    slot = tail_load<kLdsPay>(tq, seq % kTailRing, p);
                    __hip_atomic_store(ring_turn(seq), ring_turn_value(seq, 2u), __ATOMIC_RELEASE,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
                } else {  // the record was never written (its sample slot is unknown here: ADVICE r03): skip it;
                    live = false;  // the error bit fails the call
                }
            }
        } else {  // new paths
            const uint32_t qc = __builtin_amdgcn_readfirstlane(b) >> 6;
            const uint32_t fr = job.n_frames > 1 ? qc / cpf : 0u;
            const uint32_t path = (qc - fr * cpf) * 64u + lane;
            live = path < n_paths;
            if (live) {
                const uint32_t pix = path / spp, smp = path - pix * spp;
                const uint32_t j = pix / job.w, i = pix - j * job.w;
                const uint32_t px = job.x0 + i, py = job.y0 + j * job.y_stride;
                p.seed = seed_tile(py * job.view_w + px, smp, job.e.frame + fr);
                p.dir = jitter(primary_dir(job.u, px, py), p.seed);
                p.ori = ori;
                p.T = F3{1.0f, 1.0f, 1.0f};
                p.L = F3{0.0f, 0.0f, 0.0f};
                p.n = 0;
                p.mh = 0;
                slot = fr * n_paths + path;
            }
        }
        if (live) {
            MM_LANE_STAT(kLpChunk);
            bool overflow = false;
            uint32_t seq = 0;
            // A claimed tail chunk of <= defer_lanes paths runs with deferral off: it would re-park at the top of
            // its first bounce without running it, and a wave alone in its block could cycle the same tails
            // through the ring forever (round 3, 64-lane deferral: tests/test_ring_model.py).  In the main phase
            // a claim takes 64 tails, so this is off at defer_lanes < 64; every claim runs >= 1 bounce.
            const int df = (k && k <= job.defer_lanes) ? (1 << 30) : defer_from;
            const bool deferred = bounce_loop_r<kStats>(
                sc, q, p, (int)job.e.bounce_limit, (int)job.e.mirror_limit, stack, c, overflow,
                df, job.defer_lanes, [&]() { return ring_reserve(seq); });
            if (overflow) atomicOr(err, kErrStack);
            if (deferred) {
                // MM_OPT_FAULT_INJECT 4 (tests): the launch's first deferred path is lost -- its entry
                // is reserved but never written, so its reader's wait times out
                if (job.fault == 4u && !(atomicOr(err, kErrLost) & kErrLost)) {
                    poison(samples, slot, n_slots);
                } else if (ring_wait(seq, 0u, 2u, job, err)) {
                    tail_store<kLdsPay>(tq, seq % kTailRing, p, slot);
                    __hip_atomic_store(ring_turn(seq), ring_turn_value(seq, 1u), __ATOMIC_RELEASE,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
                } else {
                    poison(samples, slot, n_slots);
                }
            } else {
                const F3 s = path_value(p);
                samples[slot] = s;
                paths++;
            }
        }
#ifdef MM_RING_CLOCKS
        {
            const uint64_t dt = wall_clock64() - rc_t0;
            if (k) rc_tail += dt; else rc_main += dt;
        }
#endif
    }
#ifdef MM_RING_CLOCKS
    if (job.wave_ts && lane == 0) {
        const uint32_t wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6) + 16384u;
        if (wid < job.wave_ts_cap) {
            job.wave_ts[4 * wid + 0] = rc_main;
            job.wave_ts[4 * wid + 1] = rc_tail;
            job.wave_ts[4 * wid + 2] = chunks;
            job.wave_ts[4 * wid + 3] = rc_idle;
        }
    }
#endif
    if (kStats) flush_stats(stats, c, paths);
    return chunks;
}

// LDS modes (what a resident block stages before tracing; the rest is read
// through L1/L2):
//   0  nothing (nodes, records global)           BVH form 5
//   1  BVH nodes                                  BVH form 5 (general rect test)
//   3  BVH nodes + compact slot records           BVH forms 5 / 7
//   11 the whole grid image                       grid search
//   12 grid cells + lists, records + boxes global grid search
//   13 nothing (the grid image global)             grid search
//   14 grid records + class table + cells + lists, grid search (compact records: the maze forms)
//      leaf boxes global
// stage_and_run fills the block's LDS for the mode and calls body(query).
//
// Modes 11 and 14 stage the grid image into a STATIC LDS array (grid_lds):
// its address is a compile-time constant, so the class table (LDS offset 0 of
// the image) and record k (kGridClassBytes + 16 k) are read with the
// constant folded into the ds_read instruction's immediate offset.  (The
// base of the dynamic extern __shared__ array is a link-time relocation:
// every address built on it costs a VALU add, and the three-operand
// v_lshl_add_u32 and the SGPR-operand v_add_u32 it becomes cannot pair with
// another wave's VALU op in a quad-cycle -- scripts/isa_dual.hip,
// DESIGN.md s10.)  Each instance's array takes what the block's 80 KB leave
// after its other static LDS (two 1024-thread blocks per CU).
constexpr uint32_t kLdsPerBlock = 80 * 1024;
template <int kRing>
constexpr uint32_t grid_lds_cap() {
    uint32_t other = kClaimWords * 16u * 4u + 64u;  // claimed queue ranges + alignment slack
    if (kRing != 0) other += (4u + kTailRing) * 4u;  // ring counters and turn words
    if (kRing == 2) other += 4u * kTailRing * 16u;   // ring payload
#ifdef MM_LANE_STATS
    other += 2u * kLpCount * 4u;
#endif
    return (kLdsPerBlock - other) & ~15u;
}
template <uint32_t kBytes>
__device__ __forceinline__ uint4* grid_lds() {
    __shared__ uint4 g[kBytes / 16u];
    return g;
}

template <int kLds, int kForm, bool kStats, int kRing, typename F>
__device__ __forceinline__ uint32_t stage_and_run(const DevScene& sc, const TileJob& job, F&& body) {
    extern __shared__ float4 lds[];
    auto staged = [&]() {  // diagnostics: time at which the block's LDS staging completed (wave timeline)
        if (job.wave_ts && (threadIdx.x & 63u) == 0) {
            const uint32_t wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
#ifndef MM_PHASE_CLOCKS
            if (wid < job.wave_ts_cap) job.wave_ts[4 * wid + 1] = (unsigned long long)wall_clock64();
#endif
        }
    };
    if constexpr (kLds == 11 || kLds == 14) {
        // the data -- class table + records (+ boxes: mode 11) -- first, at the
        // static array's start (compile-time offsets in the rect test), then
        // cells + lists
        const uint32_t d0 = sc.grid.off_data, end = kLds == 11 ? sc.grid.bytes : sc.grid.off_box;
        const uint32_t nr16 = (end - d0) / 16u, ni16 = d0 / 16u;
        uint4* img = grid_lds<grid_lds_cap<kRing>()>();
        const uint4* src = sc.grid.image;
        for (uint32_t i = threadIdx.x; i < nr16; i += blockDim.x) img[i] = src[ni16 + i];
        {  // cells (their first-entry fields as LDS byte addresses: grid_stage_cells), then lists
            const uint32_t nc16 = sc.grid.off_list / 16u, lbase = lds_addr(img + nr16) + sc.grid.off_list;
            for (uint32_t i = threadIdx.x; i < ni16; i += blockDim.x)
                img[nr16 + i] = i < nc16 ? grid_stage_cells<grid_wide(kForm)>(src[i], lbase) : src[i];
        }
        __syncthreads();
        staged();
        const char* base = reinterpret_cast<const char*>(img);
        const char* index = base + 16u * nr16;
        // compact records: the class table at offset 0, record k at kGridClassBytes + 16 k; else records at 0
        const auto recs = reinterpret_cast<const uint4*>(base + (grid_flat(kForm) ? kGridClassBytes : 0u));
        const auto cls = reinterpret_cast<const float4*>(base);
        const auto run = [&](auto box) {
            const auto gv = grid_view(LdsCells{lds_addr(index)}, LdsList{lds_addr(index + sc.grid.off_list)},
                                      recs, box, cls);
            return body(GridQuery<kStats, grid_slow(kForm), grid_wide(kForm), grid_flat(kForm), decltype(gv)>{sc, gv});
        };
        if constexpr (kLds == 11)
            return run(reinterpret_cast<const float2*>(base + (sc.grid.off_box - d0)));
        else
            return run(sc.grid.box);
    } else if constexpr (kLds == 12) {
        const uint32_t n16 = sc.grid.off_data / 16u, nc16 = sc.grid.off_list / 16u;
        uint4* img = reinterpret_cast<uint4*>(lds);
        const uint32_t lbase = lds_addr(img) + sc.grid.off_list;
        for (uint32_t i = threadIdx.x; i < n16; i += blockDim.x)
            img[i] = i < nc16 ? grid_stage_cells<grid_wide(kForm)>(sc.grid.image[i], lbase) : sc.grid.image[i];
        __syncthreads();
        staged();
        const char* base = reinterpret_cast<const char*>(lds);
        const auto gv = grid_view(LdsCells{lds_addr(base)}, LdsList{lds_addr(base + sc.grid.off_list)},
                                  sc.grid.recs, sc.grid.box, sc.grid.cls);
        return body(GridQuery<kStats, grid_slow(kForm), grid_wide(kForm), grid_flat(kForm), decltype(gv)>{sc, gv});
    } else if constexpr (kLds == 13) {
        const auto gv = grid_view(GlobalCells{reinterpret_cast<const char*>(sc.grid.cells)}, GlobalList{sc.grid.list},
                                  sc.grid.recs, sc.grid.box, sc.grid.cls);
        return body(GridQuery<kStats, grid_slow(kForm), grid_wide(kForm), grid_flat(kForm), decltype(gv)>{sc, gv});
    } else if constexpr (kLds == 1 || kLds == 3) {
        for (uint32_t i = threadIdx.x; i < 2 * sc.n_nodes; i += blockDim.x) lds[i] = sc.nodes[i];
        uint2* lds_recs = reinterpret_cast<uint2*>(lds + 2 * sc.n_nodes);
        if constexpr (kLds == 3)
            for (uint32_t i = threadIdx.x; i < 5 * sc.n_rects; i += blockDim.x) lds_recs[i] = sc.recs[i];
        __syncthreads();
        staged();
        if constexpr (kLds == 3) {
            const auto v = view(static_cast<float4*>(lds), lds_recs);
            return body(BvhQuery<kStats, kForm, decltype(v)>{sc, v});
        } else {
            const auto v = view(static_cast<float4*>(lds));
            return body(BvhQuery<kStats, kForm, decltype(v)>{sc, v});
        }
    } else {
        const auto v = view(sc.nodes);
        return body(BvhQuery<kStats, kForm, decltype(v)>{sc, v});
    }
}

// Timeline records (mm_set_wave_timeline): wave wid's (entry, staged, exit, chunks) at 4 * wid, its (last
// chunk start, XCC id, HW_ID, chunks) at 4 * (wid + kTimelineWaves) when the buffer holds them.
[[maybe_unused]] constexpr uint32_t kTimelineWaves = 32768;
// Per-wave diagnostics record and the self-cleaning counter pair shared by the
// persistent kernels (counter[0] = next item, counter[1] = waves done; the
// last wave to finish re-zeroes the words, so the next launch needs no memset
// -- a fill kernel queued between two frames on another stream would wait for
// free CUs and serialise overlapping frames).
// The last wave also publishes the launch's error flag into its status word
// (TileJob::status) and clears the flag for the next launch on the stream.
__device__ __forceinline__ void persistent_exit(const TileJob& job, uint32_t chunks, unsigned long long t_entry,
                                                uint32_t* counter, uint32_t* err) {
    if (job.wave_ts && (threadIdx.x & 63u) == 0) {
        const uint32_t wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        if (wid < job.wave_ts_cap) {
#ifdef MM_PHASE_CLOCKS  // (entry, query cycles, exit, shade cycles), s_memtime
            job.wave_ts[4 * wid + 0] = t_entry;
            job.wave_ts[4 * wid + 2] = (unsigned long long)wall_clock64();
#else
            job.wave_ts[4 * wid + 0] = t_entry;
            job.wave_ts[4 * wid + 2] = (unsigned long long)wall_clock64();
            job.wave_ts[4 * wid + 3] = chunks;
#endif
        }
    }
#ifdef MM_TAIL_CLOCKS
    if (job.wave_ts && (threadIdx.x & 63u) == 0) {
        // more records per wave (index wid + kTimelineWaves, wid + 2 kTimelineWaves): its last chunk's start
        // (bit 63: a tail chunk), where it ran -- HW_REG_XCC_ID (the XCD, 0-7) and HW_REG_HW_ID (CU, SIMD,
        // shader engine; MI355X_MICROARCH.md) --, chunks; its longest chunk (10 ns), chunks over 100 us, the
        // clock when it saw the global queue out, the clock at its exit
        const uint32_t wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6) + kTimelineWaves;
        if (wid + kTimelineWaves < job.wave_ts_cap) {
            const uint32_t* cw = claim_words();
            const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);   // hwreg(HW_REG_XCC_ID, 0, 4)
            const uint32_t hwid = __builtin_amdgcn_s_getreg((31 << 11) | 4);  // hwreg(HW_REG_HW_ID, 0, 32)
            job.wave_ts[4 * wid + 0] = cw[4] | (unsigned long long)cw[5] << 32;
            job.wave_ts[4 * wid + 1] = xcc;
            job.wave_ts[4 * wid + 2] = hwid;
            job.wave_ts[4 * wid + 3] = chunks;
            const uint32_t w2 = wid + kTimelineWaves;
            job.wave_ts[4 * w2 + 0] = cw[6];
            job.wave_ts[4 * w2 + 1] = cw[7];
            job.wave_ts[4 * w2 + 2] = cw[8] | (unsigned long long)cw[9] << 32;
            job.wave_ts[4 * w2 + 3] = (unsigned long long)wall_clock64();
            const uint32_t w3 = w2 + kTimelineWaves;  // per chunk kind: (sum << 32 | count), longest
            if (w3 < job.wave_ts_cap) {
                job.wave_ts[4 * w3 + 0] = (unsigned long long)cw[10] << 32 | cw[11];
                job.wave_ts[4 * w3 + 1] = (unsigned long long)cw[12] << 32 | cw[13];
                job.wave_ts[4 * w3 + 2] = cw[14];
                job.wave_ts[4 * w3 + 3] = cw[15];
            }
        }
    }
#endif
    if ((threadIdx.x & 63u) == 0) {
        __threadfence();
        const uint32_t total = gridDim.x * (blockDim.x >> 6);
        if (atomicAdd(counter + kDoneWord, 1u) == total - 1) {
            atomicExch(counter, 0u);
            atomicExch(counter + kDoneWord, 0u);
            if (job.status) {
                const uint32_t e = atomicExch(err, 0u);
                __hip_atomic_store(job.status, e | kStatusDone, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

__global__ void k_publish_status(uint32_t* err, uint32_t* status) {
    const uint32_t e = atomicExch(err, 0u);
    __hip_atomic_store(status, e | kStatusDone, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_publish_status(uint32_t* err, uint32_t* status, hipStream_t s) {
    hipLaunchKernelGGL(k_publish_status, dim3(1), dim3(1), 0, s, err, status);  // one lane
    return hipGetLastError();
}

// 1024-thread blocks at 8 waves per SIMD (<= 64 VGPRs).  With the grid search,
// 768-thread blocks at 6 waves (80 VGPRs, no VGPR spills) measured 6.21 vs
// 5.87 ms on C3 (profiles/r02/ab_grid_variants.txt).  (A/B builds:
// -DMM_WP_THREADS=896 -DMM_WP_WAVES=7 and the like.)
#ifndef MM_WP_THREADS
#define MM_WP_THREADS 1024
#endif
#ifndef MM_WP_WAVES
#define MM_WP_WAVES 8
#endif
constexpr uint32_t kWpThreads = MM_WP_THREADS;
// kRing: 0 no tail deferral; 1 tail rings, payload in global records; 2 tail rings, payload in LDS.
template <bool kStats, int kLds, int kForm, int kRing>
__global__ __launch_bounds__(MM_WP_THREADS, MM_WP_WAVES) void k_trace_wavepersist(DevScene sc, TileJob job, Sample* __restrict__ samples,
                                                               unsigned long long* stats, uint32_t* err,
                                                               uint32_t* work) {
    if constexpr (kRing != 0) {  // the block's tail ring: counters and turn words zero
        for (uint32_t i = threadIdx.x; i < 4u + kTailRing; i += blockDim.x) ring_ctl()[i] = 0u;
        __syncthreads();
    }
    if (job.fault == 1u && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(err, kErrInjected);
#ifdef MM_LANE_STATS
    if (threadIdx.x < 2u * kLpCount) lane_stat_words()[threadIdx.x] = 0u;
    __syncthreads();
#endif
#ifdef MM_PHASE_CLOCKS
    const unsigned long long t_entry = job.wave_ts ? (unsigned long long)wall_clock64() : 0ull;
#else
    const unsigned long long t_entry = job.wave_ts ? (unsigned long long)wall_clock64() : 0ull;
#endif
    const uint32_t chunks = stage_and_run<kLds, kForm, kStats, kRing>(sc, job, [&](const auto& q) {
        if constexpr (kRing != 0)
            return wavepersist_ring_body<kStats, kRing == 2>(sc, q, job, samples, stats, err, work);
        else
            return wavepersist_body<kStats>(sc, q, job, samples, stats, err, work);
    });
#ifdef MM_LANE_STATS
    __syncthreads();  // every wave of the block is done: add its counts to the timeline buffer
    if (job.wave_ts && job.wave_ts_cap >= kLaneStatRecord + (2u * kLpCount + 3u) / 4u &&
        threadIdx.x < 2u * kLpCount)
        atomicAdd(job.wave_ts + 4u * kLaneStatRecord + threadIdx.x, (unsigned long long)lane_stat_words()[threadIdx.x]);
#endif
    persistent_exit(job, chunks, t_entry, work, err);
}

uint32_t wavepersist_grid_cap(int ring) {
    return ring == 2 ? grid_lds_cap<2>() : ring == 1 ? grid_lds_cap<1>() : grid_lds_cap<0>();
}

size_t wavepersist_lds_bytes(const DevScene& sc, int lds_mode) {
    switch (lds_mode) {
        case 11: return sc.grid.bytes;
        case 12: return sc.grid.off_data;
        case 14: return sc.grid.off_box;
        case 1: return 2 * (size_t)sc.n_nodes * sizeof(float4);
        case 3: return 2 * (size_t)sc.n_nodes * sizeof(float4) + 5 * (size_t)sc.n_rects * sizeof(uint2);
        default: return 0;
    }
}

// Resident grid of a persistent kernel: blocks per CU from the occupancy API x
// CUs (minus MM_OPT_RESERVE_CUS), capped by the work.
template <typename K>
static uint32_t persistent_grid(K kern, size_t lds, uint32_t reserve_cus, uint64_t items) {
    int per_cu = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kWpThreads, lds) != hipSuccess) return 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int cus_used = std::max(1, cus - (int)reserve_cus);
    uint64_t grid = (uint64_t)std::max(1, per_cu) * (uint64_t)cus_used;
    return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(grid, (items + kWpThreads - 1) / kWpThreads));
}

template <int kLds, int kForm, int kRing>
static hipError_t launch_wavepersist_t(const DevScene& sc, const TileJob& job, Sample* samples,
                                       unsigned long long* stats, uint32_t* err, uint32_t* work, bool count_stats,
                                       hipStream_t s) {
    // modes 11 / 14 stage into the kernel's static grid array (stage_and_run): no dynamic LDS, and an image
    // larger than the array is refused here (the host picks the ring kind so that it fits)
    if ((kLds == 11 || kLds == 14) && wavepersist_lds_bytes(sc, kLds) > grid_lds_cap<kRing>())
        return hipErrorInvalidValue;
    const size_t lds = (kLds == 11 || kLds == 14) ? 0 : wavepersist_lds_bytes(sc, kLds);
    auto kern = count_stats ? k_trace_wavepersist<true, kLds, kForm, kRing>
                            : k_trace_wavepersist<false, kLds, kForm, kRing>;
    const uint32_t grid =
        persistent_grid(kern, lds, job.reserve_cus, (uint64_t)job.w * job.h * job.e.spp * job.n_frames);
    if (!grid) return hipErrorInvalidValue;
    if (kRing == 1 && (uint64_t)grid * kTailRing > job.tail.cap) return hipErrorInvalidValue;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kWpThreads), lds, s, sc, job, samples, stats, err, work);
    return hipGetLastError();
}

// (LDS mode, form) pairs; the tail-deferral variant (MM_OPT_DEFER) is built
// for the grid search and the lean BVH form with records in LDS.  The build
// holds what MM_PIPE_AUTO can select: the grid search, and the BVH forms for
// scenes the grid cannot take (nodes + records in LDS, nodes only, nothing).
// (The A/B-only placements -- split node cache, nodes with global records,
// dictionary nodes, loop form 0 -- measured slower and were removed in round
// 6)  The maze forms (flat grid walk,
// compact records; grid_build.cpp decides) in every grid placement: a maze
// grid's compact records are read by no other form.  (No SLOW records in
// maze grids: no slow maze forms.)
#define MM_FLAT_INSTANCES(X)                                                                                  \
    X(11, kFormGridWide + kFormGridFlat) X(11, kFormGrid + kFormGridFlat) X(14, kFormGrid + kFormGridFlat)     \
    X(12, kFormGrid + kFormGridFlat) X(13, kFormGridWide + kFormGridFlat) X(13, kFormGrid + kFormGridFlat)
#define MM_DEFER_INSTANCES(X)                                                                                 \
    X(11, kFormGrid) X(12, kFormGrid) X(13, kFormGrid)                                                        \
    X(11, kFormGridSlow) X(12, kFormGridSlow) X(13, kFormGridSlow)                                            \
    X(11, kFormGridWide) X(13, kFormGridWide) X(11, kFormGridWideSlow) X(13, kFormGridWideSlow)               \
    MM_FLAT_INSTANCES(X) X(3, kFormLean)
#define MM_WP_INSTANCES(X)                                                                                    \
    MM_DEFER_INSTANCES(X) X(0, kFormLeafInterior) X(1, kFormLeafInterior) X(3, kFormLeafInterior)

bool wavepersist_built(int lds_mode, int form) {
#define MM_WP(L, F) if (lds_mode == L && form == F) return true;
    MM_WP_INSTANCES(MM_WP)
#undef MM_WP
    return false;
}

bool wavepersist_defer_built(int lds_mode, int form) {
#define MM_WP(L, F) if (lds_mode == L && form == F) return true;
    MM_DEFER_INSTANCES(MM_WP)
#undef MM_WP
    return false;
}

hipError_t launch_trace_wavepersist(const DevScene& sc, const TileJob& job, Sample* samples,
                                    unsigned long long* stats, uint32_t* err, uint32_t* work, bool count_stats,
                                    int lds_mode, int form, hipStream_t s) {
    const int ring = job.defer_from < (1u << 30) ? (job.ring_lds ? 2 : 1) : 0;
#define MM_WP(L, F)                                                                                          \
    if (lds_mode == L && form == F && ring == 1)                                                             \
        return launch_wavepersist_t<L, F, 1>(sc, job, samples, stats, err, work, count_stats, s);            \
    if (lds_mode == L && form == F && ring == 2)                                                             \
        return launch_wavepersist_t<L, F, 2>(sc, job, samples, stats, err, work, count_stats, s);
    MM_DEFER_INSTANCES(MM_WP)
#undef MM_WP
#define MM_WP(L, F)                                                                                          \
    if (lds_mode == L && form == F && ring == 0)                                                             \
        return launch_wavepersist_t<L, F, 0>(sc, job, samples, stats, err, work, count_stats, s);
    MM_WP_INSTANCES(MM_WP)
#undef MM_WP
    return hipErrorInvalidValue;
}

hipError_t wavepersist_attributes(int lds_mode, int form, int ring, hipFuncAttributes* a) {
#define MM_WP(L, F)                                                                                          \
    if (lds_mode == L && form == F && ring == 1)                                                             \
        return hipFuncGetAttributes(a, reinterpret_cast<const void*>(k_trace_wavepersist<false, L, F, 1>));  \
    if (lds_mode == L && form == F && ring == 2)                                                             \
        return hipFuncGetAttributes(a, reinterpret_cast<const void*>(k_trace_wavepersist<false, L, F, 2>));
    MM_DEFER_INSTANCES(MM_WP)
#undef MM_WP
#define MM_WP(L, F)                                                                                          \
    if (lds_mode == L && form == F && ring == 0)                                                             \
        return hipFuncGetAttributes(a, reinterpret_cast<const void*>(k_trace_wavepersist<false, L, F, 0>));
    MM_WP_INSTANCES(MM_WP)
#undef MM_WP
    return hipErrorInvalidValue;
}

hipError_t launch_trace_mega(const DevScene& sc, const TileJob& job, Sample* samples, unsigned long long* stats_dev,
                             uint32_t* err, bool count_stats, const MegaOpts& o, hipStream_t s) {
    if (!o.reference) return hipErrorInvalidValue;  // one thread per path: MM_PIPE_REFERENCE only
    const uint32_t n = job.w * job.h * job.e.spp;
    const dim3 grid((n + o.block - 1) / o.block);
    if (count_stats)
        hipLaunchKernelGGL(k_trace_mega<true>, grid, dim3(o.block), 0, s, sc, job, samples, stats_dev, err);
    else
        hipLaunchKernelGGL(k_trace_mega<false>, grid, dim3(o.block), 0, s, sc, job, samples, stats_dev, err);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Sample reduction: spp % 8 == 0 -> pairwise tree in blocks of 8, blocks added
// left to right (the reference order for 64 spp); otherwise left to right.
__global__ void k_resolve(TileJob job, const Sample* __restrict__ samples, void* __restrict__ out) {
    const uint32_t pix = blockIdx.x * blockDim.x + threadIdx.x;
    if (pix >= job.w * job.h) return;
    const uint32_t spp = job.e.spp;
    const Sample* s = samples + (size_t)pix * spp;
    F3 acc;
    if (spp % 8 == 0) {
        for (uint32_t b = 0; b < spp; b += 8) {
            const F3 p0 = s[b + 0] + s[b + 1], p1 = s[b + 2] + s[b + 3];
            const F3 p2 = s[b + 4] + s[b + 5], p3 = s[b + 6] + s[b + 7];
            const F3 blk = (p0 + p1) + (p2 + p3);
            acc = (b == 0) ? blk : acc + blk;
        }
    } else {
        acc = s[0];
        for (uint32_t k = 1; k < spp; ++k) acc = acc + s[k];
    }
    store_pixel(job, out, pix, pixel_mean(acc, spp));
}

// The same reduction when 64 % spp == 0, a wave per 64 consecutive samples
// (64/spp whole pixels): every load is one coalesced 1-KB wave access, and
// resolve_in_wave adds in k_resolve's order (bit-identical).  Used for spp 1,
// 2, 4 (spp % 8 == 0 takes k_resolve8).
__global__ __launch_bounds__(256) void k_resolve_wave(TileJob job, const Sample* __restrict__ samples,
                                                      void* __restrict__ out) {
    const uint32_t n = job.w * job.h * job.e.spp;
    const uint32_t path = blockIdx.x * blockDim.x + threadIdx.x;  // waves never straddle the end: n % 64 == 0
    const bool valid = path < n;                                   // unless the tile is ragged
    const Sample v = valid ? samples[path] : Sample{0.0f, 0.0f, 0.0f};
    resolve_in_wave(job, v, path, valid, out, 0);
}

// spp % 8 == 0: one thread per pixel, each block of 8 samples read as six
// 16-B loads (a pixel's samples are 96 B-aligned runs: 12 spp B per pixel),
// added in k_resolve's tree -- no cross-lane shuffles, one active lane per
// pixel instead of one in eight (mean: pixel_mean, mm_wave_util.h).
__global__ __launch_bounds__(256) void k_resolve8(TileJob job, const Sample* __restrict__ samples,
                                                  void* __restrict__ out) {
    const uint32_t pix = blockIdx.x * blockDim.x + threadIdx.x;
    if (pix >= job.w * job.h) return;
    const uint32_t spp = job.e.spp;
    const float4* q = reinterpret_cast<const float4*>(samples + (size_t)pix * spp);
    F3 acc;
    for (uint32_t b = 0; b < spp; b += 8, q += 6) {
        const float4 a0 = q[0], a1 = q[1], a2 = q[2], a3 = q[3], a4 = q[4], a5 = q[5];
        const F3 s0{a0.x, a0.y, a0.z}, s1{a0.w, a1.x, a1.y}, s2{a1.z, a1.w, a2.x}, s3{a2.y, a2.z, a2.w};
        const F3 s4{a3.x, a3.y, a3.z}, s5{a3.w, a4.x, a4.y}, s6{a4.z, a4.w, a5.x}, s7{a5.y, a5.z, a5.w};
        const F3 blk = ((s0 + s1) + (s2 + s3)) + ((s4 + s5) + (s6 + s7));
        acc = (b == 0) ? blk : acc + blk;
    }
    store_pixel(job, out, pix, pixel_mean(acc, spp));
}

hipError_t launch_resolve(const TileJob& job, const Sample* samples, void* out, hipStream_t s) {
    const uint32_t n = job.w * job.h;
    if (job.e.spp % 8 == 0) {
        hipLaunchKernelGGL(k_resolve8, dim3((n + 255) / 256), dim3(256), 0, s, job, samples, out);
    } else if (64 % job.e.spp == 0) {
        const uint32_t paths = n * job.e.spp;
        hipLaunchKernelGGL(k_resolve_wave, dim3((paths + 255) / 256), dim3(256), 0, s, job, samples, out);
    } else {
        hipLaunchKernelGGL(k_resolve, dim3((n + 255) / 256), dim3(256), 0, s, job, samples, out);
    }
    return hipGetLastError();
}

}  // namespace mm
