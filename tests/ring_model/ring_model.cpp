// ring_model.cpp -- a CPU model of the block-local tail ring of
// k_trace_wavepersist<..., kDefer = true> (mirror-maze_amd/csrc/trace_kernels.hip:
// ring_reserve, ring_claim, ring_wait, wavepersist_ring_body; mm_path.h:
// bounce_loop_r), run under a seeded random scheduler.
//
// One block: W waves of L lanes, one ring of R entries (reserved / claimed
// counters and one turn word per slot), a global queue of 64-path chunks.  Each
// scheduler step executes ONE atomic step of one wave: an LDS load, an LDS
// compare-and-swap, an LDS store, one poll of a protocol wait, one bounce of
// the wave's live lanes, one dequeue.  SIMT rule: a wave's lanes move
// together -- a wait completes only when every waiting lane's turn word has
// the wanted value (the kernel's divergent spin loop releases none of the
// lanes' entries before the last lane's wait ends), deferred lanes leave the
// bounce loop but the wave runs the loop until its last live lane is done.
//
// A path is abstracted to its bounce count T (deterministic per path id, 1..B):
// it leaves the loop after bounce T.  Deferral at the top of a bounce, as in
// bounce_loop_r: lanes with n >= defer_from take part; if at most defer_lanes
// of them run, the leader tries ONE reservation (read claimed, read reserved,
// room check, CAS); success parks them.
//
// Checks: every path finishes exactly once; the run ends -- no bounce for a
// long run of steps is a deadlock (every live wave polls a wait that cannot
// end) or a livelock (waves keep moving ring entries without a bounce); the
// longest protocol wait, in scheduler steps.
//
//   ring_model waves lanes ring chunks max_bounces defer_lanes defer_from
//              steps seed policy burst bounce_cost
//   policy bits: 0 = the round-3 kernel; bit 0: a claimed tail chunk runs with
//   deferral off when its lane count is <= defer_lanes (it would otherwise
//   re-park at once, without a bounce); bit 1: turn values modulo 2^24 (the
//   sequence counters are 32-bit: lap = seq / R wraps from 2^32 / R - 1 to 0).
//   The round-4 kernel is policy 3 (trace_kernels.hip ring_turn_value).
//   bit 2: the end-of-queue split (MM_END_SPLIT): once a wave has seen the
//   queue out, a block flag is set; a new chunk from the last 4 x waves chunks
//   then parks all its live lanes at its next bounce top (>= defer_from), and
//   every claim made while the flag is set needs 1 entry and takes
//   avail / (waves / 2) clamped to [lanes / 4, lanes].
//   seq0 (optional): the counters' start value, the turn words set as if every
//   earlier entry had been written and read (a ring near the 2^32 wrap).
//   burst: mean scheduler quantum (1 = every step a fresh random wave).
//   bounce_cost: mean scheduler steps per bounce (a bounce is ~10-100x an LDS
//   operation on the GPU).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

namespace {

constexpr uint32_t kOff = 1u << 30;

struct Lane {
    bool live = false;     // holds a path in this chunk
    bool in_loop = false;  // still in the bounce loop
    bool deferred = false;
    uint32_t path = 0, n = 0, seq = 0;
};

enum Pc {
    TOP, CLAIM_RES, CLAIM_CAS, NOCLAIM, DRAIN_RES, DEQUEUE, R_WAIT, R_LOAD, B_TOP, RES_RES, RES_CAS, B_WORK,
    AFTER, W_WAIT, W_STORE, EXITED
};
const char* pc_name(int p) {
    static const char* n[] = {"TOP", "CLAIM_RES", "CLAIM_CAS", "NOCLAIM", "DRAIN_RES", "DEQUEUE", "R_WAIT", "R_LOAD",
                              "B_TOP", "RES_RES", "RES_CAS", "B_WORK", "AFTER", "W_WAIT", "W_STORE", "EXITED"};
    return n[p];
}

struct Wave {
    Pc pc = TOP;
    bool off = false;  // has seen the global queue out (defer_from = 2^30)
    uint32_t df = 0;   // defer_from for the current chunk
    std::vector<Lane> lane;
    uint32_t c_cl = 0, c_res = 0, k = 0, first = 0, left_cl = 0;
    uint32_t r_cl = 0, r_res = 0, cnt = 0;
    uint64_t wait_start = 0;
    bool tail_chunk = false;
    bool split = false;  // policy 4: a new chunk from the queue's end zone
    bool endf = false;   // policy 4: the block flag as this wave's claim read it
    uint32_t busy = 0;  // scheduler steps left in the current bounce
};

struct Model {
    uint32_t W, L, R, Q, B, defer_lanes, defer_from;
    int policy;
    uint32_t bounce_cost = 1;  // scheduler steps per bounce (an LDS step costs 1)
    std::mt19937_64* rng = nullptr;
    // ring
    uint32_t reserved = 0, claimed = 0;
    std::vector<uint32_t> turn;
    std::vector<uint32_t> pay_path, pay_n;
    uint32_t q_next = 0;
    bool end_flag = false;  // policy 4: a wave has seen the queue out
    std::vector<Wave> w;
    std::vector<uint32_t> T;     // bounces per path
    std::vector<uint32_t> done;  // completions per path
    uint64_t step = 0, last_change = 0, last_progress = 0, bounces = 0;
    uint64_t max_wait = 0, waits = 0, parks = 0, claims = 0, reserve_fail = 0, end_parks = 0;

    uint32_t lap(uint32_t seq) const { return seq / R; }
    // turn value (2 lap + c) as the kernel computes it
    uint32_t tv(uint32_t seq, uint32_t c) const {
        const uint32_t t = 2 * lap(seq) + c;
        return (policy & 2) ? (t & 0xFFFFFFu) : t;
    }
    uint32_t slot(uint32_t seq) const { return seq % R; }

    void start_loop(Wave& v) {
        for (auto& l : v.lane) {
            l.in_loop = l.live && l.n < T[l.path];
            l.deferred = false;
        }
        v.pc = B_TOP;
    }

    // one atomic step of wave i; returns whether shared or wave state changed
    bool exec(uint32_t i) {
        Wave& v = w[i];
        switch (v.pc) {
            case TOP:  // ring_claim: lane 0 reads claimed (policy 4: the flag first) ...
                v.endf = (policy & 4) && end_flag;
                v.c_cl = claimed;
                v.pc = CLAIM_RES;
                return true;
            case CLAIM_RES: {  // ... then reserved
                v.c_res = reserved;
                const uint32_t avail = v.c_res - v.c_cl, need = (v.off || v.endf) ? 1u : L;
                if (avail < need) { v.k = 0; v.pc = NOCLAIM; return true; }
                uint32_t cap = L;
                if (v.endf) {
                    const uint32_t lo = L / 4 ? L / 4 : 1, div = W / 2 ? W / 2 : 1;
                    cap = avail / div;
                    if (cap < lo) cap = lo;
                    if (cap > L) cap = L;
                }
                v.k = avail < cap ? avail : cap;
                v.pc = CLAIM_CAS;
                return true;
            }
            case CLAIM_CAS:
                if (claimed == v.c_cl) {
                    claimed += v.k;
                    v.first = v.c_cl;
                    ++claims;
                    for (uint32_t j = 0; j < L; ++j) v.lane[j] = Lane{};
                    v.pc = R_WAIT;
                    v.wait_start = step;
                } else {
                    v.k = 0;
                    v.pc = NOCLAIM;
                }
                return true;
            case NOCLAIM:
                if (v.off) { v.left_cl = claimed; v.pc = DRAIN_RES; } else v.pc = DEQUEUE;
                return true;
            case DRAIN_RES:
                v.pc = (reserved - v.left_cl) == 0 ? EXITED : TOP;
                return true;
            case DEQUEUE:
                if (q_next >= Q) { v.off = true; end_flag = true; v.pc = TOP; return true; }
                {
                    const uint32_t c = q_next++;
                    v.split = (policy & 4) && c + 4 * W >= Q;
                    for (uint32_t j = 0; j < L; ++j) {
                        v.lane[j] = Lane{};
                        v.lane[j].live = true;
                        v.lane[j].path = c * L + j;
                    }
                    v.tail_chunk = false;
                    v.df = v.off ? kOff : defer_from;
                    start_loop(v);
                }
                return true;
            case R_WAIT: {  // every lane < k: turn == 2 lap + 1
                bool all = true;
                for (uint32_t j = 0; j < v.k && all; ++j) {
                    const uint32_t s = v.first + j;
                    all = turn[slot(s)] == tv(s, 1);
                }
                if (!all) return false;
                const uint64_t dt = step - v.wait_start;
                if (dt > max_wait) max_wait = dt;
                ++waits;
                v.pc = R_LOAD;
                return true;
            }
            case R_LOAD:  // the payload loads and the release store (2 lap + 2), lanes < k
                for (uint32_t j = 0; j < L; ++j) {
                    Lane& l = v.lane[j];
                    l = Lane{};
                    if (j >= v.k) continue;
                    const uint32_t s = v.first + j;
                    l.live = true;
                    l.path = pay_path[slot(s)];
                    l.n = pay_n[slot(s)];
                    turn[slot(s)] = tv(s, 2);
                }
                v.tail_chunk = true;
                v.split = false;
                v.df = v.off ? kOff : defer_from;
                if ((policy & 1) && v.k <= defer_lanes) v.df = kOff;  // would re-park at once
                start_loop(v);
                return true;
            case B_TOP: {
                uint32_t in = 0, elig = 0;
                for (auto& l : v.lane) {
                    if (!l.in_loop) continue;
                    ++in;
                    if (l.n >= v.df) ++elig;
                }
                if (!in) { v.pc = AFTER; return true; }
                if (elig && (elig <= defer_lanes || (v.split && end_flag))) {
                    v.cnt = elig;
                    v.r_cl = claimed;  // ring_reserve: leader reads claimed ...
                    v.pc = RES_RES;
                } else {
                    v.pc = B_WORK;
                }
                return true;
            }
            case RES_RES:  // ... then reserved, room check
                v.r_res = reserved;
                if (v.r_res + v.cnt - v.r_cl <= R) v.pc = RES_CAS;
                else { ++reserve_fail; v.pc = B_WORK; }
                return true;
            case RES_CAS:
                if (reserved == v.r_res) {
                    reserved += v.cnt;
                    uint32_t s = v.r_res;
                    for (auto& l : v.lane)
                        if (l.in_loop && l.n >= v.df) { l.in_loop = false; l.deferred = true; l.seq = s++; }
                    ++parks;
                    if (v.split && end_flag) ++end_parks;
                } else {
                    ++reserve_fail;
                }
                v.pc = B_WORK;
                return true;
            case B_WORK: {  // one bounce of the lanes still in the loop (bounce_cost steps)
                if (v.busy == 0 && bounce_cost > 1) { v.busy = 1 + (uint32_t)((*rng)() % (2 * bounce_cost)); }
                if (v.busy > 1) { --v.busy; return true; }
                v.busy = 0;
                bool any = false;
                for (auto& l : v.lane) {
                    if (!l.in_loop) continue;
                    any = true;
                    ++l.n;
                    ++bounces;
                    if (l.n >= T[l.path]) l.in_loop = false;
                }
                if (any) last_progress = step;
                v.pc = B_TOP;
                return true;
            }
            case AFTER: {
                bool defer = false;
                for (auto& l : v.lane) {
                    if (!l.live) continue;
                    if (l.deferred) defer = true;
                    else ++done[l.path];
                }
                if (defer) { v.pc = W_WAIT; v.wait_start = step; } else v.pc = TOP;
                return true;
            }
            case W_WAIT: {  // every deferred lane: turn == 2 lap
                for (auto& l : v.lane)
                    if (l.deferred && turn[slot(l.seq)] != tv(l.seq, 0)) return false;
                const uint64_t dt = step - v.wait_start;
                if (dt > max_wait) max_wait = dt;
                ++waits;
                v.pc = W_STORE;
                return true;
            }
            case W_STORE:  // payload stores and the release store (2 lap + 1)
                for (auto& l : v.lane)
                    if (l.deferred) {
                        pay_path[slot(l.seq)] = l.path;
                        pay_n[slot(l.seq)] = l.n;
                        turn[slot(l.seq)] = tv(l.seq, 1);
                    }
                v.pc = TOP;
                return true;
            case EXITED:
                return false;
        }
        return false;
    }
};

}  // namespace

int main(int argc, char** argv) {
    if (argc < 13) {
        std::fprintf(stderr, "usage: ring_model waves lanes ring chunks max_bounces defer_lanes defer_from steps seed "
                             "policy burst bounce_cost [seq0]\n");
        return 2;
    }
    Model m;
    m.W = (uint32_t)std::atoi(argv[1]);
    m.L = (uint32_t)std::atoi(argv[2]);
    m.R = (uint32_t)std::atoi(argv[3]);
    m.Q = (uint32_t)std::atoi(argv[4]);
    m.B = (uint32_t)std::atoi(argv[5]);
    m.defer_lanes = (uint32_t)std::atoi(argv[6]);
    m.defer_from = (uint32_t)std::atoi(argv[7]);
    const uint64_t max_steps = std::strtoull(argv[8], nullptr, 10);
    const uint64_t seed = std::strtoull(argv[9], nullptr, 10);
    m.policy = std::atoi(argv[10]);
    const double burst = std::atof(argv[11]);
    m.bounce_cost = (uint32_t)std::atoi(argv[12]);
    std::mt19937_64 rng(seed);
    m.rng = &rng;
    m.turn.assign(m.R, 0);
    if (argc > 13) {  // counters at seq0; slot s last read in the lap before its next entry's
        const uint32_t seq0 = (uint32_t)std::strtoul(argv[13], nullptr, 10);
        m.reserved = m.claimed = seq0;
        for (uint32_t i = 0; i < m.R; ++i) {
            const uint32_t e = seq0 + i;  // the next entry using slot e % R
            m.turn[m.slot(e)] = m.tv(e, 0);
        }
    }
    m.pay_path.assign(m.R, 0xFFFFFFFFu);
    m.pay_n.assign(m.R, 0);
    m.w.resize(m.W);
    for (auto& v : m.w) v.lane.resize(m.L);
    const uint32_t n_paths = m.Q * m.L;
    m.T.resize(n_paths);
    m.done.assign(n_paths, 0);
    for (uint32_t p = 0; p < n_paths; ++p) {  // geometric-ish bounce counts, 1..B
        uint32_t t = 1;
        while (t < m.B && (rng() % 100) < 80) ++t;
        m.T[p] = t;
    }
    const uint64_t stall = 200000;  // steps without any change (deadlock) or any bounce (livelock)
    std::geometric_distribution<int> quantum(burst > 1.0 ? 1.0 / burst : 1.0);
    std::string verdict = "ok";
    uint32_t cur = 0;
    int left_q = 0;
    for (m.step = 0; m.step < max_steps; ++m.step) {
        std::vector<uint32_t> alive;
        for (uint32_t i = 0; i < m.W; ++i)
            if (m.w[i].pc != EXITED) alive.push_back(i);
        if (alive.empty()) break;
        if (left_q <= 0 || m.w[cur].pc == EXITED) {
            cur = alive[rng() % alive.size()];
            left_q = 1 + quantum(rng);
        }
        --left_q;
        if (m.exec(cur)) m.last_change = m.step;
        if (m.step - m.last_progress > stall) {  // no bounce for `stall` steps: stuck
            verdict = (m.step - m.last_change > stall / 2) ? "deadlock" : "livelock";
            break;
        }
    }
    bool all_exited = true;
    for (auto& v : m.w) all_exited &= v.pc == EXITED;
    if (verdict == "ok" && !all_exited) verdict = "unfinished";
    uint32_t lost = 0, dup = 0;
    for (uint32_t p = 0; p < n_paths; ++p) {
        if (m.done[p] == 0) ++lost;
        if (m.done[p] > 1) ++dup;
    }
    if (verdict == "ok" && (lost || dup || m.reserved != m.claimed)) verdict = "conservation";
    std::printf("{\"verdict\": \"%s\", \"steps\": %llu, \"bounces\": %llu, \"max_wait\": %llu, \"waits\": %llu, "
                "\"parks\": %llu, \"end_parks\": %llu, \"claims\": %llu, \"reserve_fail\": %llu, \"lost\": %u, \"dup\": %u, "
                "\"reserved\": %u, \"claimed\": %u, \"states\": \"",
                verdict.c_str(), (unsigned long long)m.step, (unsigned long long)m.bounces,
                (unsigned long long)m.max_wait, (unsigned long long)m.waits, (unsigned long long)m.parks,
                (unsigned long long)m.end_parks, (unsigned long long)m.claims, (unsigned long long)m.reserve_fail, lost, dup, m.reserved, m.claimed);
    for (uint32_t i = 0; i < m.W; ++i) std::printf("%s%s%s", i ? " " : "", pc_name(m.w[i].pc), m.w[i].off ? "*" : "");
    std::printf("\"}\n");
    return verdict == "ok" ? 0 : 1;
}
