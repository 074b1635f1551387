// regroup_model.cpp -- VERDICT r03 item 2: would regrouping the paths that
// share a wave (by the next query's start cell and direction octant) raise
// the grid search's lane utilisation enough to pay for the regrouping?
//
// Input: the per-query records of scripts/grid_sim.c (DUMP=<file>; one record
// per closest-hit query of a C3 frame sample: path, bounce, start cell,
// octant, cells visited, list lengths of the first 6 cells, rejection-sampling
// trials of the shading that follows).  For each bounce index b < main_bounces
// (the bounces every path runs; C3's mirror tails past bounce 8 are the tail
// rings' business), waves of 64 paths are formed either as the kernel forms
// them (64 consecutive paths: 8 pixels x 8 samples) or by regrouping a pool of
// P paths (a resident block's 1024, or more) sorted by a key, and the wave's
// cell-synchronous loop costs are summed as the kernel runs them:
//   rect-test iterations  sum over cell steps c of max over lanes of len_c
//   cell-step iterations  max over lanes of cells visited
//   trial iterations      max over lanes of trials
// with the kernel's VALU per iteration (35 rect test, 32 cell step, 39
// trial; the default kernel's ISA) to weigh them.  No regrouping cost is
// charged: this is the upper bound of what regrouping can save.
//
//   g++ -O2 -std=c++17 -o /tmp/sim/regroup scripts/regroup_model.cpp
//   /tmp/sim/regroup /tmp/sim/q32.bin [main_bounces=8]
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <unordered_map>
#include <vector>

struct Q {  // scripts/grid_sim.c qrec_t
    uint32_t path;
    uint16_t cell0;
    uint8_t bounce, oct, ncells, trials, lens[6];
};
static_assert(sizeof(Q) == 16, "record layout");

struct Cost {
    double rect = 0, step = 0, trial = 0, lane_rect = 0, lane_step = 0, lane_trial = 0, waves = 0;
    double valu() const { return 35 * rect + 32 * step + 39 * trial; }
};

static void wave_cost(const std::vector<const Q*>& w, Cost& c) {
    if (w.empty()) return;
    int maxc = 0, maxt = 0;
    for (auto* q : w) { maxc = std::max(maxc, (int)q->ncells); maxt = std::max(maxt, (int)q->trials); }
    for (int k = 0; k < std::min(maxc, 6); ++k) {
        int m = 0;
        for (auto* q : w)
            if (q->ncells > k) m = std::max(m, (int)q->lens[k]);
        c.rect += m;
    }
    c.step += maxc;
    c.trial += maxt;
    for (auto* q : w) {
        for (int k = 0; k < std::min((int)q->ncells, 6); ++k) c.lane_rect += q->lens[k];
        c.lane_step += q->ncells;
        c.lane_trial += q->trials;
    }
    c.waves += 1;
}

int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: regroup q.bin [main_bounces]\n"); return 2; }
    const int main_b = argc > 2 ? atoi(argv[2]) : 8;
    FILE* f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 1; }
    std::vector<Q> recs;
    {
        Q buf[4096];
        size_t n;
        while ((n = fread(buf, sizeof(Q), 4096, f)) > 0) recs.insert(recs.end(), buf, buf + n);
        fclose(f);
    }
    // by bounce: the queries of every path, in path order
    std::vector<std::vector<const Q*>> by_b(main_b);
    for (auto& q : recs)
        if (q.bounce < main_b) by_b[q.bounce].push_back(&q);
    for (auto& v : by_b) std::sort(v.begin(), v.end(), [](const Q* a, const Q* b) { return a->path < b->path; });
    printf("%zu queries; per bounce:", recs.size());
    for (int b = 0; b < main_b; ++b) printf(" %zu", by_b[b].size());
    printf("\n");

    using Key = std::function<uint64_t(const Q*)>;
    struct Policy { std::string name; size_t pool; Key key; };
    const Key none = nullptr;
    std::vector<Policy> pols = {
        {"kernel: 64 consecutive paths (8 px x 8 spp)", 0, none},
        {"pool 1024, by (start cell, octant)", 1024, [](const Q* q) { return (uint64_t)q->cell0 << 3 | q->oct; }},
        {"pool 1024, by (octant, start cell)", 1024, [](const Q* q) { return (uint64_t)q->oct << 16 | q->cell0; }},
        {"pool 4096, by (start cell, octant)", 4096, [](const Q* q) { return (uint64_t)q->cell0 << 3 | q->oct; }},
        {"pool 65536, by (start cell, octant)", 65536, [](const Q* q) { return (uint64_t)q->cell0 << 3 | q->oct; }},
        {"pool 1024, by trials", 1024, [](const Q* q) { return (uint64_t)q->trials; }},
        {"pool 1024, by (start cell, octant, trials)", 1024,
         [](const Q* q) { return (uint64_t)q->cell0 << 11 | (uint64_t)q->oct << 8 | q->trials; }},
        {"pool 1024, by actual work (cells, lens): bound, not implementable", 1024,
         [](const Q* q) {
             uint64_t k = q->ncells;
             for (int i = 0; i < 6; ++i) k = k << 8 | q->lens[i];
             return k;
         }},
    };
    double base_valu = 0;
    for (auto& p : pols) {
        Cost c;
        for (int b = 0; b < main_b; ++b) {
            const auto& v = by_b[b];
            if (!p.pool) {  // the kernel's waves: 64 consecutive path ids (paths that ended are simply absent)
                std::vector<const Q*> w;
                uint32_t chunk = UINT32_MAX;
                for (auto* q : v) {
                    if (q->path / 64 != chunk) { wave_cost(w, c); w.clear(); chunk = q->path / 64; }
                    w.push_back(q);
                }
                wave_cost(w, c);
                continue;
            }
            for (size_t i0 = 0; i0 < v.size(); i0 += p.pool) {
                std::vector<const Q*> pool(v.begin() + i0, v.begin() + std::min(v.size(), i0 + p.pool));
                std::stable_sort(pool.begin(), pool.end(), [&](const Q* a, const Q* b) { return p.key(a) < p.key(b); });
                for (size_t j = 0; j < pool.size(); j += 64) {
                    std::vector<const Q*> w(pool.begin() + j, pool.begin() + std::min(pool.size(), j + 64));
                    wave_cost(w, c);
                }
            }
        }
        if (!p.pool) base_valu = c.valu();
        printf("%-66s waves %8.0f | iterations: rect %9.0f (util %.3f) step %9.0f (%.3f) trial %9.0f (%.3f) | "
               "weighted VALU %.4g (%.3f of the kernel's)\n",
               p.name.c_str(), c.waves, c.rect, c.lane_rect / (64 * c.rect), c.step, c.lane_step / (64 * c.step),
               c.trial, c.lane_trial / (64 * c.trial), c.valu(), c.valu() / base_valu);
    }
    return 0;
}
