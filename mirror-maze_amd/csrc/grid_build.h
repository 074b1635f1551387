// grid_build.h — host side of the certified grid search: the grid image
// (mm_device.h: DevGrid) built from the scene and its reference BVH.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "mm_types.h"

namespace mm {

constexpr uint32_t kMaxClasses = 64;  // threshold classes of compact records (6 bits)
constexpr uint32_t kGridClassBytes = 16 * kMaxClasses;  // the class table, ahead of the compact records

struct GridHost {
    float mn[3], mx[3], cell[3], inv[3];
    int n[3];
    uint32_t n_glob = 0;
    uint32_t glob[4] = {0, 0, 0, 0};
    uint32_t off_list = 0, off_recs = 0, off_box = 0, bytes = 0;
    uint32_t n_list = 0;
    uint32_t n_slow = 0;  // records the kernel tests with the general statement
    bool wide = true;     // 64-bit cell words with face ranges (else 32-bit: first | count << 22)
    // The maze forms (mm_grid.h kFlat): one cell along y, every listed record
    // FAST with an x or z normal, and at most kMaxClasses distinct folded
    // threshold tuples -- then the records are compact (16 B: origins + meta,
    // the thresholds in a class table at off_class) and the kernel walks x / z
    // with 2-way record selects.
    bool flat_ok = false;
    // The two global rects are y-normal FAST records in the planes y = slab_y[0] < slab_y[1] (glob[0],
    // glob[1]: the maze's floor and ceiling): a query tests only the one the ray is not moving away from
    // (mm_grid.h grid_search).
    bool slab = false;
    float slab_y[2] = {0.0f, 0.0f};
    uint32_t off_class = 0, n_class = 0;
    // Where the data after the index (cells + lists) starts: the class table of compact records (which
    // precedes their records, so a kernel that stages the data first finds the table at LDS address 0 and
    // record k at kGridClassBytes + 16 k -- compile-time offsets), else the records.
    uint32_t off_data = 0;
    std::vector<uint8_t> image;
};

// Returns false (with a reason) when the scene does not suit the search.
// merge_axes: an axis whose cells would not shorten the lists gets one cell (MM_OPT_GRID_MERGE).
// cell_scale: the first cell size tried, in units of the median rect extent (MM_OPT_GRID_CELL).
// wide: 64-bit cell words with per-face list ranges where they fit (MM_OPT_GRID_WIDE), else plain words.
bool build_grid(const mm_rect* rects, uint32_t n_rects, const mm_node* nodes, uint32_t n_nodes,
                const uint32_t* idx, size_t index_budget, GridHost& g, std::string& why, bool merge_axes = true,
                double cell_scale = 1.0, bool wide = true);

}  // namespace mm
