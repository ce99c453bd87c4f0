// tsqr_plan.hpp -- the TSQR reduction tree's level plan and workspace layout
// (host only, no HIP: also built into the sanitized host checker).
//
// Level 0 factors the n-row panel in tiles of TR rows; level l+1 factors the
// stack of level l's tile R factors (m x m each); the local root has one
// tile.  With P ranks the local roots are all-gathered into the input of the
// first global level and the global levels run redundantly on every rank.
// Offsets are in doubles from the start of the tree workspace (-1 = none).
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace cal {

struct TsqrLevelPlan {
    int src = 0;              // 0 stack, 1 direct columns, 2 formed panel
    int64_t rows = 0, tiles = 0;
    int64_t in = -1;          // stack input (src 0): m x m blocks
    int64_t up = -1;          // UP output: tiles blocks of m x m
    int64_t down = -1;        // DOWN output of a stack level (input shape)
    int64_t S = -1;           // DOWN input: the parent's blocks (-1 at the root)
};

struct TsqrPlan {
    std::vector<TsqrLevelPlan> lv;
    size_t nlocal = 0;        // levels before the gathered stack
    size_t need = 0;          // workspace doubles
};

// plan for an n x m panel (tiles of TR rows) on rank `me` of P
TsqrPlan tsqr_plan(int64_t n, int m, int64_t TR, bool form, int P, int me);

}  // namespace cal
