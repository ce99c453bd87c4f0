// tsqr_plan.cpp -- see tsqr_plan.hpp.
#include "tsqr_plan.hpp"

#include <algorithm>

namespace cal {

TsqrPlan tsqr_plan(int64_t n, int m, int64_t TR, bool form, int P, int me) {
    TsqrPlan p;
    const int64_t mm = (int64_t)m * m;
    auto push = [&](int src, int64_t rows) {
        TsqrLevelPlan L;
        L.src = src;
        L.rows = rows;
        L.tiles = (rows + TR - 1) / TR;
        p.lv.push_back(L);
        p.need += (size_t)L.tiles * mm;                   // UP output
        if (src == 0) p.need += (size_t)(rows / m) * mm;  // DOWN output (input shape)
    };
    push(form ? 2 : 1, std::max<int64_t>(n, 1));
    while (p.lv.back().tiles > 1) push(0, p.lv.back().tiles * m);
    p.nlocal = p.lv.size();
    if (P > 1) {
        push(0, (int64_t)P * m);  // the gathered local roots (the allgather's output is its input)
        p.need += (size_t)P * mm;
        while (p.lv.back().tiles > 1) push(0, p.lv.back().tiles * m);
    }
    int64_t off = 0;
    for (size_t l = 0; l < p.lv.size(); ++l) {
        TsqrLevelPlan& L = p.lv[l];
        if (P > 1 && l == p.nlocal) {  // gathered stack
            L.in = off;
            off += (int64_t)P * mm;
        }
        L.up = off;
        off += L.tiles * mm;
        if (L.src == 0) {
            L.down = off;
            off += (L.rows / m) * mm;
        }
        if (l + 1 < p.lv.size() && !(P > 1 && l + 1 == p.nlocal)) p.lv[l + 1].in = L.up;
    }
    // DOWN inputs: level l's S = level l+1's DOWN output; the local root's S =
    // this rank's block of the first global level's DOWN output
    for (size_t l = 0; l + 1 < p.lv.size(); ++l) p.lv[l].S = p.lv[l + 1].down;
    if (P > 1) p.lv[p.nlocal - 1].S = p.lv[p.nlocal].down + (int64_t)me * mm;
    p.lv.back().S = -1;
    return p;
}

}  // namespace cal
