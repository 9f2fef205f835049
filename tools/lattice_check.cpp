// CPU driver of the slot-lattice fit (shmr_amd/csrc/ptr_grid.hpp row_anchors +
// fit_slots, and fit_with_slots for a second lattice over the same slots) for
// tests/test_ptr_grid.py.  Per case: "nrows nent nent2", then nent lines
// "row j addr" (the first lattice) and nent2 lines (the second; 0: none).
// Prints "1 base bpitch spitch [base2 bpitch2 spitch2] s_0 .. s_{nrows-1}" or "0".
#include <cstdio>
#include <vector>

#include "ptr_grid.hpp"

using namespace shmr::grid;

static bool read_entries(unsigned long long n, std::vector<RowEntry>* e) {
    e->resize(n);
    for (auto& x : *e) {
        unsigned long long r, j, a;
        if (std::scanf("%llu %llu %llu", &r, &j, &a) != 3) return false;
        x = {r, j, a};
    }
    return true;
}

int main() {
    unsigned long long nrows, n1, n2;
    while (std::scanf("%llu %llu %llu", &nrows, &n1, &n2) == 3) {
        std::vector<RowEntry> e1, e2;
        if (!read_entries(n1, &e1) || !read_entries(n2, &e2)) return 2;
        uint64_t sp = 0, sp2 = 0;
        std::vector<uint64_t> anchor, anchor2, slot;
        Grid g, g2;
        bool ok = row_anchors(e1, nrows, &sp, &anchor) && fit_slots(anchor, &g, &slot);
        if (ok && n2) ok = row_anchors(e2, nrows, &sp2, &anchor2) && fit_with_slots(anchor2, slot, &g2);
        if (!ok) {
            std::printf("0\n");
            continue;
        }
        std::printf("1 %llu %llu %llu", (unsigned long long)g.base, (unsigned long long)g.bpitch,
                    (unsigned long long)sp);
        if (n2)
            std::printf(" %llu %llu %llu", (unsigned long long)g2.base, (unsigned long long)g2.bpitch,
                        (unsigned long long)sp2);
        for (uint64_t s : slot) std::printf(" %llu", (unsigned long long)s);
        std::printf("\n");
    }
    return 0;
}
