// CPU driver of shmr::grid::fit_grid (shmr_amd/csrc/ptr_grid.hpp) for
// tests/test_ptr_grid.py: reads cases "n" then n lines "b j addr" from stdin,
// prints "1 base bpitch spitch" or "0" per case.
#include <cstdio>
#include <vector>

#include "ptr_grid.hpp"

int main() {
    unsigned long long n;
    while (std::scanf("%llu", &n) == 1) {
        std::vector<shmr::grid::Entry> e(n);
        for (auto& x : e) {
            unsigned long long b, j, a;
            if (std::scanf("%llu %llu %llu", &b, &j, &a) != 3) return 2;
            x = {b, j, a};
        }
        shmr::grid::Grid g;
        if (shmr::grid::fit_grid(e, &g))
            std::printf("1 %llu %llu %llu\n", (unsigned long long)g.base, (unsigned long long)g.bpitch,
                        (unsigned long long)g.spitch);
        else
            std::printf("0\n");
    }
    return 0;
}
