// Slot grids in shard-pointer tables (the *_ptrs_dev calls; ec_api.cpp).
// Host logic only, header-only (tests/test_ptr_grid.py compiles it on the CPU).
//
// A table whose entries sit on a grid -- entry (b, j) at base + b * bpitch +
// j * spitch, as the buffers of a Block-Cache slab do (shmr_ec_device_alloc_
// shards, or any [blocks][shards][pitch] array) -- names exactly the addresses
// the strided kernels of the *_batch_dev calls compute from (base, pitches),
// in the same unsigned 64-bit arithmetic.  fit_grid finds such a grid or says
// there is none; every entry is checked, so a fit is exact by construction.
#pragma once

#include <algorithm>
#include <cstdint>
#include <vector>

namespace shmr {
namespace grid {

struct Entry {
    uint64_t b, j;
    uint64_t addr;
};

struct Grid {
    uint64_t base = 0, bpitch = 0, spitch = 0;
};

// Non-negative integers bp, sp with db * bp + dj * sp = da, where (db, dj) is
// the one direction every entry lies on (db >= 0; dj > 0 when db == 0): one
// pitch alone when it divides, else the general solution of the linear
// Diophantine equation.
inline bool solve_line(__int128 db, __int128 dj, __int128 da, __int128* bp, __int128* sp) {
    *bp = *sp = 0;
    if (db != 0 && da % db == 0 && da / db >= 0) {
        *bp = da / db;
        return true;
    }
    if (dj != 0 && da % dj == 0 && da / dj >= 0) {
        *sp = da / dj;
        return true;
    }
    if (db == 0 || dj == 0) return false;
    // extended Euclid: db * x + dj * y = g
    __int128 r0 = db, r1 = dj, x0 = 1, x1 = 0, y0 = 0, y1 = 1;
    while (r1 != 0) {
        const __int128 q = r0 / r1;
        __int128 t = r0 - q * r1;
        r0 = r1, r1 = t;
        t = x0 - q * x1, x0 = x1, x1 = t;
        t = y0 - q * y1, y0 = y1, y1 = t;
    }
    if (r0 < 0) r0 = -r0, x0 = -x0, y0 = -y0;
    if (da % r0 != 0) return false;
    const __int128 X = x0 * (da / r0), Y = y0 * (da / r0);   // one solution
    const __int128 qb = dj / r0, qs = db / r0;                // bp = X + qb t, sp = Y - qs t (qs > 0)
    auto fdiv = [](__int128 a, __int128 b) { return a / b - ((a % b != 0) && ((a < 0) != (b < 0))); };
    __int128 t_hi = fdiv(Y, qs);                              // sp >= 0
    __int128 t;
    if (qb > 0) {                                             // bp >= 0: t >= ceil(-X / qb)
        const __int128 t_lo = -fdiv(X, qb);
        if (t_lo > t_hi) return false;
        t = t_lo;
    } else {                                                  // bp >= 0: t <= floor(X / -qb)
        t = std::min(t_hi, fdiv(X, -qb));
    }
    *bp = X + qb * t;
    *sp = Y - qs * t;
    return *bp >= 0 && *sp >= 0 && db * *bp + dj * *sp == da;
}

// Entries in ascending b, then ascending j within a block.  Pitches must come
// out non-negative; a pitch no pair of entries determines is 0 (the kernels
// then never multiply it by an index that differs between entries).
inline bool fit_grid(const std::vector<Entry>& e, Grid* g) {
    *g = Grid{};
    if (e.empty()) return true;
    const Entry& e0 = e[0];
    // difference vectors (db, dj, da) of the entries against e0; solve
    //   da = db * bp + dj * sp
    // from two independent ones (Cramer's rule, exact integers), or from one
    // when every entry lies on one line of (b, j).
    __int128 v1b = 0, v1j = 0, v1a = 0;
    bool have1 = false, have2 = false;
    __int128 bp = 0, sp = 0;
    for (size_t i = 1; i < e.size() && !have2; ++i) {
        const __int128 db = __int128(e[i].b) - __int128(e0.b), dj = __int128(e[i].j) - __int128(e0.j);
        const __int128 da = __int128(e[i].addr) - __int128(e0.addr);
        if (db == 0 && dj == 0) return false;   // two entries for one (block, shard)
        if (!have1) {
            v1b = db, v1j = dj, v1a = da;
            have1 = true;
            continue;
        }
        const __int128 det = v1b * dj - v1j * db;
        if (det == 0) continue;
        const __int128 nb = v1a * dj - v1j * da, ns = v1b * da - db * v1a;
        if (nb % det != 0 || ns % det != 0) return false;
        bp = nb / det;
        sp = ns / det;
        have2 = true;
    }
    if (have1 && !have2 && !solve_line(v1b, v1j, v1a, &bp, &sp)) return false;   // collinear entries
    if (bp < 0 || sp < 0 || bp > __int128(UINT64_MAX) || sp > __int128(UINT64_MAX)) return false;
    const uint64_t ubp = uint64_t(bp), usp = uint64_t(sp);
    const uint64_t base = e0.addr - e0.b * ubp - e0.j * usp;   // wrapping, as the kernels compute
    for (const Entry& x : e)
        if (x.addr != base + x.b * ubp + x.j * usp) return false;
    g->base = base;
    g->bpitch = ubp;
    g->spitch = usp;
    return true;
}

}  // namespace grid
}  // namespace shmr
