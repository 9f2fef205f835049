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

// ---- slot lattices (r06) ------------------------------------------------------
// fit_grid takes a block's position in the table as its index.  A Block Cache
// that takes and drops blocks one at a time (a slot pool, shmr_ec_pool_*), or a
// batch merged from concurrent per-block calls, hands over rows in any order
// and with holes.  The block order of a batch does not change any byte, so a
// lattice instead FINDS each row's slot: row r's touched entries (j, addr) lie
// at base + s_r * bpitch + j * spitch, the slots s_r distinct.  The strided
// kernels then run over the slots (one arithmetic run, segment runs in the
// kernel arguments, or an uploaded block list: ec_core launch_slots).

struct RowEntry {
    uint64_t row, j;   // row of the table; shard position within the row
    uint64_t addr;
};

// The common shard pitch of the rows and each row's anchor (the address of its
// j = 0 position): entries grouped by row (ascending), every row 0 .. nrows-1
// with at least one entry.  The pitch comes from the first row holding two
// positions (exact, non-negative); rows that never hold two leave it 0 (the
// kernels then multiply it only by the one position each row touches).
inline bool row_anchors(const std::vector<RowEntry>& e, size_t nrows, uint64_t* spitch, std::vector<uint64_t>* anchor) {
    *spitch = 0;
    anchor->assign(nrows, 0);
    bool have = false;
    for (size_t i = 1; i < e.size() && !have; ++i) {
        if (e[i].row != e[i - 1].row || e[i].j == e[i - 1].j) continue;
        const __int128 dj = __int128(e[i].j) - __int128(e[i - 1].j);
        const __int128 da = __int128(e[i].addr) - __int128(e[i - 1].addr);
        if (da % dj != 0 || da / dj < 0 || da / dj > __int128(UINT64_MAX)) return false;
        *spitch = uint64_t(da / dj);
        have = true;
    }
    std::vector<bool> seen(nrows, false);
    for (const RowEntry& x : e) {
        if (x.row >= nrows) return false;
        const uint64_t a = x.addr - x.j * *spitch;   // wrapping, as the kernels compute
        if (!seen[x.row]) {
            seen[x.row] = true;
            (*anchor)[x.row] = a;
        } else if ((*anchor)[x.row] != a) {
            return false;
        }
    }
    for (bool s : seen)
        if (!s) return false;
    return true;
}

inline uint64_t gcd_u64(uint64_t a, uint64_t b) {
    while (b) {
        const uint64_t t = a % b;
        a = b;
        b = t;
    }
    return a;
}

// Slots from anchors: base = the lowest anchor, bpitch = the gcd of every
// anchor's distance from it, slot = distance / bpitch.  Distinct anchors only
// (two rows on one slot would be one block coded twice); slots < 2^32 (the
// kernels' block lists and segment runs are 32-bit).
inline bool fit_slots(const std::vector<uint64_t>& anchor, Grid* g, std::vector<uint64_t>* slot) {
    const size_t n = anchor.size();
    *g = Grid{};
    slot->assign(n, 0);
    if (n == 0) return false;
    uint64_t lo = anchor[0];
    for (uint64_t a : anchor) lo = std::min(lo, a);
    uint64_t gg = 0;
    for (uint64_t a : anchor) gg = gcd_u64(gg, a - lo);
    if (n > 1 && gg == 0) return false;
    for (size_t r = 0; r < n; ++r) {
        const uint64_t s = gg ? (anchor[r] - lo) / gg : 0;
        if (s >> 32) return false;
        (*slot)[r] = s;
    }
    std::vector<uint64_t> sorted(*slot);
    std::sort(sorted.begin(), sorted.end());
    for (size_t i = 1; i < n; ++i)
        if (sorted[i] == sorted[i - 1]) return false;
    g->base = lo;
    g->bpitch = gg;
    return true;
}

// A second lattice over the SAME slots (an encode's parity rows, a rebuild's
// compact output): anchor_r = base + slot_r * bpitch for every row, bpitch
// non-negative (from the lowest and the highest slot, exact), checked for
// every row in wrapping 64-bit arithmetic.
inline bool fit_with_slots(const std::vector<uint64_t>& anchor, const std::vector<uint64_t>& slot, Grid* g) {
    *g = Grid{};
    const size_t n = anchor.size();
    if (n == 0 || slot.size() != n) return false;
    size_t lo = 0, hi = 0;
    for (size_t r = 1; r < n; ++r) {
        if (slot[r] < slot[lo]) lo = r;
        if (slot[r] > slot[hi]) hi = r;
    }
    uint64_t bp = 0;
    if (slot[hi] != slot[lo]) {
        const __int128 d = __int128(anchor[hi]) - __int128(anchor[lo]);
        const __int128 ds = __int128(slot[hi]) - __int128(slot[lo]);
        if (d < 0 || d % ds != 0) return false;
        bp = uint64_t(d / ds);
    }
    const uint64_t base = anchor[lo] - slot[lo] * bp;
    for (size_t r = 0; r < n; ++r)
        if (anchor[r] != base + slot[r] * bp) return false;
    g->base = base;
    g->bpitch = bp;
    return true;
}

}  // namespace grid
}  // namespace shmr
