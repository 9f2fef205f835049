// Shard-pointer tables: the crate's argument shape (every shard a buffer of its
// own: ReedSolomon::encode over the Vec<u8> per shard that reference
// src/vfs/block.rs:408-419 builds, reconstruct rebuilding every None into a
// fresh buffer, :556-565) on device memory or on mapped host memory.  Used by
// the *_ptrs_dev calls (ec_api.cpp) and by the submission queue that merges
// concurrent per-block calls (submit.cpp).
//
// A table whose touched shards sit on a slot lattice (ptr_grid.hpp: a Block-
// Cache slab, a slot pool with holes, rows merged from concurrent callers in
// any order) runs through the strided kernels over its slots; any other table
// goes up (table cache, table ring or capture reserve) and runs the table
// kernels, which wait on a scalar load of each block's row.
#include <algorithm>
#include <cstring>
#include <map>
#include <numeric>
#include <vector>

#include "ec_core.hpp"
#include "ptr_grid.hpp"

namespace shmr {
namespace core {

namespace {

using grid::Grid;
using grid::RowEntry;

// The strided form of a table: a layout over slots, and the rows that do work
// ordered by slot.
struct LatticeForm {
    Layout L{nullptr, nullptr, 0, 0, 0, 0, 0};
    std::vector<size_t> rows;       // table rows with work, ascending slot
    std::vector<uint64_t> slots;    // their slots
};

// Shard indices block `pr` reads (in[0 .. *ni)) and writes (out[0 .. *no)),
// ascending, without allocating (the per-block cost of a merged batch).
void touched_into(unsigned k, unsigned t, OpClass op, bool data_only, const uint8_t* pr, unsigned* in, unsigned* ni,
                  unsigned* out, unsigned* no) {
    *ni = *no = 0;
    if (op == kEncode) {
        for (unsigned i = 0; i < k; ++i) in[(*ni)++] = i;
        for (unsigned i = k; i < t; ++i) out[(*no)++] = i;
        return;
    }
    unsigned np = 0;
    for (unsigned i = 0; i < t; ++i) np += pr[i] ? 1 : 0;
    if (np == t) return;
    for (unsigned i = 0; i < t; ++i) {
        if (pr[i]) {
            if (*ni < k) in[(*ni)++] = i;
        } else if (i < k || !data_only) {
            out[(*no)++] = i;
        }
    }
}

bool lattice_form(unsigned k, unsigned t, const uint64_t* tab, const uint8_t* present, size_t n, bool data_only,
                  OpClass op, bool host_mapped, LatticeForm* F) {
    std::vector<size_t> rows;
    rows.reserve(n);
    // entries (row, position, address): inputs at their shard index; outputs at
    // index - k (encode: the parity rows), at their rank q among the block's
    // rebuilt shards (a compact output); every touched shard at its index
    // (rebuilt in place)
    // (epres, rebuilds: every present shard of the row -- they sit on the
    // same lattice as the ones read, and pin its shard pitch when each row
    // reads only one, k = 1)
    std::vector<RowEntry> ein, eout, eall, epres;
    ein.reserve(n * k);
    eout.reserve(n * (t - k));
    if (op == kDecode) {
        eall.reserve(n * t);
        epres.reserve(n * t);
    }
    unsigned in[256], out[256], ni = 0, no = 0;
    for (size_t b = 0; b < n; ++b) {
        touched_into(k, t, op, data_only, op == kEncode ? nullptr : present + b * t, in, &ni, out, &no);
        if (no == 0) continue;
        const uint64_t r = rows.size();
        rows.push_back(b);
        const uint64_t* row = tab + b * t;
        for (unsigned q = 0; q < ni; ++q) ein.push_back({r, in[q], row[in[q]]});
        for (unsigned q = 0; q < no; ++q) eout.push_back({r, op == kEncode ? uint64_t(out[q] - k) : q, row[out[q]]});
        if (op == kDecode) {   // inputs and outputs merged in index order
            unsigned x = 0, y = 0;
            while (x < ni || y < no) {
                const unsigned i = (y >= no || (x < ni && in[x] < out[y])) ? in[x++] : out[y++];
                eall.push_back({r, i, row[i]});
            }
            const uint8_t* pr = present + b * t;
            for (unsigned i = 0; i < t; ++i)
                if (pr[i] && row[i]) epres.push_back({r, i, row[i]});   // (queue rows: 0 where not read)
        }
    }
    if (rows.empty()) return false;
    const size_t nr = rows.size();
    std::vector<uint64_t> ain, aout, slots;
    uint64_t sp_in = 0, sp_out = 0;
    Grid gi, go;
    Layout& L = F->L;
    if (op == kEncode) {   // inputs on one lattice, parity rows on another over the same slots
        if (!grid::row_anchors(ein, nr, &sp_in, &ain) || !grid::fit_slots(ain, &gi, &slots)) return false;
        if (!grid::row_anchors(eout, nr, &sp_out, &aout) || !grid::fit_with_slots(aout, slots, &go)) return false;
        L = Layout{reinterpret_cast<const uint8_t*>(uintptr_t(gi.base)), reinterpret_cast<uint8_t*>(uintptr_t(go.base)),
                   gi.bpitch, sp_in, go.bpitch, sp_out, k};
    } else if (grid::row_anchors(eall, nr, &sp_in, &ain) && grid::fit_slots(ain, &gi, &slots)) {
        // every touched shard on one lattice: rebuilt in place
        uint8_t* base = reinterpret_cast<uint8_t*>(uintptr_t(gi.base));
        L = Layout{base, base, gi.bpitch, sp_in, gi.bpitch, sp_in, 0};
    } else {
        // present shards on one lattice, rebuilt shards (q-th of the block) on
        // another: a compact output (device memory only)
        if (host_mapped) return false;
        auto fit = [&](const std::vector<RowEntry>& e) {
            return grid::row_anchors(e, nr, &sp_in, &ain) && grid::fit_slots(ain, &gi, &slots) &&
                   grid::row_anchors(eout, nr, &sp_out, &aout) && grid::fit_with_slots(aout, slots, &go);
        };
        if (!fit(epres) && !fit(ein)) return false;
        L = Layout{reinterpret_cast<const uint8_t*>(uintptr_t(gi.base)), reinterpret_cast<uint8_t*>(uintptr_t(go.base)),
                   gi.bpitch, sp_in, go.bpitch, sp_out, 0};
        L.compact = true;
    }
    L.host_mapped = host_mapped;
    std::vector<size_t> order(nr);
    std::iota(order.begin(), order.end(), size_t(0));
    std::sort(order.begin(), order.end(), [&](size_t a, size_t b) { return slots[a] < slots[b]; });
    F->rows.resize(nr);
    F->slots.resize(nr);
    for (size_t i = 0; i < nr; ++i) {
        F->rows[i] = rows[order[i]];
        F->slots[i] = slots[order[i]];
    }
    return true;
}

// Whether a lattice rebuild would need the multi-plan block list -- several
// erasure patterns of one row count whose blocks (slot order) fall into more
// runs than the kernel arguments hold (ec_core reconstruct_on_device): every
// workgroup's plan is then three dependent loads away (list, plan index, plan
// table), and the table kernels, whose rows name the addresses directly, ran
// 3-5 points faster (pool with mixed patterns, profiles/r06/s1, s2:
// ptrs_ab decode83 pool_dense 0.666 / 0.656 vs pool_dense_tab 0.714 / 0.684).
bool lattice_needs_plan_list(unsigned t, const uint8_t* present, const LatticeForm& F) {
    std::map<std::vector<uint8_t>, std::vector<uint64_t>> by_pattern;   // pattern -> slots (ascending)
    for (size_t i = 0; i < F.rows.size(); ++i) {
        const uint8_t* pr = present + F.rows[i] * t;
        by_pattern[std::vector<uint8_t>(pr, pr + t)].push_back(F.slots[i]);
    }
    std::map<unsigned, std::pair<size_t, size_t>> by_m;   // absent count -> (patterns, runs)
    for (const auto& g : by_pattern) {
        unsigned m = 0;
        for (uint8_t x : g.first) m += x ? 0 : 1;
        size_t runs = 0;
        const auto& v = g.second;
        for (size_t i = 0; i < v.size();) {
            size_t e = i + 1;
            const uint64_t st = e < v.size() ? v[e] - v[i] : 1;
            while (e < v.size() && v[e] - v[e - 1] == st) ++e;
            ++runs;
            i = e;
        }
        auto& c = by_m[m];
        c.first += 1;
        c.second += runs;
    }
    for (const auto& kv : by_m)
        if (kv.second.first > 1 && kv.second.second > kern::kMaxSegs) return true;
    return false;
}

}  // namespace

int ptrs_launch(Codec& c, const uint64_t* tab, const uint8_t* present, size_t nblocks, uint64_t len, bool data_only,
                int device, hipStream_t stream, OpClass op, bool host_mapped, bool use_cache, bool* lattice) {
    const unsigned k = c.k(), t = k + c.p();
    if (lattice) *lattice = false;
    if (nblocks == 0) return SHMR_EC_OK;
    if (ptrs_grid()) {
        LatticeForm F;
        if (lattice_form(k, t, tab, present, nblocks, data_only, op, host_mapped, &F) &&
            !(op == kDecode && lattice_needs_plan_list(t, present, F)) &&
            slots_launch_fits(op, k, F.L, F.slots.data(), F.slots.size())) {
            int rc;
            if (op == kEncode) {
                rc = encode_on_device(c, device, F.L, F.rows.size(), len, stream, F.slots.data());
            } else {
                std::vector<uint8_t> pr(F.rows.size() * t);
                for (size_t i = 0; i < F.rows.size(); ++i) std::memcpy(&pr[i * t], present + F.rows[i] * t, t);
                rc = reconstruct_on_device(c, device, F.L, pr.data(), F.rows.size(), len, data_only, stream,
                                           F.slots.data());
            }
            if (rc == SHMR_EC_OK) {
                count_device(device, kDevPtrTableGrids);
                if (lattice) *lattice = true;
            }
            return rc;
        }
    }
    int rc = device_init(device, stream);
    if (rc) return rc;
    bool aligned = true;   // every shard the launch touches 16-byte aligned
    {
        unsigned in[256], out[256], ni = 0, no = 0;
        for (size_t b = 0; b < nblocks && aligned; ++b) {
            touched_into(k, t, op, data_only, op == kEncode ? nullptr : present + b * t, in, &ni, out, &no);
            for (unsigned q = 0; q < ni; ++q) aligned = aligned && (tab[b * t + in[q]] & 15u) == 0;
            for (unsigned q = 0; q < no; ++q) aligned = aligned && (tab[b * t + out[q]] & 15u) == 0;
        }
    }
    // The kernels read each block's row in plan order (input t at [t], output
    // r at [k + r]): a reconstruct's rows are permuted here, once per call, so
    // no shard address in the kernel waits on a plan index load.  An encode
    // table is already in plan order.
    const uint64_t* table = tab;
    std::vector<uint64_t> permuted;
    if (op == kDecode) {
        permuted.resize(nblocks * t);
        permute_ptr_rows(tab, present, nblocks, k, t, data_only, permuted.data());
        table = permuted.data();
    }
    auto run = [&](const uint8_t* d_tab, size_t b0, size_t n) -> int {
        Layout L{nullptr, nullptr, 0, 0, 0, 0, 0};
        L.d_ptrs = reinterpret_cast<const uint64_t*>(d_tab);
        L.total = t;
        L.ptrs_aligned = aligned;
        L.host_mapped = host_mapped;
        if (op == kEncode) return encode_on_device(c, device, L, n, len, stream);
        return reconstruct_on_device(c, device, L, present + b0 * t, n, len, data_only, stream);
    };
    bool capturing = false;
    if ((rc = capture_state(stream, &capturing))) return rc;
    if (capturing) {   // a block of the capture reserve, returned when the graph is destroyed
        const size_t bytes = nblocks * t * sizeof(uint64_t);
        uint8_t *h = nullptr, *d = nullptr;
        rc = capture_alloc(device, stream, bytes, &h, &d);
        if (rc) return rc;
        std::memcpy(h, table, bytes);
        if (hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, stream) != hipSuccess) {
            (void)hipGetLastError();
            return SHMR_EC_DEVICE_ERROR;
        }
        return run(d, 0, nblocks);
    }
    PtrTableCache* cache = nullptr;
    if (use_cache && !host_mapped && !(cache = PtrTableCache::for_device(device, &rc))) return rc;
    UploadRing* ring = nullptr;
    const size_t per_chunk = UploadRing::kSlotBytes / (sizeof(uint64_t) * t);
    for (size_t b0 = 0; b0 < nblocks; b0 += per_chunk) {
        const size_t n = std::min(per_chunk, nblocks - b0);
        if (cache) {   // a table this stream passed before (same bytes): its device copy, no upload
            const uint8_t* dtab = nullptr;
            int entry = -1;
            rc = cache->lookup(table + b0 * t, n * t * sizeof(uint64_t), stream, &dtab, &entry);
            if (rc) return rc;
            if (dtab) {
                rc = run(dtab, b0, n);
                const int rc2 = cache->release_after(entry, stream);
                if (rc) return rc;
                if (rc2) return rc2;
                continue;
            }
        }
        if (!ring && !(ring = UploadRing::for_device(device, &rc, UploadRing::kPointers))) return rc;
        uint8_t *hslot = nullptr, *dslot = nullptr;
        int slot = -1;
        rc = ring->acquire(&hslot, &dslot, &slot);
        if (rc) return rc;
        std::memcpy(hslot, table + b0 * t, n * t * sizeof(uint64_t));
        // Mapped shards: small launches (few 4 KiB tiles) read the table from
        // the pinned slot itself, no H2D copy in front of the kernel (every
        // workgroup reads its block's row; across PCIe that costs larger
        // launches 1-4 %, so they upload it).
        const uint64_t tiles = n * ((len + 4095) / 4096);
        const uint8_t* direct = host_mapped && tiles <= ptrs_direct_max() ? ring->host_view(slot) : nullptr;
        rc = direct ? SHMR_EC_OK : ring->upload(slot, n * t * sizeof(uint64_t), stream);
        if (rc == SHMR_EC_OK) rc = run(direct ? direct : dslot, b0, n);
        const int rc2 = ring->release_after(slot, stream);
        if (rc) return rc;
        if (rc2) return rc2;
    }
    return SHMR_EC_OK;
}

}  // namespace core
}  // namespace shmr
