// Device-side core of the erasure path (see ec_core.hpp).
#include "ec_core.hpp"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <string>
#include <unordered_map>
#include <unordered_set>

namespace shmr {
namespace core {

// ===========================================================================
// Tuning.  kAuto knobs follow kern::policy_variant: the fastest variants measured
// on MI355X per launch shape (tools/tune.py, interleaved A/B in one process;
// DESIGN.md "Tuning").  set_tuning() pins a knob explicitly.
// ===========================================================================
namespace {

constexpr int kBounceKibDefault = 8192;   // measured: see bounce_limit()
constexpr int kPtrsDirectDefault = 16;    // tiles; measured: see ptrs_direct_max()
constexpr int kSyncSpinDefault = 0;       // us; measured: see sync_stream()

struct Tuning {
    std::atomic<int> u{kAuto};
    std::atomic<int> nt_load{kAuto};
    std::atomic<int> nt_store{kAuto};
    std::atomic<int> occ8{0};
    std::atomic<int> grid{-1};     // -1: one workgroup per tile
    std::atomic<int> diag{0};
    std::atomic<int> threads{256};
    std::atomic<int> depth{kAuto};
    std::atomic<int> wgs_per_cu{kAuto};
    std::atomic<int> occ{kAuto};
    std::atomic<int> early{kAuto};
    std::atomic<int> spre{kAuto};
    std::atomic<int> fuse_tail{kAuto};
    std::atomic<int> glds{kAuto};
    std::atomic<int> serial{kAuto};
    std::atomic<int> sc1_store{kAuto};
    std::atomic<int> realign{kAuto};
    std::atomic<int> peel{kAuto};
    std::atomic<int> wave_run{kAuto};
    std::atomic<int> st_align{kAuto};
    std::atomic<int> xcd{kAuto};
    std::atomic<int> pair{kAuto};
};
Tuning g_tune[2];   // [kEncode], [kDecode]
std::atomic<int> g_bounce_kib{kBounceKibDefault};
std::atomic<int> g_mirror_zc{1};
std::atomic<int> g_ptrs_direct{kPtrsDirectDefault};
std::atomic<int> g_sync_spin{kSyncSpinDefault};
std::atomic<int> g_alias_devices{0};   // tools build: alias device IDs (see ec_core.hpp)
// Reconstructs over device shard-pointer tables take segment launches (plans in
// the kernel arguments) when they fit; 0 = always the uploaded block/plan table
std::atomic<int> g_ptrs_segs{1};
// Pointer tables that name a slot grid (ec_api.cpp ptrs_as_grid) take the strided kernels
// of the *_batch_dev calls; 0 = always the table kernels
std::atomic<int> g_ptrs_grid{1};
// Misaligned device-resident shards: kAuto = the vector kernels (modes 0 / 1)
// where the device passed probe_unaligned_vector, else the realigning kernel
// (mode 3); 0 = always mode 3 (what a device that fails the probe runs: exact
// results, so the product build takes it too -- the kernel sweep test runs the
// fallback kernels of the product library this way), 1 = always modes 0 / 1
// (tools build only: wrong on a device without the unaligned mode).
std::atomic<int> g_uvec{kAuto};
// Slot lists (launch_slots): 1 = always the uploaded block list, even for one
// arithmetic run or segment runs (tools build only: measures the list's cost)
std::atomic<int> g_slots_list{0};
// Reconstructs whose patterns' blocks fit no 32 segment runs: 0 = one multi-plan
// launch set (block list + per-block plan index uploaded: each workgroup's plan
// is two dependent loads away), 1 = one single-plan launch set per pattern over
// its blocks (launch_slots: a run, segment runs or a block list)
std::atomic<int> g_pattern_launches{0};
// Lattice tables whose slots need the uploaded block list (more than 32
// arithmetic runs, or several runs where segment launches do not apply):
// 0 = the table kernels instead (measured faster: profiles/r06 s1, s3, s14,
// ptrs_ab pool_holed vs pool_holed_tab), 1 = the strided kernels over the list
std::atomic<int> g_lattice_list{0};

// The launch policy itself is kern::policy_variant (gf_apply.hpp): constexpr,
// so the product library compiles exactly the kernels it can select.  Its
// measured basis (tools/tune.py, interleaved A/B in one process):
//  * depth-2 register ring (one shard of loads in flight per wave) beats depth
//    1 / 3 / 5 / 9 on every shape; nontemporal loads + stores win with it.
//  * U = 2 (8 KiB tiles) for 4-row launches: 4-erasure RS(10,4) rebuild 73.8
//    vs 67.8-68.9 % of HBM peak; 2- and 3-row launches lose 5-7 points at U = 2.
//  * early prologue for encodes with k <= 8 (RS(8,3) on padded slots +1.2 -
//    1.4 points, RS(4,2) +1.7 - 2.6) and, with the per-dword math order, for
//    4-row encodes (+1.0 / +0.5 / +1.0 / 0.0 on four boxes).
//  * partial last tiles at the head of the full-tile grid: -5.5 % (encode) /
//    -5.8 % (decode) time against a separate tail launch.
//  * reconstructs peel the ring's tail (no look-ahead load past the last input;
//    profiles/r03/r03h/).  1-row in-place rebuilds cap residency at 7
//    workgroups per CU (+1.4 - 1.7 on two boxes).
//  * rebuilt shards into buffers of their own (compact output, device pointer
//    tables): sc1 stores, no cap (RS(10,4) 2-erasure 81.1 / 81.2 % vs 77.4 %
//    with nontemporal stores); the early prologue there only for 4-row
//    rebuilds (+1.3 / +1.8).  r04 re-judged the 2- and 3-row adoptions of r03
//    (+0.7 / +0.7 / +1.1 / -0.8 and +0.5 / +0.5: under one point, not repeated
//    on three boxes) and dropped them.
//  * mapped host shards (zero-copy across PCIe): temporal loads (72 vs 64 GB/s
//    of RS(8,3) encode traffic), the plain LDS-staged tile.
//  * device pointer tables: the early prologue (first loads addressed from
//    scalar loads of the block's table row) for RS(8,3) encode (+1.8) and
//    every rebuild (+3.4 / +8.2 with sc1); RS(10,4) encode keeps the plain tile.

bool split_key(const char* key, std::string* k, int* first, int* last) {
    if (!key) return false;
    *k = key;
    *first = kEncode;
    *last = kDecode;
    if (k->rfind("encode.", 0) == 0) {
        *first = *last = kEncode;
        *k = k->substr(7);
    } else if (k->rfind("decode.", 0) == 0) {
        *first = *last = kDecode;
        *k = k->substr(7);
    }
    return true;
}

bool aligned16(uint64_t v) { return (v & 15u) == 0; }

}  // namespace

int set_tuning(const char* key, int value) {
    std::string k;
    int first = 0, last = 1;
    if (!split_key(key, &k, &first, &last)) return SHMR_EC_INVALID_ARGUMENT;
    if (k == "bounce_kib") {   // not per op class
        if (value < 0 && value != kAuto) return SHMR_EC_INVALID_ARGUMENT;
        g_bounce_kib = value == kAuto ? kBounceKibDefault : value;
        return SHMR_EC_OK;
    }
    if (k == "mirror_zc") {
        g_mirror_zc = value == kAuto ? 1 : (value != 0);
        return SHMR_EC_OK;
    }
    if (k == "ptrs_segs") {
        g_ptrs_segs = value == kAuto ? 1 : (value != 0);
        return SHMR_EC_OK;
    }
    if (k == "ptrs_grid") {
        g_ptrs_grid = value == kAuto ? 1 : (value != 0);
        return SHMR_EC_OK;
    }
    if (k == "ptrs_direct") {
        if (value < 0 && value != kAuto) return SHMR_EC_INVALID_ARGUMENT;
        g_ptrs_direct = value == kAuto ? kPtrsDirectDefault : value;
        return SHMR_EC_OK;
    }
    if (k == "sync_spin_us") {
        if (value < 0 && value != kAuto) return SHMR_EC_INVALID_ARGUMENT;
        g_sync_spin = value == kAuto ? kSyncSpinDefault : value;
        return SHMR_EC_OK;
    }
    if (k == "uvec") {   // not per op class; the product build takes kAuto and 0
#ifdef SHMR_EC_TOOLS
        if (value != kAuto && value != 0 && value != 1) return SHMR_EC_INVALID_ARGUMENT;
#else
        if (value != kAuto && value != 0) return SHMR_EC_INVALID_ARGUMENT;
#endif
        g_uvec = value;
        return SHMR_EC_OK;
    }
    if (k == "pattern_launches") {   // not per op class
        g_pattern_launches = value == kAuto ? 0 : (value != 0);
        return SHMR_EC_OK;
    }
    if (k == "lattice_list") {   // not per op class
        if (value != kAuto && value != 0 && value != 1) return SHMR_EC_INVALID_ARGUMENT;
        g_lattice_list = value == kAuto ? 0 : value;
        return SHMR_EC_OK;
    }
    if (k == "slots_list") {   // not per op class; tools build only
        const int v = value == kAuto ? 0 : value;
#ifdef SHMR_EC_TOOLS
        if (v != 0 && v != 1) return SHMR_EC_INVALID_ARGUMENT;
        g_slots_list = v;
        return SHMR_EC_OK;
#else
        return v == 0 ? SHMR_EC_OK : SHMR_EC_INVALID_ARGUMENT;
#endif
    }
    if (k == "alias_devices") {   // not per op class; tools build only (see ec_core.hpp)
        const int v = value == kAuto ? 0 : value;
#ifdef SHMR_EC_TOOLS
        if (v < 0 || v > 32) return SHMR_EC_INVALID_ARGUMENT;
        g_alias_devices = v;
        return SHMR_EC_OK;
#else
        return v == 0 ? SHMR_EC_OK : SHMR_EC_INVALID_ARGUMENT;
#endif
    }
#ifndef SHMR_EC_TOOLS
    // Product build: the kernel variant of every launch is the measured policy
    // (kern::policy_variant), the same for every caller in the process.  Kernel knobs
    // exist to take measurements and live in the tools build
    // (libshmr_ec_tools.so); here a knob may only be "set" to its default.
    // In particular "diag" (XOR-only, wrong results) is refused.
    {
        static const std::map<std::string, int> kDefaults = {
            {"chunks", kAuto}, {"nt_load", kAuto}, {"nt_store", kAuto}, {"occ8", 0},
            {"grid", -1},      {"diag", 0},        {"threads", 256},    {"depth", kAuto},   {"wgs_per_cu", kAuto},
            {"occ", kAuto},    {"early", kAuto},   {"spre", kAuto},     {"fuse_tail", kAuto},
            {"glds", kAuto},   {"serial", kAuto},   {"sc1_store", kAuto}, {"realign", kAuto}, {"peel", kAuto}, {"wave_run", kAuto}, {"st_align", kAuto},
            {"xcd", kAuto},    {"pair", kAuto}};
        const auto it = kDefaults.find(k);
        return (it != kDefaults.end() && it->second == value) ? SHMR_EC_OK : SHMR_EC_INVALID_ARGUMENT;
    }
#endif
    for (int i = first; i <= last; ++i) {
        Tuning& T = g_tune[i];
        if (k == "chunks") {
            if (value != 1 && value != 2 && value != 4 && value != kAuto) return SHMR_EC_INVALID_ARGUMENT;
            T.u = value;
        } else if (k == "nt_load") {
            T.nt_load = value == kAuto ? kAuto : (value != 0);
        } else if (k == "nt_store") {
            T.nt_store = value == kAuto ? kAuto : (value != 0);
        } else if (k == "occ8") {
            T.occ8 = value != 0;
        } else if (k == "grid") {
            if (value < -1) return SHMR_EC_INVALID_ARGUMENT;
            T.grid = value;
        } else if (k == "diag") {
            T.diag = value != 0;
        } else if (k == "threads") {
            if (value != 128 && value != 256 && value != 512) return SHMR_EC_INVALID_ARGUMENT;
            T.threads = value;
        } else if (k == "depth") {
            if (value != 1 && value != 2 && value != 3 && value != 5 && value != 9 && value != kAuto) return SHMR_EC_INVALID_ARGUMENT;
            T.depth = value;
        } else if (k == "wgs_per_cu") {
            if ((value < 0 || value > 32) && value != kAuto) return SHMR_EC_INVALID_ARGUMENT;
            T.wgs_per_cu = value;
        } else if (k == "occ") {
            if (value != 0 && value != 5 && value != 6 && value != 7 && value != kAuto) return SHMR_EC_INVALID_ARGUMENT;
            T.occ = value;
        } else if (k == "early") {
            T.early = value == kAuto ? kAuto : (value != 0);
        } else if (k == "spre") {
            T.spre = value == kAuto ? kAuto : (value != 0);
        } else if (k == "fuse_tail") {
            T.fuse_tail = value == kAuto ? kAuto : (value != 0);
        } else if (k == "glds") {
            T.glds = value == kAuto ? kAuto : (value != 0);
        } else if (k == "serial") {
            T.serial = value == kAuto ? kAuto : (value != 0);
        } else if (k == "sc1_store") {
            T.sc1_store = value == kAuto ? kAuto : (value != 0);
        } else if (k == "realign") {
            T.realign = value == kAuto ? kAuto : (value != 0);
        } else if (k == "peel") {
            T.peel = value == kAuto ? kAuto : (value != 0);
        } else if (k == "wave_run") {
            T.wave_run = value == kAuto ? kAuto : (value != 0);
        } else if (k == "st_align") {
            T.st_align = value == kAuto ? kAuto : (value != 0);
        } else if (k == "xcd") {
            T.xcd = value == kAuto ? kAuto : (value != 0);
        } else if (k == "pair") {
            T.pair = value == kAuto ? kAuto : (value != 0);
        } else {
            return SHMR_EC_INVALID_ARGUMENT;
        }
    }
    return SHMR_EC_OK;
}

int get_tuning(const char* key) {
    std::string k;
    int first = 0, last = 1;
    if (!split_key(key, &k, &first, &last)) return SHMR_EC_INVALID_ARGUMENT;
    const Tuning& T = g_tune[first];
    if (k == "bounce_kib") return g_bounce_kib;
    if (k == "mirror_zc") return g_mirror_zc;
    if (k == "ptrs_segs") return g_ptrs_segs;
    if (k == "ptrs_grid") return g_ptrs_grid;
    if (k == "ptrs_direct") return g_ptrs_direct;
    if (k == "sync_spin_us") return g_sync_spin;
    if (k == "alias_devices") return g_alias_devices;
    if (k == "slots_list") return g_slots_list;
    if (k == "lattice_list") return g_lattice_list;
    if (k == "pattern_launches") return g_pattern_launches;
    if (k == "uvec") return g_uvec;
    if (k == "chunks") return T.u;
    if (k == "nt_load") return T.nt_load;
    if (k == "nt_store") return T.nt_store;
    if (k == "occ8") return T.occ8;
    if (k == "grid") return T.grid;
    if (k == "diag") return T.diag;
    if (k == "threads") return T.threads;
    if (k == "depth") return T.depth;
    if (k == "wgs_per_cu") return T.wgs_per_cu;
    if (k == "occ") return T.occ;
    if (k == "early") return T.early;
    if (k == "spre") return T.spre;
    if (k == "fuse_tail") return T.fuse_tail;
    if (k == "glds") return T.glds;
    if (k == "serial") return T.serial;
    if (k == "sc1_store") return T.sc1_store;
    if (k == "realign") return T.realign;
    if (k == "peel") return T.peel;
    if (k == "wave_run") return T.wave_run;
    if (k == "st_align") return T.st_align;
    if (k == "xcd") return T.xcd;
    if (k == "pair") return T.pair;
    return SHMR_EC_INVALID_ARGUMENT;
}

kern::Variant select_variant(OpClass op, const kern::LaunchShape& s) {
    kern::Variant v = kern::policy_variant(s);
#ifdef SHMR_EC_TOOLS
    // Tools build: explicit knobs override the policy (measurement variants).
    const Tuning& T = g_tune[op];
    if (T.u.load() != kAuto) v.u = T.u.load();
    if (T.nt_load.load() != kAuto) v.nt_load = T.nt_load.load() != 0;
    if (T.nt_store.load() != kAuto) v.nt_store = T.nt_store.load() != 0;
    v.occ8 = T.occ8.load() != 0;
    v.diag = T.diag.load() != 0;
    v.threads = T.threads.load();
    if (T.depth.load() != kAuto) v.depth = T.depth.load();
    if (T.wgs_per_cu.load() != kAuto) v.wgs_per_cu = T.wgs_per_cu.load();
    if (T.occ.load() != kAuto) v.occ = T.occ.load();
    if (T.early.load() != kAuto) v.early = T.early.load() != 0;
    if (T.spre.load() != kAuto) v.spre = T.spre.load() != 0;
    if (T.fuse_tail.load() == 0) v.fuse_tail = false;
    if (T.glds.load() != kAuto) v.glds = T.glds.load() != 0;
    if (T.serial.load() != kAuto) v.serial = T.serial.load() != 0;
    if (T.sc1_store.load() != kAuto) v.sc1_store = T.sc1_store.load() != 0;
    if (T.peel.load() != kAuto) v.peel = T.peel.load() != 0;
    if (T.xcd.load() != kAuto) v.xcd = T.xcd.load() != 0;
    if (T.pair.load() != kAuto) v.pair = T.pair.load() != 0;
    if (T.wave_run.load() != kAuto)
        v.wave_run = T.wave_run.load() != 0;
    else
        v.wave_run = v.u > 1 && v.nt_load && v.depth == 2 && v.threads == 256 && !v.occ8 && !s.host_mapped &&
                     !v.glds && !v.spre;
    if (v.sc1_store) v.nt_store = false;        // one store policy per kernel
    if (v.glds) v.early = v.spre = false;       // the LDS-DMA ring is a form of the plain tile
    if (v.glds || v.depth != 2) v.peel = false;   // peeling is a form of the depth-2 register ring
    if (s.ptrs) v.spre = v.glds = false;        // the plain and the early tiles read pointer tables
    if (v.sc1_store && !s.sc1_ok) {
        v.sc1_store = false;
        v.nt_store = true;
    }
#else
    (void)op;
#endif
    return v;
}

kern::LaunchShape shape_of(OpClass op, unsigned k, unsigned rows, bool host_mapped, bool ptrs, bool segs,
                           bool compact, bool sc1_ok, bool fused) {
    kern::LaunchShape s;
    s.decode = op == kDecode;
    s.small_k = k <= 8;
    s.rows = rows;
    s.host_mapped = host_mapped;
    s.ptrs = ptrs;
    s.segs = segs && (s.decode || (!ptrs && !host_mapped));
    s.compact = compact && s.decode && !ptrs && !host_mapped;
    s.sc1_ok = sc1_ok && !host_mapped;
    s.fused = fused;
    return s;
}

bool segs_supported(OpClass op, unsigned k, bool host_mapped, bool ptrs, bool compact) {
    if (op == kEncode && (host_mapped || ptrs || compact)) return false;   // device pitch layouts only (shape_valid)
#ifdef SHMR_EC_TOOLS
    for (unsigned rows = 1; rows <= kern::kMaxRowsPerLaunch; ++rows)
        for (bool sc1_ok : {false, true}) {
            const kern::LaunchShape s = shape_of(op, k, rows, host_mapped, ptrs, true, compact, sc1_ok, false);
            if (!kern::variant_compiled(select_variant(op, s), rows)) return false;
        }
#else
    (void)op, (void)k, (void)host_mapped, (void)ptrs, (void)compact;   // every policy shape is compiled
#endif
    return true;
}

void permute_ptr_rows(const uint64_t* src, const uint8_t* present, size_t n, unsigned k, unsigned t, bool data_only,
                      uint64_t* dst) {
    for (size_t b = 0; b < n; ++b) {
        const uint64_t* s = src + b * t;
        uint64_t* d = dst + b * t;
        const uint8_t* pr = present ? present + b * t : nullptr;
        unsigned np = 0;
        for (unsigned i = 0; pr && i < t; ++i) np += pr[i] ? 1 : 0;
        if (!pr || np == t) {   // encode (already in plan order), or nothing to rebuild
            std::memcpy(d, s, size_t(t) * sizeof(uint64_t));
            continue;
        }
        unsigned ni = 0, no = 0;
        for (unsigned i = 0; i < t; ++i) {
            if (pr[i]) {
                if (ni < k) d[ni++] = s[i];   // the first k present shards, in index order
            } else if (i < k || !data_only) {
                d[k + no++] = s[i];           // the absent ones, ascending
            }
        }
        for (unsigned j = k + no; j < t; ++j) d[j] = 0;
    }
}

int grid_mode(OpClass op) { return g_tune[op].grid.load(); }

uint64_t bounce_limit() { return uint64_t(g_bounce_kib.load()) << 10; }

bool mirror_zero_copy() { return g_mirror_zc.load() != 0; }

uint64_t ptrs_direct_max() { return uint64_t(g_ptrs_direct.load()); }

bool ptrs_grid() { return g_ptrs_grid.load() != 0; }

bool slots_launch_fits(OpClass op, unsigned k, const Layout& L, const uint64_t* slots, uint64_t n) {
    if (g_lattice_list.load(std::memory_order_relaxed)) return true;
    uint64_t runs = 0;
    for (uint64_t i = 0; i < n;) {   // (launch_slots' run split)
        uint64_t e = i + 1;
        const uint64_t st = e < n ? slots[e] - slots[i] : 1;
        while (e < n && slots[e] - slots[e - 1] == st) ++e;
        if (++runs > kern::kMaxSegs) return false;
        i = e;
    }
    return runs <= 1 || segs_supported(op, k, L.host_mapped, L.d_ptrs != nullptr, L.compact);
}

hipError_t sync_stream(hipStream_t stream) {
    const int spin = g_sync_spin.load();
    if (spin > 0) {
        const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(spin);
        do {
            const hipError_t e = hipStreamQuery(stream);
            if (e != hipErrorNotReady) return e;
        } while (std::chrono::steady_clock::now() < until);
    }
    return hipStreamSynchronize(stream);
}

// ===========================================================================
// Devices and plans
// ===========================================================================
int device_count() {
    // asked at every compute call (check_device): the count a process sees does
    // not change once it is known, so it is read from HIP until it is
    static std::atomic<int> known{-1};
    const int k = known.load(std::memory_order_relaxed);
    if (k > 0) return k;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    if (n > 0) known.store(n, std::memory_order_relaxed);
    return n;
}

namespace {
constexpr int kMaxDevIds = 64;
std::atomic<uint64_t> g_dev_counters[kMaxDevIds][kDevCounters];
}  // namespace

int logical_device_count() {
    const int n = device_count();
    return n > 0 ? n + g_alias_devices.load() : 0;
}

int physical_device(int dev) {
    const int n = device_count();
    return (n > 0 && dev >= n) ? dev % n : dev;
}

int check_device(int dev) {
    const int n = logical_device_count();
    if (n <= 0) return SHMR_EC_NO_DEVICE;
    if (dev < 0 || dev >= n || dev >= kMaxDevIds) return SHMR_EC_INVALID_ARGUMENT;
    return SHMR_EC_OK;
}

void count_device(int dev, DevCounter c, uint64_t n) {
    if (dev >= 0 && dev < kMaxDevIds) g_dev_counters[dev][c].fetch_add(n, std::memory_order_relaxed);
}

void device_stats(int dev, uint64_t* out, size_t n) {
    for (size_t i = 0; i < n && i < size_t(kDevCounters); ++i)
        out[i] = (dev >= 0 && dev < kMaxDevIds) ? g_dev_counters[dev][i].load() : 0;
}

uint32_t plan_tab_off(unsigned k, unsigned m) {
    return uint32_t((8 + 2 * size_t(k) + 2 * size_t(m) + 31) & ~size_t(31));
}

// ---- per-device state: unaligned-access verdict and the plan arena ----------
namespace {
constexpr size_t kArenaChunk = size_t(4) << 20;   // ~3,000 RS(10,4) plan images
constexpr size_t kArenaAlign = 256;

struct ArenaChunk {
    uint8_t* host = nullptr;   // pinned
    uint8_t* dev = nullptr;
    size_t cap = 0, used = 0;
};

// The capture reserve: tables of captured calls, first-fit over chunks of
// pinned + device memory, each block back on its chunk's free list when the
// graph that captured it is destroyed (capture_alloc).
struct CaptureChunk {
    uint8_t* host = nullptr;
    uint8_t* dev = nullptr;
    size_t cap = 0;
    std::map<size_t, size_t> free_;   // offset -> length, coalesced
};

constexpr size_t kMirrorStreams = 32;   // per device: caller streams with a mirror stream of their own

struct DeviceState {
    int dev = -1;
    bool uvec = false;             // probe verdict of the physical GPU
    hipStream_t priv = nullptr;    // private stream of init-time work
    std::mutex mmu;                // guards mirrors
    std::unordered_map<hipStream_t, hipStream_t> mirrors;   // caller stream -> its mirror stream
    std::mutex mu;                 // guards chunks
    std::vector<ArenaChunk> chunks;
    std::mutex cmu;                // guards cchunks and their free lists
    std::vector<CaptureChunk*> cchunks;   // leaked with the state (graphs may outlive everything)
};

std::mutex g_state_mu;                          // serialises device_init
std::atomic<DeviceState*> g_state[kMaxDevIds];  // leaked: in-flight kernels read the arenas
std::map<int, bool>* g_probe_verdict = new std::map<int, bool>;   // physical GPU -> verdict

DeviceState* state_of(int dev) {
    return (dev >= 0 && dev < kMaxDevIds) ? g_state[dev].load(std::memory_order_acquire) : nullptr;
}

// Blocking: pinned + device allocation.  Caller holds ds.mu (or owns ds).
int add_chunk(DeviceState& ds, size_t bytes) {
    RelaxedCapture relaxed;
    ArenaChunk c;
    c.cap = std::max(round_up(bytes, kArenaAlign), kArenaChunk);
    count_device(ds.dev, kDevBlockingCalls, 2);
    if (hipHostMalloc(reinterpret_cast<void**>(&c.host), c.cap, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        return SHMR_EC_OUT_OF_MEMORY;
    }
    if (hipMalloc(reinterpret_cast<void**>(&c.dev), c.cap) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipHostFree(c.host);
        return SHMR_EC_OUT_OF_MEMORY;
    }
    ds.chunks.push_back(c);
    return SHMR_EC_OK;
}

constexpr size_t kCaptureChunk = size_t(4) << 20;   // the reserve device init creates

// Blocking: pinned + device allocation.  Caller holds ds.cmu (or owns ds).
int add_capture_chunk(DeviceState& ds, size_t bytes) {
    RelaxedCapture relaxed;
    auto* c = new CaptureChunk;
    c->cap = round_up(bytes, kArenaAlign);
    count_device(ds.dev, kDevBlockingCalls, 2);
    if (hipHostMalloc(reinterpret_cast<void**>(&c->host), c->cap, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        delete c;
        return SHMR_EC_OUT_OF_MEMORY;
    }
    if (hipMalloc(reinterpret_cast<void**>(&c->dev), c->cap) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipHostFree(c->host);
        delete c;
        return SHMR_EC_OUT_OF_MEMORY;
    }
    c->free_[0] = c->cap;
    ds.cchunks.push_back(c);
    return SHMR_EC_OK;
}

size_t largest_free_locked(const DeviceState& ds) {
    size_t best = 0;
    for (const CaptureChunk* c : ds.cchunks)
        for (const auto& r : c->free_) best = std::max(best, r.second);
    return best;
}

void capture_free_locked(CaptureChunk* c, size_t off, size_t len) {
    auto it = c->free_.emplace(off, len).first;
    auto next = std::next(it);
    if (next != c->free_.end() && it->first + it->second == next->first) {
        it->second += next->second;
        c->free_.erase(next);
    }
    if (it != c->free_.begin()) {
        auto prev = std::prev(it);
        if (prev->first + prev->second == it->first) {
            prev->second += it->second;
            c->free_.erase(it);
        }
    }
}

// One captured call's table: returned to the reserve by the destructor of the
// HIP user object its graph holds (runs on a HIP thread: no HIP calls here).
struct CaptureBlock {
    DeviceState* ds;
    CaptureChunk* c;
    size_t off, len;
};
void release_capture_block(void* p) {
    auto* b = static_cast<CaptureBlock*>(p);
    {
        std::lock_guard<std::mutex> lock(b->ds->cmu);
        capture_free_locked(b->c, b->off, b->len);
    }
    count_device(b->ds->dev, kDevCaptureReleased);
    delete b;
}
}  // namespace

int capture_state(hipStream_t stream, bool* capturing) {
    *capturing = false;
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    // under the mode the caller entered the library with (see RelaxedCapture)
    const CaptureModeTls& t = capture_mode_tls();
    hipStreamCaptureMode m = t.caller;
    const bool swap = t.depth > 0 && hipThreadExchangeStreamCaptureMode(&m) == hipSuccess;
    const hipError_t e = hipStreamIsCapturing(stream, &st);
    if (swap) (void)hipThreadExchangeStreamCaptureMode(&m);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        // e.g. the legacy null stream while another thread captures in global
        // mode: the call would join (and break) that capture -- refuse it
        return e == hipErrorStreamCaptureImplicit ? SHMR_EC_INVALID_ARGUMENT : SHMR_EC_DEVICE_ERROR;
    }
    if (st == hipStreamCaptureStatusInvalidated) return SHMR_EC_INVALID_ARGUMENT;
    *capturing = st == hipStreamCaptureStatusActive;
    return SHMR_EC_OK;
}

namespace {
std::mutex g_own_mu;
std::unordered_set<hipStream_t>* g_own_streams = new std::unordered_set<hipStream_t>;   // leaked
}  // namespace

void register_own_stream(hipStream_t s) {
    std::lock_guard<std::mutex> lock(g_own_mu);
    g_own_streams->insert(s);
}

bool own_stream(hipStream_t s) {
    std::lock_guard<std::mutex> lock(g_own_mu);
    return g_own_streams->count(s) != 0;
}

hipError_t grow_scratch(uint8_t** p, size_t* cap, size_t bytes, bool host) {
    static std::mutex mu;
    static auto* kept = new std::vector<std::pair<void*, bool>>;   // leaked: outlives static teardown
    const size_t want = std::max(bytes, *cap * 2);
    void* q = nullptr;
    const hipError_t e = host ? hipHostMalloc(&q, want, hipHostMallocMapped | hipHostMallocPortable)
                              : hipMalloc(&q, want);
    if (e != hipSuccess) return e;
    if (*p) {
        std::lock_guard<std::mutex> lock(mu);
        kept->emplace_back(*p, host);
    }
    *p = static_cast<uint8_t*>(q);
    *cap = want;
    return hipSuccess;
}

hipError_t create_priority_stream(hipStream_t* s) {
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) {
        (void)hipGetLastError();
        return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
    }
    return hipStreamCreateWithPriority(s, hipStreamNonBlocking, greatest);
}

int record_mirrored(int dev, hipStream_t stream, hipEvent_t on_caller, hipEvent_t mirror) {
    if (own_stream(stream)) {
        if (hipEventRecord(mirror, stream) == hipSuccess) return SHMR_EC_OK;
        (void)hipGetLastError();
        return SHMR_EC_DEVICE_ERROR;
    }
    DeviceState* ds = state_of(dev);
    if (!ds) {
        const int rc = device_init(dev, nullptr);
        if (rc) return rc;
        ds = state_of(dev);
    }
    // r06: the caller stream's own mirror stream (the private stream once the
    // per-device cap is reached): a caller stream held up by something outside
    // the library then delays only its own mirrors, not every other stream's
    // (before, all of them queued on the one private stream behind its wait)
    hipStream_t ms = ds->priv;
    {
        std::lock_guard<std::mutex> lock(ds->mmu);
        auto it = ds->mirrors.find(stream);
        if (it != ds->mirrors.end()) {
            ms = it->second;
        } else if (ds->mirrors.size() < kMirrorStreams) {
            hipStream_t m = nullptr;
            if (create_priority_stream(&m) == hipSuccess) {
                ds->mirrors[stream] = m;
                register_own_stream(m);
                count_device(dev, kDevStagingStreams);
                ms = m;
            } else {
                (void)hipGetLastError();
            }
        }
    }
    if (hipEventRecord(on_caller, stream) != hipSuccess || hipStreamWaitEvent(ms, on_caller, 0) != hipSuccess ||
        hipEventRecord(mirror, ms) != hipSuccess) {
        (void)hipGetLastError();
        return SHMR_EC_DEVICE_ERROR;
    }
    return SHMR_EC_OK;
}

int device_init(int dev, hipStream_t caller) {
    if (dev < 0 || dev >= kMaxDevIds) return SHMR_EC_INVALID_ARGUMENT;
    if (state_of(dev)) return SHMR_EC_OK;
    std::lock_guard<std::mutex> lock(g_state_mu);
    if (state_of(dev)) return SHMR_EC_OK;
    // Init allocates and synchronises: inside a capture it would invalidate
    // the caller's graph, so it is refused there (nothing enqueued).
    if (caller) {
        bool cap = false;
        const int rc = capture_state(caller, &cap);
        if (rc) return rc;
        if (cap) return SHMR_EC_INVALID_ARGUMENT;
    }
    DeviceScope scope(dev);
    if (!scope.ok()) return SHMR_EC_DEVICE_ERROR;
    RelaxedCapture relaxed;
    auto* ds = new DeviceState;
    ds->dev = dev;
    count_device(dev, kDevBlockingCalls);
    if (create_priority_stream(&ds->priv) != hipSuccess) {
        (void)hipGetLastError();
        delete ds;
        return SHMR_EC_DEVICE_ERROR;
    }
    register_own_stream(ds->priv);
    int rc = add_chunk(*ds, kArenaChunk);
    if (rc) {
        (void)hipStreamDestroy(ds->priv);
        delete ds;
        return rc;
    }
    rc = add_capture_chunk(*ds, kCaptureChunk);
    if (rc) {
        (void)hipStreamDestroy(ds->priv);
        (void)hipHostFree(ds->chunks.back().host);
        (void)hipFree(ds->chunks.back().dev);
        delete ds;
        return rc;
    }
    // the probe's scratch: the head of the first chunk
    ArenaChunk& c = ds->chunks.back();
    c.used = round_up(kern::kProbeScratchBytes, kArenaAlign);
    const int phys = physical_device(dev);
    auto it = g_probe_verdict->find(phys);
    if (it == g_probe_verdict->end()) {
        bool ok = false;
        count_device(dev, kDevBlockingCalls);
        if (kern::probe_unaligned_vector(&ok, c.dev, c.host, ds->priv) != hipSuccess) {
            (void)hipGetLastError();
            ok = false;   // the realigning kernel serves misaligned shards
        }
        it = g_probe_verdict->emplace(phys, ok).first;
    }
    ds->uvec = it->second;
    g_state[dev].store(ds, std::memory_order_release);
    return SHMR_EC_OK;
}

bool unaligned_vector(int dev) {
    const int knob = g_uvec.load();
    if (knob != kAuto) return knob != 0;
    const DeviceState* ds = state_of(dev);
    return ds && ds->uvec;
}

int arena_alloc(int dev, size_t bytes, bool capturing, uint8_t** host, uint8_t** devp) {
    DeviceState* ds = state_of(dev);
    if (!ds) return SHMR_EC_INVALID_ARGUMENT;
    bytes = round_up(bytes ? bytes : 1, kArenaAlign);
    std::lock_guard<std::mutex> lock(ds->mu);
    if (ds->chunks.back().used + bytes > ds->chunks.back().cap) {
        if (capturing) return SHMR_EC_OUT_OF_MEMORY;   // growth would allocate inside the capture
        DeviceScope scope(dev);
        if (!scope.ok()) return SHMR_EC_DEVICE_ERROR;
        const int rc = add_chunk(*ds, bytes);
        if (rc) return rc;
    }
    ArenaChunk& c = ds->chunks.back();
    *host = c.host + c.used;
    *devp = c.dev + c.used;
    c.used += bytes;
    return SHMR_EC_OK;
}

int capture_reserve(int dev, size_t bytes) {
    int rc = device_init(dev, nullptr);
    if (rc) return rc;
    DeviceState* ds = state_of(dev);
    bytes = round_up(bytes ? bytes : 1, kArenaAlign);
    std::lock_guard<std::mutex> lock(ds->cmu);
    if (largest_free_locked(*ds) >= bytes) return SHMR_EC_OK;
    DeviceScope scope(dev);
    if (!scope.ok()) return SHMR_EC_DEVICE_ERROR;
    return add_capture_chunk(*ds, std::max(bytes, kCaptureChunk));
}

int capture_alloc(int dev, hipStream_t stream, size_t bytes, uint8_t** host, uint8_t** devp) {
    DeviceState* ds = state_of(dev);
    if (!ds) return SHMR_EC_INVALID_ARGUMENT;
    bytes = round_up(bytes ? bytes : 1, kArenaAlign);
    CaptureChunk* chunk = nullptr;
    size_t off = 0;
    {
        std::lock_guard<std::mutex> lock(ds->cmu);
        for (CaptureChunk* c : ds->cchunks) {
            for (auto it = c->free_.begin(); it != c->free_.end(); ++it)
                if (it->second >= bytes) {
                    chunk = c;
                    off = it->first;
                    const size_t rest = it->second - bytes;
                    c->free_.erase(it);
                    if (rest) c->free_[off + bytes] = rest;
                    break;
                }
            if (chunk) break;
        }
    }
    if (!chunk) return SHMR_EC_OUT_OF_MEMORY;   // never grown inside a capture: shmr_ec_capture_reserve
    count_device(dev, kDevCaptureTables);
    *host = chunk->host + off;
    *devp = chunk->dev + off;
    // Tie the block to the graph being captured: a user object the graph
    // retains (and every executable graph made from it) returns the block when
    // the last of them is destroyed.  Without the graph handle the block stays
    // allocated for the life of the process.
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    hipGraph_t graph = nullptr;
    const hipGraphNode_t* deps = nullptr;
    size_t ndeps = 0;
    if (hipStreamGetCaptureInfo_v2(stream, &st, &id, &graph, &deps, &ndeps) != hipSuccess || !graph) {
        (void)hipGetLastError();
        return SHMR_EC_OK;
    }
    auto* blk = new CaptureBlock{ds, chunk, off, bytes};
    hipUserObject_t obj = nullptr;
    if (hipUserObjectCreate(&obj, blk, release_capture_block, 1, hipUserObjectNoDestructorSync) != hipSuccess) {
        (void)hipGetLastError();
        delete blk;
        return SHMR_EC_OK;
    }
    if (hipGraphRetainUserObject(graph, obj, 1, hipGraphUserObjectMove) != hipSuccess) {
        (void)hipGetLastError();   // the object (and with it the block) is kept for good
    }
    return SHMR_EC_OK;
}

// ---- plan images ---------------------------------------------------------------
namespace {
// One plan image on one device ID: a permanent pinned copy and its device
// twin in the arena.  The upload runs on the stream of the first use
// (kPending, `ready` recorded behind it) until observed complete (kDone); an
// upload recorded inside a capture (kCaptured) happens only when the graph
// runs, so the next use outside a capture uploads again.
struct PlanDev {
    uint8_t* host = nullptr;
    uint8_t* dev = nullptr;
    size_t bytes = 0;
    enum State { kCaptured, kPending, kDone } state = kCaptured;
    hipStream_t stream = nullptr;
    hipEvent_t ready = nullptr;    // recorded behind the upload on the caller's stream
    hipEvent_t mready = nullptr;   // its mirror (record_mirrored): queried and waited on
};

int upload_plan(PlanDev& pd, int dev, hipStream_t stream, bool capturing) {
    if (hipMemcpyAsync(pd.dev, pd.host, pd.bytes, hipMemcpyHostToDevice, stream) != hipSuccess) {
        (void)hipGetLastError();
        return SHMR_EC_DEVICE_ERROR;
    }
    if (capturing) return SHMR_EC_OK;   // a graph node: same bytes on every replay
    for (hipEvent_t* e : {&pd.ready, &pd.mready}) {
        if (*e) continue;
        RelaxedCapture relaxed;
        if (hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            *e = nullptr;
            return SHMR_EC_DEVICE_ERROR;
        }
    }
    const int rc = record_mirrored(dev, stream, pd.ready, pd.mready);
    if (rc) return rc;
    pd.state = PlanDev::kPending;
    pd.stream = stream;
    return SHMR_EC_OK;
}
}  // namespace

int plan_on_device(Plan& plan, int dev, hipStream_t stream, bool compact, const uint8_t** out) {
    bool cap = false;
    const int crc = capture_state(stream, &cap);
    if (crc) return crc;
    std::lock_guard<std::mutex> lock(plan.dev_mu);
    void*& slot = plan.dev_image[dev * 2 + (compact ? 1 : 0)];
    auto* pd = static_cast<PlanDev*>(slot);
    if (!pd) {
        const std::vector<uint8_t> img = plan.image(compact);
        uint8_t *h = nullptr, *d = nullptr;
        const int rc = arena_alloc(dev, img.size(), cap, &h, &d);
        if (rc) return rc;
        std::memcpy(h, img.data(), img.size());
        pd = new PlanDev;
        pd->host = h;
        pd->dev = d;
        pd->bytes = img.size();
        slot = pd;
        count_device(dev, kDevPlanImages);
        const int rc2 = upload_plan(*pd, dev, stream, cap);
        if (rc2) return rc2;
    } else if (pd->state == PlanDev::kPending && !cap) {
        const hipError_t q = hipEventQuery(pd->mready);
        if (q == hipSuccess) {
            pd->state = PlanDev::kDone;
        } else if (q == hipErrorNotReady) {
            (void)hipGetLastError();
            // still in flight on another stream (which may be held up by
            // anything): upload the same bytes again on this one rather than
            // wait for it (r06; the permanent pinned image, the same device
            // slot -- a second copy of identical bytes)
            if (pd->stream != stream) {
                const int rc = upload_plan(*pd, dev, stream, false);
                if (rc) return rc;
            }
        } else {
            (void)hipGetLastError();
            return SHMR_EC_DEVICE_ERROR;
        }
    } else if (pd->state != PlanDev::kDone) {
        // captured-only upload, or capturing now before the eager upload is
        // known complete: (re)upload on this stream -- identical bytes
        const int rc = upload_plan(*pd, dev, stream, cap);
        if (rc) return rc;
    }
    *out = pd->dev;
    return SHMR_EC_OK;
}

// ===========================================================================
// Launch sets.  Rows go in groups of <= 4 per launch; each group is one
// full-tile launch (the tuned variant) plus, when len is not a multiple of the
// tile, one launch over the remaining U=1 tiles (the last partial, byte-exact
// bounds).  Misaligned device-resident layouts take the same kernels where
// the device serves unaligned vector access (unaligned_vector), else the
// realigning kernel for full 4 KiB tiles plus the byte-granular one for the
// rest; misaligned mapped host shards take the byte-granular kernel.
// ===========================================================================
int launch_set(Plan& plan, int dev, const Layout& L, const BlockSet& bs, uint64_t len, hipStream_t stream,
               OpClass op) {
    const uint64_t nblk = bs.n;
    if (nblk == 0 || plan.m == 0) return SHMR_EC_OK;
    int rc = device_init(dev, stream);
    if (rc) return rc;
    const uint8_t* dplan = nullptr;
    const uint32_t tab_off = plan_tab_off(plan.k, plan.m);
    if (!bs.d_plans && !bs.segs) {
        rc = plan_on_device(plan, dev, stream, L.compact, &dplan);
        if (rc) return rc;
    }
    if (bs.nseg > kern::kMaxSegs) return SHMR_EC_INVALID_ARGUMENT;
    bool identity = true;   // encode plans (and decodes that lost only parity) read shard t as input t
    for (uint32_t t = 0; t < plan.k; ++t) identity = identity && plan.in_idx[t] == t;
    kern::Variant tail;   // tail / unaligned launches: U = 1, plain loads
    const int cap = grid_mode(op);
    const bool ptrs = L.d_ptrs != nullptr;
    // Misaligned device-resident shards (the reference's contiguous block
    // buffer, shard i at i * S) take the same vector kernels as aligned ones
    // where the device serves unaligned 16-byte accesses (verified once per
    // device at init; every access still covers only the lane's own bytes),
    // else the realigning kernel below (pitch layouts; misaligned device
    // shard-pointer tables then take the byte-granular kernel).  Mapped host
    // shards never do: the probe covered device memory only.
    const bool out16 = aligned16(uintptr_t(L.out_base)) && aligned16(L.out_bpitch) && aligned16(L.out_spitch);
    const bool aligned16_all =
        ptrs ? L.ptrs_aligned
             : aligned16(uintptr_t(L.in_base)) && aligned16(L.in_bpitch) && aligned16(L.in_spitch) && out16;
    const bool aligned = aligned16_all || (!L.host_mapped && unaligned_vector(dev));
    for (uint32_t row0 = 0; row0 < plan.m; row0 += kern::kMaxRowsPerLaunch) {
        const uint32_t rows = std::min<uint32_t>(kern::kMaxRowsPerLaunch, plan.m - row0);
        count_device(dev, kDevLaunches);
        // sc1 stores are raw buffer stores: a 2 GiB resource per output row,
        // and 16-byte aligned outputs only (the unaligned-access probe covers
        // the global instructions); otherwise nontemporal global stores
        const bool sc1_ok = len < (uint64_t(1) << 31) - 4096 && !L.host_mapped && (ptrs ? L.ptrs_aligned : out16);
        kern::LaunchShape shape = shape_of(op, plan.k, rows, L.host_mapped, ptrs, bs.segs != nullptr, L.compact,
                                           sc1_ok, false);
        kern::Variant var = select_variant(op, shape);
        {   // fused tails: the partial last tile of every block leads the full-tile grid
            const uint64_t tb0 = kern::tile_bytes(var.u, var.threads);
            if (len >= tb0 && len % tb0 != 0) {
                shape.fused = true;
                const kern::Variant fv = select_variant(op, shape);
                if (fv.fuse_tail && kern::variant_compiled(fv, rows)) var = fv;
            }
        }
        // Misaligned shards on a device with unaligned vector access: the
        // policy's kernels as they are, or (knob "realign", tools build) the
        // realigning-load form of the plain tile
        if (!aligned16_all && g_tune[op].realign.load() == 1 && !ptrs) {
            var.realign = true;
            var.early = var.spre = var.glds = var.peel = var.wave_run = false;   // the realigning tile keeps its own ring
        }
        // Misaligned output rows (knob "st_align", tools build): aligned
        // stores realigned across lanes in the full tiles
        if (!out16 && !ptrs && g_tune[op].st_align.load() == 1 && !var.realign) {
            var.st_align = true;
            if (op == kDecode) var.early = false;   // measured (and compiled) on the plain rebuild tile
        }
        const uint64_t tb = kern::tile_bytes(var.u, var.threads);
        kern::ApplyArgs a{};
        a.in_base = L.in_base;
        a.out_base = L.out_base;
        a.in_bpitch = L.in_bpitch;
        a.in_spitch = L.in_spitch;
        a.out_bpitch = L.out_bpitch;
        a.out_spitch = L.out_spitch;
        a.out_bias = L.out_bias;
        a.blk_list = bs.d_list;
        a.blk_first = bs.first;
        a.blk_stride = bs.stride;
        a.nblk = nblk;
        a.plan_table = bs.d_plans;
        a.blk_plan = bs.d_plan_idx;
        a.len = len;
        a.k = plan.k;
        a.m = plan.m;
        a.row0 = row0;
        a.plan = dplan;
        a.tab_off = tab_off;
        a.in_identity = (bs.d_plans || bs.segs) ? 0u : uint32_t(identity);
        a.nseg = bs.segs ? bs.nseg : 0;
        for (uint32_t i = 0; i < a.nseg; ++i) a.segs[i] = bs.segs[i];
        a.shard_ptrs = L.d_ptrs;
        a.total = L.total;
        if (!aligned) {
            // Device-resident shards off 16-byte alignment (the reference's
            // contiguous block buffer, shard i at i * S): full 4 KiB tiles in
            // the realigning vector kernel (mode 3), the rest byte-granular.
            // Mapped host shards stay byte-granular: their loads cross PCIe,
            // where mode 3's second (overlapping) load would be paid again.
            const uint64_t tb1 = kern::tile_bytes(1);
            const uint64_t full1 = (ptrs || L.host_mapped) ? 0 : len / tb1;
            if (full1) {
                a.col_base = 0;
                a.tiles_per_block = uint32_t(full1);
                a.ntiles = nblk * full1;
                SHMR_HIP_TRY(kern::launch_apply(a, rows, tail, 3, cap, stream));
            }
            if (len > full1 * tb1) {
                a.col_base = full1 * tb1;
                a.tiles_per_block = uint32_t((len - full1 * tb1 + tb1 - 1) / tb1);
                a.ntiles = nblk * a.tiles_per_block;
                SHMR_HIP_TRY(kern::launch_apply(a, rows, tail, 2, cap, stream));
            }
            continue;
        }
        const uint64_t full = len / tb;
        const bool fused = var.fuse_tail && full > 0 && len % tb != 0;
        var.fuse_tail = fused;
        if (full) {
            a.col_base = 0;
            a.tiles_per_block = uint32_t(full);
            a.lead_tails = fused ? nblk : 0;
            a.ntiles = nblk * full + a.lead_tails;
            const hipError_t e = kern::launch_apply(a, rows, var, 0, cap, stream);
            if (e == hipErrorInvalidValue) return SHMR_EC_INVALID_ARGUMENT;   // variant not compiled
            if (e != hipSuccess) return SHMR_EC_DEVICE_ERROR;
            a.lead_tails = 0;
        }
        if (len % tb && !fused) {
            const uint64_t tb1 = kern::tile_bytes(1);
            a.col_base = full * tb;
            a.tiles_per_block = uint32_t((len - full * tb + tb1 - 1) / tb1);
            a.ntiles = nblk * a.tiles_per_block;
            SHMR_HIP_TRY(kern::launch_apply(a, rows, tail, 1, cap, stream));
        }
    }
    return SHMR_EC_OK;
}

namespace {
// A launch's table in device memory: inside a capture a block of the capture
// reserve (every replay re-reads it; returned when the graph is destroyed),
// else a slot of the device's table ring, released behind the launch.
// fill(host) writes the bytes; launch(device copy) enqueues the kernels.
template <class Fill, class Launch>
int with_table(int dev, hipStream_t stream, size_t bytes, Fill fill, Launch launch) {
    bool capturing = false;
    int rc = capture_state(stream, &capturing);
    if (rc) return rc;
    uint8_t *h = nullptr, *d = nullptr;
    if (capturing) {
        rc = capture_alloc(dev, stream, bytes, &h, &d);
        if (rc) return rc;
        fill(h);
        if (hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, stream) != hipSuccess) {
            (void)hipGetLastError();
            return SHMR_EC_DEVICE_ERROR;
        }
        return launch(d);
    }
    if (bytes > UploadRing::kSlotBytes) return SHMR_EC_INVALID_ARGUMENT;
    UploadRing* ring = UploadRing::for_device(dev, &rc);
    if (!ring) return rc;
    int slot = -1;
    rc = ring->acquire(&h, &d, &slot);
    if (rc) return rc;
    fill(h);
    rc = ring->upload(slot, bytes, stream);
    if (rc == SHMR_EC_OK) rc = launch(d);
    const int rc2 = ring->release_after(slot, stream);
    return rc ? rc : rc2;
}
}  // namespace

int launch_slots(Plan& plan, int dev, const Layout& L, const uint64_t* slots, uint64_t n, uint64_t len,
                 hipStream_t stream, OpClass op) {
    if (n == 0) return SHMR_EC_OK;
    // maximal arithmetic runs of the (ascending) slots
    std::vector<kern::Seg> segs;
    bool fits = true;
    for (uint64_t i = 0; i < n;) {
        uint64_t e = i + 1;
        const uint64_t st = e < n ? slots[e] - slots[i] : 1;
        while (e < n && slots[e] - slots[e - 1] == st) ++e;
        if (segs.size() == kern::kMaxSegs) {
            fits = false;
            break;
        }
        kern::Seg sg{};
        sg.start = uint32_t(i);
        sg.first = uint32_t(slots[i]);
        sg.stride = e - i > 1 ? uint32_t(st) : 1u;
        segs.push_back(sg);
        i = e;
    }
    if (g_slots_list.load(std::memory_order_relaxed)) fits = false;   // (tools: the list, measured)
    if (fits && segs.size() == 1) {   // one run: the plain strided launch
        BlockSet bs;
        bs.first = slots[0];
        bs.stride = segs[0].stride;
        bs.n = n;
        return launch_set(plan, dev, L, bs, len, stream, op);
    }
    if (fits && segs_supported(op, plan.k, L.host_mapped, L.d_ptrs != nullptr, L.compact)) {
        const uint8_t* dp = nullptr;
        int rc = device_init(dev, stream);
        if (rc) return rc;
        rc = plan_on_device(plan, dev, stream, L.compact, &dp);
        if (rc) return rc;
        for (auto& sg : segs) sg.plan = dp;
        BlockSet bs;
        bs.n = n;
        bs.segs = segs.data();
        bs.nseg = uint32_t(segs.size());
        return launch_set(plan, dev, L, bs, len, stream, op);
    }
    // an uploaded block list, a ring slot per chunk
    const uint64_t per = UploadRing::kSlotBytes / sizeof(uint32_t);
    for (uint64_t c0 = 0; c0 < n; c0 += per) {
        const uint64_t cnt = std::min(per, n - c0);
        const int rc = with_table(
            dev, stream, size_t(cnt) * sizeof(uint32_t),
            [&](uint8_t* h) {
                uint32_t* l = reinterpret_cast<uint32_t*>(h);
                for (uint64_t j = 0; j < cnt; ++j) l[j] = uint32_t(slots[c0 + j]);
            },
            [&](const uint8_t* d) {
                BlockSet bs;
                bs.n = cnt;
                bs.d_list = reinterpret_cast<const uint32_t*>(d);
                return launch_set(plan, dev, L, bs, len, stream, op);
            });
        if (rc) return rc;
    }
    return SHMR_EC_OK;
}

int encode_on_device(Codec& c, int dev, const Layout& L, uint64_t nblocks, uint64_t len, hipStream_t stream,
                     const uint64_t* slots) {
    // (first: segment launches upload the plan before launch_set would init
    // the device -- r06 s30, a pool encode as a process's first call)
    const int rc = device_init(dev, stream);
    if (rc) return rc;
    count_device(dev, kDevBlocksEncoded, nblocks);
    if (slots) return launch_slots(*c.encode_plan(), dev, L, slots, nblocks, len, stream, kEncode);
    BlockSet bs;
    bs.n = nblocks;
    return launch_set(*c.encode_plan(), dev, L, bs, len, stream, kEncode);
}

int validate_presence(const Codec& c, const uint8_t* present, uint64_t nblocks) {
    const unsigned k = c.k(), t = k + c.p();
    for (uint64_t b = 0; b < nblocks; ++b) {
        unsigned np = 0;
        for (unsigned i = 0; i < t; ++i) np += present[b * t + i] ? 1 : 0;
        if (np != t && np < k) return SHMR_EC_TOO_FEW_SHARDS_PRESENT;
    }
    return SHMR_EC_OK;
}

int reconstruct_on_device(Codec& c, int dev, uint8_t* d_shards, uint64_t shard_pitch, uint64_t block_pitch,
                          const uint8_t* present, uint64_t nblocks, uint64_t len, bool data_only,
                          hipStream_t stream) {
    const Layout L{d_shards, d_shards, block_pitch, shard_pitch, block_pitch, shard_pitch, 0};
    return reconstruct_on_device(c, dev, L, present, nblocks, len, data_only, stream);
}

int reconstruct_on_device(Codec& c, int dev, const Layout& L, const uint8_t* present, uint64_t nblocks, uint64_t len,
                          bool data_only, hipStream_t stream, const uint64_t* slots) {
    const unsigned k = c.k(), t = k + c.p();
    int rc = device_init(dev, stream);
    if (rc) return rc;
    std::map<std::vector<uint8_t>, std::vector<uint64_t>> groups;   // pattern -> blocks
    for (uint64_t b = 0; b < nblocks; ++b) {
        const uint8_t* pr = present + b * t;
        unsigned np = 0;
        for (unsigned i = 0; i < t; ++i) np += pr[i] ? 1 : 0;
        if (np == t) continue;                          // crate: all present -> Ok(())
        if (np < k) return SHMR_EC_TOO_FEW_SHARDS_PRESENT;
        std::vector<uint8_t> key(t);
        for (unsigned i = 0; i < t; ++i) key[i] = pr[i] ? 1 : 0;
        groups[key].push_back(slots ? slots[b] : b);
    }
    if (groups.empty()) return SHMR_EC_OK;
    for (auto& g : groups) count_device(dev, kDevBlocksReconstructed, g.second.size());
    // Patterns with the same number of rebuilt shards share one multi-plan
    // launch set: the kernel picks each block's plan from a device table, so a
    // batch with many erasure patterns is still one launch (plus a tail).
    struct Group {
        std::vector<std::shared_ptr<Plan>> plans;
        std::vector<uint32_t> blocks;
        std::vector<uint16_t> plan_idx;
    };
    std::map<unsigned, Group> by_m;
    for (auto& g : groups) {
        auto plan = c.reconstruct_plan(g.first, data_only);
        if (plan->m == 0) continue;
        Group& grp = by_m[plan->m];
        const uint16_t pi = uint16_t(grp.plans.size());
        grp.plans.push_back(plan);
        for (uint64_t b : g.second) {
            grp.blocks.push_back(uint32_t(b));
            grp.plan_idx.push_back(pi);
        }
    }
    for (auto& kv : by_m) {
        Group& grp = kv.second;
        // A single pattern over an arithmetic block sequence needs no upload.
        bool arith = grp.plans.size() == 1;
        const uint64_t stride = grp.blocks.size() > 1 ? uint64_t(grp.blocks[1]) - grp.blocks[0] : 1;
        for (size_t i = 1; arith && i < grp.blocks.size(); ++i)
            arith = uint64_t(grp.blocks[i]) - grp.blocks[i - 1] == stride;
        if (arith) {
            BlockSet bs;
            bs.first = grp.blocks[0];
            bs.stride = stride;
            bs.n = grp.blocks.size();
            rc = launch_set(*grp.plans[0], dev, L, bs, len, stream, kDecode);
            if (rc) return rc;
            continue;
        }
        // Few patterns whose blocks form few arithmetic runs (a failed disk,
        // or the b-mod-k erasures of the benchmark): the runs and their plans
        // travel in the kernel arguments -- no table upload on the stream and
        // no dependent table loads in the kernel prologue.
        {
            std::vector<kern::Seg> segs;
            // (device shard-pointer tables: knob "ptrs_segs")
            bool fits = (!(L.d_ptrs && !L.host_mapped) || g_ptrs_segs.load() != 0) &&
                        segs_supported(kDecode, c.k(), L.host_mapped, L.d_ptrs != nullptr, L.compact);
            for (size_t i = 0; i < grp.blocks.size() && fits;) {
                size_t e = i + 1;
                const uint32_t st = e < grp.blocks.size() ? grp.blocks[e] - grp.blocks[i] : 1;
                while (e < grp.blocks.size() && grp.plan_idx[e] == grp.plan_idx[i] &&
                       grp.blocks[e] > grp.blocks[e - 1] && grp.blocks[e] - grp.blocks[e - 1] == st)
                    ++e;
                if (segs.size() == kern::kMaxSegs) {
                    fits = false;
                    break;
                }
                kern::Seg sg{};
                sg.start = uint32_t(i);
                sg.first = grp.blocks[i];
                sg.stride = e - i > 1 ? st : 1;
                segs.push_back(sg);
                // remember the plan index in pad_ until the device pointers are known
                segs.back().pad_ = grp.plan_idx[i];
                i = e;
            }
            if (fits) {
                for (auto& sg : segs) {
                    const uint8_t* dp = nullptr;
                    rc = plan_on_device(*grp.plans[sg.pad_], dev, stream, L.compact, &dp);
                    if (rc) return rc;
                    sg.plan = dp;
                    sg.pad_ = 0;
                }
                BlockSet bs;
                bs.n = grp.blocks.size();
                bs.segs = segs.data();
                bs.nseg = uint32_t(segs.size());
                rc = launch_set(*grp.plans[0], dev, L, bs, len, stream, kDecode);
                if (rc) return rc;
                continue;
            }
        }
        if (g_pattern_launches.load(std::memory_order_relaxed)) {   // a single-plan launch set per pattern
            std::vector<std::vector<uint64_t>> per(grp.plans.size());
            for (size_t i = 0; i < grp.blocks.size(); ++i) per[grp.plan_idx[i]].push_back(grp.blocks[i]);
            for (size_t pi = 0; pi < per.size(); ++pi) {
                rc = launch_slots(*grp.plans[pi], dev, L, per[pi].data(), per[pi].size(), len, stream, kDecode);
                if (rc) return rc;
            }
            continue;
        }
        if (grp.plans.size() > 65535) return SHMR_EC_INVALID_ARGUMENT;
        std::vector<const uint8_t*> dplans(grp.plans.size());
        for (size_t i = 0; i < grp.plans.size(); ++i) {
            rc = plan_on_device(*grp.plans[i], dev, stream, L.compact, &dplans[i]);
            if (rc) return rc;
        }
        const size_t ptab_bytes = (dplans.size() * sizeof(void*) + 15) & ~size_t(15);
        bool capturing = false;
        rc = capture_state(stream, &capturing);
        if (rc) return rc;
        if (capturing) {
            // Inside a capture the tables must outlive every replay: a block of
            // the capture reserve, returned when the graph is destroyed.
            const size_t n = grp.blocks.size();
            const size_t list_off = ptab_bytes;
            const size_t pidx_off = (list_off + n * sizeof(uint32_t) + 15) & ~size_t(15);
            const size_t total = pidx_off + n * sizeof(uint16_t);
            uint8_t *h = nullptr, *d = nullptr;
            rc = capture_alloc(dev, stream, total, &h, &d);
            if (rc) return rc;
            std::memcpy(h, dplans.data(), dplans.size() * sizeof(void*));
            std::memcpy(h + list_off, grp.blocks.data(), n * sizeof(uint32_t));
            std::memcpy(h + pidx_off, grp.plan_idx.data(), n * sizeof(uint16_t));
            if (hipMemcpyAsync(d, h, total, hipMemcpyHostToDevice, stream) != hipSuccess) {
                (void)hipGetLastError();
                return SHMR_EC_DEVICE_ERROR;
            }
            BlockSet bs;
            bs.n = n;
            bs.d_plans = reinterpret_cast<const uint8_t* const*>(d);
            bs.d_list = reinterpret_cast<const uint32_t*>(d + list_off);
            bs.d_plan_idx = reinterpret_cast<const uint16_t*>(d + pidx_off);
            rc = launch_set(*grp.plans[0], dev, L, bs, len, stream, kDecode);
            if (rc) return rc;
            continue;
        }
        UploadRing* ring = UploadRing::for_device(dev, &rc);
        if (!ring) return rc;
        const size_t table_bytes = ptab_bytes;
        if (table_bytes + 64 > UploadRing::kSlotBytes) return SHMR_EC_INVALID_ARGUMENT;
        const size_t per_chunk = (UploadRing::kSlotBytes - table_bytes - 32) / (sizeof(uint32_t) + sizeof(uint16_t));
        for (size_t c0 = 0; c0 < grp.blocks.size(); c0 += per_chunk) {
            const size_t n = std::min(per_chunk, grp.blocks.size() - c0);
            uint8_t *hslot = nullptr, *dslot = nullptr;
            int slot = -1;
            rc = ring->acquire(&hslot, &dslot, &slot);
            if (rc) return rc;
            const size_t list_off = table_bytes;
            const size_t pidx_off = (list_off + n * sizeof(uint32_t) + 15) & ~size_t(15);
            const size_t total = pidx_off + n * sizeof(uint16_t);
            std::memcpy(hslot, dplans.data(), dplans.size() * sizeof(void*));
            std::memcpy(hslot + list_off, grp.blocks.data() + c0, n * sizeof(uint32_t));
            std::memcpy(hslot + pidx_off, grp.plan_idx.data() + c0, n * sizeof(uint16_t));
            rc = ring->upload(slot, total, stream);
            BlockSet bs;
            bs.n = n;
            bs.d_plans = reinterpret_cast<const uint8_t* const*>(dslot);
            bs.d_list = reinterpret_cast<const uint32_t*>(dslot + list_off);
            bs.d_plan_idx = reinterpret_cast<const uint16_t*>(dslot + pidx_off);
            if (rc == SHMR_EC_OK) rc = launch_set(*grp.plans[0], dev, L, bs, len, stream, kDecode);
            const int rc2 = ring->release_after(slot, stream);
            if (rc) return rc;
            if (rc2) return rc2;
        }
    }
    return SHMR_EC_OK;
}

// ===========================================================================
// Upload ring
// ===========================================================================
UploadRing* UploadRing::for_device(int dev, int* rc, Kind kind) {
    static std::mutex mu;
    static auto* rings = new std::map<std::pair<int, int>, UploadRing*>;   // leaked: outlives static teardown
    std::lock_guard<std::mutex> lock(mu);
    auto& r = (*rings)[{dev, int(kind)}];
    if (!r) {
        RelaxedCapture relaxed;
        auto* ring = new UploadRing;
        ring->dev_id_ = dev;
        // on failure nothing is kept: the next call retries from scratch
        auto give_up = [&](int code) -> UploadRing* {
            for (int i = 0; i < kSlots; ++i) {
                if (ring->ev_[i]) (void)hipEventDestroy(ring->ev_[i]);
                if (ring->mev_[i]) (void)hipEventDestroy(ring->mev_[i]);
            }
            if (ring->dev_) (void)hipFree(ring->dev_);
            if (ring->host_) (void)hipHostFree(ring->host_);
            (void)hipGetLastError();
            delete ring;
            *rc = code;
            return nullptr;
        };
        count_device(dev, kDevBlockingCalls, 2);
        if (hipHostMalloc(reinterpret_cast<void**>(&ring->host_), kSlots * kSlotBytes, hipHostMallocDefault) !=
                hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&ring->dev_), kSlots * kSlotBytes) != hipSuccess)
            return give_up(SHMR_EC_OUT_OF_MEMORY);
        for (int i = 0; i < kSlots; ++i)
            if (hipEventCreateWithFlags(&ring->ev_[i], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&ring->mev_[i], hipEventDisableTiming) != hipSuccess)
                return give_up(SHMR_EC_DEVICE_ERROR);
        void* hd = nullptr;
        ring->host_unified_ = hipHostGetDevicePointer(&hd, ring->host_, 0) == hipSuccess && hd == ring->host_;
        if (!ring->host_unified_) (void)hipGetLastError();
        r = ring;
        count_device(dev, kDevUploadRings);
    }
    *rc = SHMR_EC_OK;
    return r;
}

int UploadRing::acquire(uint8_t** host, uint8_t** dev, int* slot) {
    std::unique_lock<std::mutex> lock(mu_);
    for (;;) {
        // r06: a free slot whose last reader has finished, if there is one --
        // never wait behind a reader held up on some stream while other slots
        // are ready (a caller stream held by a host-released wait)
        int ready = -1, any = -1;
        for (int n = 0; n < kSlots && ready < 0; ++n) {
            const int i = (next_ + n) % kSlots;
            if (inuse_[i]) continue;
            if (any < 0) any = i;
            if (!armed_[i]) {
                ready = i;
            } else {
                const hipError_t q = hipEventQuery(mev_[i]);
                if (q == hipSuccess) {
                    armed_[i] = false;
                    ready = i;
                } else if (q == hipErrorNotReady) {
                    (void)hipGetLastError();
                } else {
                    (void)hipGetLastError();
                    ready = i;   // (an error surfaces below, on the slot's own wait)
                }
            }
        }
        for (int i = ready >= 0 ? ready : any; i >= 0;) {
            inuse_[i] = true;
            next_ = (i + 1) % kSlots;
            const bool armed = armed_[i];
            lock.unlock();
            if (armed) {
                hipError_t q = hipEventQuery(mev_[i]);
                if (q == hipErrorNotReady) {   // the slot's last reader is still queued
                    (void)hipGetLastError();
                    count_device(dev_id_, kDevBlockingCalls);
                    q = hipEventSynchronize(mev_[i]);
                }
                if (q != hipSuccess) {
                    (void)hipGetLastError();
                    release_now(i);
                    return SHMR_EC_DEVICE_ERROR;
                }
            }
            *host = host_ + size_t(i) * kSlotBytes;
            *dev = dev_ + size_t(i) * kSlotBytes;
            *slot = i;
            return SHMR_EC_OK;
        }
        cv_.wait(lock);
    }
}

int UploadRing::upload(int slot, size_t bytes, hipStream_t stream) {
    const size_t off = size_t(slot) * kSlotBytes;
    return hipMemcpyAsync(dev_ + off, host_ + off, bytes, hipMemcpyHostToDevice, stream) == hipSuccess
               ? SHMR_EC_OK
               : SHMR_EC_DEVICE_ERROR;
}

int UploadRing::release_after(int slot, hipStream_t stream) {
    const bool ok = record_mirrored(dev_id_, stream, ev_[slot], mev_[slot]) == SHMR_EC_OK;
    std::lock_guard<std::mutex> lock(mu_);
    armed_[slot] = ok;
    inuse_[slot] = false;
    cv_.notify_one();
    return ok ? SHMR_EC_OK : SHMR_EC_DEVICE_ERROR;
}

void UploadRing::release_now(int slot) {
    std::lock_guard<std::mutex> lock(mu_);
    inuse_[slot] = false;
    cv_.notify_one();
}

// ===========================================================================
// Shard-pointer table cache
// ===========================================================================
PtrTableCache* PtrTableCache::for_device(int dev, int* rc) {
    static std::mutex mu;
    static auto* caches = new std::map<int, PtrTableCache*>;   // leaked: in-flight kernels read the entries
    std::lock_guard<std::mutex> lock(mu);
    auto& c = (*caches)[dev];
    if (!c) {
        c = new PtrTableCache;
        c->dev_id_ = dev;
    }
    *rc = SHMR_EC_OK;
    return c;
}

namespace {
uint64_t fnv1a64(const void* p, size_t bytes) {
    const uint8_t* b = static_cast<const uint8_t*>(p);
    uint64_t h = 1469598103934665603ull;
    size_t i = 0;
    for (; i + 8 <= bytes; i += 8) {
        uint64_t w;
        std::memcpy(&w, b + i, 8);
        h = (h ^ w) * 1099511628211ull;
    }
    for (; i < bytes; ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}

bool event_done(hipEvent_t e) {
    const hipError_t q = hipEventQuery(e);
    if (q == hipSuccess) return true;
    (void)hipGetLastError();
    return false;
}
}  // namespace

int PtrTableCache::lookup(const void* tab, size_t bytes, hipStream_t stream, const uint8_t** d_tab, int* entry) {
    *d_tab = nullptr;
    *entry = -1;
    if (bytes > UploadRing::kSlotBytes) return SHMR_EC_OK;
    const uint64_t h = fnv1a64(tab, bytes);
    std::lock_guard<std::mutex> lock(mu_);
    for (int i = 0; i < kEntries; ++i) {
        Entry& e = e_[i];
        if (e.valid && e.stream == stream && e.bytes == bytes && e.hash == h && std::memcmp(e.host, tab, bytes) == 0) {
            // (a stream handle reused after its stream was destroyed: wait on the device).
            // The upload's own event, not its mirror: it was recorded on this
            // stream, which is not capturing (the cache serves no captured call),
            // and the mirror may queue behind other streams' events.
            if (!event_done(e.up) && hipStreamWaitEvent(stream, e.up, 0) != hipSuccess) {
                (void)hipGetLastError();
                return SHMR_EC_DEVICE_ERROR;
            }
            ++e.busy;
            e.tick = ++tick_;
            count_device(dev_id_, kDevPtrTableHits);
            *d_tab = e.dev;
            *entry = i;
            return SHMR_EC_OK;
        }
    }
    // miss: a never-used entry, else the least recently used free one whose
    // pinned copy the last upload has left and whose readers on another
    // stream are done
    int victim = -1;
    for (int i = 0; i < kEntries && victim < 0; ++i)
        if (!e_[i].host) victim = i;
    if (victim < 0) {
        for (int i = 0; i < kEntries; ++i) {
            Entry& e = e_[i];
            // (readers on the same stream included: a destroyed stream's handle
            // may come back for a new stream while its kernels still run)
            // (an entry of this stream -- not capturing -- may use its own events)
            const bool mine = e.stream == stream;
            if (e.busy || !event_done(mine ? e.up : e.mup)) continue;
            if (e.used_armed && !event_done(mine ? e.used : e.mused)) continue;
            if (victim < 0 || e.tick < e_[victim].tick) victim = i;
        }
    }
    if (victim < 0) return SHMR_EC_OK;   // every entry busy: the caller uses the upload ring
    Entry& e = e_[victim];
    if (!e.host) {
        // (no arena memory or events for a new entry: the caller takes the upload ring)
        uint8_t *hblk = nullptr, *dblk = nullptr;
        if (arena_alloc(dev_id_, UploadRing::kSlotBytes, false, &hblk, &dblk) != SHMR_EC_OK) return SHMR_EC_OK;
        RelaxedCapture relaxed;
        if (hipEventCreateWithFlags(&e.up, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&e.used, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&e.mup, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&e.mused, hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            return SHMR_EC_OK;   // the arena block is abandoned (permanent memory)
        }
        e.host = hblk;
        e.dev = dblk;
    }
    e.valid = false;
    std::memcpy(e.host, tab, bytes);
    if (hipMemcpyAsync(e.dev, e.host, bytes, hipMemcpyHostToDevice, stream) != hipSuccess) {
        (void)hipGetLastError();
        return SHMR_EC_DEVICE_ERROR;
    }
    if (record_mirrored(dev_id_, stream, e.up, e.mup) != SHMR_EC_OK) return SHMR_EC_DEVICE_ERROR;
    e.bytes = bytes;
    e.hash = h;
    e.stream = stream;
    e.valid = true;
    e.used_armed = false;
    ++e.busy;
    e.tick = ++tick_;
    *d_tab = e.dev;
    *entry = victim;
    return SHMR_EC_OK;
}

int PtrTableCache::release_after(int entry, hipStream_t stream) {
    std::lock_guard<std::mutex> lock(mu_);
    Entry& e = e_[entry];
    --e.busy;
    if (record_mirrored(dev_id_, stream, e.used, e.mused) != SHMR_EC_OK) {
        e.valid = false;
        return SHMR_EC_DEVICE_ERROR;
    }
    e.used_armed = true;
    return SHMR_EC_OK;
}

// ===========================================================================
// Staging pool
// ===========================================================================
StagingPool& StagingPool::get() {
    static StagingPool* p = new StagingPool;   // leaked: outlives static teardown
    return *p;
}

Staging* StagingPool::acquire(int dev, size_t bytes, int* rc) {
    Staging* s = nullptr;
    {
        std::lock_guard<std::mutex> lock(mu_);
        auto& lst = free_[dev];
        if (!lst.empty()) {
            s = lst.back();
            lst.pop_back();
        }
    }
    RelaxedCapture relaxed;
    if (!s) {
        s = new Staging;
        s->dev = dev;
        // (greatest priority like the library's other streams: a stream of
        // its own among the hardware queues, not one a held caller stream may
        // share -- r06 s33, tests/test_gpu_hol.py)
        DeviceScope scope(dev);
        if (!scope.ok() || create_priority_stream(&s->stream) != hipSuccess) {
            (void)hipGetLastError();
            delete s;
            *rc = SHMR_EC_DEVICE_ERROR;
            return nullptr;
        }
        register_own_stream(s->stream);
        count_device(dev, kDevStagingStreams);
    }
    if (s->cap < bytes) {
        DeviceScope scope(dev);
        if (!scope.ok() || grow_scratch(&s->dbuf, &s->cap, bytes, false) != hipSuccess) {
            (void)hipGetLastError();
            release(s);
            *rc = SHMR_EC_OUT_OF_MEMORY;
            return nullptr;
        }
    }
    *rc = SHMR_EC_OK;
    return s;
}

void StagingPool::release(Staging* s) {
    std::lock_guard<std::mutex> lock(mu_);
    free_[s->dev].push_back(s);
}

}  // namespace core
}  // namespace shmr
