// C ABI of the MI355X erasure path (include/shmr_ec.h).
//
// Validation in the crate's order, then device work through ec_core (device
// batches) or host_engine (host-buffer batches).  There is deliberately no
// CPU compute path: without a GPU every compute entry point fails with
// SHMR_EC_NO_DEVICE.
#include "shmr_ec.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <vector>

#include "ec_core.hpp"
#include "host_engine.hpp"
#include "submit.hpp"

using shmr::core::Codec;
using shmr::core::Plan;
namespace core = shmr::core;

namespace {
// No C++ exception (allocation failure, thread or stream creation) crosses the
// C ABI: it becomes a status code, so a Rust/C caller never sees an abort.
// Every entry point runs under the relaxed capture mode (core::RelaxedCapture).
template <class F>
int guarded(F&& f) noexcept {
    try {
        core::RelaxedCapture relaxed;
        return f();
    } catch (const std::bad_alloc&) {
        return SHMR_EC_OUT_OF_MEMORY;
    } catch (...) {
        return SHMR_EC_DEVICE_ERROR;
    }
}
// The submission queue's per-block entry points make no HIP call in the
// caller's thread except through the queue (whose launches, watcher and
// creation enter the relaxed mode themselves): no mode switch per call -- two
// runtime calls per block that the 16-thread per-block shape pays in
// contention (r06, tools/perblock_dev.cpp).
template <class F>
int guarded_light(F&& f) noexcept {
    try {
        return f();
    } catch (const std::bad_alloc&) {
        return SHMR_EC_OUT_OF_MEMORY;
    } catch (...) {
        return SHMR_EC_DEVICE_ERROR;
    }
}
// Slabs handed out by shmr_ec_device_alloc_shards (base -> device; `freeing`
// while a shmr_ec_device_free_shards of it runs: one of two racing frees wins,
// and a failed free leaves the entry, so the slab can still be freed).
struct SlabEntry {
    int device;
    bool freeing;
};
std::mutex g_slab_mu;
std::map<uintptr_t, SlabEntry> g_slabs;
}  // namespace

extern "C" {

const char* shmr_ec_status_name(int st) {
    switch (st) {
        case SHMR_EC_OK: return "Ok";
        case SHMR_EC_TOO_FEW_SHARDS: return "TooFewShards";
        case SHMR_EC_TOO_MANY_SHARDS: return "TooManyShards";
        case SHMR_EC_TOO_FEW_DATA_SHARDS: return "TooFewDataShards";
        case SHMR_EC_TOO_MANY_DATA_SHARDS: return "TooManyDataShards";
        case SHMR_EC_TOO_FEW_PARITY_SHARDS: return "TooFewParityShards";
        case SHMR_EC_TOO_MANY_PARITY_SHARDS: return "TooManyParityShards";
        case SHMR_EC_TOO_FEW_BUFFER_SHARDS: return "TooFewBufferShards";
        case SHMR_EC_TOO_MANY_BUFFER_SHARDS: return "TooManyBufferShards";
        case SHMR_EC_INCORRECT_SHARD_SIZE: return "IncorrectShardSize";
        case SHMR_EC_TOO_FEW_SHARDS_PRESENT: return "TooFewShardsPresent";
        case SHMR_EC_EMPTY_SHARD: return "EmptyShard";
        case SHMR_EC_INVALID_SHARD_FLAGS: return "InvalidShardFlags";
        case SHMR_EC_INVALID_INDEX: return "InvalidIndex";
        case SHMR_EC_INVALID_ARGUMENT: return "InvalidArgument";
        case SHMR_EC_NO_DEVICE: return "NoDevice";
        case SHMR_EC_DEVICE_ERROR: return "DeviceError";
        case SHMR_EC_OUT_OF_MEMORY: return "OutOfMemory";
        default: return "Unknown";
    }
}

#ifndef SHMR_EC_KERNEL_ID
#define SHMR_EC_KERNEL_ID "unknown"
#endif
#ifdef SHMR_EC_TOOLS
#define SHMR_EC_FLAVOUR "tools"
#else
#define SHMR_EC_FLAVOUR "product"
#endif

const char* shmr_ec_version(void) { return "shmr_ec 0.3.0 (gfx950, " SHMR_EC_FLAVOUR ")"; }

const char* shmr_ec_build_id(void) { return SHMR_EC_KERNEL_ID; }

int shmr_ec_is_tools_build(void) {
#ifdef SHMR_EC_TOOLS
    return 1;
#else
    return 0;
#endif
}

size_t shmr_ec_shard_size(uint64_t length, uint32_t data_shards) {
    if (data_shards == 0) return 0;
    // Rust: (length as f32 / data_shards as f32).ceil() as usize
    const float q = static_cast<float>(length) / static_cast<float>(data_shards);
    const float c = std::ceil(q);
    if (!(c > 0.0f)) return 0;
    if (c >= 18446744073709551615.0f) return SIZE_MAX;
    return static_cast<size_t>(c);
}

int shmr_ec_new(uint32_t data_shards, uint32_t parity_shards, shmr_ec_t** out) {
    if (!out) return SHMR_EC_INVALID_ARGUMENT;
    *out = nullptr;
    if (data_shards == 0) return SHMR_EC_TOO_FEW_DATA_SHARDS;
    if (parity_shards == 0) return SHMR_EC_TOO_FEW_PARITY_SHARDS;
    if (uint64_t(data_shards) + parity_shards > 256) return SHMR_EC_TOO_MANY_SHARDS;
    try {
        auto* rs = new shmr_ec;
        rs->codec = shmr::gf::get_codec(data_shards, parity_shards);
        *out = rs;
    } catch (...) {
        return SHMR_EC_OUT_OF_MEMORY;
    }
    return SHMR_EC_OK;
}

void shmr_ec_free(shmr_ec_t* rs) { delete rs; }

uint32_t shmr_ec_data_shard_count(const shmr_ec_t* rs) { return rs ? rs->codec->k() : 0; }
uint32_t shmr_ec_parity_shard_count(const shmr_ec_t* rs) { return rs ? rs->codec->p() : 0; }
uint32_t shmr_ec_total_shard_count(const shmr_ec_t* rs) { return rs ? rs->codec->k() + rs->codec->p() : 0; }

int shmr_ec_matrix(const shmr_ec_t* rs, uint8_t* out, size_t out_len) {
    if (!rs || !out) return SHMR_EC_INVALID_ARGUMENT;
    const auto& m = rs->codec->matrix();
    if (out_len < m.d.size()) return SHMR_EC_INVALID_ARGUMENT;
    std::memcpy(out, m.d.data(), m.d.size());
    return SHMR_EC_OK;
}

int shmr_ec_reconstruct_plan(shmr_ec_t* rs, const uint8_t* present, size_t nshards, int data_only,
                             uint16_t* in_idx, uint16_t* out_idx, uint8_t* out_rows, size_t out_rows_len,
                             uint32_t* n_out) {
    return guarded([&]() -> int {
        if (!rs || !present || !in_idx || !out_idx || !out_rows || !n_out) return SHMR_EC_INVALID_ARGUMENT;
        const unsigned k = rs->codec->k(), t = k + rs->codec->p();
        if (nshards < t) return SHMR_EC_TOO_FEW_SHARDS;
        if (nshards > t) return SHMR_EC_TOO_MANY_SHARDS;
        unsigned np = 0;
        for (unsigned i = 0; i < t; ++i) np += present[i] ? 1 : 0;
        if (np == t) {
            *n_out = 0;
            return SHMR_EC_OK;
        }
        if (np < k) return SHMR_EC_TOO_FEW_SHARDS_PRESENT;
        std::vector<uint8_t> pr(present, present + t);
        auto plan = rs->codec->reconstruct_plan(pr, data_only != 0);
        if (out_rows_len < size_t(plan->m) * k) return SHMR_EC_INVALID_ARGUMENT;
        std::memcpy(in_idx, plan->in_idx.data(), 2 * size_t(k));
        std::memcpy(out_idx, plan->out_idx.data(), 2 * size_t(plan->m));
        std::memcpy(out_rows, plan->rows.d.data(), size_t(plan->m) * k);
        *n_out = plan->m;
        return SHMR_EC_OK;
    });
}

int shmr_ec_set_device(shmr_ec_t* rs, int device) {
    if (!rs || device < 0) return SHMR_EC_INVALID_ARGUMENT;
    rs->device = device;
    return SHMR_EC_OK;
}

int shmr_ec_set_tuning(const char* key, int value) {
    return guarded([&]() -> int {
        if (!key) return SHMR_EC_INVALID_ARGUMENT;
        bool known = false;
        const int rc = core::set_submit_tuning(key, value, &known);
        return known ? rc : core::set_tuning(key, value);
    });
}
int shmr_ec_get_tuning(const char* key) {
    return guarded([&]() -> int {
        if (!key) return SHMR_EC_INVALID_ARGUMENT;
        bool known = false;
        const int v = core::get_submit_tuning(key, &known);
        return known ? v : core::get_tuning(key);
    });
}

int shmr_ec_queue_stats(int device, uint64_t* out, size_t n) {
    if (!out || device < 0) return SHMR_EC_INVALID_ARGUMENT;
    core::submit_stats(device, out, n);
    return SHMR_EC_OK;
}

int shmr_ec_describe_variant(int decode, uint32_t data_shards, uint32_t rows, char* buf, size_t len) {
    if (!buf || len == 0 || rows == 0) return SHMR_EC_INVALID_ARGUMENT;
    if (decode < 0 || decode > 4) return SHMR_EC_INVALID_ARGUMENT;
    const core::OpClass op = (decode == 1 || decode == 2 || decode == 4) ? core::kDecode : core::kEncode;
    const uint32_t r = std::min<uint32_t>(rows, shmr::kern::kMaxRowsPerLaunch);
    // 3 / 4: encode / reconstruct over device shard-pointer tables (aligned
    // shards); the variant of a shard length with a partial last tile
    const shmr::kern::LaunchShape s =
        core::shape_of(op, data_shards, r, false, decode >= 3, false, decode == 2, true, true);
    const auto v = core::select_variant(op, s);
    auto lean = v;   // the full-tile kernel without fused tails must always exist
    lean.fuse_tail = false;
    const bool compiled = shmr::kern::variant_compiled(lean, r) && (!v.fuse_tail || shmr::kern::variant_compiled(v, r));
    std::snprintf(buf, len,
                  "chunks=%d nt_load=%d nt_store=%d occ8=%d threads=%d grid=%d diag=%d depth=%d "
                  "wgs_per_cu=%d occ=%d early=%d spre=%d fuse_tail=%d compiled=%d",
                  v.u, int(v.nt_load), int(v.nt_store), int(v.occ8), v.threads,
                  core::grid_mode(op), int(v.diag), v.depth, v.wgs_per_cu, v.occ, int(v.early), int(v.spre), int(v.fuse_tail),
                  int(compiled));
    // appended only when set: records keyed by the string stay valid
    for (const auto& kv : {std::make_pair(v.glds, " glds=1"), std::make_pair(v.serial, " serial=1"),
                           std::make_pair(v.sc1_store, " sc1_store=1"), std::make_pair(v.realign, " realign=1"),
                           std::make_pair(v.peel, " peel=1"), std::make_pair(v.wave_run, " wave_run=1"),
                           std::make_pair(v.st_align, " st_align=1"), std::make_pair(v.xcd, " xcd=1"), std::make_pair(v.pair, " pair=1")}) {
        const size_t n = std::strlen(buf);
        if (kv.first && n + 1 < len) std::snprintf(buf + n, len - n, "%s", kv.second);
    }
    return SHMR_EC_OK;
}

size_t shmr_ec_kernel_inventory(shmr_ec_kernel_info* out, size_t cap) {
    static_assert(sizeof(shmr_ec_kernel_info) == sizeof(shmr::kern::KernelInfo), "kernel info layout");
    return shmr::kern::kernel_inventory(reinterpret_cast<shmr::kern::KernelInfo*>(out), out ? cap : 0);
}

int shmr_ec_cache_stats(const shmr_ec_t* rs, uint64_t* hits, uint64_t* misses) {
    if (!rs) return SHMR_EC_INVALID_ARGUMENT;
    if (hits) *hits = rs->codec->decode_cache_hits();
    if (misses) *misses = rs->codec->decode_cache_misses();
    return SHMR_EC_OK;
}

int shmr_ec_device_count(void) { return core::device_count(); }

int shmr_ec_device_init(int device) {
    return guarded([&]() -> int {
        const int rc = core::check_device(device);
        if (rc) return rc;
        return core::device_init(device, nullptr);
    });
}

int shmr_ec_capture_reserve(int device, size_t bytes) {
    return guarded([&]() -> int {
        const int rc = core::check_device(device);
        if (rc) return rc;
        return core::capture_reserve(device, bytes);
    });
}

int shmr_ec_device_stats(int device, uint64_t* out, size_t n) {
    if (!out || device < 0) return SHMR_EC_INVALID_ARGUMENT;
    core::device_stats(device, out, n);
    return SHMR_EC_OK;
}

int shmr_ec_path_stats(uint64_t* zero_copy_blocks, uint64_t* staged_blocks) {
    core::path_stats(zero_copy_blocks, staged_blocks);
    return SHMR_EC_OK;
}

// ---- device memory for batches -------------------------------------------------
int shmr_ec_device_alloc(int device, size_t bytes, int contiguous, void** out) {
    return guarded([&]() -> int {
        if (!out) return SHMR_EC_INVALID_ARGUMENT;
        *out = nullptr;
        int rc = core::check_device(device);
        if (rc) return rc;
        hipError_t e;
        {
            core::DeviceScope scope(device);
            if (!scope.ok()) return SHMR_EC_DEVICE_ERROR;
            const size_t n = bytes ? bytes : 1;
            core::RelaxedCapture relaxed;
            e = contiguous ? hipExtMallocWithFlags(out, n, hipDeviceMallocContiguous) : hipMalloc(out, n);
        }
        if (e != hipSuccess) {
            (void)hipGetLastError();
            *out = nullptr;
            return SHMR_EC_OUT_OF_MEMORY;
        }
        return SHMR_EC_OK;
    });
}

int shmr_ec_device_free(int device, void* p) {
    return guarded([&]() -> int {
        if (!p) return SHMR_EC_OK;
        int rc = core::check_device(device);
        if (rc) return rc;
        // A slab freed this way leaves no registry entry for a later allocation
        // at the same address to inherit: dropped now (the address is still
        // ours) -- unless free_shards is freeing it, which keeps the entry until
        // the memory is gone, so a failed free can be retried.
        {
            std::lock_guard<std::mutex> lk(g_slab_mu);
            auto it = g_slabs.find(uintptr_t(p));
            if (it != g_slabs.end() && it->second.device == device && !it->second.freeing) g_slabs.erase(it);
        }
        {
            core::DeviceScope scope(device);
            if (!scope.ok()) return SHMR_EC_DEVICE_ERROR;
            core::RelaxedCapture relaxed;
            if (hipFree(p) != hipSuccess) {
                (void)hipGetLastError();
                return SHMR_EC_DEVICE_ERROR;
            }
        }
        std::lock_guard<std::mutex> lk(g_slab_mu);
        auto it = g_slabs.find(uintptr_t(p));   // (an entry a new slab at this address made is not ours)
        if (it != g_slabs.end() && it->second.device == device && it->second.freeing) g_slabs.erase(it);
        return SHMR_EC_OK;
    });
}

// ---- shard buffers in slot placement (pointer-table calls) ----------------------
int shmr_ec_device_alloc_shards(int device, size_t nblocks, size_t shards_per_block, size_t shard_len,
                                uint8_t** out_ptrs) {
    return guarded([&]() -> int {
        if (!out_ptrs || nblocks == 0 || shards_per_block == 0 || shard_len == 0) return SHMR_EC_INVALID_ARGUMENT;
        const uint64_t n = uint64_t(nblocks) * shards_per_block;
        if (n / nblocks != shards_per_block) return SHMR_EC_INVALID_ARGUMENT;
        // page-aligned slots, one page more for a
        // power-of-two stride (the bench layout's placement)
        uint64_t pitch = core::round_up(shard_len, 4096);
        if (pitch % 65536 == 0) pitch += 4096;
        if (pitch < shard_len || n > UINT64_MAX / pitch) return SHMR_EC_INVALID_ARGUMENT;
        void* slab = nullptr;
        const int rc = shmr_ec_device_alloc(device, size_t(n * pitch), 0, &slab);
        if (rc) return rc;
        try {
            std::lock_guard<std::mutex> lk(g_slab_mu);
            g_slabs[uintptr_t(slab)] = SlabEntry{device, false};
        } catch (...) {
            (void)shmr_ec_device_free(device, slab);
            throw;
        }
        uint8_t* base = static_cast<uint8_t*>(slab);
        for (uint64_t j = 0; j < n; ++j) out_ptrs[j] = base + j * pitch;
        return SHMR_EC_OK;
    });
}

int shmr_ec_device_free_shards(int device, uint8_t* first) {
    return guarded([&]() -> int {
        if (!first) return SHMR_EC_OK;
        {
            std::lock_guard<std::mutex> lk(g_slab_mu);
            auto it = g_slabs.find(uintptr_t(first));
            if (it == g_slabs.end() || it->second.device != device || it->second.freeing)
                return SHMR_EC_INVALID_ARGUMENT;
            it->second.freeing = true;   // under the lock: one of two racing frees wins
        }
        const int rc = shmr_ec_device_free(device, first);   // erases the entry once freed
        if (rc) {
            std::lock_guard<std::mutex> lk(g_slab_mu);
            auto it = g_slabs.find(uintptr_t(first));
            if (it != g_slabs.end()) it->second.freeing = false;   // still allocated: freeable again
        }
        return rc;
    });
}

// ---- pinned host memory (Block Cache buffers) --------------------------------
// Mapped + portable: every GPU of the node can address it, so the host-buffer
// entry points run their kernels on it in place (zero-copy).
int shmr_ec_host_alloc(size_t bytes, void** out) {
    return guarded([&]() -> int {
        if (!out) return SHMR_EC_INVALID_ARGUMENT;
        *out = nullptr;
        int rc = core::check_device(0);
        if (rc) return rc;
        const size_t n = bytes ? bytes : 1;
        core::RelaxedCapture relaxed;
        if (hipHostMalloc(out, n, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess) {
            (void)hipGetLastError();
            *out = nullptr;
            return SHMR_EC_OUT_OF_MEMORY;
        }
        void* dev = nullptr;
        if (hipHostGetDevicePointer(&dev, *out, 0) == hipSuccess && dev) {
            try {
                core::mapped_add(*out, n, dev);
            } catch (...) {   // registry allocation failed: hand nothing out
                (void)hipHostFree(*out);
                *out = nullptr;
                throw;
            }
        } else {
            (void)hipGetLastError();   // still pinned: the staged DMA path takes it
        }
        return SHMR_EC_OK;
    });
}

void shmr_ec_host_free(void* p) {
    if (!p) return;
    core::mapped_remove(p);
    core::RelaxedCapture relaxed;
    if (hipHostFree(p) != hipSuccess) (void)hipGetLastError();
}

int shmr_ec_host_register(void* p, size_t bytes) {
    return guarded([&]() -> int {
        if (!p || bytes == 0) return SHMR_EC_INVALID_ARGUMENT;
        int rc = core::check_device(0);
        if (rc) return rc;
        core::RelaxedCapture relaxed;
        if (hipHostRegister(p, bytes, hipHostRegisterMapped | hipHostRegisterPortable) != hipSuccess) {
            (void)hipGetLastError();
            return SHMR_EC_DEVICE_ERROR;
        }
        void* dev = nullptr;
        if (hipHostGetDevicePointer(&dev, p, 0) != hipSuccess || !dev) {
            (void)hipGetLastError();
            (void)hipHostUnregister(p);
            return SHMR_EC_DEVICE_ERROR;
        }
        try {
            core::mapped_add(p, bytes, dev);
        } catch (...) {
            (void)hipHostUnregister(p);
            throw;
        }
        return SHMR_EC_OK;
    });
}

int shmr_ec_host_unregister(void* p) {
    return guarded([&]() -> int {
        if (!p || !core::mapped_remove(p)) return SHMR_EC_INVALID_ARGUMENT;
        core::RelaxedCapture relaxed;
        if (hipHostUnregister(p) == hipSuccess) return SHMR_EC_OK;
        (void)hipGetLastError();
        return SHMR_EC_DEVICE_ERROR;
    });
}

}  // extern "C"

// ---- validation in the crate's order (shared by host and device forms) -------------
namespace {
// ReedSolomon::encode: check_piece_count!(all), then check_slices!(multi).
int check_encode(shmr_ec_t* rs, uint8_t* const* shards, const size_t* shard_lens, size_t nshards, size_t* len) {
    if (!rs || !shards || !shard_lens) return SHMR_EC_INVALID_ARGUMENT;
    const unsigned t = rs->codec->k() + rs->codec->p();
    if (nshards < t) return SHMR_EC_TOO_FEW_SHARDS;
    if (nshards > t) return SHMR_EC_TOO_MANY_SHARDS;
    *len = shard_lens[0];
    if (*len == 0) return SHMR_EC_EMPTY_SHARD;
    for (unsigned i = 0; i < t; ++i)
        if (shard_lens[i] != *len) return SHMR_EC_INCORRECT_SHARD_SIZE;
    for (unsigned i = 0; i < t; ++i)
        if (!shards[i]) return SHMR_EC_INVALID_ARGUMENT;
    return SHMR_EC_OK;
}

// ReedSolomon::reconstruct{,_data}: per present shard len 0 -> EmptyShard,
// mismatch -> IncorrectShardSize, in index order; then the presence count.
// *plan = nullptr: every shard present (the crate returns Ok without work).
int check_reconstruct(shmr_ec_t* rs, uint8_t* const* shards, const size_t* shard_lens, const uint8_t* present,
                      size_t nshards, int data_only, size_t* len, std::shared_ptr<Plan>* plan) {
    if (!rs || !shards || !shard_lens || !present) return SHMR_EC_INVALID_ARGUMENT;
    Codec& c = *rs->codec;
    const unsigned k = c.k(), t = k + c.p();
    if (nshards < t) return SHMR_EC_TOO_FEW_SHARDS;
    if (nshards > t) return SHMR_EC_TOO_MANY_SHARDS;
    unsigned np = 0;
    bool have_len = false;
    *len = 0;
    for (unsigned i = 0; i < t; ++i) {
        if (!present[i]) continue;
        if (shard_lens[i] == 0) return SHMR_EC_EMPTY_SHARD;
        ++np;
        if (have_len && shard_lens[i] != *len) return SHMR_EC_INCORRECT_SHARD_SIZE;
        *len = shard_lens[i];
        have_len = true;
    }
    plan->reset();
    if (np == t) return SHMR_EC_OK;
    if (np < k) return SHMR_EC_TOO_FEW_SHARDS_PRESENT;
    std::vector<uint8_t> pr(present, present + t);
    auto pl = c.reconstruct_plan(pr, data_only != 0);
    for (unsigned m = 0; m < pl->m; ++m)
        if (!shards[pl->out_idx[m]]) return SHMR_EC_INVALID_ARGUMENT;
    for (unsigned i = 0; i < k; ++i)
        if (!shards[pl->in_idx[i]]) return SHMR_EC_INVALID_ARGUMENT;
    if (pl->m) *plan = pl;
    return SHMR_EC_OK;
}

// A queue request for one validated block (row: device addresses, shard
// index order, 0 where the call touches nothing).
std::unique_ptr<core::SubmitReq> make_req(shmr_ec_t* rs, core::OpClass op, bool data_only, bool host_mapped,
                                          size_t len, int dev, std::vector<uint64_t> row, const uint8_t* present) {
    std::unique_ptr<core::SubmitReq> r(new core::SubmitReq);
    r->codec = rs->codec.get();
    r->op = op;
    r->data_only = data_only;
    r->host_mapped = host_mapped;
    r->len = len;
    r->dev = dev;
    r->set_row(row.data(), present, unsigned(row.size()));   // (after len and host_mapped: its time estimate)
    return r;
}

// Submits r; with `queued` (a *_start call) hands it over pending, else waits.
int run_req(std::unique_ptr<core::SubmitReq> r, core::SubmitReq** queued) {
    const int rc = core::submit(r.get());
    if (rc) return rc;
    if (queued) {
        *queued = r.release();
        return SHMR_EC_OK;
    }
    return core::wait(r.get());
}
}  // namespace

extern "C" {

// ---- host-buffer encode (ReedSolomon::encode) --------------------------------------
// async != nullptr (shmr_ec_encode_start): shards in mapped memory are coded by
// kernels left running (a pooled stream in *async, or -- through the
// submission queue, knob "coalesce" -- a request in *queued); every other path
// finishes here.
static int encode_impl(shmr_ec_t* rs, uint8_t* const* shards, const size_t* shard_lens, size_t nshards,
                       core::Staging** async, core::SubmitReq** queued) {
    return guarded([&]() -> int {
        size_t len = 0;
        int rc = check_encode(rs, shards, shard_lens, nshards, &len);
        if (rc) return rc;
        Codec& c = *rs->codec;
        const unsigned k = c.k(), p = c.p(), t = k + p;
        const int dev = rs->device;
        rc = core::check_device(dev);
        if (rc) return rc;
        if (core::coalesce_host()) {   // mapped shards: merged with concurrent calls, coded in place
            const core::HostJob job{c, core::kEncode, false, shards, nullptr, 1, len, 0, 1};
            std::vector<uint64_t> row;
            if (core::map_rows(job, &row)) {
                core::count_blocks(true, 1);
                return run_req(make_req(rs, core::kEncode, false, true, len, dev, std::move(row), nullptr),
                               async ? queued : nullptr);
            }
        }
        {   // shards in mapped memory: the kernel encodes them in place (zero-copy)
            const core::HostJob job{c, core::kEncode, false, shards, nullptr, 1, len, 0, 1};
            bool handled = false;
            rc = core::run_mapped_job(job, &dev, 1, &handled, true, async);
            if (handled || rc) return rc;
        }
        if (uint64_t(t) * len <= core::bounce_limit()) {   // pageable, small: one bounce, one launch
            const core::HostJob job{c, core::kEncode, false, shards, nullptr, 1, len, 0, 1};
            return core::run_bounced_job(job, dev);
        }
        core::count_blocks(false, 1);
        core::DeviceScope scope(dev);
        if (!scope.ok()) return SHMR_EC_DEVICE_ERROR;
        const uint64_t pitch = core::round_up(len, 256);
        core::StagingLease lease;
        lease.s = core::StagingPool::get().acquire(dev, pitch * t, &rc);
        if (!lease.s) return rc;
        core::Staging& s = *lease.s;
        for (unsigned i = 0; i < k; ++i)
            SHMR_HIP_TRY(hipMemcpyAsync(s.dbuf + i * pitch, shards[i], len, hipMemcpyHostToDevice, s.stream));
        const core::Layout L{s.dbuf, s.dbuf, 0, pitch, 0, pitch, 0};
        rc = core::encode_on_device(c, dev, L, 1, len, s.stream);
        if (rc) return rc;
        for (unsigned r = 0; r < p; ++r)
            SHMR_HIP_TRY(hipMemcpyAsync(shards[k + r], s.dbuf + (k + r) * pitch, len, hipMemcpyDeviceToHost, s.stream));
        SHMR_HIP_TRY(core::sync_stream(s.stream));
        return SHMR_EC_OK;
    });
}

// ---- host-buffer reconstruct (ReedSolomon::reconstruct{,_data}) ---------------------
static int reconstruct_impl(shmr_ec_t* rs, uint8_t* const* shards, const size_t* shard_lens, const uint8_t* present,
                            size_t nshards, int data_only, core::Staging** async, core::SubmitReq** queued) {
    return guarded([&]() -> int {
        size_t len = 0;
        std::shared_ptr<Plan> plan;
        int rc = check_reconstruct(rs, shards, shard_lens, present, nshards, data_only, &len, &plan);
        if (rc || !plan) return rc;
        Codec& c = *rs->codec;
        const unsigned k = c.k(), t = k + c.p();
        const int dev = rs->device;
        rc = core::check_device(dev);
        if (rc) return rc;
        if (core::coalesce_host()) {   // mapped shards: merged with concurrent calls, rebuilt in place
            const core::HostJob job{c, core::kDecode, data_only != 0, shards, present, 1, len, 0, 1};
            std::vector<uint64_t> row;
            if (core::map_rows(job, &row)) {
                core::count_blocks(true, 1);
                return run_req(make_req(rs, core::kDecode, data_only != 0, true, len, dev, std::move(row), present),
                               async ? queued : nullptr);
            }
        }
        {   // shards in mapped memory: rebuilt in place by the kernel (zero-copy)
            const core::HostJob job{c, core::kDecode, data_only != 0, shards, present, 1, len, 0, 1};
            bool handled = false;
            rc = core::run_mapped_job(job, &dev, 1, &handled, true, async);
            if (handled || rc) return rc;
        }
        if (uint64_t(t) * len <= core::bounce_limit()) {   // pageable, small: one bounce, one launch
            const core::HostJob job{c, core::kDecode, data_only != 0, shards, present, 1, len, 0, 1};
            return core::run_bounced_job(job, dev);
        }
        core::count_blocks(false, 1);
        core::DeviceScope scope(dev);
        if (!scope.ok()) return SHMR_EC_DEVICE_ERROR;
        const uint64_t pitch = core::round_up(len, 256);
        core::StagingLease lease;
        lease.s = core::StagingPool::get().acquire(dev, pitch * t, &rc);
        if (!lease.s) return rc;
        core::Staging& s = *lease.s;
        for (unsigned i = 0; i < k; ++i) {
            const unsigned idx = plan->in_idx[i];
            SHMR_HIP_TRY(hipMemcpyAsync(s.dbuf + idx * pitch, shards[idx], len, hipMemcpyHostToDevice, s.stream));
        }
        rc = core::reconstruct_on_device(c, dev, s.dbuf, pitch, pitch * t, present, 1, len, data_only != 0, s.stream);
        if (rc) return rc;
        for (unsigned m = 0; m < plan->m; ++m) {
            const unsigned idx = plan->out_idx[m];
            SHMR_HIP_TRY(hipMemcpyAsync(shards[idx], s.dbuf + idx * pitch, len, hipMemcpyDeviceToHost, s.stream));
        }
        SHMR_HIP_TRY(core::sync_stream(s.stream));
        return SHMR_EC_OK;
    });
}

// ---- one block on device buffers, through the submission queue -----------------
// The crate's encode / reconstruct of ONE block (block.rs:427, :560) whose
// shards are device buffers; concurrent calls on the device merge into batch
// launches (submit.hpp).
static int encode_dev_impl(shmr_ec_t* rs, uint8_t* const* d_shards, const size_t* shard_lens, size_t nshards,
                           int device, core::SubmitReq** queued) {
    return guarded_light([&]() -> int {
        size_t len = 0;
        int rc = check_encode(rs, d_shards, shard_lens, nshards, &len);
        if (rc) return rc;
        if ((rc = core::check_device(device))) return rc;
        std::vector<uint64_t> row(nshards);
        for (size_t i = 0; i < nshards; ++i) row[i] = uint64_t(uintptr_t(d_shards[i]));
        return run_req(make_req(rs, core::kEncode, false, false, len, device, std::move(row), nullptr), queued);
    });
}

static int reconstruct_dev_impl(shmr_ec_t* rs, uint8_t* const* d_shards, const size_t* shard_lens,
                                const uint8_t* present, size_t nshards, int data_only, int device,
                                core::SubmitReq** queued) {
    return guarded_light([&]() -> int {
        size_t len = 0;
        std::shared_ptr<Plan> plan;
        int rc = check_reconstruct(rs, d_shards, shard_lens, present, nshards, data_only, &len, &plan);
        if (rc || !plan) return rc;
        if ((rc = core::check_device(device))) return rc;
        std::vector<uint64_t> row(nshards, 0);
        for (unsigned i = 0; i < plan->k; ++i) row[plan->in_idx[i]] = uint64_t(uintptr_t(d_shards[plan->in_idx[i]]));
        for (unsigned m = 0; m < plan->m; ++m) row[plan->out_idx[m]] = uint64_t(uintptr_t(d_shards[plan->out_idx[m]]));
        return run_req(make_req(rs, core::kDecode, data_only != 0, false, len, device, std::move(row), present), queued);
    });
}

int shmr_ec_encode(shmr_ec_t* rs, uint8_t* const* shards, const size_t* shard_lens, size_t nshards) {
    return encode_impl(rs, shards, shard_lens, nshards, nullptr, nullptr);
}

int shmr_ec_reconstruct(shmr_ec_t* rs, uint8_t* const* shards, const size_t* shard_lens, const uint8_t* present,
                        size_t nshards, int data_only) {
    return reconstruct_impl(rs, shards, shard_lens, present, nshards, data_only, nullptr, nullptr);
}

int shmr_ec_encode_dev(shmr_ec_t* rs, uint8_t* const* d_shards, const size_t* shard_lens, size_t nshards,
                       int device) {
    return encode_dev_impl(rs, d_shards, shard_lens, nshards, device, nullptr);
}

int shmr_ec_reconstruct_dev(shmr_ec_t* rs, uint8_t* const* d_shards, const size_t* shard_lens, const uint8_t* present,
                            size_t nshards, int data_only, int device) {
    return reconstruct_dev_impl(rs, d_shards, shard_lens, present, nshards, data_only, device, nullptr);
}

// ---- asynchronous single-block calls -----------------------------------------------
struct shmr_ec_op {
    core::Staging* s = nullptr;     // pending zero-copy kernels' stream, or none
    core::SubmitReq* req = nullptr; // or a request of the submission queue
};

static int start_op(int rc, core::Staging* s, core::SubmitReq* req, shmr_ec_op_t** op) {
    auto drop = [&] {
        if (s) (void)core::finish_async(s);
        if (req) {
            (void)core::wait(req);
            delete req;
        }
    };
    if (rc != SHMR_EC_OK) {
        drop();
        return rc;
    }
    return guarded_light([&]() -> int {
        try {
            *op = new shmr_ec_op;
        } catch (...) {
            drop();
            throw;
        }
        (*op)->s = s;
        (*op)->req = req;
        return SHMR_EC_OK;
    });
}

int shmr_ec_encode_start(shmr_ec_t* rs, uint8_t* const* shards, const size_t* shard_lens, size_t nshards,
                         shmr_ec_op_t** op) {
    if (!op) return SHMR_EC_INVALID_ARGUMENT;
    *op = nullptr;
    core::Staging* s = nullptr;
    core::SubmitReq* q = nullptr;
    const int rc = encode_impl(rs, shards, shard_lens, nshards, &s, &q);
    return start_op(rc, s, q, op);
}

int shmr_ec_reconstruct_start(shmr_ec_t* rs, uint8_t* const* shards, const size_t* shard_lens, const uint8_t* present,
                              size_t nshards, int data_only, shmr_ec_op_t** op) {
    if (!op) return SHMR_EC_INVALID_ARGUMENT;
    *op = nullptr;
    core::Staging* s = nullptr;
    core::SubmitReq* q = nullptr;
    const int rc = reconstruct_impl(rs, shards, shard_lens, present, nshards, data_only, &s, &q);
    return start_op(rc, s, q, op);
}

int shmr_ec_encode_dev_start(shmr_ec_t* rs, uint8_t* const* d_shards, const size_t* shard_lens, size_t nshards,
                             int device, shmr_ec_op_t** op) {
    if (!op) return SHMR_EC_INVALID_ARGUMENT;
    *op = nullptr;
    core::SubmitReq* q = nullptr;
    const int rc = encode_dev_impl(rs, d_shards, shard_lens, nshards, device, &q);
    return start_op(rc, nullptr, q, op);
}

int shmr_ec_reconstruct_dev_start(shmr_ec_t* rs, uint8_t* const* d_shards, const size_t* shard_lens,
                                  const uint8_t* present, size_t nshards, int data_only, int device,
                                  shmr_ec_op_t** op) {
    if (!op) return SHMR_EC_INVALID_ARGUMENT;
    *op = nullptr;
    core::SubmitReq* q = nullptr;
    const int rc = reconstruct_dev_impl(rs, d_shards, shard_lens, present, nshards, data_only, device, &q);
    return start_op(rc, nullptr, q, op);
}

int shmr_ec_op_wait(shmr_ec_op_t* op) {
    if (!op) return SHMR_EC_INVALID_ARGUMENT;
    int rc = SHMR_EC_OK;
    if (op->s) rc = guarded([&] { return core::finish_async(op->s); });
    if (op->req) {
        rc = guarded_light([&] { return core::wait(op->req); });
        delete op->req;
    }
    delete op;
    return rc;
}

// ---- device-resident batches --------------------------------------------------------
int shmr_ec_encode_batch_dev(shmr_ec_t* rs, const uint8_t* d_data, size_t data_shard_pitch, size_t data_block_pitch,
                             uint8_t* d_parity, size_t parity_shard_pitch, size_t parity_block_pitch, size_t nblocks,
                             size_t shard_len, int device, void* stream) {
    return guarded([&]() -> int {
        if (!rs) return SHMR_EC_INVALID_ARGUMENT;
        if (nblocks == 0) return SHMR_EC_OK;
        if (shard_len == 0) return SHMR_EC_EMPTY_SHARD;
        if (!d_data || !d_parity) return SHMR_EC_INVALID_ARGUMENT;
        int rc = core::check_device(device);
        if (rc) return rc;
        core::DeviceScope scope(device);
        if (!scope.ok()) return SHMR_EC_DEVICE_ERROR;
        Codec& c = *rs->codec;
        const core::Layout L{d_data, d_parity, data_block_pitch, data_shard_pitch, parity_block_pitch, parity_shard_pitch,
                             c.k()};
        return core::encode_on_device(c, device, L, nblocks, shard_len, static_cast<hipStream_t>(stream));
    });
}

int shmr_ec_reconstruct_batch_dev(shmr_ec_t* rs, uint8_t* d_shards, size_t shard_pitch, size_t block_pitch,
                                  const uint8_t* present, size_t nblocks, size_t shard_len, int data_only, int device,
                                  void* stream) {
    return guarded([&]() -> int {
        if (!rs || !present) return SHMR_EC_INVALID_ARGUMENT;
        if (nblocks == 0) return SHMR_EC_OK;
        if (shard_len == 0) return SHMR_EC_EMPTY_SHARD;
        if (!d_shards) return SHMR_EC_INVALID_ARGUMENT;
        Codec& c = *rs->codec;
        int rc = core::validate_presence(c, present, nblocks);   // no launch on a bad batch
        if (rc) return rc;
        rc = core::check_device(device);
        if (rc) return rc;
        core::DeviceScope scope(device);
        if (!scope.ok()) return SHMR_EC_DEVICE_ERROR;
        return core::reconstruct_on_device(c, device, d_shards, shard_pitch, block_pitch, present, nblocks, shard_len,
                                           data_only != 0, static_cast<hipStream_t>(stream));
    });
}

int shmr_ec_reconstruct_batch_dev_out(shmr_ec_t* rs, const uint8_t* d_shards, size_t shard_pitch, size_t block_pitch,
                                      const uint8_t* present, size_t nblocks, size_t shard_len, int data_only,
                                      uint8_t* d_out, size_t out_shard_pitch, size_t out_block_pitch, int device,
                                      void* stream) {
    return guarded([&]() -> int {
        if (!rs || !present) return SHMR_EC_INVALID_ARGUMENT;
        if (nblocks == 0) return SHMR_EC_OK;
        if (shard_len == 0) return SHMR_EC_EMPTY_SHARD;
        if (!d_shards || !d_out) return SHMR_EC_INVALID_ARGUMENT;
        Codec& c = *rs->codec;
        int rc = core::validate_presence(c, present, nblocks);   // no launch on a bad batch
        if (rc) return rc;
        rc = core::check_device(device);
        if (rc) return rc;
        core::DeviceScope scope(device);
        if (!scope.ok()) return SHMR_EC_DEVICE_ERROR;
        core::Layout L{d_shards, d_out, block_pitch, shard_pitch, out_block_pitch, out_shard_pitch, 0};
        L.compact = true;
        return core::reconstruct_on_device(c, device, L, present, nblocks, shard_len, data_only != 0,
                                           static_cast<hipStream_t>(stream));
    });
}

// ---- device-resident shards anywhere: shard-pointer tables --------------------------
// The crate's own shape (block.rs:408-427: every shard its own Vec<u8>; :556-565:
// every None shard rebuilt into a fresh buffer) on device memory: validation
// here, dispatch in core::ptrs_launch (a slot lattice -> the strided kernels over
// its slots; else the table, from the device's table cache or uploaded on the
// caller's stream; inside a capture into the capture reserve).
static int ptrs_dev(shmr_ec_t* rs, uint8_t* const* d_shards, const uint8_t* present, size_t nblocks,
                    size_t shard_len, int data_only, int device, void* stream_, core::OpClass op) {
    return guarded([&]() -> int {
        if (!rs || !d_shards) return SHMR_EC_INVALID_ARGUMENT;
        if (op == core::kDecode && !present) return SHMR_EC_INVALID_ARGUMENT;
        if (nblocks == 0) return SHMR_EC_OK;
        if (shard_len == 0) return SHMR_EC_EMPTY_SHARD;
        Codec& c = *rs->codec;
        const unsigned k = c.k(), t = k + c.p();
        int rc = SHMR_EC_OK;
        if (op == core::kDecode && (rc = core::validate_presence(c, present, nblocks))) return rc;
        for (size_t b = 0; b < nblocks; ++b)
            for (unsigned i = 0; i < t; ++i) {
                // absent parity under data_only is neither read nor written
                const bool needed = op == core::kEncode || present[b * t + i] || i < k || !data_only;
                if (needed && !d_shards[b * t + i]) return SHMR_EC_INVALID_ARGUMENT;
            }
        rc = core::check_device(device);
        if (rc) return rc;
        core::DeviceScope scope(device);
        if (!scope.ok()) return SHMR_EC_DEVICE_ERROR;
        static_assert(sizeof(uint8_t*) == sizeof(uint64_t), "64-bit device pointers");
        return core::ptrs_launch(c, reinterpret_cast<const uint64_t*>(d_shards), present, nblocks, shard_len,
                                 data_only != 0, device, static_cast<hipStream_t>(stream_), op, false, true);
    });
}

int shmr_ec_encode_ptrs_dev(shmr_ec_t* rs, uint8_t* const* d_shards, size_t nblocks, size_t shard_len, int device,
                            void* stream) {
    return ptrs_dev(rs, d_shards, nullptr, nblocks, shard_len, 0, device, stream, core::kEncode);
}

int shmr_ec_reconstruct_ptrs_dev(shmr_ec_t* rs, uint8_t* const* d_shards, const uint8_t* present, size_t nblocks,
                                 size_t shard_len, int data_only, int device, void* stream) {
    return ptrs_dev(rs, d_shards, present, nblocks, shard_len, data_only, device, stream, core::kDecode);
}

// ---- host-buffer batches over one or more GPUs -------------------------------------
static int host_batch(shmr_ec_t* rs, uint8_t* const* host_shards, const uint8_t* present, size_t nblocks,
                      size_t shard_len, int data_only, const int* devices, int ndev, core::OpClass op) {
    return guarded([&]() -> int {
        if (!rs || !host_shards || !devices || ndev <= 0) return SHMR_EC_INVALID_ARGUMENT;
        if (op == core::kDecode && !present) return SHMR_EC_INVALID_ARGUMENT;
        if (nblocks == 0) return SHMR_EC_OK;
        if (shard_len == 0) return SHMR_EC_EMPTY_SHARD;
        Codec& c = *rs->codec;
        const unsigned t = c.k() + c.p();
        for (size_t b = 0; b < nblocks; ++b)
            for (unsigned i = 0; i < t; ++i) {
                // absent shards of a decode still need an output buffer (unless
                // they are parity under data_only)
                const bool needed = op == core::kEncode || present[b * t + i] || i < c.k() || !data_only;
                if (needed && !host_shards[b * t + i]) return SHMR_EC_INVALID_ARGUMENT;
            }
        for (int d = 0; d < ndev; ++d) {
            int rc = core::check_device(devices[d]);
            if (rc) return rc;
        }
        core::HostJob job{c, op, data_only != 0, host_shards, present, nblocks, shard_len, 64ull << 20,
                          core::copy_threads_default()};
        return core::run_host_job(job, devices, ndev);
    });
}

int shmr_ec_encode_blocks_host(shmr_ec_t* rs, uint8_t* const* host_shards, size_t nblocks, size_t shard_len,
                               const int* devices, int ndev) {
    return host_batch(rs, host_shards, nullptr, nblocks, shard_len, 0, devices, ndev, core::kEncode);
}

int shmr_ec_reconstruct_blocks_host(shmr_ec_t* rs, uint8_t* const* host_shards, const uint8_t* present,
                                    size_t nblocks, size_t shard_len, int data_only, const int* devices, int ndev) {
    return host_batch(rs, host_shards, present, nblocks, shard_len, data_only, devices, ndev, core::kDecode);
}

}  // extern "C"
