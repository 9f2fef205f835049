// C ABI of the MI355X erasure path (include/shmr_ec.h).
//
// Host-side orchestration only: validation in the crate's order, plan
// selection (gf256.cpp), device staging and kernel launches (gf_apply.hip).
// There is deliberately no CPU compute path here.
#include "shmr_ec.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "gf256.hpp"
#include "gf_apply.hpp"

using shmr::gf::Codec;
using shmr::gf::Plan;

struct shmr_ec {
    std::shared_ptr<Codec> codec;
    std::atomic<int> device{0};
};

namespace {

// Kernel tuning per operation class (encode / reconstruct), process-wide.
// kAuto knobs follow variant_policy(), the fastest variants measured on MI355X
// per launch shape (DESIGN.md "Tuning"); set_tuning() pins a knob explicitly.
constexpr int kAuto = -2;
struct Tuning {
    std::atomic<int> u{kAuto};
    std::atomic<int> nt_load{kAuto};
    std::atomic<int> nt_store{kAuto};
    std::atomic<int> scalar_tabs{0};
    std::atomic<int> occ8{0};
    std::atomic<int> grid{-1};     // -1: one workgroup per tile
    std::atomic<int> diag{0};
    std::atomic<int> threads{256};
};
Tuning g_tune[2];   // [0] encode, [1] reconstruct
enum OpClass { kEncode = 0, kDecode = 1 };

// Measured (tools/tune.py, interleaved A/B in one process, MI355X):
//  encode RS(8,3): NT loads+stores, U=1 (78 %); RS(4,2): NT stores only (77 %
//  vs 72 % with NT loads); RS(10,4) (4 rows per launch): U=2 (71 % vs 66 %);
//  reconstruct: NT loads+stores, U=1.
shmr::kern::Variant variant_policy(OpClass op, unsigned k, unsigned rows) {
    shmr::kern::Variant v;
    v.u = (op == kEncode && rows >= 4) ? 2 : 1;
    v.nt_store = true;
    v.nt_load = op == kDecode || k >= 8;
    return v;
}

shmr::kern::Variant resolve_variant(OpClass op, unsigned k, unsigned rows) {
    const Tuning& T = g_tune[op];
    shmr::kern::Variant v = variant_policy(op, k, rows);
    if (T.u.load() != kAuto) v.u = T.u.load();
    if (T.nt_load.load() != kAuto) v.nt_load = T.nt_load.load() != 0;
    if (T.nt_store.load() != kAuto) v.nt_store = T.nt_store.load() != 0;
    v.scalar_tabs = T.scalar_tabs.load() != 0;
    v.occ8 = T.occ8.load() != 0;
    v.diag = T.diag.load() != 0;
    v.threads = T.threads.load();
    return v;
}

#define HIP_TRY(expr)                                     \
    do {                                                  \
        hipError_t _e = (expr);                           \
        if (_e != hipSuccess) return SHMR_EC_DEVICE_ERROR; \
    } while (0)

int device_count() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// Sets the calling thread's device for the scope, restoring the previous one.
class DeviceScope {
public:
    explicit DeviceScope(int dev) {
        ok_ = hipGetDevice(&prev_) == hipSuccess && hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceScope() {
        if (ok_) (void)hipSetDevice(prev_);
    }
    bool ok() const { return ok_; }

private:
    int prev_ = 0;
    bool ok_ = false;
};

int check_device(int dev) {
    const int n = device_count();
    if (n <= 0) return SHMR_EC_NO_DEVICE;
    if (dev < 0 || dev >= n) return SHMR_EC_INVALID_ARGUMENT;
    return SHMR_EC_OK;
}

// Device image of a plan, uploaded once per device (synchronously, on first
// use) and kept for the codec's lifetime.
int plan_on_device(Plan& plan, int dev, const uint8_t** out, uint32_t* tab_off) {
    size_t hdr = 8 + 2 * size_t(plan.k) + 2 * size_t(plan.m);
    *tab_off = uint32_t((hdr + 31) & ~size_t(31));
    std::lock_guard<std::mutex> lock(plan.dev_mu);
    auto it = plan.dev_image.find(dev);
    if (it != plan.dev_image.end()) {
        *out = static_cast<const uint8_t*>(it->second);
        return SHMR_EC_OK;
    }
    std::vector<uint8_t> img = plan.image();
    void* d = nullptr;
    if (hipMalloc(&d, img.size()) != hipSuccess) return SHMR_EC_OUT_OF_MEMORY;
    if (hipMemcpy(d, img.data(), img.size(), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(d);
        return SHMR_EC_DEVICE_ERROR;
    }
    plan.dev_image[dev] = d;
    *out = static_cast<const uint8_t*>(d);
    return SHMR_EC_OK;
}

struct Layout {
    const uint8_t* in_base;
    uint8_t* out_base;
    uint64_t in_bpitch, in_spitch, out_bpitch, out_spitch;
    uint32_t out_bias;   // subtracted from plan out_idx (encode into a parity-only buffer)
};

bool aligned16(uint64_t v) { return (v & 15u) == 0; }

// Enqueues the plan over blocks {first + j * stride, j < nblk} on the current
// device.  Rows are processed in groups of <= 4 per launch.
// Blocks covered by one launch set: {first + j * stride} or, with d_list, the
// device list d_list[j]; multi-plan sets also carry a per-block plan index into
// the device table d_plans (all plans share k and m).
struct BlockSet {
    uint64_t first = 0, stride = 1, n = 0;
    const uint32_t* d_list = nullptr;
    const uint16_t* d_plan_idx = nullptr;
    const uint8_t* const* d_plans = nullptr;
};

uint32_t plan_tab_off(unsigned k, unsigned m) {
    return uint32_t((8 + 2 * size_t(k) + 2 * size_t(m) + 31) & ~size_t(31));
}

// Enqueues out = rows (x) in for a block set on the current device.  `shape`
// supplies k and m (and the device image for single-plan sets); rows are
// processed in groups of <= 4 per launch.
int launch_set(Plan& shape, int dev, const Layout& L, const BlockSet& bs, uint64_t len, hipStream_t stream,
               OpClass op) {
    const uint64_t nblk = bs.n;
    Plan& plan = shape;
    if (nblk == 0 || plan.m == 0) return SHMR_EC_OK;
    const uint8_t* dplan = nullptr;
    const uint32_t tab_off = plan_tab_off(plan.k, plan.m);
    if (!bs.d_plans) {
        uint32_t off = 0;
        int rc = plan_on_device(plan, dev, &dplan, &off);
        if (rc) return rc;
    }
    const Tuning& T = g_tune[op];
    shmr::kern::Variant tail;   // tail / unaligned launches: U = 1, plain loads
    const int cap = T.grid.load();
    const bool aligned = aligned16(uintptr_t(L.in_base)) && aligned16(uintptr_t(L.out_base)) &&
                         aligned16(L.in_bpitch) && aligned16(L.in_spitch) && aligned16(L.out_bpitch) &&
                         aligned16(L.out_spitch);
    for (uint32_t row0 = 0; row0 < plan.m; row0 += shmr::kern::kMaxRowsPerLaunch) {
        const uint32_t rows = std::min<uint32_t>(shmr::kern::kMaxRowsPerLaunch, plan.m - row0);
        const shmr::kern::Variant var = resolve_variant(op, plan.k, rows);
        const uint64_t tb = shmr::kern::tile_bytes(var.u, var.threads);
        shmr::kern::ApplyArgs a{};
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
        if (!aligned) {
            const uint64_t tb1 = shmr::kern::tile_bytes(1);
            a.col_base = 0;
            a.tiles_per_block = uint32_t((len + tb1 - 1) / tb1);
            a.ntiles = nblk * a.tiles_per_block;
            HIP_TRY(shmr::kern::launch_apply(a, rows, tail, 2, cap, stream));
            continue;
        }
        const uint64_t full = len / tb;
        if (full) {
            a.col_base = 0;
            a.tiles_per_block = uint32_t(full);
            a.ntiles = nblk * full;
            const hipError_t e = shmr::kern::launch_apply(a, rows, var, 0, cap, stream);
            if (e == hipErrorInvalidValue) return SHMR_EC_INVALID_ARGUMENT;   // variant not compiled
            if (e != hipSuccess) return SHMR_EC_DEVICE_ERROR;
        }
        if (len % tb) {
            // remaining columns [full*tb, len): U = 1 tiles, the last one partial
            const uint64_t tb1 = shmr::kern::tile_bytes(1);
            a.col_base = full * tb;
            a.tiles_per_block = uint32_t((len - full * tb + tb1 - 1) / tb1);
            a.ntiles = nblk * a.tiles_per_block;
            HIP_TRY(shmr::kern::launch_apply(a, rows, tail, 1, cap, stream));
        }
    }
    return SHMR_EC_OK;
}

int run_plan(Plan& plan, int dev, const Layout& L, uint64_t first, uint64_t stride, uint64_t nblk,
             uint64_t len, hipStream_t stream, OpClass op) {
    BlockSet bs;
    bs.first = first;
    bs.stride = stride;
    bs.n = nblk;
    return launch_set(plan, dev, L, bs, len, stream, op);
}

// ---------------------------------------------------------------------------
// Per-device ring of pinned upload slots for small per-call tables (block
// lists, per-block plan indices, plan pointer tables).  A slot is reused only
// after the event recorded behind the kernels that read it has completed.
// ---------------------------------------------------------------------------
class UploadRing {
public:
    static constexpr int kSlots = 32;
    static constexpr size_t kSlotBytes = 256 * 1024;

    static UploadRing* for_device(int dev, int* rc) {
        static std::mutex mu;
        static auto* rings = new std::map<int, UploadRing*>;   // leaked: outlives static teardown
        std::lock_guard<std::mutex> lock(mu);
        auto& r = (*rings)[dev];
        if (!r) {
            auto* ring = new UploadRing;
            if (hipHostMalloc(reinterpret_cast<void**>(&ring->host_), kSlots * kSlotBytes, hipHostMallocDefault) !=
                    hipSuccess ||
                hipMalloc(reinterpret_cast<void**>(&ring->dev_), kSlots * kSlotBytes) != hipSuccess) {
                *rc = SHMR_EC_OUT_OF_MEMORY;
                return nullptr;
            }
            for (int i = 0; i < kSlots; ++i) {
                if (hipEventCreateWithFlags(&ring->ev_[i], hipEventDisableTiming) != hipSuccess) {
                    *rc = SHMR_EC_DEVICE_ERROR;
                    return nullptr;
                }
            }
            r = ring;
        }
        *rc = SHMR_EC_OK;
        return r;
    }

    // Claims a slot; *host/*dev point at its kSlotBytes of pinned / device memory.
    int acquire(uint8_t** host, uint8_t** dev, int* slot) {
        std::unique_lock<std::mutex> lock(mu_);
        for (;;) {
            for (int n = 0; n < kSlots; ++n) {
                const int i = (next_ + n) % kSlots;
                if (inuse_[i]) continue;
                inuse_[i] = true;
                next_ = (i + 1) % kSlots;
                const bool armed = armed_[i];
                lock.unlock();
                if (armed && hipEventSynchronize(ev_[i]) != hipSuccess) {
                    release_now(i);
                    return SHMR_EC_DEVICE_ERROR;
                }
                *host = host_ + size_t(i) * kSlotBytes;
                *dev = dev_ + size_t(i) * kSlotBytes;
                *slot = i;
                return SHMR_EC_OK;
            }
            cv_.wait(lock);
        }
    }
    // Copies the first `bytes` of the slot to the device on `stream`.
    int upload(int slot, size_t bytes, hipStream_t stream) {
        const size_t off = size_t(slot) * kSlotBytes;
        return hipMemcpyAsync(dev_ + off, host_ + off, bytes, hipMemcpyHostToDevice, stream) == hipSuccess
                   ? SHMR_EC_OK
                   : SHMR_EC_DEVICE_ERROR;
    }
    // Releases the slot once all work enqueued on `stream` so far has finished.
    int release_after(int slot, hipStream_t stream) {
        const bool ok = hipEventRecord(ev_[slot], stream) == hipSuccess;
        std::lock_guard<std::mutex> lock(mu_);
        armed_[slot] = ok;
        inuse_[slot] = false;
        cv_.notify_one();
        return ok ? SHMR_EC_OK : SHMR_EC_DEVICE_ERROR;
    }

private:
    void release_now(int slot) {
        std::lock_guard<std::mutex> lock(mu_);
        inuse_[slot] = false;
        cv_.notify_one();
    }
    uint8_t* host_ = nullptr;
    uint8_t* dev_ = nullptr;
    hipEvent_t ev_[kSlots] = {};
    bool armed_[kSlots] = {};
    bool inuse_[kSlots] = {};
    int next_ = 0;
    std::mutex mu_;
    std::condition_variable cv_;
};

// ---------------------------------------------------------------------------
// Device staging for the host-buffer entry points.
// ---------------------------------------------------------------------------
struct Staging {
    int dev = -1;
    hipStream_t stream = nullptr;
    uint8_t* dbuf = nullptr;
    size_t cap = 0;
};

class StagingPool {
public:
    static StagingPool& get() {
        static StagingPool* p = new StagingPool;   // leaked: outlives static teardown
        return *p;
    }
    // Returns a staging object on `dev` with >= bytes of device memory.
    Staging* acquire(int dev, size_t bytes, int* rc) {
        Staging* s = nullptr;
        {
            std::lock_guard<std::mutex> lock(mu_);
            auto& lst = free_[dev];
            if (!lst.empty()) {
                s = lst.back();
                lst.pop_back();
            }
        }
        if (!s) {
            s = new Staging;
            s->dev = dev;
            if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) {
                delete s;
                *rc = SHMR_EC_DEVICE_ERROR;
                return nullptr;
            }
        }
        if (s->cap < bytes) {
            if (s->dbuf) (void)hipFree(s->dbuf);
            s->dbuf = nullptr;
            s->cap = 0;
            if (hipMalloc(reinterpret_cast<void**>(&s->dbuf), bytes) != hipSuccess) {
                release(s);
                *rc = SHMR_EC_OUT_OF_MEMORY;
                return nullptr;
            }
            s->cap = bytes;
        }
        *rc = SHMR_EC_OK;
        return s;
    }
    void release(Staging* s) {
        std::lock_guard<std::mutex> lock(mu_);
        free_[s->dev].push_back(s);
    }

private:
    std::mutex mu_;
    std::map<int, std::vector<Staging*>> free_;
};

struct StagingLease {
    Staging* s = nullptr;
    ~StagingLease() {
        if (s) StagingPool::get().release(s);
    }
};

uint64_t round_up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

}  // namespace

// ===========================================================================
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

const char* shmr_ec_version(void) { return "shmr_ec 0.1.0 (gfx950)"; }

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
}

int shmr_ec_set_device(shmr_ec_t* rs, int device) {
    if (!rs || device < 0) return SHMR_EC_INVALID_ARGUMENT;
    rs->device = device;
    return SHMR_EC_OK;
}

int shmr_ec_set_tuning(const char* key, int value) {
    if (!key) return SHMR_EC_INVALID_ARGUMENT;
    std::string k(key);
    int first = 0, last = 1;
    if (k.rfind("encode.", 0) == 0) {
        first = last = kEncode;
        k = k.substr(7);
    } else if (k.rfind("decode.", 0) == 0) {
        first = last = kDecode;
        k = k.substr(7);
    }
    for (int i = first; i <= last; ++i) {
        Tuning& T = g_tune[i];
        if (k == "chunks") {
            if (value != 1 && value != 2 && value != 4 && value != kAuto) return SHMR_EC_INVALID_ARGUMENT;
            T.u = value;
        } else if (k == "nt_load") {
            T.nt_load = value == kAuto ? kAuto : (value != 0);
        } else if (k == "nt_store") {
            T.nt_store = value == kAuto ? kAuto : (value != 0);
        } else if (k == "scalar_tabs") {
            T.scalar_tabs = value != 0;
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
        } else {
            return SHMR_EC_INVALID_ARGUMENT;
        }
    }
    return SHMR_EC_OK;
}

int shmr_ec_get_tuning(const char* key) {
    if (!key) return SHMR_EC_INVALID_ARGUMENT;
    std::string k(key);
    int op = kEncode;
    if (k.rfind("encode.", 0) == 0) {
        k = k.substr(7);
    } else if (k.rfind("decode.", 0) == 0) {
        op = kDecode;
        k = k.substr(7);
    }
    const Tuning& T = g_tune[op];
    if (k == "chunks") return T.u;
    if (k == "nt_load") return T.nt_load;
    if (k == "nt_store") return T.nt_store;
    if (k == "scalar_tabs") return T.scalar_tabs;
    if (k == "occ8") return T.occ8;
    if (k == "grid") return T.grid;
    if (k == "diag") return T.diag;
    if (k == "threads") return T.threads;
    return SHMR_EC_INVALID_ARGUMENT;
}

int shmr_ec_describe_variant(int decode, uint32_t data_shards, uint32_t rows, char* buf, size_t len) {
    if (!buf || len == 0 || rows == 0) return SHMR_EC_INVALID_ARGUMENT;
    const OpClass op = decode ? kDecode : kEncode;
    const shmr::kern::Variant v = resolve_variant(op, data_shards, std::min<uint32_t>(rows, shmr::kern::kMaxRowsPerLaunch));
    std::snprintf(buf, len, "chunks=%d nt_load=%d nt_store=%d scalar_tabs=%d occ8=%d threads=%d grid=%d diag=%d", v.u,
                  int(v.nt_load), int(v.nt_store), int(v.scalar_tabs), int(v.occ8), v.threads,
                  g_tune[op].grid.load(), int(v.diag));
    return SHMR_EC_OK;
}

int shmr_ec_cache_stats(const shmr_ec_t* rs, uint64_t* hits, uint64_t* misses) {
    if (!rs) return SHMR_EC_INVALID_ARGUMENT;
    if (hits) *hits = rs->codec->decode_cache_hits();
    if (misses) *misses = rs->codec->decode_cache_misses();
    return SHMR_EC_OK;
}

int shmr_ec_device_count(void) { return device_count(); }

// ---- host-buffer encode ------------------------------------------------------
int shmr_ec_encode(shmr_ec_t* rs, uint8_t* const* shards, const size_t* shard_lens, size_t nshards) {
    if (!rs || !shards || !shard_lens) return SHMR_EC_INVALID_ARGUMENT;
    Codec& c = *rs->codec;
    const unsigned k = c.k(), p = c.p(), t = k + p;
    // crate check_piece_count!(all) then check_slices!(multi)
    if (nshards < t) return SHMR_EC_TOO_FEW_SHARDS;
    if (nshards > t) return SHMR_EC_TOO_MANY_SHARDS;
    const size_t len = shard_lens[0];
    if (len == 0) return SHMR_EC_EMPTY_SHARD;
    for (unsigned i = 0; i < t; ++i)
        if (shard_lens[i] != len) return SHMR_EC_INCORRECT_SHARD_SIZE;
    for (unsigned i = 0; i < t; ++i)
        if (!shards[i]) return SHMR_EC_INVALID_ARGUMENT;
    const int dev = rs->device;
    int rc = check_device(dev);
    if (rc) return rc;
    DeviceScope scope(dev);
    if (!scope.ok()) return SHMR_EC_DEVICE_ERROR;
    const uint64_t pitch = round_up(len, 256);
    StagingLease lease;
    lease.s = StagingPool::get().acquire(dev, pitch * t, &rc);
    if (!lease.s) return rc;
    Staging& s = *lease.s;
    for (unsigned i = 0; i < k; ++i)
        HIP_TRY(hipMemcpyAsync(s.dbuf + i * pitch, shards[i], len, hipMemcpyHostToDevice, s.stream));
    Layout L{s.dbuf, s.dbuf, 0, pitch, 0, pitch, 0};
    rc = run_plan(*c.encode_plan(), dev, L, 0, 1, 1, len, s.stream, kEncode);
    if (rc) return rc;
    for (unsigned r = 0; r < p; ++r)
        HIP_TRY(hipMemcpyAsync(shards[k + r], s.dbuf + (k + r) * pitch, len, hipMemcpyDeviceToHost, s.stream));
    HIP_TRY(hipStreamSynchronize(s.stream));
    return SHMR_EC_OK;
}

// ---- host-buffer reconstruct --------------------------------------------------
int shmr_ec_reconstruct(shmr_ec_t* rs, uint8_t* const* shards, const size_t* shard_lens,
                        const uint8_t* present, size_t nshards, int data_only) {
    if (!rs || !shards || !shard_lens || !present) return SHMR_EC_INVALID_ARGUMENT;
    Codec& c = *rs->codec;
    const unsigned k = c.k(), p = c.p(), t = k + p;
    if (nshards < t) return SHMR_EC_TOO_FEW_SHARDS;
    if (nshards > t) return SHMR_EC_TOO_MANY_SHARDS;
    // crate reconstruct_internal: per present shard, len 0 -> EmptyShard,
    // mismatch -> IncorrectShardSize, in index order.
    unsigned np = 0;
    size_t len = 0;
    bool have_len = false;
    for (unsigned i = 0; i < t; ++i) {
        if (!present[i]) continue;
        if (shard_lens[i] == 0) return SHMR_EC_EMPTY_SHARD;
        ++np;
        if (have_len && shard_lens[i] != len) return SHMR_EC_INCORRECT_SHARD_SIZE;
        len = shard_lens[i];
        have_len = true;
    }
    if (np == t) return SHMR_EC_OK;
    if (np < k) return SHMR_EC_TOO_FEW_SHARDS_PRESENT;
    std::vector<uint8_t> pr(present, present + t);
    auto plan = c.reconstruct_plan(pr, data_only != 0);
    for (unsigned m = 0; m < plan->m; ++m)
        if (!shards[plan->out_idx[m]]) return SHMR_EC_INVALID_ARGUMENT;
    for (unsigned i = 0; i < k; ++i)
        if (!shards[plan->in_idx[i]]) return SHMR_EC_INVALID_ARGUMENT;
    if (plan->m == 0) return SHMR_EC_OK;
    const int dev = rs->device;
    int rc = check_device(dev);
    if (rc) return rc;
    DeviceScope scope(dev);
    if (!scope.ok()) return SHMR_EC_DEVICE_ERROR;
    const uint64_t pitch = round_up(len, 256);
    StagingLease lease;
    lease.s = StagingPool::get().acquire(dev, pitch * t, &rc);
    if (!lease.s) return rc;
    Staging& s = *lease.s;
    for (unsigned i = 0; i < k; ++i) {
        const unsigned idx = plan->in_idx[i];
        HIP_TRY(hipMemcpyAsync(s.dbuf + idx * pitch, shards[idx], len, hipMemcpyHostToDevice, s.stream));
    }
    Layout L{s.dbuf, s.dbuf, 0, pitch, 0, pitch, 0};
    rc = run_plan(*plan, dev, L, 0, 1, 1, len, s.stream, kDecode);
    if (rc) return rc;
    for (unsigned m = 0; m < plan->m; ++m) {
        const unsigned idx = plan->out_idx[m];
        HIP_TRY(hipMemcpyAsync(shards[idx], s.dbuf + idx * pitch, len, hipMemcpyDeviceToHost, s.stream));
    }
    HIP_TRY(hipStreamSynchronize(s.stream));
    return SHMR_EC_OK;
}

// ---- device-resident batch ----------------------------------------------------
int shmr_ec_encode_batch_dev(shmr_ec_t* rs, const uint8_t* d_data, size_t data_shard_pitch,
                             size_t data_block_pitch, uint8_t* d_parity, size_t parity_shard_pitch,
                             size_t parity_block_pitch, size_t nblocks, size_t shard_len, int device,
                             void* stream) {
    if (!rs) return SHMR_EC_INVALID_ARGUMENT;
    if (nblocks == 0) return SHMR_EC_OK;
    if (shard_len == 0) return SHMR_EC_EMPTY_SHARD;
    if (!d_data || !d_parity) return SHMR_EC_INVALID_ARGUMENT;
    int rc = check_device(device);
    if (rc) return rc;
    DeviceScope scope(device);
    if (!scope.ok()) return SHMR_EC_DEVICE_ERROR;
    Codec& c = *rs->codec;
    Layout L{d_data, d_parity, data_block_pitch, data_shard_pitch, parity_block_pitch, parity_shard_pitch, c.k()};
    return run_plan(*c.encode_plan(), device, L, 0, 1, nblocks, shard_len, static_cast<hipStream_t>(stream), kEncode);
}

int shmr_ec_reconstruct_batch_dev(shmr_ec_t* rs, uint8_t* d_shards, size_t shard_pitch, size_t block_pitch,
                                  const uint8_t* present, size_t nblocks, size_t shard_len, int data_only,
                                  int device, void* stream) {
    if (!rs || !present) return SHMR_EC_INVALID_ARGUMENT;
    if (nblocks == 0) return SHMR_EC_OK;
    if (shard_len == 0) return SHMR_EC_EMPTY_SHARD;
    if (!d_shards) return SHMR_EC_INVALID_ARGUMENT;
    Codec& c = *rs->codec;
    const unsigned k = c.k(), t = k + c.p();
    // Validate every block first (no launch on a bad batch).
    std::map<std::vector<uint8_t>, std::vector<uint64_t>> groups;
    for (size_t b = 0; b < nblocks; ++b) {
        const uint8_t* pr = present + b * t;
        unsigned np = 0;
        for (unsigned i = 0; i < t; ++i) np += pr[i] ? 1 : 0;
        if (np == t) continue;
        if (np < k) return SHMR_EC_TOO_FEW_SHARDS_PRESENT;
        std::vector<uint8_t> key(t);
        for (unsigned i = 0; i < t; ++i) key[i] = pr[i] ? 1 : 0;
        groups[key].push_back(b);
    }
    if (groups.empty()) return SHMR_EC_OK;
    int rc = check_device(device);
    if (rc) return rc;
    DeviceScope scope(device);
    if (!scope.ok()) return SHMR_EC_DEVICE_ERROR;
    Layout L{d_shards, d_shards, block_pitch, shard_pitch, block_pitch, shard_pitch, 0};
    hipStream_t s = static_cast<hipStream_t>(stream);
    // Plans with the same number of rebuilt shards share one multi-plan launch
    // set: the kernel picks each block's plan from a device table, so a batch
    // with many erasure patterns is still one launch (plus a tail launch).
    struct Group {
        std::vector<std::shared_ptr<Plan>> plans;
        std::vector<uint32_t> blocks;
        std::vector<uint16_t> plan_idx;
    };
    std::map<unsigned, Group> by_m;
    for (auto& g : groups) {
        auto plan = c.reconstruct_plan(g.first, data_only != 0);
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
            rc = run_plan(*grp.plans[0], device, L, grp.blocks[0], stride, grp.blocks.size(), shard_len, s, kDecode);
            if (rc) return rc;
            continue;
        }
        if (grp.plans.size() > 65535) return SHMR_EC_INVALID_ARGUMENT;
        std::vector<const uint8_t*> dplans(grp.plans.size());
        for (size_t i = 0; i < grp.plans.size(); ++i) {
            uint32_t off = 0;
            rc = plan_on_device(*grp.plans[i], device, &dplans[i], &off);
            if (rc) return rc;
        }
        UploadRing* ring = UploadRing::for_device(device, &rc);
        if (!ring) return rc;
        const size_t table_bytes = (dplans.size() * sizeof(void*) + 15) & ~size_t(15);
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
            rc = ring->upload(slot, total, s);
            BlockSet bs;
            bs.n = n;
            bs.d_plans = reinterpret_cast<const uint8_t* const*>(dslot);
            bs.d_list = reinterpret_cast<const uint32_t*>(dslot + list_off);
            bs.d_plan_idx = reinterpret_cast<const uint16_t*>(dslot + pidx_off);
            if (rc == SHMR_EC_OK) rc = launch_set(*grp.plans[0], device, L, bs, shard_len, s, kDecode);
            const int rc2 = ring->release_after(slot, s);
            if (rc) return rc;
            if (rc2) return rc2;
        }
    }
    return SHMR_EC_OK;
}

// ---- multi-GPU host batch -----------------------------------------------------
int shmr_ec_encode_blocks_host(shmr_ec_t* rs, uint8_t* const* host_shards, size_t nblocks, size_t shard_len,
                               const int* devices, int ndev) {
    if (!rs || !host_shards || !devices || ndev <= 0) return SHMR_EC_INVALID_ARGUMENT;
    if (nblocks == 0) return SHMR_EC_OK;
    if (shard_len == 0) return SHMR_EC_EMPTY_SHARD;
    Codec& c = *rs->codec;
    const unsigned k = c.k(), p = c.p(), t = k + p;
    for (size_t i = 0; i < nblocks * t; ++i)
        if (!host_shards[i]) return SHMR_EC_INVALID_ARGUMENT;
    for (int d = 0; d < ndev; ++d) {
        int rc = check_device(devices[d]);
        if (rc) return rc;
    }
    const uint64_t pitch = round_up(shard_len, 256);
    constexpr size_t kChunk = 16;   // blocks per H2D/kernel/D2H round
    std::vector<int> results(size_t(ndev), SHMR_EC_OK);
    auto worker = [&](int di) {
        const int dev = devices[di];
        DeviceScope scope(dev);
        if (!scope.ok()) {
            results[di] = SHMR_EC_DEVICE_ERROR;
            return;
        }
        int rc = SHMR_EC_OK;
        StagingLease lease;
        lease.s = StagingPool::get().acquire(dev, pitch * t * kChunk, &rc);
        if (!lease.s) {
            results[di] = rc;
            return;
        }
        Staging& s = *lease.s;
        std::vector<size_t> mine;
        for (size_t b = size_t(di); b < nblocks; b += size_t(ndev)) mine.push_back(b);
        for (size_t c0 = 0; c0 < mine.size(); c0 += kChunk) {
            const size_t n = std::min(kChunk, mine.size() - c0);
            for (size_t j = 0; j < n; ++j)
                for (unsigned i = 0; i < k; ++i)
                    if (hipMemcpyAsync(s.dbuf + (j * t + i) * pitch, host_shards[mine[c0 + j] * t + i], shard_len,
                                       hipMemcpyHostToDevice, s.stream) != hipSuccess) {
                        results[di] = SHMR_EC_DEVICE_ERROR;
                        return;
                    }
            Layout L{s.dbuf, s.dbuf, pitch * t, pitch, pitch * t, pitch, 0};
            rc = run_plan(*c.encode_plan(), dev, L, 0, 1, n, shard_len, s.stream, kEncode);
            if (rc) {
                results[di] = rc;
                return;
            }
            for (size_t j = 0; j < n; ++j)
                for (unsigned r = 0; r < p; ++r)
                    if (hipMemcpyAsync(host_shards[mine[c0 + j] * t + k + r], s.dbuf + (j * t + k + r) * pitch,
                                       shard_len, hipMemcpyDeviceToHost, s.stream) != hipSuccess) {
                        results[di] = SHMR_EC_DEVICE_ERROR;
                        return;
                    }
            if (hipStreamSynchronize(s.stream) != hipSuccess) {
                results[di] = SHMR_EC_DEVICE_ERROR;
                return;
            }
        }
    };
    std::vector<std::thread> th;
    for (int d = 1; d < ndev; ++d) th.emplace_back(worker, d);
    worker(0);
    for (auto& x : th) x.join();
    for (int r : results)
        if (r) return r;
    return SHMR_EC_OK;
}

}  // extern "C"
