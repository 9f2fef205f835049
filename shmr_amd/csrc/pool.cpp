// Device Block Cache slots (include/shmr_ec.h shmr_ec_pool_*).
//
// The reference's Block Cache takes and drops one block's buffers at a time
// (VirtualBlock::{populate,drop_buffer}, src/vfs/block.rs:148-152, :586-608;
// every shard a Vec<u8> of its own for the crate, :408-419, :556-565).  A slab
// from shmr_ec_device_alloc_shards can only be freed whole.  A pool carves
// block slots -- all k + p shards of one block, at the slot pitch of the
// device-resident batches -- from large device slabs, hands them out and takes
// them back one block at a time (lowest free slot first, so live blocks stay
// dense), and never moves a live slot.  Pointer tables over pool blocks, in any
// order and with holes, lie on the slab's slot lattice (ptr_grid.hpp): the
// *_ptrs_dev calls and the submission queue run them through the strided
// kernels over their slots (one run, segment runs, or a block list).
#include <algorithm>
#include <mutex>
#include <new>
#include <set>
#include <vector>

#include "ec_core.hpp"
#include "shmr_ec.h"

namespace core = shmr::core;

struct shmr_ec_pool {
    int device = 0;
    uint64_t spb = 0, len = 0, pitch = 0, bpitch = 0, per_slab = 0;
    struct Slab {
        uint8_t* base = nullptr;
        std::set<uint64_t> free_;   // free slot indices of this slab
    };
    std::vector<Slab> slabs;
    uint64_t in_use = 0;
    std::mutex mu;
};

namespace {
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
}  // namespace

extern "C" {

int shmr_ec_pool_new(int device, size_t shards_per_block, size_t shard_len, size_t slots_per_slab,
                     shmr_ec_pool_t** out) {
    return guarded([&]() -> int {
        if (!out) return SHMR_EC_INVALID_ARGUMENT;
        *out = nullptr;
        if (shards_per_block == 0 || shard_len == 0 || slots_per_slab == 0 || shards_per_block > 256)
            return SHMR_EC_INVALID_ARGUMENT;
        const int rc = core::check_device(device);
        if (rc) return rc;
        auto* p = new shmr_ec_pool;
        p->device = device;
        p->spb = shards_per_block;
        p->len = shard_len;
        // the slot placement of the batches: 4 KiB pages,
        // one more for a power-of-two stride
        p->pitch = core::round_up(shard_len, 4096);
        if (p->pitch % 65536 == 0) p->pitch += 4096;
        p->bpitch = p->pitch * shards_per_block;
        p->per_slab = slots_per_slab;
        if (p->pitch < shard_len || p->bpitch / shards_per_block != p->pitch ||
            slots_per_slab > (UINT64_MAX >> 1) / p->bpitch) {
            delete p;
            return SHMR_EC_INVALID_ARGUMENT;
        }
        *out = p;
        return SHMR_EC_OK;
    });
}

int shmr_ec_pool_alloc(shmr_ec_pool_t* pool, uint8_t** out_ptrs) {
    return guarded([&]() -> int {
        if (!pool || !out_ptrs) return SHMR_EC_INVALID_ARGUMENT;
        std::lock_guard<std::mutex> lk(pool->mu);
        shmr_ec_pool::Slab* sl = nullptr;
        for (auto& s : pool->slabs)
            if (!s.free_.empty()) {
                sl = &s;
                break;
            }
        if (!sl) {   // a new slab (blocking device allocation)
            void* mem = nullptr;
            const int rc = shmr_ec_device_alloc(pool->device, size_t(pool->per_slab * pool->bpitch), 0, &mem);
            if (rc) return rc;
            shmr_ec_pool::Slab s;
            s.base = static_cast<uint8_t*>(mem);
            try {
                for (uint64_t i = 0; i < pool->per_slab; ++i) s.free_.insert(s.free_.end(), i);
                pool->slabs.push_back(std::move(s));
            } catch (...) {
                (void)shmr_ec_device_free(pool->device, mem);
                throw;
            }
            sl = &pool->slabs.back();
        }
        const uint64_t slot = *sl->free_.begin();   // lowest free slot: live blocks stay dense
        sl->free_.erase(sl->free_.begin());
        ++pool->in_use;
        uint8_t* b = sl->base + slot * pool->bpitch;
        for (uint64_t i = 0; i < pool->spb; ++i) out_ptrs[i] = b + i * pool->pitch;
        return SHMR_EC_OK;
    });
}

int shmr_ec_pool_free(shmr_ec_pool_t* pool, uint8_t* first) {
    return guarded([&]() -> int {
        if (!pool || !first) return SHMR_EC_INVALID_ARGUMENT;
        std::lock_guard<std::mutex> lk(pool->mu);
        for (auto& s : pool->slabs) {
            if (first < s.base || first >= s.base + pool->per_slab * pool->bpitch) continue;
            const uint64_t off = uint64_t(first - s.base);
            if (off % pool->bpitch != 0) return SHMR_EC_INVALID_ARGUMENT;
            const uint64_t slot = off / pool->bpitch;
            if (!s.free_.insert(slot).second) return SHMR_EC_INVALID_ARGUMENT;   // freed twice
            --pool->in_use;
            return SHMR_EC_OK;
        }
        return SHMR_EC_INVALID_ARGUMENT;
    });
}

int shmr_ec_pool_destroy(shmr_ec_pool_t* pool) {
    return guarded([&]() -> int {
        if (!pool) return SHMR_EC_OK;
        int rc = SHMR_EC_OK;
        for (auto& s : pool->slabs) {
            const int r = shmr_ec_device_free(pool->device, s.base);
            if (r && rc == SHMR_EC_OK) rc = r;
        }
        delete pool;
        return rc;
    });
}

int shmr_ec_pool_stats(shmr_ec_pool_t* pool, uint64_t* slabs, uint64_t* slots, uint64_t* in_use) {
    if (!pool) return SHMR_EC_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> lk(pool->mu);
    if (slabs) *slabs = pool->slabs.size();
    if (slots) *slots = pool->slabs.size() * pool->per_slab;
    if (in_use) *in_use = pool->in_use;
    return SHMR_EC_OK;
}

}  // extern "C"
