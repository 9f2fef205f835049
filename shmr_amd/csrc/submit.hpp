// Submission queue (submit.cpp): per-block calls from concurrent threads merged
// into batch launches.  Not part of the public interface.
//
// The reference codes one block per call from rayon workers
// (src/vfs/mod.rs:91-97 -> VirtualBlock::sync_data -> ReedSolomon::encode at
// src/vfs/block.rs:427; load_block -> reconstruct at :560).  One launch per
// 4 MiB block leaves the GPU launch-bound (a single-block RS(8,3) kernel is
// ~6 us on the GPU for 0.9 us of HBM work), so per device ID the
// library keeps one queue: a call whose inputs are ready pushes its block's
// shard row into a lock-free inbox; the queue's watcher thread, its one
// launcher, launches at once when nothing runs, and calls that arrive while a
// batch runs (or, knob coalesce_us, within a window) merge into the next
// launch, which it issues shortly before the running batch's estimated end
// (knob coalesce_lead_us) -- every pending request of every codec, grouped per
// (codec, op, length, data_only, memory kind), each group one pointer-table
// call (a slot lattice runs the strided kernels, core::ptrs_launch).
// Completion is in launch order on the one stream: a mark kernel behind every
// batch stores its sequence number into a pinned host word, on which the
// batch's callers spin before they sleep; the watcher wakes the sleepers.
#pragma once

#include <atomic>
#include <memory>
#include <string>
#include <vector>

#include "ec_core.hpp"

namespace shmr {
namespace core {

struct SubmitReq {
    const Codec* codec = nullptr;   // a registry codec (gf::get_codec: never freed)
    OpClass op = kEncode;
    bool data_only = false;
    bool host_mapped = false;       // row addresses are mapped host memory
    uint64_t len = 0;
    int dev = 0;
    // The block's row -- total device addresses in shard index order (0: not
    // touched) -- and, for a reconstruct, its presence flags: in the request
    // itself up to kInline shards (the launcher reads one object per request,
    // no second cache miss), else in the vectors.  set_row() fills them.
    static constexpr unsigned kInline = 24;
    unsigned total = 0;
    double est_ns = 0;              // the block's estimated GPU time (bytes at a nominal rate)
    uint64_t row_inline[kInline];
    uint8_t present_inline[kInline];
    std::vector<uint64_t> row;
    std::vector<uint8_t> present;
    const uint64_t* row_data() const { return total <= kInline ? row_inline : row.data(); }
    const uint8_t* present_data() const { return total <= kInline ? present_inline : present.data(); }
    void set_row(const uint64_t* r, const uint8_t* pr, unsigned t);
    // completion: the batch's sequence number (its completion mark), set
    // when the request is launched; done = 1 when its status is final without
    // a mark (a failed launch)
    std::atomic<uint64_t> seq{0};
    std::atomic<int> done{0};
    int rc = SHMR_EC_OK;
};

// Queues r (validated by the caller: crate checks, non-NULL touched shards,
// device ID) on its device's queue; may launch.  On an error nothing is
// queued.  The caller keeps r alive until wait(r) returns.
int submit(SubmitReq* r);
// Waits until r's batch has completed on the GPU; returns r's status.
int wait(SubmitReq* r);

// Knobs (set_tuning): "coalesce" (0/1: the host-buffer entry points on mapped
// memory go through the queue), "coalesce_depth" (batches in flight before
// calls wait to merge), "coalesce_target" (pending calls that launch anyway),
// "coalesce_us" (window a launch from an idle queue waits for more calls),
// "coalesce_max" (blocks per launch), "coalesce_spin_us" (a waiter spins on
// the completion word this long before it sleeps), "coalesce_watch_us" (the
// watcher spins this long before it blocks on the batch's event),
// "coalesce_lead_us" (the watcher launches the calls that arrived while one
// batch runs this long before that batch's estimated end, so the next batch
// is queued behind it and the GPU does not idle between batches; 0: only at
// its completion).
bool coalesce_host();
int set_submit_tuning(const std::string& key, int value, bool* known);
int get_submit_tuning(const std::string& key, bool* known);

// Queue statistics of a device ID: requests, launches (batches), the largest
// batch, waits that slept (blocking event sync) -- shmr_ec_queue_stats.
void submit_stats(int dev, uint64_t* out, size_t n);

}  // namespace core
}  // namespace shmr
