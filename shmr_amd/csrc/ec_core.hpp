// Internal device-side core of the erasure path: tuning policy, plan images on
// the device, launch sets over block batches, the per-device upload ring and
// staging pool.  Used by the C ABI (ec_api.cpp) and the host-buffer pipeline
// (host_engine.cpp).  Not part of the public interface.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "gf256.hpp"
#include "gf_apply.hpp"
#include "shmr_ec.h"

namespace shmr {
namespace core {

using gf::Codec;
using gf::Plan;

#define SHMR_HIP_TRY(expr)                                 \
    do {                                                   \
        hipError_t _e = (expr);                            \
        if (_e != hipSuccess) return SHMR_EC_DEVICE_ERROR; \
    } while (0)

// ---- tuning ---------------------------------------------------------------
enum OpClass { kEncode = 0, kDecode = 1 };
constexpr int kAuto = -2;

int set_tuning(const char* key, int value);
int get_tuning(const char* key);
// The full-tile variant of a launch shape: kern::policy_variant (gf_apply.hpp),
// plus the tools build's kernel knobs.
kern::Variant select_variant(OpClass op, const kern::LaunchShape& s);
kern::LaunchShape shape_of(OpClass op, unsigned k, unsigned rows, bool host_mapped, bool ptrs, bool segs,
                           bool compact, bool sc1_ok, bool fused);
// Whether segment launches are compiled for this op's current tuning (always,
// in the product build).
bool segs_supported(OpClass op, unsigned k, bool host_mapped, bool ptrs, bool compact = false);
// Shard-pointer table rows in plan order (kern::ApplyArgs::shard_ptrs): input t
// at [t], output row r at [k + r].  src / dst: n rows of t entries.  present ==
// nullptr (encode): the rows are already in plan order and are copied.  A
// reconstruct's plan reads the first k present shards and writes the absent
// ones in ascending index (data_only: the absent data shards only;
// gf256.cpp Codec::reconstruct_plan); rows with every shard present are copied.
void permute_ptr_rows(const uint64_t* src, const uint8_t* present, size_t n, unsigned k, unsigned t, bool data_only,
                      uint64_t* dst);
int grid_mode(OpClass op);
// Largest block ((k+p) * shard bytes) a pageable single-block call bounces
// through a mapped buffer instead of per-shard DMA copies (knob "bounce_kib").
uint64_t bounce_limit();
// Pageable host batches: code the pinned mirror in place (zero-copy) instead
// of DMA-ing it to device staging (knob "mirror_zc").
bool mirror_zero_copy();
// Zero-copy launches of at most this many 4 KiB tiles (blocks x tiles per
// shard) read their shard-pointer table straight from the pinned upload slot
// across PCIe instead of uploading it first (knob "ptrs_direct"; 0 = always
// upload).
uint64_t ptrs_direct_max();
// Device pointer tables whose shards form a slot grid (entry (b, j) at base +
// b * block_pitch + j * shard_pitch: a Block-Cache slab, shmr_ec_device_alloc_shards)
// run through the strided kernels of the *_batch_dev calls (knob "ptrs_grid",
// default 1; 0 = always the table kernels).
bool ptrs_grid();
// Waits for `stream`: polls it for up to the "sync_spin_us" knob before a
// blocking hipStreamSynchronize (short single-block calls finish within the
// spin and skip the blocking wake-up).
hipError_t sync_stream(hipStream_t stream);

// ---- devices --------------------------------------------------------------
// Device IDs.  Every per-device object (plan images, upload rings, staging
// pools and pipes, the counters below) is keyed by the caller's device ID.
// The tools build can add alias IDs (knob "alias_devices" = a): IDs n .. n+a-1
// of an n-GPU process run on physical GPU (id mod n) but keep their own
// per-device state -- a one-GPU rehearsal of the multi-device bookkeeping.
int device_count();           // physical GPUs
int logical_device_count();   // physical + alias IDs (0 without a GPU)
int physical_device(int dev);
int check_device(int dev);   // SHMR_EC_OK / NO_DEVICE / INVALID_ARGUMENT

// Per-device counters (shmr_ec_device_stats; index order of the header's
// SHMR_EC_DEV_* constants).
enum DevCounter {
    kDevBlocksEncoded = 0,
    kDevBlocksReconstructed,
    kDevLaunches,
    kDevPlanImages,
    kDevUploadRings,
    kDevStagingStreams,
    kDevBlockingCalls,
    kDevPtrTableHits,
    kDevCaptureTables,
    kDevCaptureReleased,
    kDevPtrTableGrids,
    kDevCounters
};
void count_device(int dev, DevCounter c, uint64_t n = 1);
void device_stats(int dev, uint64_t* out, size_t n);

// Sets the calling thread's device for the scope, restoring the previous one.
class DeviceScope {
public:
    explicit DeviceScope(int dev) {
        ok_ = hipGetDevice(&prev_) == hipSuccess && hipSetDevice(physical_device(dev)) == hipSuccess;
    }
    ~DeviceScope() {
        if (ok_) (void)hipSetDevice(prev_);
    }
    bool ok() const { return ok_; }

private:
    int prev_ = 0;
    bool ok_ = false;
};

// Every C-ABI entry point runs under the relaxed stream-capture mode (the
// calling thread's mode is restored on return).  Under the default (global)
// mode HIP refuses the library's allocation and synchronisation calls
// (hipMalloc / hipFree / hipHostMalloc / hipHostRegister, hipStreamSynchronize
// of its own streams ...) while ANY thread of the process captures a graph --
// and the refused call invalidates that capture -- although none of them
// touches a captured stream (measured: profiles/r04/s8, tools/capture_probe_hip.py).
// The caller's own capture is checked separately, under the mode the caller
// entered with (capture_state): nothing allocates or synchronises inside it.
struct CaptureModeTls {
    int depth = 0;
    hipStreamCaptureMode caller = hipStreamCaptureModeGlobal;
};
inline CaptureModeTls& capture_mode_tls() {
    static thread_local CaptureModeTls t;
    return t;
}
// (-DSHMR_EC_NO_RELAXED_CAPTURE compiles the guard out: the measurement build of
// tools/guard_ab.cpp; never the product.)
class RelaxedCapture {
public:
#ifdef SHMR_EC_NO_RELAXED_CAPTURE
    RelaxedCapture() {}
    ~RelaxedCapture() {}
#else
    RelaxedCapture() {
        ok_ = hipThreadExchangeStreamCaptureMode(&prev_) == hipSuccess;
        if (!ok_) {
            (void)hipGetLastError();
            return;
        }
        CaptureModeTls& t = capture_mode_tls();
        if (t.depth++ == 0) t.caller = prev_;
    }
    ~RelaxedCapture() {
        if (!ok_) return;
        --capture_mode_tls().depth;
        (void)hipThreadExchangeStreamCaptureMode(&prev_);
    }
#endif
    RelaxedCapture(const RelaxedCapture&) = delete;
    RelaxedCapture& operator=(const RelaxedCapture&) = delete;

private:
    hipStreamCaptureMode prev_ = hipStreamCaptureModeRelaxed;
    bool ok_ = false;
};

// ---- per-device state --------------------------------------------------------
// Created once per device ID, by the first call that touches the device or by
// shmr_ec_device_init, synchronously and on a private stream (never the
// caller's): the unaligned-access probe of the physical GPU, and the first
// chunk of the plan arena (pinned host + device memory).  Afterwards the
// device-resident entry points make no blocking HIP call: a plan image is
// written once into a permanent pinned slot and uploaded with hipMemcpyAsync
// on the caller's stream, so a graph capture records the upload and a replay
// re-copies the same bytes.  Inside a stream capture the state must already
// exist (SHMR_EC_INVALID_ARGUMENT otherwise: nothing is enqueued).
int device_init(int dev, hipStream_t caller = nullptr);
// Whether misaligned device-resident shards may take the vector kernels (the
// probe's verdict for the device, or the tools knob "uvec").  Needs the state.
bool unaligned_vector(int dev);
// Whether `stream` is being captured into a graph.  An error (e.g. the legacy
// null stream while another thread captures in global mode:
// INVALID_ARGUMENT; an invalidated capture: INVALID_ARGUMENT) is the caller's
// status -- never taken for either answer.
int capture_state(hipStream_t stream, bool* capturing);
// The capture reserve (shmr_ec_capture_reserve): per-device pinned + device
// memory for the tables of captured calls (shard-pointer tables of *_ptrs_dev,
// block tables of multi-pattern reconstructs), which every replay re-reads.
// Device init creates 4 MiB; capture_reserve makes sure one free range of
// `bytes` exists (blocking; not inside a capture).  capture_alloc never grows
// it (OUT_OF_MEMORY when no range fits) and ties the block to the graph being
// captured on `stream`: it returns to the reserve when that graph and every
// executable graph made from it are destroyed.
int capture_reserve(int dev, size_t bytes);
int capture_alloc(int dev, hipStream_t stream, size_t bytes, uint8_t** host, uint8_t** devp);

// Device image of a plan (compact: the compact-output form, Plan::image),
// written to the device's arena on first use and uploaded on `stream`; later
// uses on another stream wait for that upload (an event, no host block).
int plan_on_device(Plan& plan, int dev, hipStream_t stream, bool compact, const uint8_t** out);
uint32_t plan_tab_off(unsigned k, unsigned m);
// Permanent device memory from the device's plan arena (plus its pinned host
// twin): multi-plan tables of captured launches, which a replay re-reads.
int arena_alloc(int dev, size_t bytes, bool capturing, uint8_t** host, uint8_t** devp);

// ---- launches -----------------------------------------------------------------
struct Layout {
    const uint8_t* in_base;
    uint8_t* out_base;
    uint64_t in_bpitch, in_spitch, out_bpitch, out_spitch;
    uint32_t out_bias;   // subtracted from plan out_idx (encode into a parity-only buffer)
    // Shard-pointer layout (bases/pitches unused): shard i of block b at
    // d_ptrs[b * total + i], a device-visible table.  ptrs_aligned: every
    // address the launch touches is 16-byte aligned.  host_mapped: the shards
    // are mapped host memory (zero-copy; selects the PCIe variant policy).
    const uint64_t* d_ptrs = nullptr;
    uint32_t total = 0;
    bool ptrs_aligned = false;
    bool host_mapped = false;
    // Reconstruct into a compact output: rebuilt shard j (index order) of block
    // b at out_base + b * out_bpitch + j * out_spitch (compact plan images).
    bool compact = false;
};

// Blocks covered by one launch set: {first + j * stride} or, with d_list, the
// device list d_list[j]; multi-plan sets also carry a per-block plan index into
// the device table d_plans (all plans share k and m).
struct BlockSet {
    uint64_t first = 0, stride = 1, n = 0;
    const uint32_t* d_list = nullptr;
    const uint16_t* d_plan_idx = nullptr;
    const uint8_t* const* d_plans = nullptr;
    // or: up to kern::kMaxSegs arithmetic runs with their device plans, passed
    // in the kernel arguments (no upload)
    const kern::Seg* segs = nullptr;
    uint32_t nseg = 0;
};

// Enqueues out = rows (x) in over a block set on the current device (= dev).
int launch_set(Plan& shape, int dev, const Layout& L, const BlockSet& bs, uint64_t len, hipStream_t stream,
               OpClass op);

// Whether a lattice launch over these (ascending) slots runs without the
// uploaded block list: one arithmetic run, or segment runs (knob
// "lattice_list" = 1: always true -- the list is used).
bool slots_launch_fits(OpClass op, unsigned k, const Layout& L, const uint64_t* slots, uint64_t n);

// Encode nblocks blocks laid out per `L` (plan = the codec's parity rows).
// slots (r06, nullable): batch block j is layout block slots[j] (ascending,
// distinct, < 2^32) -- a slot lattice (ptr_grid.hpp) of a pool or of merged
// per-block calls; one arithmetic run is one strided launch, several runs travel
// in the kernel arguments where the op's segment kernels exist, else an
// uploaded block list (launch_slots).
int encode_on_device(Codec& c, int dev, const Layout& L, uint64_t nblocks, uint64_t len, hipStream_t stream,
                     const uint64_t* slots = nullptr);
// The blocks slots[0 .. n) (ascending, distinct) of a single-plan launch set.
int launch_slots(Plan& plan, int dev, const Layout& L, const uint64_t* slots, uint64_t n, uint64_t len,
                 hipStream_t stream, OpClass op);

// Reconstruct in place: all shards of block b at base + b*block_pitch +
// i*shard_pitch; present = host flags [nblocks][total].  Validates every block
// before enqueueing anything.  Caller has set the device.
int reconstruct_on_device(Codec& c, int dev, uint8_t* d_shards, uint64_t shard_pitch, uint64_t block_pitch,
                          const uint8_t* present, uint64_t nblocks, uint64_t len, bool data_only,
                          hipStream_t stream);

// Same over any layout (e.g. a shard-pointer table, or a compact output).
// slots (r06, nullable): batch block b is layout block slots[b] (ascending,
// distinct, < 2^32), as encode_on_device.
int reconstruct_on_device(Codec& c, int dev, const Layout& L, const uint8_t* present, uint64_t nblocks, uint64_t len,
                          bool data_only, hipStream_t stream, const uint64_t* slots = nullptr);

// A shard-pointer table call (ptrs.cpp): tab[b * total + i] is the device
// address of shard i of block b (0 for a shard the call does not touch),
// validated by the caller.  A table on a slot lattice runs the strided kernels
// over its slots (*lattice = true; counted as SHMR_EC_DEV_PTR_TABLE_GRIDS),
// any other the table kernels, its table uploaded on `stream` (use_cache: the
// device's table cache first; capture reserve inside a capture).  host_mapped:
// the addresses are mapped host memory (zero-copy across PCIe).
int ptrs_launch(Codec& c, const uint64_t* tab, const uint8_t* present, size_t nblocks, uint64_t len, bool data_only,
                int device, hipStream_t stream, OpClass op, bool host_mapped, bool use_cache, bool* lattice = nullptr);

// Validation shared by every reconstruct entry point.
int validate_presence(const Codec& c, const uint8_t* present, uint64_t nblocks);

// ---- per-device ring of pinned upload slots ------------------------------
// Small per-call tables (block lists, per-block plan indices, plan pointer
// tables).  A slot is reused only after the event recorded behind the
// kernels that read it has completed.
class UploadRing {
public:
    static constexpr int kSlots = 32;
    static constexpr size_t kSlotBytes = 256 * 1024;
    // Ring kTables carries multi-plan tables, kPointers shard-pointer tables:
    // a caller holding a kPointers slot may acquire a kTables slot, never the
    // reverse, so concurrent callers cannot deadlock on slots.
    enum Kind { kTables = 0, kPointers = 1 };
    static UploadRing* for_device(int dev, int* rc, Kind kind = kTables);
    int acquire(uint8_t** host, uint8_t** dev, int* slot);
    int upload(int slot, size_t bytes, hipStream_t stream);
    int release_after(int slot, hipStream_t stream);
    // Device address of the slot's pinned HOST copy (kernels can read the
    // table across PCIe without an upload), or nullptr if the host ring is not
    // mapped at the same address.
    const uint8_t* host_view(int slot) const {
        return host_unified_ ? host_ + size_t(slot) * kSlotBytes : nullptr;
    }

private:
    void release_now(int slot);
    int dev_id_ = 0;
    bool host_unified_ = false;
    uint8_t* host_ = nullptr;
    uint8_t* dev_ = nullptr;
    hipEvent_t ev_[kSlots] = {};    // recorded on the caller's stream
    hipEvent_t mev_[kSlots] = {};   // its mirror (record_mirrored): the one acquire() waits on
    bool armed_[kSlots] = {};
    bool inuse_[kSlots] = {};
    int next_ = 0;
    std::mutex mu_;
    std::condition_variable cv_;
};

// Events the library later queries, or makes another stream wait on, from any
// thread are never used as recorded on a caller's stream: that stream may have
// begun a graph capture since: a query of an event whose stream is capturing
// fails with hipErrorCapturedEvent and invalidates that capture, a wait on it
// fails with hipErrorStreamCaptureIsolation (measured: profiles/r04/s8).  `on_caller` is recorded on `stream`;
// the device's private stream waits for it and records `mirror`, which every
// later query and cross-stream wait uses (complete no earlier than on_caller).
// A library-owned stream (staging, host pipelines, the private stream: never
// captured) records `mirror` itself -- no private-stream wait, which would put
// a barrier on a shared hardware queue for every per-block host call.
int record_mirrored(int dev, hipStream_t stream, hipEvent_t on_caller, hipEvent_t mirror);
// A library stream at the device's greatest stream priority (r06): the
// runtime multiplexes streams of one priority onto a few hardware queues, so a
// caller's stream held by a host-released wait blocks whatever else shares
// its queue; the library's own queue, mirror and private streams sit in the
// high-priority pool instead (tests/test_gpu_hol.py).  Current device.
hipError_t create_priority_stream(hipStream_t* s);
// Grows a reusable scratch buffer (device memory, or mapped pinned host
// memory with `host`) to at least `bytes`, doubling, without freeing the old
// one: hipFree / hipHostFree synchronize the whole device, so a caller stream
// held by a host-released wait would hold this call (r06 s40,
// tests/test_gpu_hol.py).  The old buffer is kept for the process's life
// (doubling bounds what is kept to the final size); its caller has drained
// the work that used it.  *p / *cap unchanged on failure.
hipError_t grow_scratch(uint8_t** p, size_t* cap, size_t bytes, bool host);
// Streams the library creates (registered once, never destroyed).
void register_own_stream(hipStream_t s);
bool own_stream(hipStream_t s);

// ---- per-device cache of shard-pointer tables (the *_ptrs_dev calls) -------
// A table passed again with the same bytes on the same stream (a device Block
// Cache whose shard buffers stay put) is not uploaded again: the launch reads
// the device copy made by the earlier call, which the stream's order already
// places before it.  Entries live in permanent arena memory; an entry takes
// another table only once its upload has left the pinned copy and, for another
// stream, once its last reader has finished (no host wait: a busy cache sends
// the call through the upload ring instead).
class PtrTableCache {
public:
    static constexpr int kEntries = 8;
    static PtrTableCache* for_device(int dev, int* rc);
    // *d_tab: the device copy of tab[0, bytes), ordered before work enqueued
    // next on `stream`; nullptr when no entry is free (nothing enqueued).
    int lookup(const void* tab, size_t bytes, hipStream_t stream, const uint8_t** d_tab, int* entry);
    // After the launches that read `entry` are enqueued on `stream`.
    int release_after(int entry, hipStream_t stream);

private:
    struct Entry {
        uint8_t* host = nullptr;   // pinned copy (the upload's source)
        uint8_t* dev = nullptr;
        size_t bytes = 0;
        uint64_t hash = 0, tick = 0;
        hipStream_t stream = nullptr;
        hipEvent_t up = nullptr, used = nullptr;     // recorded on the caller's stream
        hipEvent_t mup = nullptr, mused = nullptr;   // their mirrors (record_mirrored): queried / waited on
        bool valid = false, used_armed = false;
        int busy = 0;
    };
    int dev_id_ = 0;
    Entry e_[kEntries];
    uint64_t tick_ = 0;
    std::mutex mu_;
};

// ---- device staging for the single-call host-buffer entry points ---------
struct Staging {
    int dev = -1;
    hipStream_t stream = nullptr;
    uint8_t* dbuf = nullptr;
    size_t cap = 0;
};

class StagingPool {
public:
    static StagingPool& get();
    Staging* acquire(int dev, size_t bytes, int* rc);
    void release(Staging* s);

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

inline uint64_t round_up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

}  // namespace core
}  // namespace shmr

struct shmr_ec {
    std::shared_ptr<shmr::gf::Codec> codec;
    std::atomic<int> device{0};
};
