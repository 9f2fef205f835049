// Host-buffer batch engine: StorageBlocks that start and end in host memory
// (the reference's Block Cache buffers / shard files), encoded or rebuilt on
// one or more MI355X.  Whole blocks go round-robin to devices (block b ->
// devices[b % ndev]); on each device a worker pipelines chunks of blocks
// through NS staging sets so the H2D copy of chunk c+1, the kernel of chunk c
// and the D2H copy of chunk c-1 overlap on separate streams.
//
// Host buffers in mapped memory (shmr_ec_host_alloc -- the MI355X-native Block
// Cache -- or ranges given to shmr_ec_host_register) skip all of that: the
// kernels read the data shards and write the rebuilt/parity shards in place
// across PCIe through a device table of shard pointers (zero-copy; measured
// 1.5x the staged DMA pipeline, tools/pcie_probe.py).  Other pinned buffers
// are DMA'd directly; pageable buffers (plain Vec<u8>/malloc) are first
// gathered into a mapped pinned mirror by a crew of copy threads, which the
// kernels then code in place (zero-copy; DMA staging if "mirror_zc" is off).
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "ec_core.hpp"
#include "host_engine.hpp"

namespace shmr {
namespace core {

namespace {

// A crew of threads that runs batches of memcpy tasks in parallel (the caller
// thread participates).  Lives for the duration of one device worker.
class CopyCrew {
public:
    explicit CopyCrew(int n) {
        for (int i = 1; i < n; ++i) th_.emplace_back([this] { loop(); });
    }
    ~CopyCrew() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    struct Task {
        void* dst;
        const void* src;
        size_t n;
    };
    void run(std::vector<Task>& tasks) {
        // split large copies into 1 MiB pieces for balance
        pieces_.clear();
        constexpr size_t kPiece = 1 << 20;
        for (auto& t : tasks)
            for (size_t off = 0; off < t.n; off += kPiece)
                pieces_.push_back(Task{static_cast<uint8_t*>(t.dst) + off, static_cast<const uint8_t*>(t.src) + off,
                                       std::min(kPiece, t.n - off)});
        {
            std::lock_guard<std::mutex> lk(mu_);
            next_ = 0;
            active_ = int(th_.size());
            ++gen_;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [this] { return active_ == 0; });
    }

private:
    void work() {
        for (;;) {
            const size_t i = next_.fetch_add(1);
            if (i >= pieces_.size()) break;
            std::memcpy(pieces_[i].dst, pieces_[i].src, pieces_[i].n);
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
            }
            work();
            std::lock_guard<std::mutex> lk(mu_);
            if (--active_ == 0) done_cv_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::vector<Task> pieces_;
    std::atomic<size_t> next_{0};
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    uint64_t gen_ = 0;
    int active_ = 0;
    bool stop_ = false;
};

bool is_pinned(const void* p) {
    hipPointerAttribute_t attr{};
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();   // pageable memory reports an error: clear it
        return false;
    }
    return attr.type == hipMemoryTypeHost;
}

struct StageSet {
    uint8_t* dbuf = nullptr;   // [C][t][pitch] device
    uint8_t* hbuf = nullptr;   // pinned mirror (pageable mode), mapped
    bool hbuf_unified = false; // hbuf's device address is hbuf: kernels can run on it in place
    size_t dcap = 0, hcap = 0;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    std::vector<size_t> blocks;   // global block ids of the chunk in flight
    bool pending = false;
};

constexpr int kStageSets = 3;

// Staging sets of one device, kept across jobs (allocating hundreds of MB of
// device and pinned memory per call would cost as much as the copies).  One
// job per device at a time holds `mu`.
struct DevicePipe {
    std::mutex mu;
    StageSet sets[kStageSets];
    int ensure(int dev, size_t dbytes, size_t hbytes) {
        RelaxedCapture relaxed;
        for (auto& s : sets) {
            if (!s.stream) {
                if (create_priority_stream(&s.stream) != hipSuccess ||   // (as the library's other streams)
                    hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess) {
                    (void)hipGetLastError();
                    return SHMR_EC_DEVICE_ERROR;
                }
                register_own_stream(s.stream);
                count_device(dev, kDevStagingStreams);
            }
            // (grown without a free: a hipFree would wait for every stream of
            // the device, a held caller stream included)
            if (s.dcap < dbytes && grow_scratch(&s.dbuf, &s.dcap, dbytes, false) != hipSuccess) {
                (void)hipGetLastError();
                return SHMR_EC_OUT_OF_MEMORY;
            }
            if (s.hcap < hbytes) {
                if (grow_scratch(&s.hbuf, &s.hcap, hbytes, true) != hipSuccess) {
                    (void)hipGetLastError();
                    return SHMR_EC_OUT_OF_MEMORY;
                }
                s.hbuf_unified = false;
                void* d = nullptr;
                s.hbuf_unified = hipHostGetDevicePointer(&d, s.hbuf, 0) == hipSuccess && d == s.hbuf;
                if (!s.hbuf_unified) (void)hipGetLastError();
            }
            s.pending = false;
            s.blocks.clear();
        }
        return SHMR_EC_OK;
    }
};

DevicePipe& pipe_for(int dev) {
    static std::mutex mu;
    static auto* pipes = new std::map<int, DevicePipe*>;   // leaked: outlives static teardown
    std::lock_guard<std::mutex> lock(mu);
    auto& p = (*pipes)[dev];
    if (!p) p = new DevicePipe;
    return *p;
}

// Enqueues copies of shards idx[...] (ascending) of one block between host
// pointers and the device block image (pitch apart).  Runs of shards that are
// adjacent both in host memory and in the device image (pitch == len) become a
// single hipMemcpyAsync.
int copy_runs(uint8_t* const* host, const std::vector<unsigned>& idx, uint8_t* dev_block, uint64_t pitch,
              uint64_t len, bool h2d, hipStream_t stream) {
    size_t i = 0;
    while (i < idx.size()) {
        size_t j = i + 1;
        while (j < idx.size() && idx[j] == idx[j - 1] + 1 && pitch == len &&
               host[idx[j]] == host[idx[j - 1]] + len)
            ++j;
        const uint64_t bytes = uint64_t(j - i) * len;
        uint8_t* d = dev_block + uint64_t(idx[i]) * pitch;
        const hipError_t e = h2d ? hipMemcpyAsync(d, host[idx[i]], bytes, hipMemcpyHostToDevice, stream)
                                 : hipMemcpyAsync(host[idx[i]], d, bytes, hipMemcpyDeviceToHost, stream);
        if (e != hipSuccess) return SHMR_EC_DEVICE_ERROR;
        i = j;
    }
    return SHMR_EC_OK;
}

struct MappedRange {
    size_t bytes;
    uintptr_t dev;
};
// Zero-copy takes a range only when its device address equals its host
// address (unified addressing: then it is the same on every GPU of the node);
// otherwise the range stays registered (pinned, DMA'd) but is staged.
std::mutex g_mapped_mu;
std::map<uintptr_t, MappedRange>& mapped_ranges() {
    static auto* m = new std::map<uintptr_t, MappedRange>;   // leaked: outlives static teardown
    return *m;
}

// Input / output shard indices of block b of a job (the first k present
// shards in index order are the inputs, as the crate's reconstruct picks them).
void job_io(const HostJob& job, size_t b, std::vector<unsigned>& in, std::vector<unsigned>& out) {
    const unsigned k = job.codec.k(), t = k + job.codec.p();
    in.clear();
    out.clear();
    if (job.op == kEncode) {
        for (unsigned i = 0; i < k; ++i) in.push_back(i);
        for (unsigned i = k; i < t; ++i) out.push_back(i);
        return;
    }
    const uint8_t* pr = job.present + b * t;
    unsigned np = 0;
    for (unsigned i = 0; i < t; ++i) np += pr[i] ? 1 : 0;
    if (np == t) return;   // nothing to rebuild
    for (unsigned i = 0; i < t; ++i) {
        if (pr[i]) {
            if (in.size() < k) in.push_back(i);
        } else if (i < k || !job.data_only) {
            out.push_back(i);
        }
    }
}

// Translation under g_mapped_mu (held by the caller); `hint` caches the
// range of the previous hit (a batch's shards usually share one allocation).
bool translate_locked(const void* p, size_t len, uint64_t* dev, std::map<uintptr_t, MappedRange>::const_iterator* hint) {
    const auto& m = mapped_ranges();
    const uintptr_t a = uintptr_t(p);
    auto inside = [&](std::map<uintptr_t, MappedRange>::const_iterator it) {
        return a >= it->first && a - it->first <= it->second.bytes && len <= it->second.bytes - (a - it->first);
    };
    if (!p) return false;
    if (*hint == m.end() || !inside(*hint)) {
        auto it = m.upper_bound(a);
        if (it == m.begin()) return false;
        --it;
        if (!inside(it)) return false;
        *hint = it;
    }
    if ((*hint)->second.dev != (*hint)->first) return false;
    *dev = uint64_t((*hint)->second.dev + (a - (*hint)->first));
    return true;
}

// Device addresses of every shard the job touches (0 for untouched ones);
// false if any touched shard is not in mapped host memory.
bool map_job(const HostJob& job, std::vector<uint64_t>* dptrs, bool* aligned) {
    const unsigned t = job.codec.k() + job.codec.p();
    dptrs->assign(job.nblocks * t, 0);
    *aligned = true;
    std::vector<unsigned> in, out;
    std::lock_guard<std::mutex> lock(g_mapped_mu);
    if (mapped_ranges().empty()) return false;
    auto hint = mapped_ranges().cend();
    for (size_t b = 0; b < job.nblocks; ++b) {
        job_io(job, b, in, out);
        for (const auto* v : {&in, &out})
            for (unsigned i : *v) {
                uint64_t d = 0;
                if (!translate_locked(job.host_shards[b * t + i], job.len, &d, &hint)) return false;
                (*dptrs)[b * t + i] = d;
                *aligned = *aligned && (d & 15u) == 0;
            }
    }
    return true;
}

// Zero-copy: per device, the blocks' shard-pointer tables go up through the
// device's pointer ring and the kernels run on the host buffers in place.
int run_mapped(const HostJob& job, const std::vector<uint64_t>& dptrs, bool aligned, const int* devices, int ndev,
               Staging** async) {
    Codec& c = job.codec;
    const unsigned t = c.k() + c.p();
    std::vector<int> results(size_t(ndev), SHMR_EC_OK);
    auto worker = [&](int di) {
        RelaxedCapture relaxed;   // devices 1.. run on threads of their own (default mode)
        int& result = results[size_t(di)];
        const int dev = devices[di];
        DeviceScope scope(dev);
        if (!scope.ok()) {
            result = SHMR_EC_DEVICE_ERROR;
            return;
        }
        std::vector<size_t> mine;
        for (size_t b = size_t(di); b < job.nblocks; b += size_t(ndev)) mine.push_back(b);
        if (mine.empty()) return;
        int rc = SHMR_EC_OK;
        StagingLease lease;   // a pooled stream (no device buffer)
        lease.s = StagingPool::get().acquire(dev, 0, &rc);
        if (!lease.s) {
            result = rc;
            return;
        }
        const hipStream_t stream = lease.s->stream;
        UploadRing* ring = UploadRing::for_device(dev, &rc, UploadRing::kPointers);
        if (!ring) {
            result = rc;
            return;
        }
        const size_t per_chunk = UploadRing::kSlotBytes / (sizeof(uint64_t) * t);
        std::vector<uint8_t> present;
        for (size_t c0 = 0; c0 < mine.size() && rc == SHMR_EC_OK; c0 += per_chunk) {
            const size_t n = std::min(per_chunk, mine.size() - c0);
            uint8_t *hslot = nullptr, *dslot = nullptr;
            int slot = -1;
            rc = ring->acquire(&hslot, &dslot, &slot);
            if (rc) break;
            // rows in plan order (kern::ApplyArgs::shard_ptrs): reconstructs permuted per block
            uint64_t* tab = reinterpret_cast<uint64_t*>(hslot);
            for (size_t j = 0; j < n; ++j)
                permute_ptr_rows(dptrs.data() + mine[c0 + j] * t,
                                 job.op == kEncode ? nullptr : job.present + mine[c0 + j] * t, 1, c.k(), t,
                                 job.data_only, tab + j * t);
            // small launches (few 4 KiB tiles) read the table from the pinned slot
            // itself: no H2D copy in front of the kernel.  Larger ones upload it --
            // every workgroup reads its block's table, and across PCIe that costs
            // concurrent per-block calls 1-4 % of throughput.
            const uint64_t tiles = n * ((job.len + 4095) / 4096);
            const uint8_t* direct = tiles <= ptrs_direct_max() ? ring->host_view(slot) : nullptr;
            if (!direct) rc = ring->upload(slot, n * t * sizeof(uint64_t), stream);
            Layout L{nullptr, nullptr, 0, 0, 0, 0, 0};
            L.d_ptrs = reinterpret_cast<const uint64_t*>(direct ? direct : dslot);
            L.total = t;
            L.ptrs_aligned = aligned;
            L.host_mapped = true;
            if (rc == SHMR_EC_OK) {
                if (job.op == kEncode) {
                    rc = encode_on_device(c, dev, L, n, job.len, stream);
                } else {
                    present.resize(n * t);
                    for (size_t j = 0; j < n; ++j)
                        std::memcpy(present.data() + j * t, job.present + mine[c0 + j] * t, t);
                    rc = reconstruct_on_device(c, dev, L, present.data(), n, job.len, job.data_only, stream);
                }
            }
            const int rc2 = ring->release_after(slot, stream);
            if (rc == SHMR_EC_OK) rc = rc2;
        }
        if (async && rc == SHMR_EC_OK) {   // the caller waits (finish_async)
            *async = lease.s;
            lease.s = nullptr;
        } else if (sync_stream(stream) != hipSuccess && rc == SHMR_EC_OK) {
            rc = SHMR_EC_DEVICE_ERROR;
        }
        result = rc;
    };
    std::vector<std::thread> th;
    for (int d = 1; d < ndev; ++d) th.emplace_back(worker, d);
    worker(0);
    for (auto& x : th) x.join();
    for (int r : results)
        if (r) return r;
    return SHMR_EC_OK;
}

}  // namespace

namespace {
std::atomic<uint64_t> g_zero_copy_blocks{0}, g_staged_blocks{0};
}

void count_blocks(bool zero_copy, uint64_t nblocks) {
    (zero_copy ? g_zero_copy_blocks : g_staged_blocks).fetch_add(nblocks, std::memory_order_relaxed);
}

void path_stats(uint64_t* zero_copy_blocks, uint64_t* staged_blocks) {
    if (zero_copy_blocks) *zero_copy_blocks = g_zero_copy_blocks.load();
    if (staged_blocks) *staged_blocks = g_staged_blocks.load();
}

void mapped_add(const void* host, size_t bytes, const void* dev) {
    std::lock_guard<std::mutex> lock(g_mapped_mu);
    mapped_ranges()[uintptr_t(host)] = MappedRange{bytes, uintptr_t(dev)};
}

bool mapped_remove(const void* host) {
    std::lock_guard<std::mutex> lock(g_mapped_mu);
    return mapped_ranges().erase(uintptr_t(host)) != 0;
}

bool mapped_translate(const void* p, size_t len, uint64_t* dev) {
    std::lock_guard<std::mutex> lock(g_mapped_mu);
    auto hint = mapped_ranges().cend();
    return translate_locked(p, len, dev, &hint);
}

namespace {

// Pool of mapped (pinned, device-visible) bounce buffers for run_bounced_job.
class BouncePool {
public:
    static BouncePool& get() {
        static BouncePool* p = new BouncePool;   // leaked: outlives static teardown
        return *p;
    }
    uint8_t* acquire(size_t bytes) {
        {
            std::lock_guard<std::mutex> lock(mu_);
            for (size_t i = 0; i < free_.size(); ++i)
                if (free_[i].second >= bytes) {
                    uint8_t* p = free_[i].first;
                    free_.erase(free_.begin() + long(i));
                    return p;
                }
        }
        void* p = nullptr;
        RelaxedCapture relaxed;
        if (hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        void* dev = nullptr;
        if (hipHostGetDevicePointer(&dev, p, 0) != hipSuccess || dev != p) {   // zero-copy needs unified addresses
            (void)hipGetLastError();
            (void)hipHostFree(p);
            return nullptr;
        }
        mapped_add(p, bytes, dev);
        std::lock_guard<std::mutex> lock(mu_);
        size_[static_cast<uint8_t*>(p)] = bytes;
        return static_cast<uint8_t*>(p);
    }
    void release(uint8_t* p) {
        std::lock_guard<std::mutex> lock(mu_);
        if (free_.size() >= kKeep) {   // keep a bounded pool
            mapped_remove(p);
            RelaxedCapture relaxed;
            if (hipHostFree(p) != hipSuccess) (void)hipGetLastError();
            size_.erase(p);
            return;
        }
        free_.emplace_back(p, size_[p]);
    }

private:
    static constexpr size_t kKeep = 32;
    std::mutex mu_;
    std::vector<std::pair<uint8_t*, size_t>> free_;
    std::map<uint8_t*, size_t> size_;
};

}  // namespace

int run_bounced_job(const HostJob& job, int device) {
    const unsigned t = job.codec.k() + job.codec.p();
    const size_t len = job.len;
    std::vector<unsigned> in, out;
    job_io(job, 0, in, out);
    if (out.empty()) return SHMR_EC_OK;
    uint8_t* bounce = BouncePool::get().acquire(size_t(t) * len);
    if (!bounce) return SHMR_EC_OUT_OF_MEMORY;
    std::vector<uint8_t*> ptrs(t);
    for (unsigned i = 0; i < t; ++i) ptrs[i] = bounce + size_t(i) * len;
    for (unsigned i : in) std::memcpy(ptrs[i], job.host_shards[i], len);
    HostJob bj = job;
    bj.host_shards = ptrs.data();
    bool handled = false;
    int rc = run_mapped_job(bj, &device, 1, &handled, false);
    count_blocks(false, 1);
    if (rc == SHMR_EC_OK && !handled) rc = SHMR_EC_DEVICE_ERROR;
    if (rc == SHMR_EC_OK)
        for (unsigned i : out) std::memcpy(job.host_shards[i], ptrs[i], len);
    BouncePool::get().release(bounce);
    return rc;
}

int finish_async(Staging* s) {
    StagingLease lease;
    lease.s = s;
    DeviceScope scope(s->dev);
    if (!scope.ok()) return SHMR_EC_DEVICE_ERROR;
    return sync_stream(s->stream) == hipSuccess ? SHMR_EC_OK : SHMR_EC_DEVICE_ERROR;
}

bool map_rows(const HostJob& job, std::vector<uint64_t>* dptrs) {
    bool aligned = true;
    return map_job(job, dptrs, &aligned);
}

int run_mapped_job(const HostJob& job, const int* devices, int ndev, bool* handled, bool count, Staging** async) {
    *handled = false;
    if (async && ndev != 1) return SHMR_EC_INVALID_ARGUMENT;
    if (job.op == kDecode) {
        const int rc = validate_presence(job.codec, job.present, job.nblocks);
        if (rc) return rc;
    }
    std::vector<uint64_t> dptrs;
    bool aligned = true;
    if (!map_job(job, &dptrs, &aligned)) return SHMR_EC_OK;
    *handled = true;
    if (count) count_blocks(true, job.nblocks);
    return run_mapped(job, dptrs, aligned, devices, ndev, async);
}

int copy_threads_default() {
    const unsigned hw = std::thread::hardware_concurrency();
    return int(std::max(1u, std::min(8u, hw ? hw : 1u)));
}

int run_host_job(const HostJob& job, const int* devices, int ndev) {
    Codec& c = job.codec;
    const unsigned k = c.k(), t = k + c.p();
    const uint64_t len = job.len;
    const uint64_t pitch = round_up(len, 256);
    // Every block is validated before any device work starts.
    if (job.op == kDecode) {
        int rc = validate_presence(c, job.present, job.nblocks);
        if (rc) return rc;
    }
    {
        bool handled = false;
        const int rc = run_mapped_job(job, devices, ndev, &handled);
        if (handled || rc) return rc;
    }
    count_blocks(false, job.nblocks);
    const bool pinned = is_pinned(job.host_shards[0]);
    std::vector<int> results(size_t(ndev), SHMR_EC_OK);

    auto worker = [&](int di) {
        RelaxedCapture relaxed;   // devices 1.. run on threads of their own (default mode)
        int& result = results[size_t(di)];
        const int dev = devices[di];
        DeviceScope scope(dev);
        if (!scope.ok()) {
            result = SHMR_EC_DEVICE_ERROR;
            return;
        }
        std::vector<size_t> mine;
        for (size_t b = size_t(di); b < job.nblocks; b += size_t(ndev)) mine.push_back(b);
        if (mine.empty()) return;
        const uint64_t block_bytes = uint64_t(t) * pitch;
        const size_t C = std::max<size_t>(1, std::min<size_t>(mine.size(), size_t((job.chunk_bytes + block_bytes - 1) /
                                                                                     block_bytes)));
        constexpr int NS = kStageSets;
        DevicePipe& dp = pipe_for(dev);
        std::lock_guard<std::mutex> pipe_lock(dp.mu);
        StageSet* sets = dp.sets;
        auto cleanup = [&] {
            for (int i = 0; i < NS; ++i)
                if (sets[i].stream) (void)hipStreamSynchronize(sets[i].stream);
        };
        {
            const int rc = dp.ensure(dev, C * block_bytes, pinned ? 0 : C * block_bytes);
            if (rc) {
                result = rc;
                return;
            }
        }
        CopyCrew crew(pinned ? 1 : job.copy_threads);
        std::vector<CopyCrew::Task> tasks;
        std::vector<uint8_t> present;

        // input / output shard indices of one block
        auto io = [&](size_t b, std::vector<unsigned>& in, std::vector<unsigned>& out) { job_io(job, b, in, out); };
        std::vector<unsigned> in, out;
        // staged mode: pinned mirror -> user output buffers of a finished chunk
        auto drain = [&](StageSet& s) -> int {
            if (!s.pending) return SHMR_EC_OK;
            if (hipEventSynchronize(s.done) != hipSuccess) return SHMR_EC_DEVICE_ERROR;
            s.pending = false;
            if (pinned) return SHMR_EC_OK;
            tasks.clear();
            for (size_t j = 0; j < s.blocks.size(); ++j) {
                io(s.blocks[j], in, out);
                for (unsigned i : out)
                    tasks.push_back({job.host_shards[s.blocks[j] * t + i], s.hbuf + (j * t + i) * pitch, len});
            }
            crew.run(tasks);
            return SHMR_EC_OK;
        };

        size_t chunk = 0;
        for (size_t c0 = 0; c0 < mine.size(); c0 += C, ++chunk) {
            StageSet& s = sets[chunk % NS];
            int rc = drain(s);
            if (rc) {
                result = rc;
                break;
            }
            const size_t n = std::min(C, mine.size() - c0);
            s.blocks.assign(mine.begin() + long(c0), mine.begin() + long(c0 + n));
            // gather inputs (pageable: into the pinned mirror first)
            if (!pinned) {
                tasks.clear();
                for (size_t j = 0; j < n; ++j) {
                    io(s.blocks[j], in, out);
                    for (unsigned i : in)
                        tasks.push_back({s.hbuf + (j * t + i) * pitch, job.host_shards[s.blocks[j] * t + i], len});
                }
                crew.run(tasks);
            }
            // Pageable mode with a unified mirror: the kernel codes the mirror in
            // place across PCIe (zero-copy) -- no H2D / D2H copies.
            const bool zc = !pinned && s.hbuf_unified && mirror_zero_copy();
            for (size_t j = 0; j < n && rc == SHMR_EC_OK && !zc; ++j) {
                io(s.blocks[j], in, out);
                if (job.op == kEncode && !pinned) {   // k data shards are contiguous in the mirror
                    if (hipMemcpyAsync(s.dbuf + j * block_bytes, s.hbuf + j * block_bytes, (k - 1) * pitch + len,
                                       hipMemcpyHostToDevice, s.stream) != hipSuccess)
                        rc = SHMR_EC_DEVICE_ERROR;
                    continue;
                }
                if (pinned) {
                    rc = copy_runs(job.host_shards + s.blocks[j] * t, in, s.dbuf + j * block_bytes, pitch, len, true,
                                   s.stream);
                    continue;
                }
                for (unsigned i : in) {
                    if (hipMemcpyAsync(s.dbuf + (j * t + i) * pitch, s.hbuf + (j * t + i) * pitch, len,
                                       hipMemcpyHostToDevice, s.stream) != hipSuccess)
                        rc = SHMR_EC_DEVICE_ERROR;
                }
            }
            // compute
            if (rc == SHMR_EC_OK) {
                uint8_t* base = zc ? s.hbuf : s.dbuf;
                Layout L{base, base, block_bytes, pitch, block_bytes, pitch, 0};
                L.host_mapped = zc;
                if (job.op == kEncode) {
                    rc = encode_on_device(c, dev, L, n, len, s.stream);
                } else {
                    present.assign(n * t, 1);
                    for (size_t j = 0; j < n; ++j)
                        std::memcpy(present.data() + j * t, job.present + s.blocks[j] * t, t);
                    rc = reconstruct_on_device(c, dev, L, present.data(), n, len, job.data_only, s.stream);
                }
            }
            // outputs
            for (size_t j = 0; j < n && rc == SHMR_EC_OK && !zc; ++j) {
                io(s.blocks[j], in, out);
                if (job.op == kEncode && !pinned) {   // p parity shards are contiguous too
                    if (hipMemcpyAsync(s.hbuf + (j * t + k) * pitch, s.dbuf + (j * t + k) * pitch,
                                       (t - k - 1) * pitch + len, hipMemcpyDeviceToHost, s.stream) != hipSuccess)
                        rc = SHMR_EC_DEVICE_ERROR;
                    continue;
                }
                if (pinned) {
                    rc = copy_runs(job.host_shards + s.blocks[j] * t, out, s.dbuf + j * block_bytes, pitch, len,
                                   false, s.stream);
                    continue;
                }
                for (unsigned i : out) {
                    if (hipMemcpyAsync(s.hbuf + (j * t + i) * pitch, s.dbuf + (j * t + i) * pitch, len,
                                       hipMemcpyDeviceToHost, s.stream) != hipSuccess)
                        rc = SHMR_EC_DEVICE_ERROR;
                }
            }
            if (rc == SHMR_EC_OK && hipEventRecord(s.done, s.stream) != hipSuccess) rc = SHMR_EC_DEVICE_ERROR;
            s.pending = rc == SHMR_EC_OK;
            if (rc) {
                result = rc;
                break;
            }
        }
        for (int i = 0; i < NS; ++i) {
            const int rc = drain(sets[i]);
            if (rc && result == SHMR_EC_OK) result = rc;
        }
        cleanup();
    };

    std::vector<std::thread> th;
    for (int d = 1; d < ndev; ++d) th.emplace_back(worker, d);
    worker(0);
    for (auto& x : th) x.join();
    for (int r : results)
        if (r) return r;
    return SHMR_EC_OK;
}

}  // namespace core
}  // namespace shmr
