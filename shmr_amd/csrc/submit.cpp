// Submission queue: concurrent per-block calls merged into batch launches (see
// submit.hpp).
//
// Completion: after a batch's kernels the queue's stream runs a one-wave mark
// kernel that stores the batch's sequence number into a pinned host word
// (kern::launch_mark, a system-scope release store).  A waiting caller spins
// on that word -- a plain load, no HIP call, no lock -- for "coalesce_spin_us"
// and then sleeps on a condition.  One watcher thread per queue follows the
// oldest batch in flight (spinning on the word for "coalesce_watch_us", then
// asleep in hipEventSynchronize on a blocking-sync event recorded behind the
// mark), wakes the sleepers when it completes, and
// launches what was held back for merging -- so no caller's thread is spent
// on other callers' completions.
#include "submit.hpp"

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <thread>
#include <tuple>

#include "gf_apply.hpp"

namespace shmr {
namespace core {

namespace {

using Clock = std::chrono::steady_clock;

std::atomic<int> g_coalesce{0};      // host-buffer entry points on mapped memory through the queue
std::atomic<int> g_depth{1};         // batches in flight before pending calls wait to merge
std::atomic<int> g_target{64};       // ... unless this many are pending (a launch of its own)
std::atomic<int> g_window_us{0};     // an idle queue's launch waits this long for more calls
std::atomic<int> g_max{1024};        // blocks per launch
std::atomic<int> g_spin_us{30};      // a waiter spins this long before it sleeps
std::atomic<int> g_watch_us{200};    // the watcher spins this long before it sleeps on the event
std::atomic<int> g_mark{1};          // 1: a mark kernel advances the word; 0: the watcher does, from the event
constexpr int kDepthDefault = 1, kTargetDefault = 64, kWindowDefault = 0, kMaxDefault = 1024, kSpinDefault = 30,
              kWatchDefault = 200;

constexpr int kMaxQueues = 64;   // device IDs (ec_core kMaxDevIds)
enum { kReqs = 0, kBatches, kMaxBatch, kSleeps, kStatCount };
std::atomic<uint64_t> g_stats[kMaxQueues][kStatCount];

inline void cpu_relax() { __builtin_ia32_pause(); }

class Queue {
public:
    explicit Queue(int dev) : dev_(dev) {}

    int init() {
        RelaxedCapture relaxed;
        int rc = device_init(dev_, nullptr);
        if (rc) return rc;
        DeviceScope scope(dev_);
        if (!scope.ok()) return SHMR_EC_DEVICE_ERROR;
        if (create_priority_stream(&stream_) != hipSuccess) {
            (void)hipGetLastError();
            return SHMR_EC_DEVICE_ERROR;
        }
        void* w = nullptr;
        if (hipHostMalloc(&w, 64, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess) {
            (void)hipGetLastError();
            return SHMR_EC_OUT_OF_MEMORY;
        }
        void* dw = nullptr;
        if (hipHostGetDevicePointer(&dw, w, 0) != hipSuccess || !dw) {
            (void)hipGetLastError();
            return SHMR_EC_DEVICE_ERROR;
        }
        word_ = static_cast<uint64_t*>(w);
        dword_ = static_cast<uint64_t*>(dw);
        __atomic_store_n(word_, 0, __ATOMIC_RELEASE);
        register_own_stream(stream_);
        count_device(dev_, kDevStagingStreams);
        std::thread([this] { watch(); }).detach();   // lives with the (leaked) queue
        return SHMR_EC_OK;
    }

    void submit(SubmitReq* r) {
        g_stats[dev_][kReqs].fetch_add(1, std::memory_order_relaxed);
        std::unique_lock<std::mutex> lk(mu_);
        if (pending_.empty()) first_arrival_ = Clock::now();
        pending_.push_back(r);
        pump(lk);
        lk.unlock();
        cv_work_.notify_one();
    }

    int wait(SubmitReq* r) {
        if (!r->seq.load(std::memory_order_acquire) && !r->done.load(std::memory_order_acquire)) {
            // waited for before it was launched (held back to merge): nothing
            // else may come to merge with it -- launch what is pending now
            std::unique_lock<std::mutex> lk(mu_);
            pump(lk, true);
        }
        const auto t0 = Clock::now();
        const auto spin = std::chrono::microseconds(g_spin_us.load(std::memory_order_relaxed));
        for (uint32_t i = 0;; ++i) {   // spin on the host word
            if (finished(r)) return result(r);
            if ((i & 63) == 63 && Clock::now() - t0 >= spin) break;
            cpu_relax();
        }
        std::unique_lock<std::mutex> lk(mu_);   // sleep: the watcher wakes us
        cv_done_.wait(lk, [&] { return finished(r); });
        return result(r);
    }

private:
    struct Batch {
        uint64_t seq = 0;
        hipEvent_t ev = nullptr;
    };

    uint64_t completed() const { return __atomic_load_n(word_, __ATOMIC_ACQUIRE); }
    // The host's own advance of the word (knob coalesce_mark=0; only the
    // watcher writes it then, in launch order).
    void advance(uint64_t seq) {
        if (completed() < seq) __atomic_store_n(word_, seq, __ATOMIC_RELEASE);
    }

    bool finished(const SubmitReq* r) const {
        if (r->done.load(std::memory_order_acquire)) return true;   // failed launch, or a broken queue
        const uint64_t s = r->seq.load(std::memory_order_acquire);
        return (s && completed() >= s) || broken_.load(std::memory_order_acquire);
    }

    // A finished request's status: its own, or DEVICE_ERROR when the queue
    // broke before its batch completed.
    int result(const SubmitReq* r) const {
        if (r->done.load(std::memory_order_acquire)) return r->rc;
        const uint64_t s = r->seq.load(std::memory_order_acquire);
        return (s && completed() >= s) ? r->rc : SHMR_EC_DEVICE_ERROR;
    }

    // Drops finished batches (their events back to the pool).  mu_ held.
    void reap() {
        const uint64_t c = completed();
        while (!inflight_.empty() && inflight_.front().seq <= c) {
            if (inflight_.front().ev) events_.push_back(inflight_.front().ev);
            inflight_.pop_front();
        }
    }

    // Launches pending requests: at once while fewer than `depth` batches are
    // in flight, or when `target` requests are pending; otherwise they wait
    // (and merge) until a batch completes.  One launcher at a time.  mu_ held.
    // force: launch whatever is pending (a caller waits for a held-back call).
    void pump(std::unique_lock<std::mutex>& lk, bool force = false) {
        for (;;) {
            if (launching_ || pending_.empty()) return;
            reap();
            const size_t depth = size_t(std::max(1, g_depth.load(std::memory_order_relaxed)));
            const size_t target = size_t(std::max(1, g_target.load(std::memory_order_relaxed)));
            if (!force && inflight_.size() >= depth && pending_.size() < target) return;
            force = false;
            const size_t maxn = size_t(std::max(1, g_max.load(std::memory_order_relaxed)));
            const int window = g_window_us.load(std::memory_order_relaxed);
            launching_ = true;
            if (window > 0 && inflight_.empty() && pending_.size() < maxn) {
                const auto until = first_arrival_ + std::chrono::microseconds(window);
                if (Clock::now() < until) {   // an idle queue: give other callers the window
                    lk.unlock();
                    while (Clock::now() < until) std::this_thread::yield();
                    lk.lock();
                }
            }
            const size_t n = std::min(maxn, pending_.size());
            take_.assign(pending_.begin(), pending_.begin() + long(n));
            pending_.erase(pending_.begin(), pending_.begin() + long(n));
            if (!pending_.empty()) first_arrival_ = Clock::now();
            const uint64_t seq = ++launched_;
            hipEvent_t ev = nullptr;   // (a blocking-sync event from the pool, or made by launch)
            if (!events_.empty()) {
                ev = events_.back();
                events_.pop_back();
            }
            lk.unlock();
            const bool queued = launch(take_, seq, &ev);
            lk.lock();
            launching_ = false;
            if (queued) {
                inflight_.push_back(Batch{seq, ev});
                cv_work_.notify_one();
            } else {   // nothing left running (failed and drained): every status is final
                if (ev) events_.push_back(ev);
                for (SubmitReq* q : take_) q->done.store(1, std::memory_order_release);
                cv_done_.notify_all();
            }
            take_.clear();
        }
    }

    // Enqueues one batch on the queue's stream: one pointer-table call per
    // group of compatible requests, the completion mark, the batch's event.
    // A group's error is its requests' status.  false: nothing will mark the
    // batch (every status is final; the stream is drained).
    bool launch(std::vector<SubmitReq*>& reqs, uint64_t seq, hipEvent_t* ev) {
        RelaxedCapture relaxed;
        DeviceScope scope(dev_);
        if (!scope.ok()) {
            for (SubmitReq* q : reqs) q->rc = SHMR_EC_DEVICE_ERROR;
            return false;
        }
        using Key = std::tuple<const Codec*, int, bool, bool, uint64_t>;
        std::map<Key, std::vector<SubmitReq*>> groups;
        for (SubmitReq* q : reqs) {
            groups[Key{q->codec.get(), int(q->op), q->data_only, q->host_mapped, q->len}].push_back(q);
            q->seq.store(seq, std::memory_order_release);   // the mark for seq comes after its kernels
        }
        for (auto& g : groups) {
            std::vector<SubmitReq*>& v = g.second;
            Codec& c = *v[0]->codec;
            const unsigned t = c.k() + c.p();
            const size_t n = v.size();
            tab_.resize(n * t);
            for (size_t b = 0; b < n; ++b) std::memcpy(&tab_[b * t], v[b]->row.data(), t * sizeof(uint64_t));
            if (v[0]->op == kDecode) {
                present_.resize(n * t);
                for (size_t b = 0; b < n; ++b) std::memcpy(&present_[b * t], v[b]->present.data(), t);
            }
            int rc;
            try {
                rc = ptrs_launch(c, tab_.data(), v[0]->op == kDecode ? present_.data() : nullptr, n, v[0]->len,
                                 v[0]->data_only, dev_, stream_, v[0]->op, v[0]->host_mapped, false);
            } catch (const std::bad_alloc&) {
                rc = SHMR_EC_OUT_OF_MEMORY;
            } catch (...) {
                rc = SHMR_EC_DEVICE_ERROR;
            }
            if (rc)
                for (SubmitReq* q : v) q->rc = rc;
        }
        g_stats[dev_][kBatches].fetch_add(1, std::memory_order_relaxed);
        uint64_t m = g_stats[dev_][kMaxBatch].load(std::memory_order_relaxed);
        while (reqs.size() > m && !g_stats[dev_][kMaxBatch].compare_exchange_weak(m, reqs.size())) {
        }
        const bool mark = g_mark.load(std::memory_order_relaxed) != 0;
        if (!mark) {   // the watcher advances the word once the batch's event completes
            if (!*ev && hipEventCreateWithFlags(ev, hipEventDisableTiming | hipEventBlockingSync) != hipSuccess) {
                (void)hipGetLastError();
                *ev = nullptr;
            }
            if (*ev && hipEventRecord(*ev, stream_) == hipSuccess) return true;
            (void)hipGetLastError();
            if (hipStreamSynchronize(stream_) != hipSuccess) {   // no event: drained, statuses final
                (void)hipGetLastError();
                broken_.store(true, std::memory_order_release);
            }
            for (SubmitReq* q : reqs)
                if (q->rc == SHMR_EC_OK) q->rc = SHMR_EC_DEVICE_ERROR;
            return false;
        }
        if (kern::launch_mark(dword_, seq, stream_) != hipSuccess) {
            (void)hipGetLastError();
            // no mark: drain the stream so no request completes early
            if (hipStreamSynchronize(stream_) != hipSuccess) {
                (void)hipGetLastError();
                broken_.store(true, std::memory_order_release);
            }
            for (SubmitReq* q : reqs)
                if (q->rc == SHMR_EC_OK) q->rc = SHMR_EC_DEVICE_ERROR;
            return false;
        }
        // From here on the batch's waiters may return (and free their
        // requests) at any moment: nothing below touches them.  The event
        // (recorded behind the mark) lets the watcher sleep instead of spin;
        // without one it follows the word only.
        if (!*ev && hipEventCreateWithFlags(ev, hipEventDisableTiming | hipEventBlockingSync) != hipSuccess) {
            (void)hipGetLastError();
            *ev = nullptr;
        }
        if (*ev && hipEventRecord(*ev, stream_) != hipSuccess) {
            (void)hipGetLastError();
            (void)hipEventDestroy(*ev);
            *ev = nullptr;
        }
        return true;
    }

    // The watcher: follows the oldest batch in flight -- the host word, then
    // (after coalesce_watch_us) hipEventSynchronize on its event; an error
    // there means the device failed: the queue is broken and every waiter
    // returns DEVICE_ERROR -- wakes the sleeping callers when it completes, and
    // launches what pump() held back.
    void watch() {
        RelaxedCapture relaxed;
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_work_.wait(lk, [&] { return !inflight_.empty() || (!pending_.empty() && !launching_); });
            pump(lk);
            if (inflight_.empty()) continue;
            const uint64_t target = inflight_.front().seq;
            const hipEvent_t ev = inflight_.front().ev;
            lk.unlock();
            const auto t0 = Clock::now();
            const auto spin = std::chrono::microseconds(g_watch_us.load(std::memory_order_relaxed));
            bool seen = false;
            for (uint32_t i = 0;; ++i) {
                if (completed() >= target) {
                    seen = true;
                    break;
                }
                if (ev && !g_mark.load(std::memory_order_relaxed) && (i & 15) == 15) {   // no mark kernel:
                    const hipError_t q = hipEventQuery(ev);                               // poll the event
                    if (q == hipSuccess) {
                        advance(target);
                        seen = true;
                        break;
                    }
                    if (q != hipErrorNotReady) {
                        (void)hipGetLastError();
                        break;   // (the blocking wait below reports it)
                    }
                    (void)hipGetLastError();
                }
                if ((i & 255) == 255 && Clock::now() - t0 >= spin) break;
                cpu_relax();
            }
            if (!seen && ev) {   // sleep until the GPU signals the event (behind the mark)
                DeviceScope scope(dev_);
                if (hipEventSynchronize(ev) != hipSuccess) {
                    (void)hipGetLastError();
                    broken_.store(true, std::memory_order_release);
                } else if (!g_mark.load(std::memory_order_relaxed)) {
                    advance(target);
                }
                g_stats[dev_][kSleeps].fetch_add(1, std::memory_order_relaxed);
            }
            lk.lock();
            reap();
            lk.unlock();
            cv_done_.notify_all();
            lk.lock();
            if (broken_.load(std::memory_order_acquire)) {   // nothing will complete: release everyone
                for (SubmitReq* q : pending_) {
                    q->rc = SHMR_EC_DEVICE_ERROR;
                    q->done.store(1, std::memory_order_release);
                }
                pending_.clear();
                while (!inflight_.empty()) inflight_.pop_front();
                cv_done_.notify_all();
            }
        }
    }

    const int dev_;
    hipStream_t stream_ = nullptr;
    uint64_t* word_ = nullptr;    // completion mark (host view)
    uint64_t* dword_ = nullptr;   // ... its device address
    std::mutex mu_;
    std::condition_variable cv_work_, cv_done_;
    std::vector<SubmitReq*> pending_, take_;
    std::deque<Batch> inflight_;
    std::vector<hipEvent_t> events_;
    std::vector<uint64_t> tab_;
    std::vector<uint8_t> present_;
    uint64_t launched_ = 0;
    bool launching_ = false;
    std::atomic<bool> broken_{false};
    Clock::time_point first_arrival_{};
};

std::mutex g_queues_mu;
std::atomic<Queue*> g_queues[kMaxQueues];   // leaked: waiters may outlive static teardown

Queue* queue_for(int dev, int* rc) {
    if (dev < 0 || dev >= kMaxQueues) {
        *rc = SHMR_EC_INVALID_ARGUMENT;
        return nullptr;
    }
    *rc = SHMR_EC_OK;
    if (Queue* q = g_queues[dev].load(std::memory_order_acquire)) return q;
    std::lock_guard<std::mutex> lock(g_queues_mu);
    if (Queue* q = g_queues[dev].load(std::memory_order_acquire)) return q;
    auto* q = new Queue(dev);
    *rc = q->init();
    if (*rc) {
        delete q;   // (its stream and word, if made, are abandoned: a failing device)
        return nullptr;
    }
    g_queues[dev].store(q, std::memory_order_release);
    return q;
}

}  // namespace

int submit(SubmitReq* r) {
    int rc = SHMR_EC_OK;
    Queue* q = queue_for(r->dev, &rc);
    if (!q) return rc;
    q->submit(r);
    return SHMR_EC_OK;
}

int wait(SubmitReq* r) {
    int rc = SHMR_EC_OK;
    Queue* q = queue_for(r->dev, &rc);
    if (!q) return rc;
    return q->wait(r);
}

bool coalesce_host() { return g_coalesce.load(std::memory_order_relaxed) != 0; }

int set_submit_tuning(const std::string& key, int value, bool* known) {
    *known = true;
    auto set = [&](std::atomic<int>& v, int dflt, int lo, int hi) {
        if (value == kAuto) value = dflt;
        if (value < lo || value > hi) return SHMR_EC_INVALID_ARGUMENT;
        v = value;
        return SHMR_EC_OK;
    };
    if (key == "coalesce") return set(g_coalesce, 0, 0, 1);
    if (key == "coalesce_depth") return set(g_depth, kDepthDefault, 1, 64);
    if (key == "coalesce_target") return set(g_target, kTargetDefault, 1, 65536);
    if (key == "coalesce_us") return set(g_window_us, kWindowDefault, 0, 100000);
    if (key == "coalesce_max") return set(g_max, kMaxDefault, 1, 65536);
    if (key == "coalesce_spin_us") return set(g_spin_us, kSpinDefault, 0, 10000000);
    if (key == "coalesce_watch_us") return set(g_watch_us, kWatchDefault, 0, 10000000);
    if (key == "coalesce_mark") return set(g_mark, 1, 0, 1);
    *known = false;
    return SHMR_EC_INVALID_ARGUMENT;
}

int get_submit_tuning(const std::string& key, bool* known) {
    *known = true;
    if (key == "coalesce") return g_coalesce;
    if (key == "coalesce_depth") return g_depth;
    if (key == "coalesce_target") return g_target;
    if (key == "coalesce_us") return g_window_us;
    if (key == "coalesce_max") return g_max;
    if (key == "coalesce_spin_us") return g_spin_us;
    if (key == "coalesce_watch_us") return g_watch_us;
    if (key == "coalesce_mark") return g_mark;
    *known = false;
    return SHMR_EC_INVALID_ARGUMENT;
}

void submit_stats(int dev, uint64_t* out, size_t n) {
    for (size_t i = 0; i < n && i < size_t(kStatCount); ++i)
        out[i] = (dev >= 0 && dev < kMaxQueues) ? g_stats[dev][i].load() : 0;
}

}  // namespace core
}  // namespace shmr
