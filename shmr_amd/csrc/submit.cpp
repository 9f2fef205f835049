// Submission queue: concurrent per-block calls merged into batch launches (see
// submit.hpp).
//
// Submission: a call puts its request into the queue's inbox, a ring of
// request pointers (one fetch_add; r06 s13: 16 threads on one mutex convoyed,
// the aggregate submission rate fell below one thread's), and wakes the watcher
// if it sleeps.  The callers' threads make no HIP call: the queue's watcher
// thread is its one launcher (r06 s15-s23: a thread's first HIP calls cost
// tens of microseconds, and new callers' first calls queued behind each
// other in the runtime while every block waited).  It launches at once when
// nothing is in flight (or `coalesce_depth` allows more, or `coalesce_target`
// calls are pending, or a caller waits for a call not yet launched);
// otherwise calls wait to merge.  A launch drains the inbox, groups the
// requests and enqueues them.
//
// Completion: after a batch's kernels the queue's stream runs a one-wave mark
// kernel that stores the batch's sequence number into a pinned host word
// (kern::launch_mark, a system-scope release store).  A waiting caller spins
// on that word -- a plain load, no HIP call, no lock -- for "coalesce_spin_us"
// and then sleeps on a condition.  One watcher thread per queue follows the
// oldest batch in flight (spinning on the word for "coalesce_watch_us", then
// asleep in hipEventSynchronize on a blocking-sync event recorded behind the
// mark), wakes the sleepers when it completes, and launches what was held
// back for merging: `coalesce_lead_us` before the running batch's estimated
// end (its bytes at a nominal rate), so that batch's successor is already
// queued on the stream when it finishes, or at its completion.
#include "submit.hpp"

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <thread>
#include <tuple>

#include "gf_apply.hpp"

namespace shmr {
namespace core {

namespace {

using Clock = std::chrono::steady_clock;

std::atomic<int> g_coalesce{0};      // host-buffer entry points on mapped memory through the queue
std::atomic<int> g_depth{1};         // batches in flight the watcher adds to at once
std::atomic<int> g_target{64};       // ... or this many pending calls launch anyway
std::atomic<int> g_window_us{0};     // an idle queue's launch waits this long for more calls
std::atomic<int> g_max{1024};        // blocks per launch
std::atomic<int> g_spin_us{30};      // a waiter spins this long before it sleeps
std::atomic<int> g_watch_us{200};    // the watcher spins this long before it sleeps on the event
std::atomic<int> g_mark{1};          // 1: a mark kernel advances the word; 0: the watcher does, from the event
std::atomic<int> g_lead_us{30};      // the watcher's early launch, before the running batch's estimated end
std::atomic<int> g_idle_us{1000};    // the watcher spins this long for calls on an idle queue before it sleeps
constexpr int kDepthDefault = 1, kTargetDefault = 64, kWindowDefault = 0, kMaxDefault = 1024, kSpinDefault = 30,
              kWatchDefault = 200, kLeadDefault = 30, kIdleDefault = 1000;
constexpr int kMaxInflight = 8;      // batches on the stream, whatever the target rule says
// A batch's estimated GPU time: a launch's fixed cost plus its algorithmic
// bytes at a nominal rate (device memory; mapped host memory crosses PCIe).
constexpr int64_t kFixedNs = 5000;
constexpr double kDevBytesPerNs = 6400.0;   // 6.4 TB/s = 6,400 bytes per ns
constexpr double kHostBytesPerNs = 50.0;     // 50 GB/s = 50 bytes per ns

constexpr int kMaxQueues = 64;   // device IDs (ec_core kMaxDevIds)
enum { kReqs = 0, kBatches, kMaxBatch, kSleeps, kAhead, kStatCount };
std::atomic<uint64_t> g_stats[kMaxQueues][kStatCount];

inline void cpu_relax() { __builtin_ia32_pause(); }

// Diagnostic event log (environment SHMR_QUEUE_TRACE=1; printed to stderr at
// exit): launches (start, end, mode, blocks, batches in flight) and the
// watcher's completions, microseconds from the first event.
struct TraceEv {
    int64_t t0, t1;
    int kind, mode, n, f;
};
struct Trace {
    bool on = std::getenv("SHMR_QUEUE_TRACE") != nullptr;
    std::mutex mu;
    std::vector<TraceEv> ev;
    void add(int kind, int mode, int n, int f, int64_t t0, int64_t t1) {
        if (!on) return;
        std::lock_guard<std::mutex> lk(mu);
        if (ev.size() < 200000) ev.push_back(TraceEv{t0, t1, kind, mode, n, f});
    }
    ~Trace() {
        if (!on || ev.empty()) return;
        const int64_t base = ev.front().t0;
        std::fprintf(stderr, "QTRACE base_ns=%lld\n", (long long)base);
        for (const TraceEv& e : ev)
            std::fprintf(stderr, "QTRACE %s mode=%d n=%d f=%d t0=%.1f t1=%.1f\n",
                         e.kind == 0 ? "launch" : e.kind == 1 ? "reaped" : e.kind == 3 ? "phase" : "other", e.mode, e.n, e.f,
                         double(e.t0 - base) / 1e3, double(e.t1 - base) / 1e3);
    }
};
Trace g_trace;
inline int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count();
}

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
        if (queued_.fetch_add(1, std::memory_order_seq_cst) == 0 && g_window_us.load(std::memory_order_relaxed) > 0)
            first_arrival_ns_.store(now_ns(), std::memory_order_relaxed);
        const uint64_t t = tail_.fetch_add(1, std::memory_order_seq_cst);
        while (t - head_pub_.load(std::memory_order_acquire) >= kRing) std::this_thread::yield();   // full (rare)
        ring_[t & (kRing - 1)].store(r, std::memory_order_seq_cst);
        wake_watcher();
    }

    int wait(SubmitReq* r) {
        // waited for before it was launched (held back to merge): nothing else
        // may come to merge with it -- the watcher launches what is pending
        // now; wait for that launch (briefly spinning, then asleep)
        for (uint32_t i = 0; !launched(r); ++i) {
            if (i == 0 || (i >= 64 && (i & 7) == 0)) {
                force_.store(true, std::memory_order_seq_cst);
                wake_watcher();
            }
            if (i < 64) {
                cpu_relax();
                continue;
            }
            forced_waiters_.fetch_add(1, std::memory_order_seq_cst);
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_done_.wait_for(lk, std::chrono::microseconds(500), [&] { return launched(r); });
            }
            forced_waiters_.fetch_sub(1, std::memory_order_seq_cst);
        }
        const auto t0 = Clock::now();
        const auto spin = std::chrono::microseconds(g_spin_us.load(std::memory_order_relaxed));
        for (uint32_t i = 0;; ++i) {   // spin on the host word
            if (finished(r)) return result(r);
            if ((i & 63) == 63 && Clock::now() - t0 >= spin) break;
            cpu_relax();
        }
        {
            std::unique_lock<std::mutex> lk(mu_);   // sleep: the watcher wakes us
            cv_done_.wait(lk, [&] { return finished(r); });
        }
        return result(r);
    }

private:
    enum Mode { kForced, kByWatcher };
    struct Batch {
        uint64_t seq = 0;
        hipEvent_t ev = nullptr;
        int64_t est_end_ns = 0;
    };

    // A caller's work for the watcher (a call pushed, a launch forced): wake
    // it if it sleeps.  (sleeping_ is set before the watcher's last look
    // under imu_, and read here after the caller's own store: one of the
    // two sees the other.)
    void wake_watcher() {
        if (!sleeping_.load(std::memory_order_seq_cst)) return;
        { std::lock_guard<std::mutex> lk(imu_); }
        cv_work_.notify_one();
    }

    uint64_t completed() const { return __atomic_load_n(word_, __ATOMIC_ACQUIRE); }
    // The host's own advance of the word (knob coalesce_mark=0; only the
    // watcher writes it then, in launch order).
    void advance(uint64_t seq) {
        if (completed() < seq) __atomic_store_n(word_, seq, __ATOMIC_RELEASE);
    }

    bool launched(const SubmitReq* r) const {
        return r->seq.load(std::memory_order_acquire) || r->done.load(std::memory_order_acquire) ||
               broken_.load(std::memory_order_acquire);
    }
    bool finished(const SubmitReq* r) const {
        if (r->done.load(std::memory_order_acquire)) return true;   // failed launch
        const uint64_t s = r->seq.load(std::memory_order_acquire);
        return (s && completed() >= s) || broken_.load(std::memory_order_acquire);
    }

    // A finished request's status: its own, or DEVICE_ERROR when the queue
    // broke before its batch completed.
    // (A request the queue still holds -- the launcher's, when the queue broke
    // under it -- is returned only after the launcher let go: the caller
    // frees it next.)
    int result(const SubmitReq* r) const {
        if (r->done.load(std::memory_order_acquire)) return r->rc;
        const uint64_t s = r->seq.load(std::memory_order_acquire);
        if (s && completed() >= s) return r->rc;
        while (launching_.load(std::memory_order_acquire)) std::this_thread::yield();
        return SHMR_EC_DEVICE_ERROR;
    }

    // Whether a launcher of this kind should take the pending calls now.
    bool wanted(Mode mode) const {
        if (broken_.load(std::memory_order_acquire)) return false;
        const int64_t q = queued_.load(std::memory_order_seq_cst);
        if (q <= 0) return false;
        if (mode == kForced) return true;
        const int f = inflight_n_.load(std::memory_order_seq_cst);
        if (f == 0) return true;
        if (f < std::max(1, g_depth.load(std::memory_order_relaxed))) return true;
        if (q >= std::max(1, g_target.load(std::memory_order_relaxed)) && f < kMaxInflight) return true;
        return mode == kByWatcher && f == 1 && now_ns() >= ahead_at_ns_.load(std::memory_order_relaxed);
    }

    // Launches the pending calls while `wanted` (the watcher only: callers'
    // threads make no HIP call -- r06 s15/s23: a thread's first HIP calls
    // cost tens of microseconds, and 16-32 new threads' first calls queued
    // behind each other in the runtime for up to 0.5 ms while every
    // caller's block waited).  launching_ marks the launch in progress.
    void launch_some(Mode mode) {
        while (wanted(mode)) {
            if (launching_.exchange(true, std::memory_order_seq_cst)) return;
            const int f = inflight_n_.load(std::memory_order_seq_cst);
            const int window = g_window_us.load(std::memory_order_relaxed);
            if (mode != kForced && f == 0 && window > 0) {   // an idle queue: give other callers the window
                const int64_t until = first_arrival_ns_.load(std::memory_order_relaxed) + int64_t(window) * 1000;
                while (now_ns() < until && queued_.load(std::memory_order_relaxed) < g_max.load())
                    std::this_thread::yield();
            }
            if (wanted(mode)) {
                if (mode == kByWatcher && f == 1 &&
                    queued_.load(std::memory_order_relaxed) < std::max(1, g_target.load(std::memory_order_relaxed)) &&
                    g_depth.load(std::memory_order_relaxed) <= 1)   // (not the target or depth rule)
                    g_stats[dev_][kAhead].fetch_add(1, std::memory_order_relaxed);
                const int64_t ta = g_trace.on ? now_ns() : 0;
                const int64_t qa = queued_.load(std::memory_order_relaxed);
                launch_pending();
                if (g_trace.on) g_trace.add(0, int(mode), int(qa), f, ta, now_ns());
            }
            launching_.store(false, std::memory_order_seq_cst);
            if (forced_waiters_.load(std::memory_order_seq_cst) > 0) {   // callers asleep in wait() for a launch
                { std::lock_guard<std::mutex> lk(mu_); }
                cv_done_.notify_all();
            }
            if (mode == kForced) mode = kByWatcher;   // one forced launch; then the usual rule
        }
    }

    // Takes up to coalesce_max pending calls and enqueues them.  launching_ held.
    void launch_pending() {
        // the inbox in arrival order, up to the first slot whose caller has
        // taken its index but not yet stored (it comes with the next launch)
        for (;;) {
            std::atomic<SubmitReq*>& slot = ring_[head_ & (kRing - 1)];
            SubmitReq* r = slot.load(std::memory_order_acquire);
            if (!r) break;
            slot.store(nullptr, std::memory_order_relaxed);
            pending_.push_back(r);
            ++head_;
        }
        head_pub_.store(head_, std::memory_order_release);
        if (pending_.empty()) return;
        const size_t maxn = size_t(std::max(1, g_max.load(std::memory_order_relaxed)));
        const size_t n = std::min(maxn, pending_.size());
        take_.assign(pending_.begin(), pending_.begin() + long(n));
        pending_.erase(pending_.begin(), pending_.begin() + long(n));
        queued_.fetch_sub(int64_t(n), std::memory_order_seq_cst);
        const uint64_t seq = ++launched_;
        double bytes_ns = 0;   // the batch's estimated GPU time
        for (const SubmitReq* q : take_) bytes_ns += q->est_ns;
        hipEvent_t ev = nullptr;   // (a blocking-sync event from the pool, or made by launch)
        {
            std::lock_guard<std::mutex> lk(imu_);
            if (!events_.empty()) {
                ev = events_.back();
                events_.pop_back();
            }
        }
        const bool queued = launch(take_, seq, &ev);
        const int64_t t = now_ns();
        {
            std::lock_guard<std::mutex> lk(imu_);
            if (queued) {
                const int64_t start = std::max(t, inflight_.empty() ? t : inflight_.back().est_end_ns);
                inflight_.push_back(Batch{seq, ev, start + kFixedNs + int64_t(bytes_ns)});
                publish_inflight();
            } else {   // nothing left running (failed and drained): every status is final
                if (ev) events_.push_back(ev);
                for (SubmitReq* q : take_) q->done.store(1, std::memory_order_release);
            }
        }
        take_.clear();
        if (queued) {
            cv_work_.notify_one();
        } else {
            { std::lock_guard<std::mutex> lk(mu_); }
            cv_done_.notify_all();
        }
    }

    // inflight_ changed: its size and the watcher's early-launch time.  imu_ held.
    void publish_inflight() {
        inflight_n_.store(int(inflight_.size()), std::memory_order_seq_cst);
        front_end_ns_.store(inflight_.empty() ? INT64_MAX : inflight_.front().est_end_ns, std::memory_order_relaxed);
        const int lead = g_lead_us.load(std::memory_order_relaxed);
        ahead_at_ns_.store(inflight_.size() == 1 && lead > 0 ? inflight_.front().est_end_ns - int64_t(lead) * 1000
                                                            : INT64_MAX,
                           std::memory_order_relaxed);
    }

    // Drops finished batches (their events back to the pool).  imu_ held.
    void reap() {
        const uint64_t c = completed();
        bool changed = false;
        while (!inflight_.empty() && inflight_.front().seq <= c) {
            if (inflight_.front().ev) events_.push_back(inflight_.front().ev);
            inflight_.pop_front();
            changed = true;
        }
        if (changed) publish_inflight();
    }

    // Enqueues one batch on the queue's stream: one pointer-table call per
    // group of compatible requests, the completion mark, the batch's event.
    // A group's error is its requests' status.  false: nothing will mark the
    // batch (every status is final; the stream is drained).
    bool launch(std::vector<SubmitReq*>& reqs, uint64_t seq, hipEvent_t* ev) {
        const int64_t tl0 = g_trace.on ? now_ns() : 0;
        RelaxedCapture relaxed;
        DeviceScope scope(dev_);
        if (!scope.ok()) {
            for (SubmitReq* q : reqs) q->rc = SHMR_EC_DEVICE_ERROR;
            return false;
        }
        using Key = std::tuple<const Codec*, int, bool, bool, uint64_t>;
        std::map<Key, std::vector<SubmitReq*>> groups;
        for (SubmitReq* q : reqs) {
            groups[Key{q->codec, int(q->op), q->data_only, q->host_mapped, q->len}].push_back(q);
            q->seq.store(seq, std::memory_order_release);   // the mark for seq comes after its kernels
        }
        if (g_trace.on) g_trace.add(3, 0, int(reqs.size()), 0, tl0, now_ns());
        for (auto& g : groups) {
            std::vector<SubmitReq*>& v = g.second;
            Codec& c = *const_cast<Codec*>(v[0]->codec);
            const unsigned t = c.k() + c.p();
            const size_t n = v.size();
            tab_.resize(n * t);
            for (size_t b = 0; b < n; ++b) std::memcpy(&tab_[b * t], v[b]->row_data(), t * sizeof(uint64_t));
            if (v[0]->op == kDecode) {
                present_.resize(n * t);
                for (size_t b = 0; b < n; ++b) std::memcpy(&present_[b * t], v[b]->present_data(), t);
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
        if (g_trace.on) g_trace.add(3, 1, int(reqs.size()), 0, tl0, now_ns());
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

    // Launches what is due: everything pending when a caller forced it,
    // otherwise what `wanted` allows.
    void launch_due() {
        if (force_.exchange(false, std::memory_order_seq_cst))
            launch_some(kForced);
        else if (wanted(kByWatcher))
            launch_some(kByWatcher);
    }

    // The watcher, the queue's one launcher: launches what is due, follows
    // the oldest batch in flight -- the host word, then (after
    // coalesce_watch_us, and past the early-launch time while calls could
    // still arrive) hipEventSynchronize on its event; an error there means
    // the device failed: the queue is broken and every waiter returns
    // DEVICE_ERROR -- wakes the sleeping callers when it completes, and with
    // nothing in flight spins coalesce_idle_us for calls before it sleeps.
    void watch() {
        RelaxedCapture relaxed;
        std::unique_lock<std::mutex> lk(imu_);
        lk.unlock();
        for (;;) {
            launch_due();
            lk.lock();
            if (broken_.load(std::memory_order_acquire)) {
                release_all(lk);
                continue;
            }
            if (inflight_.empty()) {   // idle: spin for calls, then sleep
                lk.unlock();
                const auto t0 = Clock::now();
                const auto idle = std::chrono::microseconds(g_idle_us.load(std::memory_order_relaxed));
                bool work = false;
                for (uint32_t i = 0;; ++i) {
                    if (queued_.load(std::memory_order_seq_cst) > 0 || force_.load(std::memory_order_seq_cst)) {
                        work = true;
                        break;
                    }
                    if ((i & 255) == 255 && Clock::now() - t0 >= idle) break;
                    cpu_relax();
                }
                if (work) continue;
                lk.lock();
                sleeping_.store(true, std::memory_order_seq_cst);
                cv_work_.wait(lk, [&] {
                    return queued_.load(std::memory_order_seq_cst) > 0 || force_.load(std::memory_order_seq_cst) ||
                           !inflight_.empty() || broken_.load(std::memory_order_acquire);
                });
                sleeping_.store(false, std::memory_order_seq_cst);
                lk.unlock();
                continue;
            }
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
                if ((i & 15) == 15) {
                    launch_due();   // the early launch, the target rule, forced launches
                    if (ev && !g_mark.load(std::memory_order_relaxed)) {   // no mark kernel: poll the event
                        const hipError_t q = hipEventQuery(ev);
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
                }
                if ((i & 255) == 255 && Clock::now() - t0 >= spin) {
                    // With an early launch still to make, keep following the
                    // word up to the batch's estimated end (dozing through
                    // most of a long batch), so calls that arrive meanwhile
                    // are launched behind it; past that end by 100 us, or with
                    // no early launch to make, sleep on the event.
                    if (ahead_at_ns_.load(std::memory_order_relaxed) == INT64_MAX) break;
                    const int64_t end = front_end_ns_.load(std::memory_order_relaxed), now = now_ns();
                    if (end == INT64_MAX || now > end + 100000) break;
                    if (end - now > 5000000) std::this_thread::sleep_for(std::chrono::nanoseconds(end - now - 2000000));
                }
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
            if (g_trace.on) g_trace.add(1, seen ? 1 : 0, int(target), int(inflight_.size()), now_ns(), now_ns());
            lk.unlock();
            launch_due();   // what waited for this batch (before waking the sleepers: the GPU first)
            { std::lock_guard<std::mutex> g(mu_); }   // (no caller between its check and its sleep)
            cv_done_.notify_all();
        }
    }

    // A broken queue: nothing will complete.  Every waiter returns through
    // broken_ (finished / result); the lists are dropped without touching
    // their requests, which their callers may already have freed.  imu_ held.
    void release_all(std::unique_lock<std::mutex>& lk) {
        lk.unlock();
        while (launching_.exchange(true, std::memory_order_seq_cst)) std::this_thread::yield();
        for (auto& slot : ring_) slot.store(nullptr, std::memory_order_relaxed);
        head_ = tail_.load(std::memory_order_seq_cst);
        head_pub_.store(head_, std::memory_order_release);
        pending_.clear();
        queued_.store(0, std::memory_order_seq_cst);
        launching_.store(false, std::memory_order_seq_cst);
        lk.lock();
        inflight_.clear();
        publish_inflight();
        lk.unlock();
        { std::lock_guard<std::mutex> g(mu_); }
        cv_done_.notify_all();
        lk.lock();
        cv_work_.wait(lk, [] { return false; });   // (the queue is dead: the watcher parks)
    }

    const int dev_;
    hipStream_t stream_ = nullptr;
    uint64_t* word_ = nullptr;    // completion mark (host view)
    uint64_t* dword_ = nullptr;   // ... its device address
    // The shared atomics each on a cache line of their own, apart from the
    // launcher's private state (r06 s19: callers hammering a line the
    // launcher also used slowed its launches several-fold).
    // The inbox: a ring of request pointers.  A caller takes an index
    // (fetch_add) and stores its request there; the launcher reads the slots
    // in order -- independent loads from one array (r06 s25: walking a
    // linked list of requests made by other threads' cores cost ~0.25 us of
    // dependent cache misses per request, 57 us for a 215-block batch).
    static constexpr uint64_t kRing = 1u << 16;
    std::vector<std::atomic<SubmitReq*>> ring_ = std::vector<std::atomic<SubmitReq*>>(kRing);
    alignas(64) std::atomic<uint64_t> tail_{0};            // next index a caller takes
    alignas(64) std::atomic<uint64_t> head_pub_{0};        // the launcher's head, for the full check
    uint64_t head_ = 0;                                    // launcher only
    alignas(64) std::atomic<int64_t> queued_{0};           // calls submitted and not yet launched
    alignas(64) std::atomic<bool> launching_{false};
    alignas(64) std::atomic<int> forced_waiters_{0};       // wait() callers asleep until a launch ends
    alignas(64) std::atomic<bool> force_{false};           // a caller waits for a call not yet launched
    alignas(64) std::atomic<bool> sleeping_{false};        // the watcher sleeps on cv_work_
    std::atomic<int64_t> first_arrival_ns_{0};
    alignas(64) std::vector<SubmitReq*> pending_, take_;   // launcher only
    std::vector<uint64_t> tab_;                // launcher only
    std::vector<uint8_t> present_;             // launcher only
    uint64_t launched_ = 0;                    // launcher only
    // Two locks: callers asleep in wait() (cv_done_) never stand in the
    // launcher's way to inflight_ (r06 s22: a notify_all woke 16-32 sleepers
    // whose turns at one mutex delayed launches by 100-400 us).
    alignas(64) std::mutex mu_;                // cv_done_: callers asleep until a batch completes or a launch ends
    alignas(64) std::mutex imu_;               // inflight_, events_, cv_work_ (launcher and watcher)
    std::condition_variable cv_work_, cv_done_;
    std::deque<Batch> inflight_;
    alignas(64) std::atomic<int> inflight_n_{0};
    std::atomic<int64_t> ahead_at_ns_{INT64_MAX};   // early launch behind the one batch in flight
    std::atomic<int64_t> front_end_ns_{INT64_MAX};  // the oldest batch's estimated end
    std::vector<hipEvent_t> events_;
    std::atomic<bool> broken_{false};
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

void SubmitReq::set_row(const uint64_t* r, const uint8_t* pr, unsigned t) {
    total = t;
    uint64_t* dst = row_inline;
    uint8_t* pdst = present_inline;
    if (t > kInline) {
        row.resize(t);
        dst = row.data();
        if (pr) {
            present.resize(t);
            pdst = present.data();
        }
    }
    size_t touched = 0;
    for (unsigned i = 0; i < t; ++i) {
        dst[i] = r[i];
        touched += r[i] != 0;
    }
    if (pr) std::memcpy(pdst, pr, t);
    est_ns = double(touched) * double(len) / (host_mapped ? kHostBytesPerNs : kDevBytesPerNs);
}

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
    if (key == "coalesce_lead_us") return set(g_lead_us, kLeadDefault, 0, 10000000);
    if (key == "coalesce_idle_us") return set(g_idle_us, kIdleDefault, 0, 10000000);
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
    if (key == "coalesce_lead_us") return g_lead_us;
    if (key == "coalesce_idle_us") return g_idle_us;
    *known = false;
    return SHMR_EC_INVALID_ARGUMENT;
}

void submit_stats(int dev, uint64_t* out, size_t n) {
    for (size_t i = 0; i < n && i < size_t(kStatCount); ++i)
        out[i] = (dev >= 0 && dev < kMaxQueues) ? g_stats[dev][i].load() : 0;
}

}  // namespace core
}  // namespace shmr
