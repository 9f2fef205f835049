// C++ host mirror of the reference's StorageBlock layer.  See vfs.hpp.
// Citations are into the reference tree (volfco/shmr @ 2024-08-07).
#include "vfs.hpp"

#include <fcntl.h>
#include <sys/stat.h>
#include <sys/statfs.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <future>
#include <map>
#include <memory>
#include <new>
#include <thread>
#include <tuple>

namespace shmr {

namespace {

ShmrError fs_error(int err) { return ShmrError{ShmrError::FsError, err}; }
ShmrError ec_error(int code) { return ShmrError{ShmrError::EcError, code}; }

// write_path (block.rs:611-634): pwrite at offset 0, then fsync.
Status write_path(int fd, const uint8_t* buf, size_t len, bool sync = true) {
    size_t done = 0;
    while (done < len) {
        const ssize_t n = ::pwrite(fd, buf + done, len - done, off_t(done));
        if (n < 0) {
            if (errno == EINTR) continue;
            return fs_error(errno);
        }
        done += size_t(n);
    }
    if (sync && ::fsync(fd) != 0) return fs_error(errno);
    return std::nullopt;
}

// Persistent worker pool behind parallel_for: the host path fans out hundreds
// of small file and memcpy tasks per flush / load batch, and spawning threads
// per call cost milliseconds per batch.  A caller always works on its own job
// and, once its indices are exhausted, withdraws helper slots no worker has
// picked up yet, so nested parallel_for calls cannot deadlock.
class WorkPool {
public:
    static WorkPool& get() {
        static WorkPool* p = new WorkPool(32);   // leaked: outlives static teardown
        return *p;
    }
    void run(size_t n, size_t threads, const std::function<void(size_t)>& fn) {
        auto job = std::make_shared<Job>();
        job->n = n;
        job->fn = &fn;
        const size_t helpers = std::min(threads, n) - 1;
        {
            std::lock_guard<std::mutex> lock(mu_);
            for (size_t h = 0; h < helpers; ++h) queue_.push_back(job);
            job->pending = helpers;
        }
        if (helpers == 1) cv_.notify_one();
        else if (helpers > 1) cv_.notify_all();
        work(*job);
        std::unique_lock<std::mutex> lock(mu_);
        for (auto it = queue_.begin(); it != queue_.end();) {   // withdraw unstarted helper slots
            if (*it == job) {
                it = queue_.erase(it);
                --job->pending;
            } else {
                ++it;
            }
        }
        done_cv_.wait(lock, [&] { return job->pending == 0; });
    }

private:
    struct Job {
        std::atomic<size_t> next{0};
        size_t n = 0;
        const std::function<void(size_t)>* fn = nullptr;
        size_t pending = 0;   // helper slots queued or running (under mu_)
    };
    explicit WorkPool(size_t workers) {
        for (size_t i = 0; i < workers; ++i) std::thread([this] { loop(); }).detach();
    }
    static void work(Job& j) {
        for (size_t i = j.next++; i < j.n; i = j.next++) (*j.fn)(i);
    }
    void loop() {
        for (;;) {
            std::shared_ptr<Job> job;
            {
                std::unique_lock<std::mutex> lock(mu_);
                cv_.wait(lock, [&] { return !queue_.empty(); });
                job = queue_.front();
                queue_.pop_front();
            }
            work(*job);
            std::lock_guard<std::mutex> lock(mu_);
            if (--job->pending == 0) done_cv_.notify_all();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    std::deque<std::shared_ptr<Job>> queue_;
};

// Runs fn(i) for i < n on up to `threads` threads (the reference's rayon fan-out).
template <class F>
void parallel_for(size_t n, size_t threads, F fn) {
    threads = std::max<size_t>(1, std::min(threads, n));
    if (threads == 1) {
        for (size_t i = 0; i < n; ++i) fn(i);
        return;
    }
    const std::function<void(size_t)> f = std::ref(fn);
    WorkPool::get().run(n, threads, f);
}

}  // namespace

std::string ShmrError::what() const {
    static const char* names[] = {"InvalidPoolId", "InvalidBucketId", "OutOfSpace", "EndOfFile",
                                  "FsError", "EcError", "ShardOpened", "ShardMissing",
                                  "InvalidInodeType", "InodeNotExist", "BlockIndexOutOfBounds"};
    std::string s = names[kind];
    if (kind == FsError) s += std::string("(") + std::strerror(code) + ")";
    if (kind == EcError) s += std::string("(") + shmr_ec_status_name(code) + ")";
    return s;
}

// ---------------------------------------------------------------------------
// BlockTopology (block.rs:32-98)
// ---------------------------------------------------------------------------
namespace {
std::string trim(const std::string& s) {
    size_t a = 0, b = s.size();
    while (a < b && std::isspace(static_cast<unsigned char>(s[a]))) ++a;
    while (b > a && std::isspace(static_cast<unsigned char>(s[b - 1]))) --b;
    return s.substr(a, b - a);
}
bool parse_u8(const std::string& s, uint8_t* out) {
    if (s.empty() || s.size() > 3) return false;
    unsigned v = 0;
    for (char ch : s) {
        if (ch < '0' || ch > '9') return false;
        v = v * 10 + unsigned(ch - '0');
    }
    if (v > 255) return false;
    *out = uint8_t(v);
    return true;
}
std::string rstrip_paren(std::string s) {
    while (!s.empty() && s.back() == ')') s.pop_back();
    return s;
}
}  // namespace

std::optional<BlockTopology> BlockTopology::try_from(const std::string& value, std::string* err) {
    auto fail = [&](const std::string& m) -> std::optional<BlockTopology> {
        if (err) *err = m;
        return std::nullopt;
    };
    const size_t lp = value.find('(');
    if (lp == std::string::npos) return fail("'" + value + "' does not have '('");
    const std::string name = value.substr(0, lp);
    std::string arg = value.substr(lp + 1);
    if (!arg.empty()) arg.pop_back();   // arg.pop()
    if (name == "Single") return BlockTopology::single();
    if (name == "Mirror") {
        uint8_t n;
        if (!parse_u8(rstrip_paren(arg), &n)) return fail("Unable to parse " + value + ". " + name + " - " + arg);
        return BlockTopology::mirror(n);
    }
    if (name == "Erasure") {
        std::vector<std::string> params;   // splitn(3, ',')
        size_t start = 0;
        for (int i = 0; i < 2; ++i) {
            const size_t c = arg.find(',', start);
            if (c == std::string::npos) break;
            params.push_back(arg.substr(start, c - start));
            start = c + 1;
        }
        params.push_back(arg.substr(start));
        uint8_t v, d, p;
        if (!parse_u8(trim(params[0]), &v)) return fail("Unable to parse version");
        if (!parse_u8(trim(params.size() > 1 ? params[1] : ""), &d)) return fail("Unable to parse data shards");
        if (!parse_u8(rstrip_paren(trim(params.size() > 2 ? params[2] : "")), &p))
            return fail("Unable to parse parity shards");
        return BlockTopology::erasure(v, d, p);
    }
    return fail("Unable to parse " + value + ". " + name + " - " + arg);
}

std::string BlockTopology::to_string() const {
    switch (kind) {
        case Single: return "Single";
        case Mirror: return "Mirror(" + std::to_string(n) + ")";
        default:
            return "Erasure(" + std::to_string(version) + ", " + std::to_string(data) + ", " +
                   std::to_string(parity) + ")";
    }
}

// ---------------------------------------------------------------------------
// ShmrFsConfig::select_buckets (config.rs:46-85), VirtualPath (path.rs:29-83)
// ---------------------------------------------------------------------------
Status ShmrFsConfig::select_buckets(const std::string& pool, size_t count, std::vector<std::string>* out) const {
    auto it = pools.find(pool);
    if (it == pools.end()) return ShmrError{ShmrError::InvalidPoolId};
    std::vector<std::pair<std::string, const Bucket*>> possible;
    for (auto& kv : it->second)
        if (kv.second.priority > BucketPriority::Ignore) possible.emplace_back(kv.first, &kv.second);
    std::stable_sort(possible.begin(), possible.end(), [](auto& a, auto& b) {
        if (a.second->priority != b.second->priority) return a.second->priority < b.second->priority;
        return a.second->available < b.second->available;
    });
    out->clear();
    if (possible.empty()) {
        // The reference loops forever extending an empty list (config.rs:71-74).
        return count == 0 ? Status{} : Status{ShmrError{ShmrError::InvalidBucketId}};
    }
    const auto copy = possible;
    while (possible.size() < count) possible.insert(possible.end(), copy.begin(), copy.end());
    for (size_t i = 0; i < count; ++i) out->push_back(possible[i].first);
    return std::nullopt;
}

Status VirtualPath::resolve(const ShmrFsConfig& cfg, fs::path* file, fs::path* dir) const {
    auto p = cfg.pools.find(pool);
    if (p == cfg.pools.end()) return ShmrError{ShmrError::InvalidPoolId};
    auto b = p->second.find(bucket);
    if (b == p->second.end()) return ShmrError{ShmrError::InvalidBucketId};
    const fs::path& base = b->second.path;
    fs::path d = base / filename.substr(0, 2);   // first two characters of the filename
    d /= filename.substr(2, 2);                   // next two characters
    if (file) *file = base / filename;
    if (dir) *dir = d;
    return std::nullopt;
}

Status VirtualPath::create(const ShmrFsConfig& cfg) const {
    fs::path file, dir;
    if (auto e = resolve(cfg, &file, &dir)) return e;
    std::error_code ec;
    if (!fs::exists(dir, ec)) fs::create_directories(dir, ec);
    if (ec) return fs_error(ec.value());
    const int fd = ::open(file.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
    if (fd < 0) return fs_error(errno);
    ::close(fd);
    return std::nullopt;
}

std::string VirtualPath::to_string() const { return pool + "(" + bucket + "):" + filename; }

// ---------------------------------------------------------------------------
// Block Cache buffer: `len` logical bytes (the reference's Vec<u8> length)
// inside one allocation of `cap` bytes, pinned when asked.  Bytes past `len`
// are scratch (zero padding, parity slots); growing `len` zero-fills.
// ---------------------------------------------------------------------------
namespace {

// Process-wide free lists of Block Cache allocations, by exact capacity
// (blocks of one topology share it): pinning memory costs far more than
// copying into it, so buffers dropped by drop_buffer are kept for the next
// block instead of being returned to the driver.
class BufferPool {
public:
    static BufferPool& get() {
        static BufferPool* p = new BufferPool();   // leaked: outlives static destructors
        return *p;
    }
    uint8_t* take(size_t cap, bool pinned) {
        std::lock_guard<std::mutex> lock(mu_);
        auto& m = pinned ? pinned_ : pageable_;
        auto it = m.find(cap);
        if (it == m.end()) return nullptr;
        uint8_t* p = it->second;
        m.erase(it);
        cached_ -= cap;
        return p;
    }
    // Returns false if the pool is full (the caller frees).
    bool give(uint8_t* p, size_t cap, bool pinned) {
        std::lock_guard<std::mutex> lock(mu_);
        if (cached_ + cap > limit_) return false;
        (pinned ? pinned_ : pageable_).emplace(cap, p);
        cached_ += cap;
        return true;
    }
    size_t trim() {
        std::lock_guard<std::mutex> lock(mu_);
        size_t freed = cached_;
        for (auto& kv : pinned_) shmr_ec_host_free(kv.second);
        for (auto& kv : pageable_) std::free(kv.second);
        pinned_.clear();
        pageable_.clear();
        cached_ = 0;
        return freed;
    }

private:
    std::mutex mu_;
    std::multimap<size_t, uint8_t*> pinned_, pageable_;
    size_t cached_ = 0;
    size_t limit_ = size_t(16) << 30;
};

class BlockBuffer {
public:
    BlockBuffer() = default;
    BlockBuffer(const BlockBuffer&) = delete;
    BlockBuffer& operator=(const BlockBuffer&) = delete;
    ~BlockBuffer() { release(); }

    size_t size() const { return len_; }
    bool empty() const { return len_ == 0; }
    uint8_t* data() { return p_; }
    const uint8_t* data() const { return p_; }
    bool pinned() const { return pinned_alloc_; }
    void want_pinned(bool p) { want_pinned_ = p; }

    void reserve(size_t cap) {
        if (cap <= cap_) return;
        bool pinned = false;
        uint8_t* q = nullptr;
        if (want_pinned_) {
            q = BufferPool::get().take(cap, true);
            if (q) {
                pinned = true;
            } else {
                void* v = nullptr;
                if (shmr_ec_host_alloc(cap, &v) == SHMR_EC_OK) {
                    q = static_cast<uint8_t*>(v);
                    pinned = true;
                }
            }
        }
        if (!q) q = BufferPool::get().take(cap, false);
        if (!q) q = static_cast<uint8_t*>(std::aligned_alloc(4096, (cap + 4095) & ~size_t(4095)));
        if (!q) throw std::bad_alloc();
        if (len_) std::memcpy(q, p_, len_);
        free_mem();
        p_ = q;
        cap_ = cap;
        pinned_alloc_ = pinned;
    }
    // Grows the logical length, zero-filling the new bytes (Vec::resize).
    void resize(size_t n) {
        reserve(n);
        if (n > len_) std::memset(p_ + len_, 0, n - len_);
        len_ = n;
    }
    // Sets the logical length without initialising: for loads that overwrite
    // every byte of [0, n) before anyone reads it.
    void set_len_uninit(size_t n) {
        reserve(n);
        len_ = n;
    }
    void release() {
        free_mem();
        p_ = nullptr;
        len_ = cap_ = 0;
    }

private:
    void free_mem() {
        if (!p_) return;
        if (!BufferPool::get().give(p_, cap_, pinned_alloc_)) {
            if (pinned_alloc_) shmr_ec_host_free(p_);
            else std::free(p_);
        }
        pinned_alloc_ = false;
    }
    uint8_t* p_ = nullptr;
    size_t len_ = 0, cap_ = 0;
    bool want_pinned_ = false, pinned_alloc_ = false;
};

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Reads shard file `fd` into its S-byte slot the way load_block treats the
// result of read_to_end (block.rs:540-553): returns 0 and sets *present for a
// readable file; a file of length != S is zero-padded/truncated to S and
// flagged (*odd = true).  The reference reads from the handle's cursor and
// leaves it at EOF; pread_from_start reads from offset 0 instead.
int read_slot(int fd, uint8_t* slot, size_t S, bool from_start, bool* odd) {
    size_t got = 0;
    while (got < S) {
        const ssize_t n = from_start ? ::pread(fd, slot + got, S - got, off_t(got)) : ::read(fd, slot + got, S - got);
        if (n < 0) {
            if (errno == EINTR) continue;
            return errno;
        }
        if (n == 0) break;
        got += size_t(n);
    }
    bool longer = false;
    if (got == S) {   // probe: is there more than S bytes?
        uint8_t b;
        ssize_t n;
        do {
            n = from_start ? ::pread(fd, &b, 1, off_t(S)) : ::read(fd, &b, 1);
        } while (n < 0 && errno == EINTR);
        if (n < 0) return errno;
        longer = n > 0;
    }
    if (!from_start && longer) ::lseek(fd, 0, SEEK_END);   // read_to_end drains the handle
    if (got < S) std::memset(slot + got, 0, S - got);
    *odd = got != S || longer;
    return 0;
}

std::atomic<uint64_t> g_shard_reads{0};   // shard files read by loads (shard_reads_total)

int read_slot_counted(int fd, uint8_t* slot, size_t S, bool from_start, bool* odd) {
    g_shard_reads.fetch_add(1, std::memory_order_relaxed);
    return read_slot(fd, slot, S, from_start, odd);
}

// ---- direct I/O (VfsOptions::direct_io) -------------------------------------
// Shard files read into / written from the Block-Cache slots with O_DIRECT:
// the bytes move between the disk and the (page-aligned, possibly mapped)
// slot with no page-cache copy.  Only whole 4 KiB-aligned slots qualify (S a
// multiple of 4096 -- RS(8,3) 4 MiB blocks; RS(10,4) 16 MiB's S = 1,677,722
// does not); everything else, and every file system that refuses O_DIRECT
// (tmpfs, overlay: EINVAL at open), takes the buffered path.  The on-disk
// format is unchanged: raw S bytes per shard at offset 0 (block.rs:611-634).
constexpr size_t kDirectAlign = 4096;
struct DirectStats {
    std::atomic<uint64_t> reads{0}, writes{0}, fallbacks{0}, refusals{0};
    std::mutex mu;
    int refused_errno = 0;
    std::string refused_fs;
    int io_errno = 0;   // first O_DIRECT read/write error (e.g. EFAULT: a buffer the kernel cannot pin)
};
DirectStats& g_direct() {
    static DirectStats* d = new DirectStats;   // leaked: outlives static destructors
    return *d;
}
void note_direct_io_error(int err) {
    DirectStats& d = g_direct();
    std::lock_guard<std::mutex> lock(d.mu);
    if (!d.io_errno) d.io_errno = err;
}
bool direct_eligible(const void* p, size_t S) {
    return S > 0 && S % kDirectAlign == 0 && (uintptr_t(p) % kDirectAlign) == 0;
}
std::string fs_name(const fs::path& file) {
    struct statfs sf {};
    if (::statfs(file.parent_path().c_str(), &sf) != 0) return "unknown";
    switch (static_cast<unsigned long>(sf.f_type)) {
        case 0x01021994UL: return "tmpfs";
        case 0x794c7630UL: return "overlayfs";
        case 0xEF53UL: return "ext4";
        case 0x58465342UL: return "xfs";
        case 0x9123683EUL: return "btrfs";
        case 0x6969UL: return "nfs";
        case 0x65735546UL: return "fuse";
        default: {
            char b[32];
            std::snprintf(b, sizeof b, "0x%lx", static_cast<unsigned long>(sf.f_type));
            return b;
        }
    }
}
// An O_DIRECT descriptor of `file`, or -1 (refusal recorded once per errno).
int open_direct(const fs::path& file) {
    const int fd = ::open(file.c_str(), O_RDWR | O_CREAT | O_DIRECT, 0644);
    if (fd >= 0) return fd;
    const int err = errno;
    DirectStats& d = g_direct();
    d.refusals.fetch_add(1, std::memory_order_relaxed);
    std::lock_guard<std::mutex> lock(d.mu);
    if (!d.refused_errno) {
        d.refused_errno = err;
        d.refused_fs = fs_name(file);
    }
    return -1;
}
// pwrite of a whole aligned slot at offset 0 (+ fdatasync): write_path's
// twin.  Returns 0, or the errno of a failed write (the caller then writes
// the shard buffered: O_DIRECT can refuse a buffer, e.g. EFAULT for memory
// the kernel cannot pin, or EINVAL).
int write_direct(int fd, const uint8_t* buf, size_t len, bool sync) {
    size_t done = 0;
    while (done < len) {
        const ssize_t n = ::pwrite(fd, buf + done, len - done, off_t(done));
        if (n < 0) {
            if (errno == EINTR) continue;
            return errno;
        }
        if (n == 0) return EIO;
        done += size_t(n);
    }
    if (sync && ::fdatasync(fd) != 0) return errno;
    g_direct().writes.fetch_add(1, std::memory_order_relaxed);
    return 0;
}
// read_slot's twin for a file of exactly S bytes (from offset 0); returns -1
// when the file has another length (the caller reads it buffered: the
// reference's zero-pad / drain rules need the exact byte count).
int read_slot_direct(int fd, uint8_t* slot, size_t S, bool* odd) {
    struct stat st {};
    if (::fstat(fd, &st) != 0) return errno;
    if (uint64_t(st.st_size) != S) return -1;
    size_t got = 0;
    while (got < S) {
        const ssize_t n = ::pread(fd, slot + got, S - got, off_t(got));
        if (n < 0) {
            if (errno == EINTR) continue;
            return errno;
        }
        if (n == 0) break;
        got += size_t(n);
    }
    if (got != S) return -1;
    *odd = false;
    g_shard_reads.fetch_add(1, std::memory_order_relaxed);
    g_direct().reads.fetch_add(1, std::memory_order_relaxed);
    return 0;
}

// VfsOptions::read_needed_shards: which shard files of an Erasure block a
// load reads (plan[i]: kRead, kPresentUnread, or kAbsent).  The reference
// reads all k+p (block.rs:531-556) and returns ec_data[..size] (block.rs:576).  The file sizes
// decide: a shard whose file is exactly S bytes is intact; the first k intact
// shards in index order -- exactly the reconstruct's inputs (first k present,
// the crate's rule) -- are read, the other intact ones count as present
// without being read.  Their slots are never observable: a load returns
// [..size] with size <= k*S (checked by the caller), and every flush
// re-encodes parity from the data.  A missing file is absent; a file of
// another length is absent under short_shard_is_erasure, and otherwise the
// reference's zero-pad-and-keep rule needs its bytes, so everything is read
// (returns false).  If a planned read fails, the caller reads the rest.
enum ReadPlan : uint8_t { kAbsent = 0, kRead = 1, kPresentUnread = 2 };
bool plan_needed_reads(const int* fds, size_t n, size_t k, size_t S, bool short_is_erasure, uint8_t* plan) {
    size_t inputs = 0;
    for (size_t i = 0; i < n; ++i) {
        plan[i] = kAbsent;
        if (fds[i] < 0) continue;
        struct stat st {};
        if (::fstat(fds[i], &st) != 0) return false;
        if (uint64_t(st.st_size) != S) {
            if (!short_is_erasure) return false;
            continue;
        }
        plan[i] = inputs < k ? kRead : kPresentUnread;
        inputs += plan[i] == kRead;
    }
    return true;
}

}  // namespace

// ---------------------------------------------------------------------------
// VirtualBlock
// ---------------------------------------------------------------------------
struct VirtualBlock::State {
    std::mutex handles_mu;
    std::vector<std::pair<VirtualPath, int>> handles;   // fd -1: missing (opt-in)
    std::atomic<bool> shard_loaded{false};
    std::atomic<bool> should_flush{false};
    std::atomic<bool> buffer_loaded{false};
    std::mutex buf_mu;
    BlockBuffer buffer;
    // A handle recorded as missing (VfsOptions::missing_shard_is_erasure) is
    // recreated on the next flush, which repairs the shard file.
    Status ensure_fd(size_t i, const ShmrFsConfig& cfg) {
        if (handles[i].second >= 0) return std::nullopt;
        fs::path file;
        if (auto e = handles[i].first.resolve(cfg, &file, nullptr)) return e;
        const int fd = ::open(file.c_str(), O_RDWR | O_CREAT, 0644);
        if (fd < 0) return fs_error(errno);
        handles[i].second = fd;
        return std::nullopt;
    }
    // VfsOptions::direct_io: shard i's O_DIRECT descriptor, opened on first
    // use (creating the file like ensure_fd); -1 when the file system refuses
    // it (then never retried for this handle).  The block operation that
    // calls this holds handles_mu; its parallel shard workers each touch only
    // their own i (dfds is sized with the handles by open_handles, before
    // that parallel shard I/O starts).
    int direct_fd(size_t i, const ShmrFsConfig& cfg) {
        if (i >= dfds.size()) return -1;
        if (dfds[i] >= 0 || dfds[i] == -2) return dfds[i] >= 0 ? dfds[i] : -1;
        fs::path file;
        if (handles[i].first.resolve(cfg, &file, nullptr)) return -1;
        const int fd = open_direct(file);
        dfds[i] = fd >= 0 ? fd : -2;
        return fd;
    }
    void close_handles() {
        for (auto& h : handles)
            if (h.second >= 0) ::close(h.second);
        handles.clear();
        for (int fd : dfds)
            if (fd >= 0) ::close(fd);
        dfds.clear();
    }
    // Writes shard i from `buf` (write_path; O_DIRECT under direct_io when the
    // slot qualifies).
    Status write_shard(size_t i, const ShmrFsConfig& cfg, const VfsOptions& o, const uint8_t* buf, size_t len) {
        if (auto e = ensure_fd(i, cfg)) return e;
        if (o.direct_io) {
            const int dfd = direct_eligible(buf, len) ? direct_fd(i, cfg) : -1;
            if (dfd >= 0) {
                const int err = write_direct(dfd, buf, len, o.fsync_shards);
                if (err == 0) return std::nullopt;
                note_direct_io_error(err);
            }
            g_direct().fallbacks.fetch_add(1, std::memory_order_relaxed);
        }
        return write_path(handles[i].second, buf, len, o.fsync_shards);
    }
    // Reads shard i into its slot (read_slot; O_DIRECT under direct_io for an
    // intact file into a qualifying slot, read from offset 0).
    int read_shard(size_t i, int fd, const ShmrFsConfig& cfg, const VfsOptions& o, uint8_t* slot, size_t S,
                   bool* odd) {
        if (o.direct_io && o.pread_from_start && i < handles.size() && handles[i].second >= 0) {
            const int dfd = direct_eligible(slot, S) ? direct_fd(i, cfg) : -1;
            if (dfd >= 0) {
                const int rc = read_slot_direct(dfd, slot, S, odd);
                if (rc == 0) return 0;
                if (rc > 0) note_direct_io_error(rc);   // read buffered below (-1: not exactly S bytes)
            }
            g_direct().fallbacks.fetch_add(1, std::memory_order_relaxed);
        }
        return read_slot_counted(fd, slot, S, o.pread_from_start, odd);
    }
    std::vector<int> dfds;   // O_DIRECT descriptors (direct_io), -1 unopened, -2 refused
    ~State() { close_handles(); }
};

namespace {

// The Erasure arm's shard set, in place (block.rs:404-423): data chunks of S
// at i*S (the buffer itself), the last one zero-padded, then zero data shards
// up to k, then p parity slots -- i.e. the buffer zero-extended to k*S with
// parity at k*S.  Caller holds the buffer lock.
//
// A buffer longer than k*S (only past calculate_shard_size's f32 hazard,
// e.g. 16,777,217 B at k = 8: nchunks = k + 1) makes block.rs:421's
// `parity + (data - nchunks as u8)` underflow.  Default: refuse with
// TooManyDataShards before any shard is written.  With
// VfsOptions::release_u8_wrap the reference's release build is reproduced
// (Cargo.toml:10-13, no overflow checks): the u8 arithmetic wraps to
// (p - e) mod 256 zero shards, encode sees exactly k+p shards when e <= p and
// writes parity over chunks k..k+e-1 -- in the shard files only: the
// reference encoded copies (chunks().to_vec()), so its Block Cache buffer
// keeps the data.  The overwritten buffer bytes [k*S, len) are saved in
// *tail and restore_tail() puts them back after the shard writes.
Status prepare_erasure(BlockBuffer& buf, const BlockTopology& t, size_t S, bool release_u8_wrap,
                       std::vector<uint8_t>* tail) {
    const size_t len = buf.size();
    const size_t kS = size_t(t.data) * S;
    tail->clear();
    if (len > kS) {
        if (!release_u8_wrap) return ec_error(SHMR_EC_TOO_MANY_DATA_SHARDS);
        const size_t nchunks = (len + S - 1) / S;
        const unsigned extra = uint8_t(t.parity + uint8_t(t.data - uint8_t(nchunks)));   // block.rs:421, wrapping
        if (nchunks + extra != size_t(t.data) + t.parity)
            return ec_error(nchunks + extra < size_t(t.data) + t.parity ? SHMR_EC_TOO_FEW_SHARDS
                                                                         : SHMR_EC_TOO_MANY_SHARDS);   // .unwrap() panics there
        buf.reserve((size_t(t.data) + t.parity) * S);
        tail->assign(buf.data() + kS, buf.data() + len);
        return std::nullopt;
    }
    buf.reserve((size_t(t.data) + t.parity) * S);
    std::memset(buf.data() + len, 0, kS - len);
    return std::nullopt;
}

void restore_tail(BlockBuffer& buf, const BlockTopology& t, size_t S, const std::vector<uint8_t>& tail) {
    if (!tail.empty()) std::memcpy(buf.data() + size_t(t.data) * S, tail.data(), tail.size());
}

void shard_ptrs(BlockBuffer& buf, size_t n, size_t S, uint8_t** out) {
    for (size_t i = 0; i < n; ++i) out[i] = buf.data() + i * S;
}

}  // namespace

VirtualBlock::VirtualBlock() : st_(std::make_shared<State>()) {}

void VirtualBlock::set_options(const VfsOptions& o) {
    opt_ = o;
    std::lock_guard<std::mutex> lock(st_->buf_mu);
    st_->buffer.want_pinned(o.pinned_buffers);
}

size_t VirtualBlock::shard_size() const { return calculate_shard_size(size, topology.data); }

Status VirtualBlock::create(uint64_t ino, uint64_t idx, std::shared_ptr<const ShmrFsConfig> cfg, uint64_t size,
                            BlockTopology topology, VirtualBlock* out) {
    const std::string pool = cfg->write_pool;
    return create_with_pool(ino, idx, pool, std::move(cfg), size, topology, out);
}

// block.rs:207-266
Status VirtualBlock::create_with_pool(uint64_t ino, uint64_t idx, const std::string& pool,
                                      std::shared_ptr<const ShmrFsConfig> cfg, uint64_t size,
                                      BlockTopology topology, VirtualBlock* out) {
    size_t needed = 1;
    std::string ident = "single";
    if (topology.kind == BlockTopology::Mirror) {
        needed = topology.n;
        ident = "mirror";
    } else if (topology.kind == BlockTopology::Erasure) {
        needed = size_t(topology.data) + topology.parity;
        ident = "ec" + std::to_string(topology.data) + std::to_string(topology.parity);
    }
    std::vector<std::string> buckets;
    if (auto e = cfg->select_buckets(pool, needed, &buckets)) return e;
    VirtualBlock b;
    b.ino = ino;
    b.idx = idx;
    b.size = size;
    b.topology = topology;
    for (size_t i = 0; i < buckets.size(); ++i) {
        VirtualPath vp{pool, buckets[i],
                       std::to_string(ino) + ":" + std::to_string(idx) + "_" + ident + "_" + std::to_string(i) + "." +
                           VP_DEFAULT_FILE_EXT};
        if (auto e = vp.create(*cfg)) return e;   // create the backing file now
        b.shards.push_back(vp);
    }
    b.cfg_ = std::move(cfg);
    *out = b;
    return std::nullopt;
}

// block.rs:269-313
Status VirtualBlock::read(uint64_t pos, uint8_t* buf, size_t len, size_t* nread) const {
    *nread = 0;
    if (len == 0) return std::nullopt;
    if (!st_->buffer_loaded.load()) {
        if (auto e = load_block()) return e;
    }
    std::lock_guard<std::mutex> lock(st_->buf_mu);
    const auto& data = st_->buffer;
    if (data.size() < pos) return ShmrError{ShmrError::OutOfSpace};
    const size_t n = std::min<size_t>(data.size() - pos, len);
    if (n) std::memcpy(buf, data.data() + pos, n);
    *nread = n;
    return std::nullopt;
}

// block.rs:315-370
Status VirtualBlock::write(uint64_t pos, const uint8_t* buf, size_t len, size_t* nwritten) const {
    *nwritten = 0;
    if (pos + len > size) return ShmrError{ShmrError::OutOfSpace};
    {
        std::lock_guard<std::mutex> lock(st_->buf_mu);
        auto& buffer = st_->buffer;
        // one allocation for the block's lifetime: (k+p)*S for Erasure
        buffer.reserve(topology.kind == BlockTopology::Erasure
                           ? std::max<size_t>(size, (size_t(topology.data) + topology.parity) * shard_size())
                           : size_t(size));
        const size_t end = size_t(pos) + len;
        if (buffer.size() < end) buffer.resize(end);   // grow to pos+len only, not to size
        if (len) std::memcpy(buffer.data() + pos, buf, len);
    }
    st_->should_flush.store(false);   // the reference stores false here (block.rs:367)
    *nwritten = len;
    return std::nullopt;
}

// block.rs:373-452
Status VirtualBlock::sync_data(bool force, int device, PhaseTimes* times) const {
    if (!force && !st_->should_flush.load()) return std::nullopt;
    if (!st_->shard_loaded.load()) {
        if (auto e = open_handles()) return e;
    }
    std::lock_guard<std::mutex> lock(st_->buf_mu);
    auto& buffer = st_->buffer;
    if (buffer.empty()) return std::nullopt;   // block.rs:389-391
    std::lock_guard<std::mutex> hl(st_->handles_mu);
    const size_t nh = st_->handles.size();
    std::vector<Status> res(nh);
    if (topology.kind == BlockTopology::Erasure) {
        EcStatus es;
        auto r = ReedSolomon::create(topology.data, topology.parity, &es);   // block.rs:405
        if (!r) return ec_error(es.code);
        if (device != 0) {
            const int rc = shmr_ec_set_device(r->handle(), device);
            if (rc != SHMR_EC_OK) return ec_error(rc);
        }
        const size_t S = shard_size();                                      // block.rs:406
        std::vector<uint8_t> tail;
        if (auto e = prepare_erasure(buffer, topology, S, opt_.release_u8_wrap, &tail)) return e;
        const size_t n = size_t(topology.data) + topology.parity;
        std::vector<uint8_t*> ptrs(n);
        shard_ptrs(buffer, n, S, ptrs.data());
        // block.rs:427 (.unwrap() in the reference).  Started: with mapped Block-
        // Cache buffers the GPU still runs when it returns, and the data shard
        // files (the encode's inputs, never written by it) go out meanwhile;
        // the parity files after the wait.  block.rs:436-439 writes all k+p.
        const double tc = times ? now_s() : 0;
        EcOp op;
        es = r->encode_start(ptrs.data(), n, S, &op);
        if (es.ok()) {
            const size_t k = topology.data, nw = std::min(n, nh);
            const double tw = times ? now_s() : 0;
            parallel_for(std::min(k, nw), 16, [&](size_t i) { res[i] = st_->write_shard(i, *cfg_, opt_, ptrs[i], S); });
            const double tw2 = times ? now_s() : 0;
            es = op.wait();
            if (es.ok() && opt_.fault_encode_wait) es = EcStatus{SHMR_EC_DEVICE_ERROR};   // test hook
            if (!es.ok()) {
                // The data shard files already hold the new bytes while the parity
                // files hold the old parity: the stripe is no codeword.  Make that
                // detectable under every option set -- every parity file unlinked
                // (its handles closed; the next flush recreates it, ensure_fd): a
                // later load fails to open it (reference rule) or, under
                // missing_shard_is_erasure, counts it as an erasure, never as a
                // present shard (a truncated file would be zero-padded and kept
                // present when short_shard_is_erasure is off, block.rs:548-551,
                // and a lost data shard then rebuilt from zeros) -- and leave the
                // block dirty so the next flush re-encodes.  (The reference
                // unwraps the encode before any write, block.rs:427.)
                for (size_t i = k; i < nw; ++i) {
                    fs::path file;
                    if (!st_->handles[i].first.resolve(*cfg_, &file, nullptr) && ::unlink(file.c_str()) == 0 &&
                        opt_.fsync_shards) {   // the unlink reaches the directory
                        const int dfd = ::open(file.parent_path().c_str(), O_RDONLY | O_DIRECTORY);
                        if (dfd >= 0) {
                            (void)::fsync(dfd);
                            ::close(dfd);
                        }
                    }
                    if (st_->handles[i].second >= 0) ::close(st_->handles[i].second);
                    st_->handles[i].second = -1;
                    if (i < st_->dfds.size()) {
                        if (st_->dfds[i] >= 0) ::close(st_->dfds[i]);
                        st_->dfds[i] = -1;
                    }
                }
                st_->should_flush.store(true);
            }
            if (times) times->codec_s += now_s() - tc - (tw2 - tw), times->io_s += tw2 - tw;
            if (es.ok() && nw > k) {
                const double tp = times ? now_s() : 0;
                parallel_for(nw - k, 16, [&](size_t j) {
                    const size_t i = k + j;
                    res[i] = st_->write_shard(i, *cfg_, opt_, ptrs[i], S);
                });
                if (times) times->io_s += now_s() - tp;
            }
        }
        if (!es.ok()) {
            restore_tail(buffer, topology, S, tail);
            return ec_error(es.code);
        }
        restore_tail(buffer, topology, S, tail);
    } else {
        const size_t copies = topology.kind == BlockTopology::Single ? 1 : std::min<size_t>(topology.n, nh);
        parallel_for(copies, 16, [&](size_t i) {
            res[i] = st_->ensure_fd(i, *cfg_);
            if (!res[i]) res[i] = write_path(st_->handles[i].second, buffer.data(), buffer.size(), opt_.fsync_shards);
        });
    }
    for (auto& e : res)
        if (e) return e;
    st_->should_flush.store(false);
    return std::nullopt;
}

// block.rs:455-493
Status VirtualBlock::open_handles() const {
    if (!cfg_) return fs_error(EINVAL);   // the reference panics: pool_map not populated
    std::lock_guard<std::mutex> lock(st_->handles_mu);
    st_->close_handles();
    for (auto& shard : shards) {
        fs::path file;
        if (auto e = shard.resolve(*cfg_, &file, nullptr)) return e;
        const int fd = ::open(file.c_str(), O_RDWR);
        if (fd < 0 && !opt_.missing_shard_is_erasure) {
            const int err = errno;
            st_->close_handles();
            return fs_error(err);
        }
        st_->handles.emplace_back(shard, fd);
    }
    st_->dfds.assign(st_->handles.size(), -1);
    st_->shard_loaded.store(true);
    return std::nullopt;
}

// block.rs:496-584
Status VirtualBlock::load_block(bool* reconstructed, int device, PhaseTimes* times,
                                const std::function<void(const uint8_t*)>* during) const {
    if (reconstructed) *reconstructed = false;
    if (!st_->shard_loaded.load()) {
        if (auto e = open_handles()) return e;
    }
    std::lock_guard<std::mutex> lock(st_->buf_mu);
    auto& buffer = st_->buffer;
    std::lock_guard<std::mutex> hl(st_->handles_mu);
    if (topology.kind == BlockTopology::Single) {
        buffer.reserve(size);
        if (buffer.size() < size) buffer.resize(size);
        const int fd = st_->handles[0].second;
        const ssize_t n = fd < 0 ? 0 : ::read(fd, buffer.data(), buffer.size());   // one read() call
        if (n < 0) return fs_error(errno);
    } else if (topology.kind == BlockTopology::Mirror) {
        return fs_error(ENOSYS);   // todo!("Implement Mirrored Read") in the reference
    } else {
        if (topology.version != 1) return fs_error(ENOSYS);   // unimplemented!()
        EcStatus es;
        auto r = ReedSolomon::create(topology.data, topology.parity, &es);
        if (!r) return ec_error(es.code);
        if (device != 0) {
            const int rc = shmr_ec_set_device(r->handle(), device);
            if (rc != SHMR_EC_OK) return ec_error(rc);
        }
        const size_t S = shard_size();
        const size_t n = st_->handles.size();
        buffer.reserve(std::max<size_t>(size, n * S));
        if (buffer.size() < size) buffer.set_len_uninit(size);   // every slot byte is overwritten below
        std::vector<uint8_t*> ptrs(n);
        shard_ptrs(buffer, n, S, ptrs.data());
        std::vector<uint8_t> present(n, 0), odd(n, 0), plan(n, kRead);
        std::vector<int> fds(n);
        for (size_t i = 0; i < n; ++i) fds[i] = st_->handles[i].second;
        const bool planned = opt_.read_needed_shards && opt_.pread_from_start && size <= size_t(topology.data) * S &&
                             plan_needed_reads(fds.data(), n, topology.data, S, opt_.short_shard_is_erasure, plan.data());
        if (!planned) std::fill(plan.begin(), plan.end(), uint8_t(kRead));
        auto read_one = [&](size_t i) {
            bool o = false;
            if (fds[i] >= 0 && st_->read_shard(i, fds[i], *cfg_, opt_, ptrs[i], S, &o) == 0) {   // Err -> None
                present[i] = !(o && opt_.short_shard_is_erasure);
                odd[i] = o;
            }
        };
        const double tr = times ? now_s() : 0;
        parallel_for(n, 16, [&](size_t i) {
            if (plan[i] == kRead) read_one(i);
            else if (plan[i] == kPresentUnread) present[i] = 1;
        });
        if (planned) {   // a planned read failed or changed length: read the rest as well
            bool redo = false;
            for (size_t i = 0; i < n; ++i) redo |= plan[i] == kRead && (!present[i] || odd[i]);
            if (redo)
                parallel_for(n, 16, [&](size_t i) {
                    if (plan[i] == kPresentUnread) {
                        present[i] = 0;
                        read_one(i);
                    }
                });
        }
        if (times) times->io_s += now_s() - tr;
        bool missing = false;
        for (size_t i = 0; i < n; ++i) missing |= !present[i] || odd[i];
        if (missing) {
            const double tc = times ? now_s() : 0;
            double td = 0;
            if (during && *during) {   // copies of the present shards overlap the GPU work
                EcOp op;
                es = r->reconstruct_start(ptrs.data(), present.data(), n, S, false, &op);   // block.rs:560
                if (es.ok()) {
                    const double t1 = now_s();
                    (*during)(present.data());
                    td = now_s() - t1;
                    es = op.wait();
                }
            } else {
                es = r->reconstruct_in_place(ptrs.data(), present.data(), n, S, false);   // block.rs:560 (unwrap)
            }
            if (times) times->codec_s += now_s() - tc - td, times->overlap_s += td;
            if (!es.ok()) return ec_error(es.code);
            if (reconstructed) *reconstructed = true;
        }
        buffer.resize(size);   // ec_data[..size] (block.rs:576); the bytes are already in place
    }
    st_->buffer_loaded.store(true);
    return std::nullopt;
}

// block.rs:586-596
Status VirtualBlock::drop_buffer() const {
    if (auto e = sync_data(true)) return e;
    std::lock_guard<std::mutex> lock(st_->buf_mu);
    st_->buffer.release();
    st_->buffer_loaded.store(false);
    return std::nullopt;
}

// block.rs:598-608.  The reference takes the handle lock and then calls
// sync_data, which takes it again (a self-deadlock whenever the buffer holds
// data); here the flush runs first.
Status VirtualBlock::drop_handles() const {
    if (auto e = sync_data(true)) return e;
    std::lock_guard<std::mutex> lock(st_->handles_mu);
    st_->close_handles();
    st_->shard_loaded.store(false);
    return std::nullopt;
}

std::vector<uint8_t> VirtualBlock::buffer_snapshot() const {
    std::lock_guard<std::mutex> lock(st_->buf_mu);
    const auto& b = st_->buffer;
    return std::vector<uint8_t>(b.data(), b.data() + b.size());
}

bool VirtualBlock::buffer_loaded() const { return st_->buffer_loaded.load(); }

size_t VirtualBlock::buffered_len() const {
    std::lock_guard<std::mutex> lock(st_->buf_mu);
    return st_->buffer.size();
}

bool VirtualBlock::buffer_pinned() const {
    std::lock_guard<std::mutex> lock(st_->buf_mu);
    return st_->buffer.pinned();
}

// ---------------------------------------------------------------------------
// VirtualFile (mod.rs:63-272)
// ---------------------------------------------------------------------------
VirtualFile VirtualFile::new_with(uint64_t ino, uint64_t size) {
    VirtualFile vf;
    vf.ino = ino;
    vf.size = size;
    return vf;
}

void VirtualFile::populate(std::shared_ptr<const ShmrFsConfig> cfg) {
    for (auto& b : blocks) b.populate(cfg);
    cfg_ = std::move(cfg);
}

void VirtualFile::set_options(const VfsOptions& o) {
    opt_ = o;
    for (auto& b : blocks) b.set_options(o);
}

size_t VirtualFile::batch_bytes(bool load) const {
    if (pipeline_batch_bytes != kAutoBatch) return pipeline_batch_bytes;
    // Measured (shmr_vfs_bench, 256 MiB file, mapped Block Cache): flushes
    // pipeline 128 MiB encode batches against the shard writes; loads pipeline
    // 64 MiB batches of shard reads against the zero-copy reconstruct (34 vs
    // 30 GiB/s one batch; 16-32 MiB batches lose to per-batch fan-out costs).
    // Pageable buffers run one batch (the staged codec competes with the
    // shard-file memcpy for host memory bandwidth).
    if (!opt_.pinned_buffers) return 0;
    return load ? size_t(64) << 20 : size_t(128) << 20;
}

Status VirtualFile::allocate_block() {
    if (!cfg_) return fs_error(EINVAL);
    VirtualBlock b;
    if (auto e = VirtualBlock::create(ino, blocks.size() + 1, cfg_, block_size, BlockTopology::single(), &b))
        return e;   // the next block number is len + 1 (mod.rs:119-127)
    b.set_options(opt_);
    blocks.push_back(b);
    return std::nullopt;
}

// The blocks VirtualFile::read's chunk loop visits for (pos, len).
std::vector<size_t> VirtualFile::blocks_for_range(uint64_t pos, size_t len) const {
    std::vector<size_t> out;
    const uint64_t start_chunk = pos / chunk_size;
    const uint64_t end_chunk = len / chunk_size + start_chunk;
    for (uint64_t c = start_chunk; c <= end_chunk; ++c) {
        const size_t b = size_t(c * chunk_size / block_size);
        if (b < blocks.size() && (out.empty() || out.back() != b)) out.push_back(b);
    }
    return out;
}

namespace {

// A run of consecutive chunks inside one block, copied as one memcpy.
struct ReadRun {
    size_t blk;
    uint64_t block_pos;
    size_t off, len;
};

}  // namespace

// Plan of VirtualFile::read: runs of consecutive chunks inside one block.
// When the block holds every byte of a run (buffered(blk) >= block_pos + n),
// the reference's per-chunk copies are one contiguous copy (same bytes, same
// count) at a known offset; planning stops at the first run that could come
// up short, and *c / *done say where the reference's chunk loop takes over.
template <class Buffered>
static std::vector<ReadRun> plan_read_runs(const std::vector<VirtualBlock>& blocks, uint64_t chunk_size,
                                           uint64_t block_size, uint64_t pos, size_t len, Buffered buffered,
                                           uint64_t* c_out, size_t* done_out) {
    const uint64_t start_chunk = pos / chunk_size;
    const uint64_t end_chunk = len / chunk_size + start_chunk;
    std::vector<ReadRun> runs;
    uint64_t c = start_chunk;
    size_t done = 0;
    for (; c <= end_chunk;) {
        const uint64_t block_idx = c * chunk_size / block_size;
        const uint64_t block_pos = c * chunk_size % block_size;
        if (block_idx >= blocks.size()) break;
        const uint64_t run = std::min<uint64_t>(end_chunk - c + 1, (block_size - block_pos + chunk_size - 1) / chunk_size);
        const size_t want = size_t(std::min<uint64_t>(uint64_t(done) + run * chunk_size, len)) - done;
        if (want > 0 && buffered(size_t(block_idx)) < block_pos + want) break;
        if (want > 0) runs.push_back({size_t(block_idx), block_pos, done, want});
        done += want;
        c += run;
    }
    *c_out = c;
    *done_out = done;
    return runs;
}

// mod.rs:137-180.  Chunks map to (block, block_pos) from chunk_idx * chunk_size,
// ignoring pos % chunk_size, exactly as the reference does.
Status VirtualFile::read(uint64_t pos, uint8_t* buf, size_t len, size_t* nread) {
    *nread = 0;
    if (!cfg_) return fs_error(EINVAL);
    if (len == 0 || size == 0) return std::nullopt;
    if (pos > size) return ShmrError{ShmrError::EndOfFile};
    // Copy-out overlapped with the load: the runs of blocks that the batched
    // load is about to bring in (an Erasure v1 block always ends with its full
    // `size` buffered) are planned up front and copied as soon as their batch
    // is loaded, while later batches are still reading / reconstructing.
    uint64_t c_early = 0;
    size_t done_early = 0;
    const std::vector<ReadRun> early = plan_read_runs(
        blocks, chunk_size, block_size, pos, len,
        [&](size_t bi) -> uint64_t {
            const VirtualBlock& b = blocks[bi];
            if (b.buffer_loaded()) return b.buffered_len();
            const bool erasure1 = b.topology.kind == BlockTopology::Erasure && b.topology.version == 1;
            return erasure1 ? b.size : 0;
        },
        &c_early, &done_early);
    std::map<size_t, std::vector<size_t>> early_of;   // block -> early run indices
    for (size_t i = 0; i < early.size(); ++i) early_of[early[i].blk].push_back(i);
    std::vector<uint8_t> copied(early.size(), 0);
    // Pieces of a run still to copy after its block's reconstruct: a run whose
    // block was rebuilt by a per-block task had its bytes in present data
    // shards copied while the GPU rebuilt the rest (during_rebuild).
    std::vector<std::vector<std::pair<uint64_t, size_t>>> rest(early.size());
    std::vector<uint8_t> split(early.size(), 0);
    auto during_rebuild = [&](size_t bi, const uint8_t* present) {
        auto it = early_of.find(bi);
        if (it == early_of.end()) return;
        const VirtualBlock& b = blocks[bi];
        const uint64_t S = b.shard_size(), k = b.topology.data;
        const auto& data = b.st_->buffer;   // locked by the load task (this thread)
        for (size_t q : it->second) {
            const ReadRun& r = early[q];
            if (data.size() < r.block_pos + r.len || S == 0) continue;
            for (uint64_t p0 = r.block_pos, end = r.block_pos + r.len; p0 < end;) {
                const uint64_t s = p0 / S, p1 = std::min(end, (s + 1) * S);
                if (s < k && present[s]) std::memcpy(buf + r.off + (p0 - r.block_pos), data.data() + p0, p1 - p0);
                else rest[q].emplace_back(p0, size_t(p1 - p0));
                p0 = p1;
            }
            split[q] = 1;
        }
    };
    auto on_batch = [&](const std::vector<size_t>& loaded) {
        std::vector<size_t> todo;
        for (size_t bi : loaded) {
            auto it = early_of.find(bi);
            if (it != early_of.end()) todo.insert(todo.end(), it->second.begin(), it->second.end());
        }
        // load_blocks holds these blocks' locks until this returns; read their
        // buffers directly (VirtualBlock::read would take the lock again)
        parallel_for(todo.size(), todo.size() > 4 ? 8 : 1, [&](size_t q) {
            const ReadRun& r = early[todo[q]];
            const auto& data = blocks[r.blk].st_->buffer;
            if (data.size() < r.block_pos + r.len) return;   // not as planned: the plan below copies it
            if (split[todo[q]]) {
                for (const auto& pc : rest[todo[q]])
                    std::memcpy(buf + r.off + (pc.first - r.block_pos), data.data() + pc.first, pc.second);
            } else {
                std::memcpy(buf + r.off, data.data() + r.block_pos, r.len);
            }
            copied[todo[q]] = 1;
        });
    };
    if (auto e = load_blocks(blocks_for_range(pos, len), on_batch, during_rebuild)) return e;
    uint64_t c = 0;
    size_t done = 0;
    std::vector<ReadRun> runs = plan_read_runs(blocks, chunk_size, block_size, pos, len,
                                               [&](size_t bi) -> uint64_t { return blocks[bi].buffered_len(); },
                                               &c, &done);
    {   // runs already copied during the load (same run, same bytes) are skipped
        std::vector<ReadRun> left;
        size_t e = 0;
        for (const ReadRun& r : runs) {
            while (e < early.size() && early[e].off < r.off) ++e;
            const bool same = e < early.size() && copied[e] && early[e].blk == r.blk &&
                              early[e].block_pos == r.block_pos && early[e].off == r.off && early[e].len == r.len;
            if (!same) left.push_back(r);
        }
        runs.swap(left);
    }
    const uint64_t end_chunk = len / chunk_size + pos / chunk_size;
    std::vector<Status> res(runs.size());
    parallel_for(runs.size(), runs.size() > 4 ? 8 : 1, [&](size_t i) {
        size_t n = 0;
        res[i] = blocks[runs[i].blk].read(runs[i].block_pos, buf + runs[i].off, runs[i].len, &n);
    });
    for (auto& e : res)
        if (e) return e;
    for (; c <= end_chunk; ++c) {   // the reference's loop for the rest
        const uint64_t block_idx = c * chunk_size / block_size;
        const uint64_t block_pos = c * chunk_size % block_size;
        const size_t end = size_t(std::min<uint64_t>(done + chunk_size, len));
        if (block_idx >= blocks.size()) return ShmrError{ShmrError::BlockIndexOutOfBounds};   // panics in the reference
        size_t n = 0;
        if (auto e = blocks[block_idx].read(block_pos, buf + done, end - done, &n)) return e;
        done += n;
    }
    *nread = done;
    return std::nullopt;
}

// mod.rs:182-242
Status VirtualFile::write(uint64_t pos, const uint8_t* buf, size_t len, size_t* nwritten) {
    *nwritten = 0;
    if (!cfg_) return fs_error(EINVAL);
    if (len == 0) return std::nullopt;
    const uint64_t start_chunk = pos / chunk_size;
    const uint64_t end_chunk = len / chunk_size + start_chunk;
    const uint64_t chk_per_blk = block_size / chunk_size;
    // Plan runs of consecutive chunks inside one block (allocating blocks in
    // the reference's order); runs that fit their block are one contiguous
    // write each, done in parallel.  From the first run that does not fit,
    // the rest goes chunk by chunk so OutOfSpace leaves exactly the bytes the
    // reference's loop leaves.
    struct Run {
        size_t blk;
        uint64_t block_pos;
        size_t off, len;
    };
    std::vector<Run> runs;
    uint64_t c = start_chunk;
    size_t written = 0;
    for (; c <= end_chunk;) {
        while (blocks.size() * chk_per_blk <= c)
            if (auto e = allocate_block()) return e;
        const uint64_t block_idx = c * chunk_size / block_size;
        const uint64_t block_pos = c * chunk_size % block_size;
        const uint64_t run = std::min<uint64_t>(end_chunk - c + 1, (block_size - block_pos + chunk_size - 1) / chunk_size);
        const size_t want = size_t(std::min<uint64_t>(uint64_t(written) + run * chunk_size, len)) - written;
        if (block_pos + want > blocks[block_idx].size) break;
        runs.push_back({size_t(block_idx), block_pos, written, want});
        written += want;
        c += run;
    }
    std::vector<Status> res(runs.size());
    parallel_for(runs.size(), runs.size() > 4 ? 8 : 1, [&](size_t i) {
        size_t n = 0;
        res[i] = blocks[runs[i].blk].write(runs[i].block_pos, buf + runs[i].off, runs[i].len, &n);
    });
    for (auto& e : res)
        if (e) return e;
    for (; c <= end_chunk; ++c) {   // the reference's loop for the rest
        while (blocks.size() * chk_per_blk <= c)
            if (auto e = allocate_block()) return e;
        const uint64_t block_idx = c * chunk_size / block_size;
        const uint64_t block_pos = c * chunk_size % block_size;
        const size_t end = size_t(std::min<uint64_t>(written + chunk_size, len));
        size_t n = 0;
        if (auto e = blocks[block_idx].write(block_pos, buf + written, end - written, &n)) return e;
        written += n;
    }
    size = std::max<uint64_t>(size, pos + len);
    *nwritten = written;
    return std::nullopt;
}

namespace {

// Locks held over a batch: every block's buffer lock, then its handle lock,
// in block order (the order VirtualBlock::sync_data / load_block take them).
struct BatchLocks {
    std::vector<std::unique_lock<std::mutex>> held;
};

struct Group {
    unsigned k = 0, p = 0;
    size_t S = 0;
    std::vector<size_t> members;   // block indices
};

}  // namespace

// mod.rs:91-103, MI355X-batched.
Status VirtualFile::sync_data(bool force) {
    last_sync = IoStats{};
    const double t0 = now_s();
    std::vector<Status> results(blocks.size());
    if (opt_.pinned_buffers && pipeline_batch_bytes == kAutoBatch) {
        // one flush task per block (mod.rs:93-96's par_iter), blocks round-robin over the GPUs
        const size_t nd = std::max<size_t>(1, devices.size());
        std::atomic<size_t> coded{0};
        std::mutex tmu;
        parallel_for(blocks.size(), per_block_tasks, [&](size_t i) {
            const VirtualBlock& b = blocks[i];
            const bool dirty = force || b.st_->should_flush.load();
            const double ts = now_s();
            PhaseTimes pt;
            results[i] = b.sync_data(force, devices.empty() ? 0 : devices[i % nd], &pt);
            if (!results[i] && dirty && b.topology.kind == BlockTopology::Erasure) ++coded;
            std::lock_guard<std::mutex> lock(tmu);
            last_sync.task_write_s += pt.io_s;
            last_sync.task_codec_s += pt.codec_s;
            last_sync.task_total_s += now_s() - ts;
            ++last_sync.tasks;
        });
        last_sync.blocks = coded.load();
        last_sync.total_s = now_s() - t0;
        for (auto& r : results)
            if (r) return r;
        return std::nullopt;
    }
    std::map<std::tuple<unsigned, unsigned, size_t>, Group> groups;
    std::vector<size_t> others;
    for (size_t i = 0; i < blocks.size(); ++i) {
        const VirtualBlock& b = blocks[i];
        if (b.topology.kind != BlockTopology::Erasure) {
            others.push_back(i);
            continue;
        }
        if (!force && !b.st_->should_flush.load()) continue;
        const size_t S = b.shard_size();
        Group& g = groups[{b.topology.data, b.topology.parity, S}];
        g.k = b.topology.data;
        g.p = b.topology.parity;
        g.S = S;
        g.members.push_back(i);
    }
    {   // open missing shard handles of every grouped block in parallel
        // (hundreds of open() calls per flush/load; block.rs:455-493 per block)
        std::vector<size_t> need;
        for (auto& kv : groups)
            for (size_t i : kv.second.members)
                if (!blocks[i].st_->shard_loaded.load()) need.push_back(i);
        parallel_for(need.size(), 16, [&](size_t j) { results[need[j]] = blocks[need[j]].open_handles(); });
    }
    BatchLocks locks;
    std::vector<std::vector<uint8_t>> tails(blocks.size());   // release_u8_wrap only
    for (auto& kv : groups) {
        Group& g = kv.second;
        std::vector<size_t> live;
        for (size_t i : g.members) {
            if (results[i]) continue;   // open failed
            VirtualBlock& b = blocks[i];
            locks.held.emplace_back(b.st_->buf_mu);
            if (b.st_->buffer.empty()) continue;   // block.rs:389-391: nothing to write
            if ((results[i] = prepare_erasure(b.st_->buffer, b.topology, g.S, b.opt_.release_u8_wrap, &tails[i])))
                continue;
            locks.held.emplace_back(b.st_->handles_mu);
            live.push_back(i);
        }
        g.members.swap(live);
    }
    last_sync.prepare_s = now_s() - t0;
    // Batches of ~64 MiB of data per (k, p, S): the encode of batch b+1 (one
    // pipelined multi-GPU call) overlaps the shard-file writes of batch b
    // (every (block, shard) file of the batch in parallel, block.rs:436-439).
    struct Batch {
        const Group* g;
        size_t b, e;   // members [b, e)
    };
    std::vector<Batch> batches;
    for (auto& kv : groups) {
        const Group& g = kv.second;
        const size_t bb = batch_bytes(false);
        const size_t per = bb == 0 ? g.members.size() : std::max<size_t>(1, bb / std::max<size_t>(1, size_t(g.k) * g.S));
        for (size_t b = 0; b < g.members.size(); b += per) batches.push_back({&g, b, std::min(g.members.size(), b + per)});
    }
    auto encode_batch = [&](const Batch& bt) {
        const Group& g = *bt.g;
        const size_t n = size_t(g.k) + g.p, nb = bt.e - bt.b;
        std::vector<uint8_t*> ptrs(nb * n);
        for (size_t j = 0; j < nb; ++j) shard_ptrs(blocks[g.members[bt.b + j]].st_->buffer, n, g.S, &ptrs[j * n]);
        EcStatus es;
        auto r = ReedSolomon::create(g.k, g.p, &es);
        const int rc = r ? shmr_ec_encode_blocks_host(r->handle(), ptrs.data(), nb, g.S, devices.data(),
                                                      int(devices.size()))
                         : es.code;
        if (rc != SHMR_EC_OK)
            for (size_t j = bt.b; j < bt.e; ++j) results[g.members[j]] = ec_error(rc);
    };
    auto write_batch = [&](const Batch& bt) {
        const Group& g = *bt.g;
        struct Task {
            size_t blk, shard;
        };
        std::vector<Task> tasks;
        for (size_t j = bt.b; j < bt.e; ++j) {
            const size_t i = g.members[j];
            if (results[i]) continue;
            for (size_t sh = 0; sh < size_t(g.k) + g.p && sh < blocks[i].st_->handles.size(); ++sh) tasks.push_back({i, sh});
        }
        std::vector<Status> task_res(tasks.size());
        parallel_for(tasks.size(), 32, [&](size_t t) {
            auto& st = *blocks[tasks[t].blk].st_;
            task_res[t] = st.write_shard(tasks[t].shard, *cfg_, blocks[tasks[t].blk].opt_,
                                         st.buffer.data() + tasks[t].shard * g.S, g.S);
        });
        for (size_t t = 0; t < tasks.size(); ++t)
            if (task_res[t] && !results[tasks[t].blk]) results[tasks[t].blk] = task_res[t];
        for (size_t j = bt.b; j < bt.e; ++j) {
            const size_t i = g.members[j];
            restore_tail(blocks[i].st_->buffer, blocks[i].topology, g.S, tails[i]);
            if (!results[i]) blocks[i].st_->should_flush.store(false);
        }
    };
    const double t1 = now_s();
    double io_busy = 0;
    std::future<void> writer;
    for (const Batch& bt : batches) {
        const double te = now_s();
        encode_batch(bt);
        last_sync.codec_s += now_s() - te;
        last_sync.blocks += bt.e - bt.b;
        if (writer.valid()) writer.get();
        writer = std::async(std::launch::async, [&, bt] {
            const double tw = now_s();
            write_batch(bt);
            io_busy += now_s() - tw;
        });
    }
    if (writer.valid()) writer.get();
    last_sync.io_s = io_busy;
    last_sync.total_s = now_s() - t1;
    locks.held.clear();
    parallel_for(others.size(), 16, [&](size_t j) { results[others[j]] = blocks[others[j]].sync_data(force); });
    for (auto& r : results)
        if (r) return r;
    return std::nullopt;
}

// Batched load_block (block.rs:496-584) over several blocks: the same rules
// per block, one reconstruct call per (k, p, S) for the blocks with erasures.
Status VirtualFile::load_blocks(const std::vector<size_t>& block_indices,
                                const std::function<void(const std::vector<size_t>&)>& on_batch,
                                const DuringRebuild& during_rebuild) {
    last_load = IoStats{};
    const double t0 = now_s();
    std::vector<Status> results(blocks.size());
    if (opt_.pinned_buffers && pipeline_batch_bytes == kAutoBatch) {
        // one load task per block (block.rs:496-584 each), blocks round-robin over the GPUs
        std::vector<size_t> todo;
        for (size_t i : block_indices) {
            if (i >= blocks.size()) return ShmrError{ShmrError::BlockIndexOutOfBounds};
            if (!blocks[i].st_->buffer_loaded.load()) todo.push_back(i);
        }
        const size_t nd = std::max<size_t>(1, devices.size());
        std::atomic<size_t> rebuilt{0};
        std::mutex tmu;
        parallel_for(todo.size(), per_block_read_tasks, [&](size_t q) {
            const size_t i = todo[q];
            const VirtualBlock& b = blocks[i];
            bool rec = false;
            const double ts = now_s();
            PhaseTimes pt;
            std::function<void(const uint8_t*)> during;
            if (during_rebuild) during = [&, i](const uint8_t* present) { during_rebuild(i, present); };
            results[i] = b.load_block(&rec, devices.empty() ? 0 : devices[i % nd], &pt, &during);
            if (rec) ++rebuilt;
            double copy_s = 0;
            if (!results[i] && on_batch && b.topology.kind == BlockTopology::Erasure) {
                std::lock_guard<std::mutex> lock(b.st_->buf_mu);   // on_batch reads the buffer unlocked
                const double tc = now_s();
                on_batch(std::vector<size_t>{i});
                copy_s = now_s() - tc;
            }
            std::lock_guard<std::mutex> lock(tmu);
            last_load.task_read_s += pt.io_s;
            last_load.task_codec_s += pt.codec_s;
            last_load.task_copy_s += copy_s;
            last_load.task_overlap_s += pt.overlap_s;
            last_load.task_total_s += now_s() - ts;
            ++last_load.tasks;
        });
        last_load.blocks = rebuilt.load();
        last_load.total_s = now_s() - t0;
        for (auto& r : results)
            if (r) return r;
        return std::nullopt;
    }
    std::map<std::tuple<unsigned, unsigned, size_t>, Group> groups;
    std::vector<size_t> others;
    for (size_t i : block_indices) {
        if (i >= blocks.size()) return ShmrError{ShmrError::BlockIndexOutOfBounds};
        const VirtualBlock& b = blocks[i];
        if (b.st_->buffer_loaded.load()) continue;
        if (b.topology.kind != BlockTopology::Erasure || b.topology.version != 1) {
            others.push_back(i);   // Single, Mirror (ENOSYS) and unknown versions: per block
            continue;
        }
        const size_t S = b.shard_size();
        Group& g = groups[{b.topology.data, b.topology.parity, S}];
        g.k = b.topology.data;
        g.p = b.topology.parity;
        g.S = S;
        g.members.push_back(i);
    }
    {   // open missing shard handles of every grouped block in parallel
        // (hundreds of open() calls per flush/load; block.rs:455-493 per block)
        std::vector<size_t> need;
        for (auto& kv : groups)
            for (size_t i : kv.second.members)
                if (!blocks[i].st_->shard_loaded.load()) need.push_back(i);
        parallel_for(need.size(), 16, [&](size_t j) { results[need[j]] = blocks[need[j]].open_handles(); });
    }
    for (auto& kv : groups) {   // blocks whose handles failed to open keep their error
        auto& m = kv.second.members;
        m.erase(std::remove_if(m.begin(), m.end(), [&](size_t i) { return bool(results[i]); }), m.end());
    }
    BatchLocks locks;
    struct Task {
        size_t blk, shard, S;
        uint8_t* slot;
        int fd;
        uint8_t plan;
    };
    std::vector<Task> tasks;
    std::map<size_t, size_t> first_task;   // block -> index of its shard 0 task
    for (auto& kv : groups) {
        Group& g = kv.second;
        const size_t n = size_t(g.k) + g.p;
        for (size_t i : g.members) {
            auto& st = *blocks[i].st_;
            locks.held.emplace_back(st.buf_mu);
            locks.held.emplace_back(st.handles_mu);
            st.buffer.reserve(std::max<size_t>(blocks[i].size, n * g.S));
            if (st.buffer.size() < blocks[i].size) st.buffer.set_len_uninit(blocks[i].size);   // slots overwritten
            first_task[i] = tasks.size();
            for (size_t s = 0; s < n; ++s)
                tasks.push_back({i, s, g.S, st.buffer.data() + s * g.S, s < st.handles.size() ? st.handles[s].second : -1,
                                 uint8_t(kRead)});
            const VfsOptions& o = blocks[i].opt_;
            if (o.read_needed_shards && o.pread_from_start && blocks[i].size <= size_t(g.k) * g.S) {
                std::vector<int> fds(n);
                std::vector<uint8_t> plan(n);
                for (size_t s = 0; s < n; ++s) fds[s] = tasks[first_task[i] + s].fd;
                if (plan_needed_reads(fds.data(), n, g.k, g.S, o.short_shard_is_erasure, plan.data()))
                    for (size_t s = 0; s < n; ++s) tasks[first_task[i] + s].plan = plan[s];
            }
        }
    }
    last_load.prepare_s = now_s() - t0;
    // Batches of ~64 MiB per (k, p, S): the shard-file reads of batch b+1
    // overlap the reconstruct of batch b (one pipelined multi-GPU call for
    // the blocks of b that have an erasure).
    struct Batch {
        const Group* g;
        size_t b, e;   // members [b, e)
    };
    std::vector<Batch> batches;
    for (auto& kv : groups) {
        const Group& g = kv.second;
        const size_t bb = batch_bytes(true);
        const size_t per = bb == 0 ? g.members.size() : std::max<size_t>(1, bb / std::max<size_t>(1, size_t(g.k) * g.S));
        for (size_t b = 0; b < g.members.size(); b += per) batches.push_back({&g, b, std::min(g.members.size(), b + per)});
    }
    std::vector<uint8_t> present(tasks.size(), 0), odd(tasks.size(), 0);
    auto read_batch = [&](const Batch& bt) {
        const size_t n = size_t(bt.g->k) + bt.g->p;
        const size_t t0b = first_task[bt.g->members[bt.b]];
        const size_t nt = (bt.e - bt.b) * n;   // a batch's tasks are contiguous
        auto read_task = [&](size_t t) {
            const Task& tk = tasks[t];
            const VfsOptions& o = blocks[tk.blk].opt_;
            bool od = false;
            if (tk.fd >= 0 && blocks[tk.blk].st_->read_shard(tk.shard, tk.fd, *cfg_, o, tk.slot, tk.S, &od) == 0) {
                present[t] = !(od && o.short_shard_is_erasure);
                odd[t] = od;
            }
        };
        parallel_for(nt, 32, [&](size_t q) {
            const size_t t = t0b + q;
            if (tasks[t].plan == kRead) read_task(t);
            else if (tasks[t].plan == kPresentUnread) present[t] = 1;
        });
        // read_needed_shards: a block whose planned read failed reads the rest too
        std::vector<size_t> redo;
        for (size_t q = 0; q < nt; ++q) {
            const size_t t = t0b + q;
            if (tasks[t].plan == kRead && (!present[t] || odd[t]))
                for (size_t s = 0; s < n; ++s) {
                    const size_t u = first_task[tasks[t].blk] + s;
                    if (tasks[u].plan == kPresentUnread) {
                        tasks[u].plan = kRead;
                        present[u] = 0;
                        redo.push_back(u);
                    }
                }
        }
        parallel_for(redo.size(), 32, [&](size_t q) { read_task(redo[q]); });
    };
    auto reconstruct_batch = [&](const Batch& bt) {
        const Group& g = *bt.g;
        const size_t n = size_t(g.k) + g.p;
        std::vector<size_t> need;
        for (size_t j = bt.b; j < bt.e; ++j) {
            const size_t i = g.members[j];
            bool missing = false;
            for (size_t sh = 0; sh < n; ++sh) missing |= !present[first_task[i] + sh] || odd[first_task[i] + sh];
            if (missing) need.push_back(i);
        }
        if (!need.empty()) {
            std::vector<uint8_t*> ptrs(need.size() * n);
            std::vector<uint8_t> pres(need.size() * n);
            for (size_t j = 0; j < need.size(); ++j)
                for (size_t sh = 0; sh < n; ++sh) {
                    ptrs[j * n + sh] = tasks[first_task[need[j]] + sh].slot;
                    pres[j * n + sh] = present[first_task[need[j]] + sh];
                }
            EcStatus es;
            auto r = ReedSolomon::create(g.k, g.p, &es);
            const int rc = r ? shmr_ec_reconstruct_blocks_host(r->handle(), ptrs.data(), pres.data(), need.size(), g.S,
                                                               0, devices.data(), int(devices.size()))
                             : es.code;
            if (rc != SHMR_EC_OK)
                for (size_t i : need) results[i] = ec_error(rc);
            last_load.blocks += need.size();
        }
        for (size_t j = bt.b; j < bt.e; ++j) {
            const size_t i = g.members[j];
            if (results[i]) continue;
            blocks[i].st_->buffer.resize(blocks[i].size);   // ec_data[..size]
            blocks[i].st_->buffer_loaded.store(true);
        }
    };
    const double t1 = now_s();
    double io_busy = 0;
    std::future<void> reader;
    auto start_read = [&](size_t bi) {
        reader = std::async(std::launch::async, [&, bi] {
            const double tr = now_s();
            read_batch(batches[bi]);
            io_busy += now_s() - tr;
        });
    };
    std::vector<std::future<void>> handed;   // on_batch calls in flight
    if (!batches.empty()) start_read(0);
    for (size_t bi = 0; bi < batches.size(); ++bi) {
        reader.get();
        if (bi + 1 < batches.size()) start_read(bi + 1);
        const double tc = now_s();
        reconstruct_batch(batches[bi]);
        last_load.codec_s += now_s() - tc;
        if (on_batch) {
            std::vector<size_t> loaded;
            for (size_t j = batches[bi].b; j < batches[bi].e; ++j) {
                const size_t i = batches[bi].g->members[j];
                if (!results[i]) loaded.push_back(i);
            }
            handed.push_back(std::async(std::launch::async, [&on_batch, loaded] { on_batch(loaded); }));
        }
    }
    last_load.io_s = io_busy;
    last_load.total_s = now_s() - t1;
    for (auto& f : handed) f.get();   // before the blocks' locks are released
    locks.held.clear();
    parallel_for(others.size(), 16, [&](size_t j) { results[others[j]] = blocks[others[j]].load_block(); });
    for (auto& r : results)
        if (r) return r;
    return std::nullopt;
}

Status VirtualFile::drop_buffers() const {
    for (auto& b : blocks)
        if (auto e = b.drop_buffer()) return e;
    return std::nullopt;
}

Status VirtualFile::drop_handles() const {
    for (auto& b : blocks)
        if (auto e = b.drop_handles()) return e;
    return std::nullopt;
}

// mod.rs:244-271
Status VirtualFile::replace_block(size_t block_idx, VirtualBlock new_block) {
    if (block_idx >= blocks.size()) return ShmrError{ShmrError::BlockIndexOutOfBounds};
    VirtualBlock& old = blocks[block_idx];
    std::vector<uint8_t> buf(old.size, 0);
    size_t n = 0;
    if (auto e = old.read(0, buf.data(), buf.size(), &n)) return e;
    if (auto e = new_block.write(0, buf.data(), buf.size(), &n)) return e;
    if (auto e = new_block.sync_data(true)) return e;
    blocks[block_idx] = new_block;
    return std::nullopt;
}

Status VirtualFile::rewrite_erasure(uint8_t data, uint8_t parity) {
    if (!cfg_) return fs_error(EINVAL);
    std::vector<size_t> todo;
    for (size_t i = 0; i < blocks.size(); ++i) {
        const auto& t = blocks[i].topology;
        if (!(t.kind == BlockTopology::Erasure && t.version == 1 && t.data == data && t.parity == parity))
            todo.push_back(i);
    }
    if (todo.empty()) return std::nullopt;
    if (auto e = load_blocks(todo)) return e;
    VirtualFile staged;   // the new blocks, flushed as one batch
    staged.cfg_ = cfg_;
    staged.opt_ = opt_;
    staged.devices = devices;
    for (size_t i : todo) {
        VirtualBlock& old = blocks[i];
        VirtualBlock nb;
        if (auto e = VirtualBlock::create(ino, old.idx, cfg_, old.size, BlockTopology::erasure(1, data, parity), &nb))
            return e;
        nb.set_options(opt_);
        std::vector<uint8_t> buf(old.size, 0);   // replace_block's full-size copy (mod.rs:253-262)
        size_t n = 0;
        if (auto e = old.read(0, buf.data(), buf.size(), &n)) return e;
        if (auto e = nb.write(0, buf.data(), buf.size(), &n)) return e;
        staged.blocks.push_back(nb);
    }
    if (auto e = staged.sync_data(true)) return e;
    last_sync = staged.last_sync;
    for (size_t j = 0; j < todo.size(); ++j) blocks[todo[j]] = staged.blocks[j];
    return std::nullopt;
}

size_t block_cache_trim() { return BufferPool::get().trim(); }

uint64_t shard_reads_total() { return g_shard_reads.load(); }

DirectIoStats direct_io_stats() {
    DirectStats& d = g_direct();
    DirectIoStats out;
    out.reads = d.reads.load();
    out.writes = d.writes.load();
    out.fallbacks = d.fallbacks.load();
    out.refusals = d.refusals.load();
    std::lock_guard<std::mutex> lock(d.mu);
    out.refused_errno = d.refused_errno;
    out.refused_fs = d.refused_fs;
    out.io_errno = d.io_errno;
    return out;
}

}  // namespace shmr
