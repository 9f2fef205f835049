// C++ host mirror of the reference's StorageBlock layer.  See vfs.hpp.
// Citations are into the reference tree (volfco/shmr @ 2024-08-07).
#include "vfs.hpp"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstring>
#include <thread>

namespace shmr {

namespace {

ShmrError fs_error(int err) { return ShmrError{ShmrError::FsError, err}; }
ShmrError ec_error(int code) { return ShmrError{ShmrError::EcError, code}; }

// write_path (block.rs:611-634): pwrite at offset 0, then fsync.
Status write_path(int fd, const uint8_t* buf, size_t len) {
    size_t done = 0;
    while (done < len) {
        const ssize_t n = ::pwrite(fd, buf + done, len - done, off_t(done));
        if (n < 0) {
            if (errno == EINTR) continue;
            return fs_error(errno);
        }
        done += size_t(n);
    }
    if (::fsync(fd) != 0) return fs_error(errno);
    return std::nullopt;
}

// Read::read_to_end from the handle's current cursor.
int read_to_end(int fd, std::vector<uint8_t>* out, bool from_start) {
    out->clear();
    uint8_t tmp[1 << 16];
    off_t off = 0;
    for (;;) {
        const ssize_t n = from_start ? ::pread(fd, tmp, sizeof(tmp), off) : ::read(fd, tmp, sizeof(tmp));
        if (n < 0) {
            if (errno == EINTR) continue;
            return errno;
        }
        if (n == 0) return 0;
        out->insert(out->end(), tmp, tmp + n);
        off += n;
    }
}

// Runs fn(i) for i < n on up to `threads` threads (the reference's rayon fan-out).
template <class F>
void parallel_for(size_t n, size_t threads, F fn) {
    threads = std::max<size_t>(1, std::min(threads, n));
    std::atomic<size_t> next{0};
    auto work = [&] {
        for (size_t i = next++; i < n; i = next++) fn(i);
    };
    std::vector<std::thread> th;
    for (size_t t = 1; t < threads; ++t) th.emplace_back(work);
    work();
    for (auto& t : th) t.join();
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
// VirtualBlock
// ---------------------------------------------------------------------------
struct VirtualBlock::State {
    std::mutex handles_mu;
    std::vector<std::pair<VirtualPath, int>> handles;   // fd -1: missing (opt-in)
    std::atomic<bool> shard_loaded{false};
    std::atomic<bool> should_flush{false};
    std::atomic<bool> buffer_loaded{false};
    std::mutex buf_mu;
    std::vector<uint8_t> buffer;
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
    void close_handles() {
        for (auto& h : handles)
            if (h.second >= 0) ::close(h.second);
        handles.clear();
    }
    ~State() { close_handles(); }
};

VirtualBlock::VirtualBlock() : st_(std::make_shared<State>()) {}

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
    std::memcpy(buf, data.data() + pos, n);
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
        const size_t end = size_t(pos) + len;
        if (buffer.size() < end) buffer.resize(end, 0);   // grow to pos+len only, not to size
        if (len) std::memcpy(buffer.data() + pos, buf, len);
    }
    st_->should_flush.store(false);   // the reference stores false here (block.rs:367)
    *nwritten = len;
    return std::nullopt;
}

bool VirtualBlock::erasure_shards_for_sync(bool force, std::vector<std::vector<uint8_t>>* shards, Status* st) const {
    *st = std::nullopt;
    if (topology.kind != BlockTopology::Erasure) return false;
    if (!force && !st_->should_flush.load()) return false;
    std::lock_guard<std::mutex> lock(st_->buf_mu);
    const auto& buffer = st_->buffer;
    if (buffer.empty()) return false;
    const unsigned data = topology.data, parity = topology.parity;
    EcStatus es;
    if (!ReedSolomon::create(data, parity, &es)) {   // ReedSolomon::new(data, parity)? (block.rs:405)
        *st = ec_error(es.code);
        return false;
    }
    const size_t S = calculate_shard_size(size, topology.data);   // block.rs:406
    shards->clear();
    for (size_t off = 0; off < buffer.size(); off += S) {           // buffer.chunks(S), zero padded
        const size_t n = std::min(S, buffer.size() - off);
        shards->emplace_back(S, 0);
        std::memcpy(shards->back().data(), buffer.data() + off, n);
    }
    if (shards->size() > data) {
        // block.rs:421 computes `data - nchunks` in u8: the reference panics
        // (debug) or overwrites a data chunk with parity (release).
        *st = ec_error(SHMR_EC_TOO_MANY_DATA_SHARDS);
        return false;
    }
    const size_t extra = parity + (data - shards->size());          // block.rs:421-423
    for (size_t i = 0; i < extra; ++i) shards->emplace_back(S, 0);
    return true;
}

Status VirtualBlock::write_shards(const std::vector<std::vector<uint8_t>>& shards) const {
    if (!st_->shard_loaded.load()) {
        if (auto e = open_handles()) return e;
    }
    std::lock_guard<std::mutex> lock(st_->handles_mu);
    for (size_t i = 0; i < shards.size() && i < st_->handles.size(); ++i) {   // block.rs:436-439
        if (auto e = st_->ensure_fd(i, *cfg_)) return e;
        if (auto e = write_path(st_->handles[i].second, shards[i].data(), shards[i].size())) return e;
    }
    st_->should_flush.store(false);
    return std::nullopt;
}

// block.rs:373-452
Status VirtualBlock::sync_data(bool force) const {
    if (!force && !st_->should_flush.load()) return std::nullopt;
    if (!st_->shard_loaded.load()) {
        if (auto e = open_handles()) return e;
    }
    if (topology.kind == BlockTopology::Erasure) {
        std::vector<std::vector<uint8_t>> shards;
        Status st;
        if (!erasure_shards_for_sync(true, &shards, &st)) return st;   // empty buffer: nothing written
        EcStatus es;
        auto r = ReedSolomon::create(topology.data, topology.parity, &es);
        if (!r) return ec_error(es.code);
        es = r->encode(shards);   // block.rs:427 (.unwrap() in the reference)
        if (!es.ok()) return ec_error(es.code);
        return write_shards(shards);
    }
    std::lock_guard<std::mutex> lock(st_->buf_mu);
    if (st_->buffer.empty()) return std::nullopt;   // block.rs:389-391
    std::lock_guard<std::mutex> hl(st_->handles_mu);
    if (topology.kind == BlockTopology::Single) {
        if (auto e = st_->ensure_fd(0, *cfg_)) return e;
        if (auto e = write_path(st_->handles[0].second, st_->buffer.data(), st_->buffer.size())) return e;
    } else {
        for (size_t i = 0; i < topology.n && i < st_->handles.size(); ++i) {
            if (auto e = st_->ensure_fd(i, *cfg_)) return e;
            if (auto e = write_path(st_->handles[i].second, st_->buffer.data(), st_->buffer.size())) return e;
        }
    }
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
        if (fd < 0) {
            if (!opt_.missing_shard_is_erasure) {
                const int err = errno;
                st_->close_handles();
                return fs_error(err);
            }
        }
        st_->handles.emplace_back(shard, fd);
    }
    st_->shard_loaded.store(true);
    return std::nullopt;
}

// block.rs:496-584
Status VirtualBlock::load_block() const {
    if (!st_->shard_loaded.load()) {
        if (auto e = open_handles()) return e;
    }
    std::lock_guard<std::mutex> lock(st_->buf_mu);
    auto& buffer = st_->buffer;
    if (buffer.size() < size) buffer.resize(size, 0);
    std::lock_guard<std::mutex> hl(st_->handles_mu);
    if (topology.kind == BlockTopology::Single) {
        const int fd = st_->handles[0].second;
        const ssize_t n = fd < 0 ? 0 : ::read(fd, buffer.data(), buffer.size());   // one read() call
        if (n < 0) return fs_error(errno);
    } else if (topology.kind == BlockTopology::Mirror) {
        return fs_error(ENOSYS);   // todo!("Implement Mirrored Read") in the reference
    } else {
        if (topology.version != 1) return fs_error(ENOSYS);   // unimplemented!()
        const size_t S = calculate_shard_size(size, topology.data);
        EcStatus es;
        auto r = ReedSolomon::create(topology.data, topology.parity, &es);
        if (!r) return ec_error(es.code);
        bool missing = false;
        std::vector<std::optional<std::vector<uint8_t>>> ec(st_->handles.size());
        for (size_t i = 0; i < st_->handles.size(); ++i) {
            const int fd = st_->handles[i].second;
            std::vector<uint8_t> b;
            if (fd < 0 || read_to_end(fd, &b, opt_.pread_from_start) != 0) {   // Err -> None
                missing = true;
                continue;
            }
            if (b.size() != S) {   // len != S: zero-pad, stays present (block.rs:548-551)
                missing = true;
                if (opt_.short_shard_is_erasure) continue;
                b.resize(S, 0);
            }
            ec[i] = std::move(b);
        }
        if (missing) {
            es = r->reconstruct(ec);   // block.rs:560 (.unwrap() in the reference)
            if (!es.ok()) return ec_error(es.code);
        }
        std::vector<uint8_t> all;
        all.reserve(ec.size() * S);
        for (auto& s : ec) all.insert(all.end(), s->begin(), s->end());
        std::memcpy(buffer.data(), all.data(), size_t(size));   // ec_data[..size]
    }
    st_->buffer_loaded.store(true);
    return std::nullopt;
}

// block.rs:586-596
Status VirtualBlock::drop_buffer() const {
    if (auto e = sync_data(true)) return e;
    std::lock_guard<std::mutex> lock(st_->buf_mu);
    st_->buffer = std::vector<uint8_t>();
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
    return st_->buffer;
}

bool VirtualBlock::buffer_loaded() const { return st_->buffer_loaded.load(); }

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

Status VirtualFile::allocate_block() {
    if (!cfg_) return fs_error(EINVAL);
    VirtualBlock b;
    if (auto e = VirtualBlock::create(ino, blocks.size() + 1, cfg_, block_size, BlockTopology::single(), &b))
        return e;   // the next block number is len + 1 (mod.rs:119-127)
    blocks.push_back(b);
    return std::nullopt;
}

// mod.rs:137-180.  Chunks map to (block, block_pos) from chunk_idx * chunk_size,
// ignoring pos % chunk_size, exactly as the reference does.
Status VirtualFile::read(uint64_t pos, uint8_t* buf, size_t len, size_t* nread) const {
    *nread = 0;
    if (!cfg_) return fs_error(EINVAL);
    if (len == 0 || size == 0) return std::nullopt;
    if (pos > size) return ShmrError{ShmrError::EndOfFile};
    const uint64_t start_chunk = pos / chunk_size;
    const uint64_t end_chunk = len / chunk_size + start_chunk;
    size_t done = 0;
    for (uint64_t c = start_chunk; c <= end_chunk; ++c) {
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
    size_t written = 0;
    for (uint64_t c = start_chunk; c <= end_chunk; ++c) {
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

// mod.rs:91-103, MI355X-batched: Erasure blocks of the same (k, p) are
// encoded in one pipelined GPU call, then every block's shard files are
// written from a thread pool (the rayon fan-out); errors are reported after
// every block was attempted.
Status VirtualFile::sync_data(bool force, const std::vector<int>& devices) const {
    std::vector<Status> results(blocks.size());
    struct Group {
        std::vector<size_t> members;
        std::vector<std::vector<std::vector<uint8_t>>> shards;
    };
    std::map<std::pair<unsigned, unsigned>, Group> groups;
    std::vector<size_t> others;
    for (size_t i = 0; i < blocks.size(); ++i) {
        const VirtualBlock& b = blocks[i];
        if (b.topology.kind != BlockTopology::Erasure) {
            others.push_back(i);
            continue;
        }
        std::vector<std::vector<uint8_t>> sh;
        Status st;
        if (!b.erasure_shards_for_sync(force, &sh, &st)) {
            results[i] = st;
            continue;
        }
        Group& g = groups[{b.topology.data, b.topology.parity}];
        g.members.push_back(i);
        g.shards.push_back(std::move(sh));
    }
    for (auto& kv : groups) {
        Group& g = kv.second;
        EcStatus es;
        auto r = ReedSolomon::create(kv.first.first, kv.first.second, &es);
        const size_t t = size_t(kv.first.first) + kv.first.second;
        // one batch per shard length (blocks of a file share it)
        std::map<size_t, std::vector<size_t>> by_len;
        for (size_t j = 0; j < g.members.size(); ++j) by_len[g.shards[j][0].size()].push_back(j);
        for (auto& lv : by_len) {
            std::vector<uint8_t*> ptrs;
            for (size_t j : lv.second)
                for (size_t i = 0; i < t; ++i) ptrs.push_back(g.shards[j][i].data());
            int rc = r ? shmr_ec_encode_blocks_host(r->handle(), ptrs.data(), lv.second.size(), lv.first,
                                                    devices.data(), int(devices.size()))
                       : es.code;
            if (rc != SHMR_EC_OK)
                for (size_t j : lv.second) results[g.members[j]] = ec_error(rc);
        }
        parallel_for(g.members.size(), 16, [&](size_t j) {
            if (!results[g.members[j]]) results[g.members[j]] = blocks[g.members[j]].write_shards(g.shards[j]);
        });
    }
    parallel_for(others.size(), 16, [&](size_t j) { results[others[j]] = blocks[others[j]].sync_data(force); });
    for (auto& r : results)
        if (r) return r;
    return std::nullopt;
}

Status VirtualFile::drop_buffers() const {
    for (auto& b : blocks)
        if (auto e = b.drop_buffer()) return e;
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

}  // namespace shmr
