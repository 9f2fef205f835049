// The reference's CPU path for BASELINE config 5 (VirtualFile write -> sync ->
// lose a shard -> read), timed beside shmr_vfs_bench in the same GPU session.
// A measurement leg with the status of bench.py's cpu_baseline: the erasure
// arithmetic is the oracle's restatement of reed-solomon-erasure's x86 AVX2
// loop (oracle/rs_oracle.c, oracle_encode / oracle_reconstruct_v variant 1);
// it links oracle/_build/librs_oracle.so and nothing of the product
// (libshmr_ec.so, libshmr_vfs.so).
//
// The flow restates the reference step by step, per 4 MiB Erasure(1, 8, 3)
// block of a 256 MiB file:
//   write  VirtualFile::write: the FUSE bytes copied into each block's Vec
//          buffer (src/vfs/block.rs:315-370).
//   flush  VirtualFile::sync_data: rayon par_iter over the blocks
//          (src/vfs/mod.rs:91-103) of VirtualBlock::sync_data (block.rs:404-440):
//          buffer.chunks(S) -> to_vec, the last chunk zero-padded, zero shards up
//          to k + p, ReedSolomon::encode, then write_path per shard in index order
//          (block.rs:611-634: write_all_at(buf, 0), sync_all -- here pwrite at 0
//          and fsync when fsync=1) on the handle open_handles opens (the files
//          themselves are created with the block, VirtualBlock::create, untimed).
//   read   VirtualFile::read (mod.rs:140-175): blocks in sequence, each
//          VirtualBlock::read -> load_block (block.rs:529-579): read_to_end of
//          every shard file (a missing file: None -- the C++ mirror's
//          missing_shard_is_erasure; the reference would fail in open_handles), a
//          short one zero-padded, ReedSolomon::reconstruct when any was missing,
//          every shard concatenated into ec_data, buffer = ec_data[..size], then the
//          block's bytes copied into the caller's buffer.  Timed twice: the
//          reference's sequential loop, and the loads fanned out over the same
//          thread pool as the flush (the parallel form the GPU path runs).
// The files are named as VirtualBlock::create names them (block.rs:207-266:
// "<ino>:<idx>_ec83_<i>.bin" in the bucket), so a GPU leg's files of the same
// (ino, idx) can be compared byte for byte (compare_dir).
//
//   ref_cpu_vfs <bucket_dir> [file_MiB=256] [block_MiB=4] [fsync=0] [reps=3] [threads=16] [compare_dir] [ino=1000]
// Build (one line): g++ -O3 -std=c++17 -o tools/_abx/ref_cpu_vfs tools/ref_cpu_vfs.cpp -Loracle/_build
//          -lrs_oracle -Wl,-rpath,'$ORIGIN/../../oracle/_build' -lpthread
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <functional>
#include <random>
#include <string>
#include <thread>
#include <vector>

extern "C" {
int oracle_encode(int variant, uint32_t k, uint32_t p, uint8_t* const* shards, size_t len);
int oracle_reconstruct_v(int variant, uint32_t k, uint32_t p, uint8_t* const* shards, const uint8_t* present,
                         size_t len, int data_only);
int oracle_has_avx2(void);
}

namespace fs = std::filesystem;

namespace {

constexpr uint32_t K = 8, P = 3, T = K + P;

double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

// calculate_shard_size (src/vfs/mod.rs:16-18): (length as f32 / data as f32).ceil()
size_t shard_size(uint64_t len, uint32_t data) { return size_t(std::ceil(float(len) / float(data))); }

std::string shard_name(uint64_t ino, uint64_t idx, uint32_t i) {
    return std::to_string(ino) + ":" + std::to_string(idx) + "_ec" + std::to_string(K) + std::to_string(P) + "_" +
           std::to_string(i) + ".bin";
}

void die(const char* what) {
    std::perror(what);
    std::exit(1);
}

// rayon's par_iter over n items on `threads` workers (the pool exists before the call)
struct Pool {
    explicit Pool(int n) : n_(n) {
        for (int i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
    }
    ~Pool() {
        stop_ = true;
        gen_.fetch_add(1);
        for (auto& t : th_) t.join();
    }
    void run(size_t items, const std::function<void(size_t)>& f) {
        f_ = &f;
        items_ = items;
        next_ = 0;
        done_ = 0;
        gen_.fetch_add(1, std::memory_order_release);
        while (done_.load(std::memory_order_acquire) != n_) std::this_thread::yield();
    }

private:
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            uint64_t g;
            while ((g = gen_.load(std::memory_order_acquire)) == seen) std::this_thread::yield();
            seen = g;
            if (stop_) return;
            for (size_t i = next_++; i < items_; i = next_++) (*f_)(i);
            done_.fetch_add(1, std::memory_order_acq_rel);
        }
    }
    const int n_;
    std::vector<std::thread> th_;
    const std::function<void(size_t)>* f_ = nullptr;
    size_t items_ = 0;
    std::atomic<size_t> next_{0};
    std::atomic<int> done_{0};
    std::atomic<uint64_t> gen_{0};
    std::atomic<bool> stop_{false};
};

struct Block {
    std::vector<uint8_t> buffer;   // the Block Cache Vec
    std::vector<std::string> files;
};

// REF_CPU_REUSE=1: every thread keeps its shard Vecs across blocks (no fresh
// allocation per flush / load) -- the CPU path's floor without the allocator;
// off (default): fresh Vecs as the reference allocates them (to_vec, vec![0; S],
// read_to_end, ec_data), through glibc malloc like Rust's default allocator.
bool g_reuse = false;
// thread time per phase of the last timed flush / parallel load (ns, summed over threads)
std::atomic<uint64_t> g_t_copy{0}, g_t_code{0}, g_t_io{0}, g_t_concat{0};
inline uint64_t ns_now() {
    return uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(
                         std::chrono::steady_clock::now().time_since_epoch()).count());
}

// VirtualBlock::sync_data, Erasure arm (block.rs:404-440)
void flush(Block& b, uint64_t size, bool do_fsync) {
    const size_t S = shard_size(size, K);
    const uint64_t t0 = ns_now();
    thread_local std::vector<std::vector<uint8_t>> kept;
    std::vector<std::vector<uint8_t>> fresh;
    std::vector<std::vector<uint8_t>>& shards = g_reuse ? kept : fresh;
    if (g_reuse) shards.resize(T);
    size_t j = 0;
    for (size_t off = 0; off < b.buffer.size(); off += S, ++j) {   // buffer.chunks(S).map(to_vec)
        const size_t n = std::min(S, b.buffer.size() - off);
        if (g_reuse) {
            shards[j].assign(b.buffer.begin() + long(off), b.buffer.begin() + long(off + n));
        } else {
            shards.emplace_back(b.buffer.begin() + long(off), b.buffer.begin() + long(off + n));
        }
        if (shards[j].size() < S) shards[j].resize(S, 0);
    }
    for (; j < T; ++j) {   // zero shards up to k + p
        if (g_reuse) shards[j].assign(S, 0);
        else shards.emplace_back(S, 0);
    }
    uint8_t* ptrs[T];
    for (uint32_t i = 0; i < T; ++i) ptrs[i] = shards[i].data();
    const uint64_t t1 = ns_now();
    if (oracle_encode(1, K, P, ptrs, S) != 0) die("encode");
    const uint64_t t2 = ns_now();
    g_t_copy += t1 - t0;
    g_t_code += t2 - t1;
    for (uint32_t i = 0; i < T; ++i) {   // write_path: write_all_at(buf, 0) + sync_all
        const int fd = ::open(b.files[i].c_str(), O_WRONLY);   // open_handles (block.rs:455-493)
        if (fd < 0) die("open for write");
        size_t done = 0;
        while (done < S) {
            const ssize_t w = ::pwrite(fd, shards[i].data() + done, S - done, off_t(done));
            if (w <= 0) die("pwrite");
            done += size_t(w);
        }
        if (do_fsync && ::fsync(fd) != 0) die("fsync");
        ::close(fd);
    }
    g_t_io += ns_now() - t2;
}

// VirtualBlock::load_block, Erasure arm (block.rs:529-579), then the read's copy-out
void load(Block& b, uint64_t size, uint8_t* out) {
    const size_t S = shard_size(size, K);
    const uint64_t t0 = ns_now();
    thread_local std::vector<std::vector<uint8_t>> kept(T);
    std::vector<std::vector<uint8_t>> fresh(T);
    std::vector<std::vector<uint8_t>>& shards = g_reuse ? kept : fresh;
    for (auto& v : shards) v.clear();
    uint8_t present[T];
    bool missing = false;
    for (uint32_t i = 0; i < T; ++i) {
        const int fd = ::open(b.files[i].c_str(), O_RDONLY);
        if (fd < 0) {   // read_to_end error -> None
            present[i] = 0;
            missing = true;
            continue;
        }
        std::vector<uint8_t>& v = shards[i];
        struct stat st{};
        if (::fstat(fd, &st) == 0) v.reserve(size_t(st.st_size));
        uint8_t tmp[1 << 16];
        for (;;) {   // read_to_end
            const ssize_t r = ::read(fd, tmp, sizeof tmp);
            if (r < 0) die("read");
            if (r == 0) break;
            v.insert(v.end(), tmp, tmp + r);
        }
        ::close(fd);
        if (v.size() != S) {
            missing = true;
            v.resize(S, 0);
        }
        present[i] = 1;
    }
    const uint64_t t1 = ns_now();
    g_t_io += t1 - t0;
    if (missing) {   // r.reconstruct(&mut ec_shards): every None filled (vec![0; S])
        uint8_t* ptrs[T];
        for (uint32_t i = 0; i < T; ++i) {
            if (!present[i]) shards[i].assign(S, 0);
            ptrs[i] = shards[i].data();
        }
        if (oracle_reconstruct_v(1, K, P, ptrs, present, S, 0) != 0) die("reconstruct");
    }
    const uint64_t t2 = ns_now();
    g_t_code += t2 - t1;
    thread_local std::vector<uint8_t> kept_data;
    std::vector<uint8_t> fresh_data;
    std::vector<uint8_t>& ec_data = g_reuse ? kept_data : fresh_data;   // every shard concatenated
    ec_data.clear();
    for (uint32_t i = 0; i < T; ++i) ec_data.insert(ec_data.end(), shards[i].begin(), shards[i].end());
    b.buffer.assign(ec_data.begin(), ec_data.begin() + long(size));   // buffer.copy_from_slice(&ec_data[..size])
    std::memcpy(out, b.buffer.data(), size);   // VirtualBlock::read into the FUSE buffer
    g_t_concat += ns_now() - t2;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <bucket_dir> [file_MiB] [block_MiB] [fsync] [reps] [threads] [compare_dir] [ino]\n",
                     argv[0]);
        return 2;
    }
    const std::string bucket = argv[1];
    const uint64_t file_mib = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 256;
    const uint64_t block_mib = argc > 3 ? std::strtoull(argv[3], nullptr, 10) : 4;
    const bool do_fsync = argc > 4 && std::atoi(argv[4]) != 0;
    const int reps = argc > 5 ? std::atoi(argv[5]) : 3;
    const int threads = argc > 6 ? std::atoi(argv[6]) : 16;
    const std::string compare = argc > 7 ? argv[7] : "";
    const uint64_t ino = argc > 8 ? std::strtoull(argv[8], nullptr, 10) : 1000;
    fs::create_directories(bucket);
    g_reuse = std::getenv("REF_CPU_REUSE") && std::atoi(std::getenv("REF_CPU_REUSE")) != 0;
    const uint64_t bsz = block_mib << 20;
    std::vector<uint8_t> src(file_mib << 20);   // shmr_vfs_bench's bytes (same generator and seed)
    std::mt19937_64 rng(0x53484D52);
    for (size_t i = 0; i + 8 <= src.size(); i += 8) {
        const uint64_t v = rng();
        std::memcpy(&src[i], &v, 8);
    }
    const size_t nblk = src.size() / bsz;
    Pool pool(threads);
    double best_w = 1e30, best_s = 1e30, best_rs = 1e30, best_rp = 1e30;
    bool verified = true;
    long compared = -1;
    double flush_ms[3] = {0, 0, 0}, load_ms[3] = {0, 0, 0};
    for (int rep = 0; rep < reps + 1; ++rep) {   // rep 0 warms the page cache and the pool
        std::vector<Block> blocks(nblk);
        for (size_t i = 0; i < nblk; ++i)
            for (uint32_t s = 0; s < T; ++s) blocks[i].files.push_back(bucket + "/" + shard_name(ino, i + 1, s));
        // VirtualBlock::create (block.rs:207-266): every shard file created (and
        // truncated) when the block is made -- before the flush, as in the GPU leg
        for (auto& b : blocks)
            for (auto& f : b.files) {
                const int fd = ::open(f.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
                if (fd < 0) die("create");
                ::close(fd);
            }
        double t = now_s();
        for (size_t i = 0; i < nblk; ++i) {   // VirtualFile::write: bytes into each block's Vec
            blocks[i].buffer.resize(bsz);
            std::memcpy(blocks[i].buffer.data(), src.data() + i * bsz, bsz);
        }
        const double w = now_s() - t;
        g_t_copy = g_t_code = g_t_io = 0;
        t = now_s();
        pool.run(nblk, [&](size_t i) { flush(blocks[i], bsz, do_fsync); });
        const double s = now_s() - t;
        if (rep == reps) {
            flush_ms[0] = g_t_copy / 1e6 / double(nblk);
            flush_ms[1] = g_t_code / 1e6 / double(nblk);
            flush_ms[2] = g_t_io / 1e6 / double(nblk);
        }
        if (rep == reps && !compare.empty()) {   // byte equality with the GPU leg's files
            compared = 0;
            for (size_t i = 0; i < nblk; ++i)
                for (uint32_t sh = 0; sh < T; ++sh) {
                    const std::string other = compare + "/" + shard_name(ino, i + 1, sh);
                    FILE* a = std::fopen(blocks[i].files[sh].c_str(), "rb");
                    FILE* c = std::fopen(other.c_str(), "rb");
                    std::vector<uint8_t> x(bsz), y(bsz);
                    const size_t nx = a ? std::fread(x.data(), 1, x.size(), a) : 0;
                    const size_t ny = c ? std::fread(y.data(), 1, y.size(), c) : size_t(-1);
                    if (a) std::fclose(a);
                    if (c) std::fclose(c);
                    if (nx != ny || std::memcmp(x.data(), y.data(), nx) != 0) {
                        std::fprintf(stderr, "file %s differs from %s\n", blocks[i].files[sh].c_str(), other.c_str());
                        verified = false;
                    }
                    ++compared;
                }
        }
        for (auto& b : blocks) std::vector<uint8_t>().swap(b.buffer);   // drop_buffers
        for (size_t i = 0; i < nblk; ++i) fs::remove(blocks[i].files[i % K]);   // lose data shard b mod 8
        std::vector<uint8_t> back(src.size());
        t = now_s();
        for (size_t i = 0; i < nblk; ++i) load(blocks[i], bsz, back.data() + i * bsz);   // mod.rs:140-175, in sequence
        const double rs = now_s() - t;
        verified = verified && back == src;
        for (auto& b : blocks) std::vector<uint8_t>().swap(b.buffer);
        std::fill(back.begin(), back.end(), 0);
        g_t_code = g_t_io = g_t_concat = 0;
        t = now_s();
        pool.run(nblk, [&](size_t i) { load(blocks[i], bsz, back.data() + i * bsz); });
        const double rp = now_s() - t;
        if (rep == reps) {
            load_ms[0] = g_t_io / 1e6 / double(nblk);
            load_ms[1] = g_t_code / 1e6 / double(nblk);
            load_ms[2] = g_t_concat / 1e6 / double(nblk);
        }
        verified = verified && back == src;
        for (auto& b : blocks)
            for (auto& f : b.files) fs::remove(f);
        if (rep == 0) continue;
        best_w = std::min(best_w, w);
        best_s = std::min(best_s, s);
        best_rs = std::min(best_rs, rs);
        best_rp = std::min(best_rp, rp);
    }
    const double GiB = double(1ull << 30), bytes = double(src.size());
    std::printf("{\"leg\": \"reference CPU path (oracle AVX2 restatement of the crate)\", \"shard_vecs\": \"%s\", "
                "\"avx2\": %s, "
                "\"threads\": %d, \"file_MiB\": %llu, \"block_MiB\": %llu, \"topology\": \"Erasure(1, 8, 3)\", "
                "\"fsync\": %d, \"reps\": %d, \"unit\": \"GiB/s of file data (best rep)\", "
                "\"write_GiBps\": %.2f, \"sync_GiBps\": %.2f, \"read_with_erasure_sequential_GiBps\": %.2f, "
                "\"read_with_erasure_parallel_GiBps\": %.2f, \"files_compared_with_gpu_leg\": %ld, "
                "\"ms_per_block_thread_time\": {\"flush_chunk_copy\": %.3f, \"flush_encode\": %.3f, "
                "\"flush_shard_writes\": %.3f, \"load_shard_reads\": %.3f, \"load_reconstruct\": %.3f, "
                "\"load_concat_copy_out\": %.3f}, \"verified\": %s}\n",
                g_reuse ? "kept per thread (allocator excluded)" : "fresh per block (the reference)",
                oracle_has_avx2() ? "true" : "false", threads, (unsigned long long)file_mib,
                (unsigned long long)block_mib, int(do_fsync), reps, bytes / best_w / GiB, bytes / best_s / GiB,
                bytes / best_rs / GiB, bytes / best_rp / GiB, compared, flush_ms[0], flush_ms[1], flush_ms[2],
                load_ms[0], load_ms[1], load_ms[2], verified ? "true" : "false");
    return verified ? 0 : 1;
}
