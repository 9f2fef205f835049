// Device-resident blocks coded one call per block -- the reference's per-block
// shape (VirtualFile::sync_data fans blocks out over rayon, src/vfs/mod.rs:93-96;
// each VirtualBlock::sync_data encodes its own block, block.rs:427) on a device
// Block Cache -- against one batched call over the same blocks.
//
// RS(8,3) 4 MiB blocks (S = 512 KiB) in padded slots of one hipMalloc'd slab.
// Modes: the batch call (HIP events); T host threads each on a stream of its
// own, each calling shmr_ec_encode_batch_dev for one block at a time, either
// waiting for every call (hipStreamSynchronize: a per-block flush that must
// know its parity is done) or only at the end (stream-ordered).  Every mode's
// parity is compared byte for byte with the batch call's.
// Build: hipcc --offload-arch=gfx950 -O2 -std=c++17 -Iinclude -o tools/_abx/perblock_dev tools/perblock_dev.cpp \
//          -Lshmr_amd/_lib -lshmr_ec -Wl,-rpath,'$ORIGIN/../../shmr_amd/_lib' -lpthread
// Usage: perblock_dev [blocks=256] [reps=5]
// Linked against libshmr_ec_tools.so instead (perblock_dev_tools), SHMR_PB_SWEEP=1
// repeats the per-block modes for kernel variants (tuning knobs), interleaved,
// so a kernel trace shows each variant's single-block kernel time.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "shmr_ec.h"

namespace {

constexpr uint32_t K = 8, P = 3, T = K + P;
constexpr size_t S = size_t(512) << 10;
constexpr size_t PITCH = S + 4096;   // the slot rule: 512 KiB is a multiple of 64 KiB -> one page more
constexpr size_t BLOCK = T * PITCH;

#define CHECK_HIP(x)                                                                  \
    do {                                                                              \
        if ((x) != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s failed at line %d\n", #x, __LINE__);            \
            std::exit(1);                                                             \
        }                                                                             \
    } while (0)

int encode_one(shmr_ec_t* rs, uint8_t* slab, size_t b, size_t n, hipStream_t s) {
    uint8_t* blk = slab + b * BLOCK;
    return shmr_ec_encode_batch_dev(rs, blk, PITCH, BLOCK, blk + K * PITCH, PITCH, BLOCK, n, S, 0, s);
}

// The crate's call on one block through the submission queue (r06):
// shmr_ec_encode_dev, or the started form (*op set) waited later.
int encode_queued(shmr_ec_t* rs, uint8_t* slab, size_t b, shmr_ec_op_t** op) {
    uint8_t* ptrs[T];
    size_t lens[T];
    for (uint32_t i = 0; i < T; ++i) {
        ptrs[i] = slab + b * BLOCK + i * PITCH;
        lens[i] = S;
    }
    return op ? shmr_ec_encode_dev_start(rs, ptrs, lens, T, 0, op) : shmr_ec_encode_dev(rs, ptrs, lens, T, 0);
}

std::vector<uint8_t> parity_of(const uint8_t* slab, size_t blocks) {
    std::vector<uint8_t> out(blocks * P * S);
    for (size_t b = 0; b < blocks; ++b)
        CHECK_HIP(hipMemcpy2D(out.data() + b * P * S, S, slab + b * BLOCK + K * PITCH, PITCH, S, P,
                              hipMemcpyDeviceToHost));
    return out;
}

__global__ void nop_kernel(uint8_t* p) {
    if (p && threadIdx.x == 1024) p[0] = 0;   // never true: an empty 256-lane workgroup
}

// The same empty kernel with a kernel-argument block the size of the GF
// kernels' ApplyArgs (~1 KiB: the segment table travels in the arguments).
struct BigArgs {
    uint8_t* p;
    uint64_t pad[127];
};
__global__ void nop_big_kernel(const BigArgs a) {
    if (a.p && threadIdx.x == 1024) a.p[a.pad[threadIdx.x & 127] & 7] = 0;   // never true
}

// GPU time of the empty kernels vs a single-block GF launch: kCalls of each,
// back to back on one stream (a kernel trace separates them by name).
void kernel_floor(shmr_ec_t* rs, uint8_t* slab, hipStream_t s) {
    constexpr int kCalls = 256;
    BigArgs big{};
    big.p = slab;
    for (int i = 0; i < kCalls; ++i) hipLaunchKernelGGL(nop_kernel, dim3(128), dim3(256), 0, s, slab);
    for (int i = 0; i < kCalls; ++i) hipLaunchKernelGGL(nop_big_kernel, dim3(128), dim3(256), 0, s, big);
    for (int i = 0; i < kCalls; ++i)
        if (encode_one(rs, slab, 0, 1, s) != 0) std::exit(1);
    CHECK_HIP(hipGetLastError());
    CHECK_HIP(hipStreamSynchronize(s));
    std::printf("{\"mode\": \"kernel_floor\", \"calls\": %d, \"sizeof_BigArgs\": %zu}\n", kCalls, sizeof(BigArgs));
    std::fflush(stdout);
}

// Host time per enqueue, one thread, one stream, nothing waited for: the
// library's per-block call against a bare hipLaunchKernelGGL of an empty
// kernel with the same grid (128 workgroups of 256 lanes).
void enqueue_cost(shmr_ec_t* rs, uint8_t* slab, size_t blocks, hipStream_t s) {
    constexpr int kCalls = 512;
    for (int rep = 0; rep < 3; ++rep) {
        CHECK_HIP(hipStreamSynchronize(s));
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < kCalls; ++i)
            if (encode_one(rs, slab, size_t(i) % blocks, 1, s) != 0) std::exit(1);
        const double lib = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        CHECK_HIP(hipStreamSynchronize(s));
        t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < kCalls; ++i) hipLaunchKernelGGL(nop_kernel, dim3(128), dim3(256), 0, s, slab);
        const double raw = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        CHECK_HIP(hipGetLastError());
        CHECK_HIP(hipStreamSynchronize(s));
        std::printf("{\"mode\": \"enqueue_cost\", \"calls\": %d, \"library_us_per_call\": %.2f, "
                    "\"bare_launch_us\": %.2f}\n", kCalls, lib / kCalls * 1e6, raw / kCalls * 1e6);
        std::fflush(stdout);
    }
}

// CPU time the process's cgroup was throttled for (its CPU quota), in us;
// UINT64_MAX where the file is missing.  (GPU boxes give a job a quota of
// host cores: threads that spin can use it up.)
uint64_t throttled_us() {
    for (const char* path : {"/sys/fs/cgroup/cpu.stat", "/sys/fs/cgroup/cpu/cpu.stat", "/sys/fs/cgroup/cpu,cpuacct/cpu.stat"}) {
        FILE* f = std::fopen(path, "r");
        if (!f) continue;
        char key[64];
        unsigned long long v = 0;
        uint64_t out = UINT64_MAX;
        while (std::fscanf(f, "%63s %llu", key, &v) == 2) {
            if (std::strcmp(key, "throttled_usec") == 0) out = v;
            if (std::strcmp(key, "throttled_time") == 0) out = v / 1000;   // cgroup v1: ns
        }
        std::fclose(f);
        if (out != UINT64_MAX) return out;
    }
    return UINT64_MAX;
}

}  // namespace

int main(int argc, char** argv) {
    const size_t blocks = argc > 1 ? std::strtoul(argv[1], nullptr, 10) : 256;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
    if (shmr_ec_device_init(0) != 0) {
        std::fprintf(stderr, "no device\n");
        return 1;
    }
    if (const char* tune = std::getenv("SHMR_PB_TUNE")) {   // "key=value,key=value": library knobs
        std::string spec(tune);
        size_t pos = 0;
        while (pos < spec.size()) {
            const size_t end = std::min(spec.find(',', pos), spec.size());
            const std::string kv = spec.substr(pos, end - pos);
            const size_t eq = kv.find('=');
            if (eq == std::string::npos || shmr_ec_set_tuning(kv.substr(0, eq).c_str(), std::atoi(kv.c_str() + eq + 1)) != 0) {
                std::fprintf(stderr, "bad knob %s\n", kv.c_str());
                return 1;
            }
            pos = end + 1;
        }
    }
    shmr_ec_t* rs = nullptr;
    if (shmr_ec_new(K, P, &rs) != 0) return 1;
    uint8_t* slab = nullptr;
    CHECK_HIP(hipMalloc(&slab, blocks * BLOCK));
    {   // random data shards, zero parity
        std::vector<uint8_t> host(blocks * BLOCK, 0);
        std::mt19937_64 rng(0x53484D52);
        for (size_t b = 0; b < blocks; ++b)
            for (uint32_t i = 0; i < K; ++i)
                for (size_t c = 0; c < S; c += 8) {
                    const uint64_t v = rng();
                    std::memcpy(&host[b * BLOCK + i * PITCH + c], &v, 8);
                }
        CHECK_HIP(hipMemcpy(slab, host.data(), host.size(), hipMemcpyHostToDevice));
    }
    const double data_gib = double(blocks) * K * S / double(1u << 30);
    hipStream_t s0;
    CHECK_HIP(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CHECK_HIP(hipEventCreate(&e0));
    CHECK_HIP(hipEventCreate(&e1));
    // batch reference (also warms plans and clocks)
    double best_batch = 1e30;
    for (int r = 0; r < reps + 2; ++r) {
        CHECK_HIP(hipEventRecord(e0, s0));
        if (encode_one(rs, slab, 0, blocks, s0) != 0) return 1;
        CHECK_HIP(hipEventRecord(e1, s0));
        CHECK_HIP(hipEventSynchronize(e1));
        float ms = 0;
        CHECK_HIP(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 2) best_batch = std::min(best_batch, double(ms) / 1e3);
    }
    const std::vector<uint8_t> want = parity_of(slab, blocks);
    enqueue_cost(rs, slab, blocks, s0);
    kernel_floor(rs, slab, s0);
    if (std::getenv("SHMR_PB_FLOOR_ONLY")) return 0;
    std::printf("{\"mode\": \"batch\", \"blocks\": %zu, \"GiBps\": %.1f, \"us_per_block\": %.2f}\n", blocks,
                data_gib / best_batch, best_batch / blocks * 1e6);
    std::fflush(stdout);
    struct Mode {
        int wait_each, threads;
        bool queue = false;   // r06: shmr_ec_encode_dev (submission queue) instead of a stream call
    };
    std::vector<Mode> modes;
    const bool queue_only = std::getenv("SHMR_PB_QUEUE_ONLY") != nullptr;
    const int only_threads = std::getenv("SHMR_PB_THREADS") ? std::atoi(std::getenv("SHMR_PB_THREADS")) : 0;
    const bool async_only = std::getenv("SHMR_PB_ASYNC_ONLY") != nullptr;
    for (int q = queue_only ? 1 : 0; q <= 1; ++q)
        for (int wait_each = async_only ? 0 : 1; wait_each >= 0; --wait_each)
            for (int threads : {1, 2, 4, 8, 16, 32})
                if (!only_threads || threads == only_threads) modes.push_back({wait_each, threads, q == 1});
    // variant sweep (tools build): knob sets, each over the latency / throughput modes
    std::vector<std::vector<std::pair<const char*, int>>> variants = {{}};
    if (std::getenv("SHMR_PB_SWEEP")) {
        // (depths 3/5/9 and the LDS-DMA ring are compiled without the early prologue)
        variants = {{{"encode.depth", 2}},
                    {{"encode.depth", 2}, {"encode.early", 0}},
                    {{"encode.depth", 3}, {"encode.early", 0}},
                    {{"encode.depth", 5}, {"encode.early", 0}},
                    {{"encode.depth", 9}, {"encode.early", 0}},
                    {{"encode.depth", 9}, {"encode.early", 0}, {"encode.glds", 1}},
                    {{"encode.threads", 128}, {"encode.depth", 2}, {"encode.early", 0}},
                    {{"encode.depth", 2}}};
        modes = {{1, 1}, {1, 16}, {0, 1}, {0, 16}};
    }
    for (const auto& knobs : variants) {
    for (const char* key : {"encode.depth", "encode.early", "encode.threads", "encode.glds"})
        (void)shmr_ec_set_tuning(key, std::strcmp(key, "encode.threads") == 0 ? 256 : -2);
    std::string label;
    for (const auto& kv : knobs) {
        if (shmr_ec_set_tuning(kv.first, kv.second) != 0) {
            std::fprintf(stderr, "knob %s=%d refused\n", kv.first, kv.second);
            return 1;
        }
        label += std::string(label.empty() ? "" : " ") + kv.first + "=" + std::to_string(kv.second);
    }
    char variant[256] = {0};
    (void)shmr_ec_describe_variant(0, K, P, variant, sizeof variant);
    for (const Mode& md : modes) {
        const int wait_each = md.wait_each, threads = md.threads;
        {
            std::vector<hipStream_t> ss(static_cast<size_t>(threads));
            for (auto& s : ss) CHECK_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            double best = 1e30, best_submit = 0;
            bool ok = true;
            const uint64_t thr0 = throttled_us();
            uint64_t q0[SHMR_EC_Q_COUNTERS] = {}, q1[SHMR_EC_Q_COUNTERS] = {};
            for (int r = 0; r < reps + 1; ++r) {
                CHECK_HIP(hipMemset2D(slab + K * PITCH, BLOCK, 0, P * PITCH, blocks));   // parity cleared
                CHECK_HIP(hipDeviceSynchronize());
                std::vector<int> rc(size_t(threads), 0);
                std::vector<std::chrono::steady_clock::time_point> sub_end{size_t(threads)};
                // r06: the workers are started before the clock and released
                // together (a rayon pool exists before the flush it serves);
                // r05's figures included the thread creation
                std::atomic<int> go{0};
                std::vector<std::thread> ts;
                for (int t = 0; t < threads; ++t)
                    ts.emplace_back([&, t] {
                        while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
                        if (md.queue) {
                            std::vector<shmr_ec_op_t*> ops;
                            for (size_t b = size_t(t); b < blocks; b += size_t(threads)) {
                                shmr_ec_op_t* op = nullptr;
                                if (encode_queued(rs, slab, b, wait_each ? nullptr : &op) != 0) rc[size_t(t)] = 1;
                                if (op) ops.push_back(op);
                            }
                            sub_end[size_t(t)] = std::chrono::steady_clock::now();
                            for (shmr_ec_op_t* op : ops)
                                if (shmr_ec_op_wait(op) != 0) rc[size_t(t)] = 1;
                            return;
                        }
                        hipStream_t s = ss[size_t(t)];
                        for (size_t b = size_t(t); b < blocks; b += size_t(threads)) {
                            if (encode_one(rs, slab, b, 1, s) != 0) rc[size_t(t)] = 1;
                            if (wait_each && hipStreamSynchronize(s) != hipSuccess) rc[size_t(t)] = 1;
                        }
                        if (hipStreamSynchronize(s) != hipSuccess) rc[size_t(t)] = 1;
                    });
                (void)shmr_ec_queue_stats(0, q0, SHMR_EC_Q_COUNTERS);
                const auto t0 = std::chrono::steady_clock::now();
                if (std::getenv("SHMR_PB_GO"))   // (steady-clock ns: lines up with SHMR_QUEUE_TRACE's base_ns)
                    std::fprintf(stderr, "PBGO threads=%d rep=%d ns=%lld\n", threads, r,
                                 (long long)std::chrono::duration_cast<std::chrono::nanoseconds>(t0.time_since_epoch()).count());
                go.store(1, std::memory_order_release);
                for (auto& th : ts) th.join();
                const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                (void)shmr_ec_queue_stats(0, q1, SHMR_EC_Q_COUNTERS);
                for (int x : rc) ok = ok && x == 0;
                double submit_s = 0;   // the last thread's submissions done (queue modes)
                for (const auto& e : sub_end)
                    if (md.queue) submit_s = std::max(submit_s, std::chrono::duration<double>(e - t0).count());
                if (r >= 1 && sec < best) {   // rep 0 warms the streams' state
                    best = sec;
                    best_submit = submit_s;
                }
            }
            const uint64_t thr1 = throttled_us();
            const bool same = parity_of(slab, blocks) == want;
            const uint64_t nb = q1[SHMR_EC_Q_BATCHES] - q0[SHMR_EC_Q_BATCHES];
            std::printf("{\"mode\": \"per_block\", \"api\": \"%s\", \"knobs\": \"%s\", \"variant\": \"%s\", "
                        "\"wait_each_call\": %s, \"threads\": %d, \"blocks\": %zu, "
                        "\"GiBps\": %.1f, \"us_per_block\": %.2f, \"of_batch\": %.3f, \"ok\": %s, "
                        "\"parity_equals_batch\": %s, \"tune\": \"%s\", \"queue_batches_last_rep\": %llu, "
                        "\"blocks_per_launch_last_rep\": %.2f, \"early_launches_last_rep\": %llu, "
                        "\"submitted_by_us\": %.1f, \"cgroup_throttled_us\": %lld}\n",
                        md.queue ? "encode_dev (queue)" : "encode_batch_dev (stream)", label.c_str(), variant,
                        wait_each ? "true" : "false", threads, blocks, data_gib / best,
                        best / blocks * 1e6, best_batch / best, ok ? "true" : "false", same ? "true" : "false",
                        std::getenv("SHMR_PB_TUNE") ? std::getenv("SHMR_PB_TUNE") : "", (unsigned long long)nb, nb ? double(blocks) / double(nb) : 0.0,
                        (unsigned long long)(q1[SHMR_EC_Q_EARLY] - q0[SHMR_EC_Q_EARLY]), best_submit * 1e6,
                        (thr0 == UINT64_MAX || thr1 == UINT64_MAX) ? -1LL : (long long)(thr1 - thr0));
            std::fflush(stdout);
            for (auto& s : ss) CHECK_HIP(hipStreamDestroy(s));
            if (!ok || !same) return 1;
        }
    }
    }
    CHECK_HIP(hipFree(slab));
    shmr_ec_free(rs);
    return 0;
}
