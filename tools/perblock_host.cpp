// The literal drop-in on host memory: one shmr_ec_encode (ReedSolomon::encode,
// reference src/vfs/block.rs:427) or shmr_ec_reconstruct (:560) per 4 MiB
// RS(8,3) block from T threads, as rayon calls them (src/vfs/mod.rs:93-96), on
// mapped Block-Cache buffers (shmr_ec_host_alloc: zero-copy), with knob
// "coalesce" off (one zero-copy launch per call) and on (the submission queue
// merges concurrent calls), interleaved rounds in one process; and the host
// batch (shmr_ec_encode_blocks_host / reconstruct) over the same blocks.
// Every mode's parity / rebuilt bytes are compared with the first encode's.
// Build: hipcc --offload-arch=gfx950 -O2 -std=c++17 -Iinclude -o tools/_abx/perblock_host tools/perblock_host.cpp
//          -Lshmr_amd/_lib -lshmr_ec -Wl,-rpath,'$ORIGIN/../../shmr_amd/_lib' -lpthread   (one line)
// Usage: perblock_host [blocks=128] [rounds=5]
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "shmr_ec.h"

namespace {
constexpr uint32_t K = 8, P = 3, T = K + P;
constexpr size_t S = size_t(512) << 10;
using Clock = std::chrono::steady_clock;

double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

// T worker threads started before the clock and released together
template <class F>
double run_threads(int threads, size_t n, F f) {
    std::atomic<int> go{0}, bad{0};
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t)
        ts.emplace_back([&, t] {
            while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
            for (size_t b = size_t(t); b < n; b += size_t(threads))
                if (f(b) != 0) bad = 1;
        });
    const auto t0 = Clock::now();
    go.store(1, std::memory_order_release);
    for (auto& x : ts) x.join();
    const double s = secs(t0, Clock::now());
    if (bad) {
        std::fprintf(stderr, "a call failed\n");
        std::exit(1);
    }
    return s;
}
}  // namespace

int main(int argc, char** argv) {
    const size_t B = argc > 1 ? std::strtoul(argv[1], nullptr, 10) : 128;
    const int rounds = argc > 2 ? std::atoi(argv[2]) : 5;
    if (shmr_ec_device_init(0) != 0) return 1;
    std::string tune_spec;
    if (const char* tune = std::getenv("SHMR_PB_TUNE")) {   // "key=value,...": knobs for the coalesce=1 legs
        tune_spec = tune;
        size_t pos = 0;
        while (pos < tune_spec.size()) {
            const size_t end = std::min(tune_spec.find(',', pos), tune_spec.size());
            const std::string kv = tune_spec.substr(pos, end - pos);
            const size_t eq = kv.find('=');
            if (eq == std::string::npos ||
                shmr_ec_set_tuning(kv.substr(0, eq).c_str(), std::atoi(kv.c_str() + eq + 1)) != 0) {
                std::fprintf(stderr, "bad knob %s\n", kv.c_str());
                return 1;
            }
            pos = end + 1;
        }
    }
    shmr_ec_t* rs = nullptr;
    if (shmr_ec_new(K, P, &rs) != 0) return 1;
    void* mem = nullptr;
    if (shmr_ec_host_alloc(B * T * S, &mem) != 0) return 1;
    uint8_t* cache = static_cast<uint8_t*>(mem);   // block b: T shards of S bytes
    std::mt19937_64 rng(7);
    for (size_t i = 0; i < B * T * S; i += 8) {
        const uint64_t v = rng();
        std::memcpy(cache + i, &v, 8);
    }
    std::vector<uint8_t*> ptrs(B * T);
    for (size_t j = 0; j < B * T; ++j) ptrs[j] = cache + j * S;
    std::vector<size_t> lens(T, S);
    auto enc = [&](size_t b) { return shmr_ec_encode(rs, ptrs.data() + b * T, lens.data(), T); };
    std::vector<uint8_t> present(B * T, 1), scratch(B * S);
    for (size_t b = 0; b < B; ++b) present[b * T + b % K] = 0;
    auto rec = [&](size_t b) {
        std::vector<size_t> l(T, S);
        l[b % K] = 0;
        return shmr_ec_reconstruct(rs, ptrs.data() + b * T, l.data(), present.data() + b * T, T, 0);
    };
    // reference bytes
    run_threads(8, B, enc);
    std::vector<uint8_t> want(cache, cache + B * T * S);
    const double gib = double(B) * K * S / double(1u << 30);
    auto check = [&](const char* what) {
        if (std::memcmp(cache, want.data(), want.size()) != 0) {
            std::fprintf(stderr, "%s: bytes differ\n", what);
            std::exit(1);
        }
    };
    struct Leg {
        std::string name;
        int coalesce, threads;
        bool decode, batch;
        double best = 1e30;
    };
    std::vector<Leg> legs;
    for (bool decode : {false, true}) {
        legs.push_back({"batch", 1, 1, decode, true});
        for (int threads : {1, 8, 16})
            for (int c : {0, 1}) legs.push_back({"per_block", c, threads, decode, false});
    }
    int dev0 = 0;
    for (int r = 0; r < rounds + 1; ++r)
        for (Leg& L : legs) {
            if (shmr_ec_set_tuning("coalesce", L.coalesce) != 0) return 1;
            if (L.decode)   // lose data shard b mod 8 of every block
                for (size_t b = 0; b < B; ++b) std::memset(ptrs[b * T + b % K], 0xEE, S);
            double s;
            if (L.batch) {
                const auto t0 = Clock::now();
                const int rc = L.decode ? shmr_ec_reconstruct_blocks_host(rs, ptrs.data(), present.data(), B, S, 0, &dev0, 1)
                                        : shmr_ec_encode_blocks_host(rs, ptrs.data(), B, S, &dev0, 1);
                s = secs(t0, Clock::now());
                if (rc) return 1;
            } else {
                s = run_threads(L.threads, B, L.decode ? std::function<int(size_t)>(rec) : std::function<int(size_t)>(enc));
            }
            check(L.name.c_str());
            if (r > 0 && s < L.best) L.best = s;
        }
    (void)shmr_ec_set_tuning("coalesce", -2);
    uint64_t q[SHMR_EC_Q_COUNTERS] = {};
    (void)shmr_ec_queue_stats(0, q, SHMR_EC_Q_COUNTERS);
    for (const Leg& L : legs)
        std::printf("{\"op\": \"%s\", \"leg\": \"%s\", \"coalesce\": %d, \"threads\": %d, \"blocks\": %zu, "
                    "\"GiBps\": %.2f, \"ms_per_block_per_thread\": %.3f, \"buffers\": \"mapped Block Cache\", "
                    "\"tune\": \"%s\"}\n",
                    L.decode ? "reconstruct" : "encode", L.name.c_str(), L.batch ? -1 : L.coalesce, L.threads, B,
                    gib / L.best, L.best / double(B) * L.threads * 1e3, tune_spec.c_str());
    std::printf("{\"queue_requests\": %llu, \"queue_batches\": %llu, \"max_batch\": %llu}\n",
                (unsigned long long)q[SHMR_EC_Q_REQUESTS], (unsigned long long)q[SHMR_EC_Q_BATCHES],
                (unsigned long long)q[SHMR_EC_Q_MAX_BATCH]);
    shmr_ec_host_free(mem);
    shmr_ec_free(rs);
    return 0;
}
