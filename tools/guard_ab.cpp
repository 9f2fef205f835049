// Cost of the relaxed-capture guard (core::RelaxedCapture: two
// hipThreadExchangeStreamCaptureMode calls around every C-ABI entry point) on
// the drop-in per-block call, in ONE process: the in-tree product library
// against a build with the guard compiled out (-DSHMR_EC_NO_RELAXED_CAPTURE),
// both dlopen'ed RTLD_LOCAL, interleaved rounds.
//   * guard alone: ns per shmr_ec_get_tuning call (a guarded call that does
//     nothing else), 1 thread
//   * shmr_ec_encode per 4 MiB RS(8,3) block from T threads (rayon's shape,
//     reference src/vfs/mod.rs:93-96), mapped (zero-copy) and pageable blocks:
//     GiB/s of data and mean per-call latency
// Usage: guard_ab <libA.so> <libB.so> [rounds] [threads]
#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

namespace {
struct Lib {
    std::string name;
    void* h = nullptr;
    int (*new_)(uint32_t, uint32_t, void**);
    int (*encode)(void*, uint8_t* const*, const size_t*, size_t);
    int (*get_tuning)(const char*);
    int (*host_alloc)(size_t, void**);
    size_t (*shard_size)(uint64_t, uint32_t);
    void* rs = nullptr;
};

template <class F>
void sym(Lib& L, F& f, const char* n) {
    f = reinterpret_cast<F>(dlsym(L.h, n));
    if (!f) {
        std::fprintf(stderr, "%s: no %s\n", L.name.c_str(), n);
        std::exit(2);
    }
}

double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

constexpr unsigned K = 8, P = 3;
constexpr size_t NB = 64;   // blocks per round

struct Blocks {
    std::vector<std::vector<uint8_t*>> ptrs;   // [NB][K+P]
    std::vector<std::vector<uint8_t>> pageable;
};

Blocks make(Lib& L, size_t S, bool mapped, std::mt19937& rng) {
    Blocks b;
    for (size_t i = 0; i < NB; ++i) {
        uint8_t* base = nullptr;
        if (mapped) {
            void* p = nullptr;
            if (L.host_alloc((K + P) * S, &p) != 0) {
                std::fprintf(stderr, "host_alloc failed\n");
                std::exit(2);
            }
            base = static_cast<uint8_t*>(p);
        } else {
            b.pageable.emplace_back((K + P) * S);
            base = b.pageable.back().data();
        }
        for (size_t j = 0; j < K * S; ++j) base[j] = uint8_t(rng());
        std::vector<uint8_t*> row;
        for (unsigned s = 0; s < K + P; ++s) row.push_back(base + s * S);
        b.ptrs.push_back(row);
    }
    return b;
}

// T threads over NB blocks, one shmr_ec_encode each; returns (seconds, mean call seconds)
std::pair<double, double> run(Lib& L, Blocks& b, size_t S, int T) {
    std::atomic<size_t> next{0};
    std::atomic<uint64_t> call_ns{0};
    std::vector<size_t> lens(K + P, S);
    const double t0 = now();
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&] {
            for (size_t i; (i = next++) < NB;) {
                const auto c0 = std::chrono::steady_clock::now();
                if (L.encode(L.rs, b.ptrs[i].data(), lens.data(), K + P) != 0) std::abort();
                call_ns += uint64_t(std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - c0).count());
            }
        });
    for (auto& x : th) x.join();
    return {now() - t0, call_ns.load() * 1e-9 / NB};
}
}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: guard_ab <libA.so> <libB.so> [rounds] [threads]\n");
        return 2;
    }
    const int rounds = argc > 3 ? std::atoi(argv[3]) : 9;
    const int T = argc > 4 ? std::atoi(argv[4]) : 8;
    std::vector<Lib> libs(2);
    for (int i = 0; i < 2; ++i) {
        Lib& L = libs[i];
        L.name = argv[1 + i];
        L.h = dlopen(argv[1 + i], RTLD_NOW | RTLD_LOCAL);
        if (!L.h) {
            std::fprintf(stderr, "dlopen %s: %s\n", argv[1 + i], dlerror());
            return 2;
        }
        sym(L, L.new_, "shmr_ec_new");
        sym(L, L.encode, "shmr_ec_encode");
        sym(L, L.get_tuning, "shmr_ec_get_tuning");
        sym(L, L.host_alloc, "shmr_ec_host_alloc");
        sym(L, L.shard_size, "shmr_ec_shard_size");
        if (L.new_(K, P, &L.rs) != 0) return 2;
    }
    const size_t S = libs[0].shard_size(4u << 20, K);
    std::mt19937 rng(7);
    std::vector<Blocks> mapped, pageable;
    for (auto& L : libs) {
        mapped.push_back(make(L, S, true, rng));
        pageable.push_back(make(L, S, false, rng));
        run(L, mapped.back(), S, T);   // warm: device state, plans, bounce buffers
        run(L, pageable.back(), S, T);
    }
    std::vector<std::vector<double>> guard_ns(2), mg(2), ml(2), pg(2), pl(2);
    for (int r = 0; r < rounds; ++r)
        for (int i = 0; i < 2; ++i) {
            Lib& L = libs[i];
            const int n = 200000;
            const double t0 = now();
            for (int j = 0; j < n; ++j) (void)L.get_tuning("bounce_kib");
            guard_ns[i].push_back((now() - t0) / n * 1e9);
            auto a = run(L, mapped[i], S, T);
            mg[i].push_back(NB * K * S / a.first / double(1 << 30));
            ml[i].push_back(a.second * 1e3);
            auto b = run(L, pageable[i], S, T);
            pg[i].push_back(NB * K * S / b.first / double(1 << 30));
            pl[i].push_back(b.second * 1e3);
        }
    auto med = [](std::vector<double> v) {
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
    };
    for (int i = 0; i < 2; ++i)
        std::printf("{\"lib\": \"%s\", \"rounds\": %d, \"threads\": %d, \"guarded_call_ns\": %.1f, "
                    "\"per_block_encode_mapped_GiBps\": %.2f, \"mapped_call_ms\": %.4f, "
                    "\"per_block_encode_pageable_GiBps\": %.2f, \"pageable_call_ms\": %.4f}\n",
                    libs[i].name.c_str(), rounds, T, med(guard_ns[i]), med(mg[i]), med(ml[i]), med(pg[i]), med(pl[i]));
    return 0;
}
