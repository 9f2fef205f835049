// Host-memory copy probe for the config-5 copy-out (VirtualFile::read copies
// each rebuilt 4 MiB block from its mapped Block-Cache slot into the caller's
// buffer while other tasks read shard files and the GPU reads slots across
// PCIe).  Times T threads copying 4 MiB blocks from a mapped pinned slab into
// a pageable buffer, with glibc memcpy and with AVX2 streaming stores (no
// read-for-ownership of the destination lines), interleaved A/B/A/B.
// Build: hipcc -O2 -std=c++17 -mavx2 -o tools/_abx/copy_probe tools/copy_probe.cpp -lpthread
// Usage: copy_probe [blocks=64] [reps=5]
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

namespace {

constexpr size_t kBlock = size_t(4) << 20;

void copy_stream(uint8_t* dst, const uint8_t* src, size_t n) {
    size_t i = 0;
    // dst and src are page-aligned in this probe; 32-byte streaming stores
    for (; i + 128 <= n; i += 128) {
        const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i));
        const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 32));
        const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 64));
        const __m256i d = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 96));
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i), a);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 32), b);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 64), c);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 96), d);
    }
    if (i < n) std::memcpy(dst + i, src + i, n - i);
    _mm_sfence();
}

double run(int mode, int threads, uint8_t* dst, const uint8_t* src, size_t blocks) {
    std::atomic<size_t> next{0};
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t)
        ts.emplace_back([&] {
            for (size_t b; (b = next.fetch_add(1)) < blocks;) {
                if (mode == 0)
                    std::memcpy(dst + b * kBlock, src + b * kBlock, kBlock);
                else
                    copy_stream(dst + b * kBlock, src + b * kBlock, kBlock);
            }
        });
    for (auto& th : ts) th.join();
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return double(blocks * kBlock) / s / double(1u << 30);
}

}  // namespace

int main(int argc, char** argv) {
    const size_t blocks = argc > 1 ? std::strtoul(argv[1], nullptr, 10) : 64;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
    void* src = nullptr;
    if (hipHostMalloc(&src, blocks * kBlock, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess) {
        std::fprintf(stderr, "hipHostMalloc failed\n");
        return 1;
    }
    std::vector<uint8_t> pageable_src(blocks * kBlock);
    uint8_t* dst = static_cast<uint8_t*>(std::aligned_alloc(4096, blocks * kBlock));
    std::memset(src, 0x5a, blocks * kBlock);
    std::memset(pageable_src.data(), 0x33, blocks * kBlock);
    std::memset(dst, 0, blocks * kBlock);
    for (int srcmode = 0; srcmode < 2; ++srcmode) {
        const uint8_t* s = srcmode == 0 ? static_cast<uint8_t*>(src) : pageable_src.data();
        for (int threads : {1, 8, 16, 24}) {
            double best[2] = {0, 0}, sum[2] = {0, 0};
            for (int r = 0; r < reps; ++r)
                for (int mode = 0; mode < 2; ++mode) {
                    const double g = run(mode, threads, dst, s, blocks);
                    best[mode] = g > best[mode] ? g : best[mode];
                    sum[mode] += g;
                }
            std::printf("{\"src\": \"%s\", \"threads\": %d, \"memcpy_best\": %.1f, \"stream_best\": %.1f, "
                        "\"memcpy_mean\": %.1f, \"stream_mean\": %.1f}\n",
                        srcmode == 0 ? "mapped" : "pageable", threads, best[0], best[1], sum[0] / reps, sum[1] / reps);
            std::fflush(stdout);
        }
    }
    if (std::memcmp(dst, pageable_src.data(), blocks * kBlock) != 0) {
        std::fprintf(stderr, "copy mismatch\n");
        return 1;
    }
    std::free(dst);
    (void)hipHostFree(src);
    return 0;
}
