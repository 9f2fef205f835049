// HBM ceiling microbenchmark for the erasure kernel's access pattern:
// K input streams -> R output streams, one workgroup per tile of U x 4 KiB
// columns of a block, XOR instead of GF math (so the numbers are the memory
// system's ceiling for that read/write mix, not a result).  Layout as
// bench.py: in [B][K][S], out [B][R][S].
//
//   hipcc -O3 --offload-arch=gfx950 tools/membench.hip -o tools/_bin/membench
//   membench [shard_bytes=524288] [blocks=512] [iters=20]
//   env: MEMBENCH_ALLOC=contig (physically contiguous VRAM), MEMBENCH_ONLY=83 | 104,
//        MEMBENCH_PITCH=<bytes> (shard slot > S: padded layout, bench.py --pitch-pad; a slot
//        off 16-byte alignment, e.g. 1677722 with S = 1671168, puts shards where the
//        reference's packed RS(10,4) block buffer has them), MEMBENCH_ONLY=102 (10 -> 2)
//
// Prints one JSON line per (pattern, variant): TB/s of algorithmic bytes
// (K + R) * S * B and the fraction of the 8 TB/s HBM peak.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_u __attribute__((aligned(1)));   // MEMBENCH_PITCH may put shards off 16-byte alignment

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            std::fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
            std::exit(1);                                                                    \
        }                                                                                    \
    } while (0)

constexpr int kNtL = 1, kNtS = 2, kRemap = 4;

template <int F>
__device__ __forceinline__ u32x4 ld(const uint8_t* p) {
    if constexpr (F & kNtL) return __builtin_nontemporal_load(reinterpret_cast<const u32x4_u*>(p));
    else return *reinterpret_cast<const u32x4_u*>(p);
}
template <int F>
__device__ __forceinline__ void st(uint8_t* p, u32x4 v) {
    if constexpr (F & kNtS) __builtin_nontemporal_store(v, reinterpret_cast<u32x4_u*>(p));
    else *reinterpret_cast<u32x4_u*>(p) = v;
}

// K == 0: write-only.  R == 0: read-only (one conditional atomic per lane).
template <int K, int R, int U, int F>
__global__ __launch_bounds__(256) void kin_rout(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                uint64_t S, uint64_t tiles_per_block, uint32_t ntiles,
                                                uint32_t* sink) {
    // S here is the shard slot (pitch); tiles_per_block covers the shard length
    uint32_t tile = blockIdx.x;
    if constexpr (F & kRemap) {
        // XCD-contiguous: dispatch puts blockIdx i on XCD i % 8; give XCD x the
        // x-th eighth of the tile range.
        const uint32_t per = ntiles / 8;
        tile = (blockIdx.x % 8) * per + blockIdx.x / 8;
    }
    const uint64_t j = tile / tiles_per_block;
    const uint64_t col = (tile - j * tiles_per_block) * (4096ull * U) + threadIdx.x * 16;
    const uint8_t* ib = in + j * K * S + col;
    constexpr int RR = R > 0 ? R : 1;
    u32x4 acc[U][RR];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < RR; ++r) acc[u][r] = u32x4{uint32_t(tile), uint32_t(r), 0, 0};
#pragma unroll
    for (int t = 0; t < K; ++t) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ld<F>(ib + t * S + u * 4096);
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int r = 0; r < RR; ++r) acc[u][r] ^= v[u] + u32x4{uint32_t(r), 0, 0, 0};
    }
    if constexpr (R == 0) {
#pragma unroll
        for (int u = 0; u < U; ++u)
            if ((acc[u][0].x ^ acc[u][0].y ^ acc[u][0].z ^ acc[u][0].w) == 0x9e3779b9u) atomicAdd(sink, 1u);
    } else {
        uint8_t* ob = out + j * R * S + col;
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u) st<F>(ob + r * S + u * 4096, acc[u][r]);
    }
}

template <int K, int R, int U, int F>
void run(const char* name, const uint8_t* in, uint8_t* out, uint64_t S, uint64_t B, uint32_t* sink, int iters) {
    const uint64_t tpb = S / (4096ull * U);
    const char* pe = std::getenv("MEMBENCH_PITCH");
    const uint64_t P = pe ? std::strtoull(pe, nullptr, 10) : S;   // shard slot
    const uint32_t grid = uint32_t(tpb * B);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int w = 0; w < 10; ++w) kin_rout<K, R, U, F><<<grid, 256>>>(in, out, P, tpb, grid, sink);
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) kin_rout<K, R, U, F><<<grid, 256>>>(in, out, P, tpb, grid, sink);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= iters;
    const double tbps = double(B) * (K + R) * S / (ms * 1e-3) / 1e12;
    std::printf("{\"pattern\": \"%din%dout\", \"variant\": \"%s\", \"U\": %d, \"ntl\": %d, \"nts\": %d, \"remap\": %d, "
                "\"pitch\": %llu, \"ms\": %.4f, \"TBps\": %.3f, \"frac\": %.4f}\n",
                K, R, name, U, (F & kNtL) ? 1 : 0, (F & kNtS) ? 1 : 0, (F & kRemap) ? 1 : 0, (unsigned long long)P, ms,
                tbps, tbps / 8.0);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

template <int K, int R>
void pattern(const uint8_t* in, uint8_t* out, uint64_t S, uint64_t B, uint32_t* sink, int iters) {
    run<K, R, 1, kNtL | kNtS>("nt", in, out, S, B, sink, iters);
    run<K, R, 1, 0>("plain", in, out, S, B, sink, iters);
    run<K, R, 1, kNtL>("ntload", in, out, S, B, sink, iters);
    run<K, R, 1, kNtS>("ntstore", in, out, S, B, sink, iters);
    run<K, R, 1, kNtL | kNtS | kRemap>("nt+remap", in, out, S, B, sink, iters);
    run<K, R, 2, kNtL | kNtS>("nt", in, out, S, B, sink, iters);
    run<K, R, 4, kNtL | kNtS>("nt", in, out, S, B, sink, iters);
}

int main(int argc, char** argv) {
    const uint64_t S = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 524288;
    const uint64_t B = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 512;
    const int iters = argc > 3 ? std::atoi(argv[3]) : 20;
    if (S % 16384 != 0 || (S / 4096 * B) % 8 != 0) {
        std::fprintf(stderr, "S must be a multiple of 16 KiB\n");
        return 2;
    }
    uint8_t *in, *out;
    uint32_t* sink;
    const char* pe = std::getenv("MEMBENCH_PITCH");
    const uint64_t P = pe ? std::strtoull(pe, nullptr, 10) : S;
    if (P < S) {
        std::fprintf(stderr, "MEMBENCH_PITCH must be >= S\n");
        return 2;
    }
    // MEMBENCH_ALLOC=contig: physically contiguous VRAM (hipDeviceMallocContiguous),
    // to separate page-translation effects from the access pattern's own ceiling.
    const char* alloc = std::getenv("MEMBENCH_ALLOC");
    const bool contig = alloc && std::strcmp(alloc, "contig") == 0;
    if (contig) {
        CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&in), B * 10 * P, hipDeviceMallocContiguous));
        CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&out), B * 4 * P, hipDeviceMallocContiguous));
    } else {
        CK(hipMalloc(&in, B * 10 * P));
        CK(hipMalloc(&out, B * 4 * P));
    }
    const char* only = std::getenv("MEMBENCH_ONLY");   // "83": the RS(8,3) encode pattern only
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(in, 0x5a, B * 10 * P));
    CK(hipMemset(out, 0, B * 4 * P));
    for (int i = 0; i < 300; ++i)   // clock ramp
        kin_rout<8, 3, 1, 3><<<uint32_t(S / 4096 * B), 256>>>(in, out, P, S / 4096, uint32_t(S / 4096 * B), sink);
    CK(hipDeviceSynchronize());
    for (int rep = 0; rep < 2; ++rep) {
        if (only && std::strcmp(only, "104") == 0) {   // the RS(10,4) encode pattern only
            run<10, 4, 1, kNtL | kNtS>("nt", in, out, S, B, sink, iters);
            run<10, 4, 2, kNtL | kNtS>("nt", in, out, S, B, sink, iters);
            continue;
        }
        if (only && std::strcmp(only, "102") == 0) {   // the RS(10,4) 2-erasure rebuild's streams
            run<10, 2, 1, kNtL | kNtS>("nt", in, out, S, B, sink, iters);
            continue;
        }
        pattern<8, 3>(in, out, S, B, sink, iters);
        if (only && std::strcmp(only, "83") == 0) continue;
        pattern<8, 1>(in, out, S, B, sink, iters);
        pattern<8, 0>(in, out, S, B, sink, iters);
        pattern<0, 3>(in, out, S, B, sink, iters);
        pattern<1, 1>(in, out, S, B, sink, iters);
        pattern<10, 4>(in, out, S, B, sink, iters);
    }
    CK(hipFree(in));
    CK(hipFree(out));
    CK(hipFree(sink));
    return 0;
}
