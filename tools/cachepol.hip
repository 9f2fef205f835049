// Cache-policy probe for the erasure kernel's access pattern (K input streams
// -> R output streams, one workgroup per 4 KiB tile, XOR instead of GF math):
// buffer loads/stores with every combination of the gfx950 CPol bits the
// builtins accept (aux: 1 = sc0, 2 = nt, 16 = sc1) against plain global
// nontemporal loads/stores (the production kernel's choice).
//
//   hipcc -O3 --offload-arch=gfx950 tools/cachepol.hip -o tools/_bin/cachepol
//   cachepol [shard_bytes=524288] [blocks=512] [iters=20]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            std::fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
            std::exit(1);                                                                    \
        }                                                                                    \
    } while (0)

// LA / SA: load / store aux bits for buffer ops; -1 = global nontemporal builtin.
// T > 0: the reconstruct layout -- one [B][T][S] shard array, block j reads
// shards 0..K of it except e = j % K and writes shard e (R = 1).  T < 0: the
// same reads, shard e written to the same place of a second [B][-T][S] array.
// T <= -100: the same reads from a [B][-T-100][S] array, shard e written to a
// compact [B][1][S] output.
template <int K, int R, int LA, int SA, int T = 0>
__global__ __launch_bounds__(256) void probe(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint64_t S,
                                             uint64_t tiles_per_block) {
    const uint32_t tile = blockIdx.x;
    const uint64_t j = tile / tiles_per_block;
    const uint32_t col = uint32_t((tile - j * tiles_per_block) * 4096ull + threadIdx.x * 16);
    const uint32_t e = uint32_t(j % K);
    constexpr int AT = T <= -100 ? -T - 100 : T < 0 ? -T : T;
    const uint8_t* ib = T ? out + j * AT * S : in + j * K * S;
    uint8_t* ob = T > 0      ? out + j * T * S + e * S
                  : T <= -100 ? const_cast<uint8_t*>(in) + j * S
                  : T < 0     ? const_cast<uint8_t*>(in) + j * AT * S + e * S
                              : out + j * R * S;
    __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void*)ib, 0, 0x7fffffff, 0x00020000);
    __amdgpu_buffer_rsrc_t rout = __builtin_amdgcn_make_buffer_rsrc((void*)ob, 0, 0x7fffffff, 0x00020000);
    u32x4 acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = u32x4{tile, uint32_t(r), 0, 0};
#pragma unroll
    for (int t0 = 0; t0 < K; ++t0) {
        const uint32_t t = T && uint32_t(t0) >= e ? t0 + 1 : t0;
        u32x4 v;
        if constexpr (LA < 0) {
            v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(ib + t * S + col));
        } else {
            v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rin, uint32_t(t * S + col), 0, LA));
        }
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] ^= v + u32x4{uint32_t(r), 0, 0, 0};
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if constexpr (SA < 0) {
            __builtin_nontemporal_store(acc[r], reinterpret_cast<u32x4*>(ob + r * S + col));
        } else {
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, acc[r]),
                                                   rout, uint32_t(r * S + col), 0, SA);
        }
    }
}

template <int K, int R, int LA, int SA, int T = 0>
void run(const uint8_t* in, uint8_t* out, uint64_t S, uint64_t B, int iters) {
    const uint64_t tpb = S / 4096;
    const uint32_t grid = uint32_t(tpb * B);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int w = 0; w < 10; ++w) probe<K, R, LA, SA, T><<<grid, 256>>>(in, out, S, tpb);
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) probe<K, R, LA, SA, T><<<grid, 256>>>(in, out, S, tpb);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= iters;
    const double tbps = double(B) * (K + R) * S / (ms * 1e-3) / 1e12;
    std::printf("{\"pattern\": \"%din%dout%s\", \"load_aux\": %d, \"store_aux\": %d, \"ms\": %.4f, \"TBps\": %.3f, "
                "\"frac\": %.4f}\n",
                K, R, T > 0 ? "_in_place" : T <= -100 ? "_compact_out" : T < 0 ? "_sparse_out" : "", LA, SA, ms, tbps,
                tbps / 8.0);
    std::fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

template <int K, int R, int LA, int T = 0>
void stores(const uint8_t* in, uint8_t* out, uint64_t S, uint64_t B, int iters) {
    run<K, R, LA, -1, T>(in, out, S, B, iters);
    run<K, R, LA, 0, T>(in, out, S, B, iters);
    run<K, R, LA, 2, T>(in, out, S, B, iters);
    run<K, R, LA, 1, T>(in, out, S, B, iters);
    run<K, R, LA, 3, T>(in, out, S, B, iters);
    run<K, R, LA, 16, T>(in, out, S, B, iters);
    run<K, R, LA, 18, T>(in, out, S, B, iters);
    run<K, R, LA, 17, T>(in, out, S, B, iters);
    run<K, R, LA, 19, T>(in, out, S, B, iters);
}

template <int K, int R, int T = 0>
void pattern(const uint8_t* in, uint8_t* out, uint64_t S, uint64_t B, int iters) {
    stores<K, R, -1, T>(in, out, S, B, iters);
    stores<K, R, 2, T>(in, out, S, B, iters);
}

int main(int argc, char** argv) {
    const uint64_t S = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 524288;
    const uint64_t B = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 512;
    const int iters = argc > 3 ? std::atoi(argv[3]) : 20;
    if (S % 4096 != 0 || 11 * S >= 0x7fffffffull) {
        std::fprintf(stderr, "S must be a multiple of 4 KiB and 11 * S < 2 GiB\n");
        return 2;
    }
    uint8_t *in, *out;
    CK(hipMalloc(&in, B * 11 * S));
    CK(hipMalloc(&out, B * 11 * S));
    CK(hipMemset(in, 0x5a, B * 11 * S));
    CK(hipMemset(out, 0x33, B * 11 * S));
    for (int i = 0; i < 300; ++i) probe<8, 3, -1, -1><<<uint32_t(S / 4096 * B), 256>>>(in, out, S, S / 4096);   // clock ramp
    CK(hipDeviceSynchronize());
    for (int rep = 0; rep < 2; ++rep) {
        pattern<8, 3>(in, out, S, B, iters);
        pattern<8, 1>(in, out, S, B, iters);
        pattern<8, 1, 11>(in, out, S, B, iters);
        pattern<8, 1, -11>(in, out, S, B, iters);
        pattern<8, 1, -111>(in, out, S, B, iters);
    }
    CK(hipFree(in));
    CK(hipFree(out));
    return 0;
}
