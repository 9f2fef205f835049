// Probe: does separating HBM reads and writes in time beat the mixed-traffic
// ceiling of the erasure access pattern?
//
// The RS(8,3) encode reads 8 shards and writes 3 per tile; every channel sees
// reads and writes interleaved (measured ceilings, profiles/r01/membench_ceilings.jsonl:
// read-only 8->0 89.5 % of 8 TB/s, write-only 0->3 82.7 %, mixed 8->3 77.8 %).
// If the memory system lost that difference to read/write turnarounds, a
// kernel whose waves all read in one time slot and all write in the next
// would approach R/0.895 + W/0.827 ~ 87 %.  Here every wave of a persistent
// grid gates itself on the SoC-wide real-time counter (100 MHz): it loads and
// XOR-reduces Q wave-tiles (8 x 1 KiB each) during the read part of each
// period, keeps the 3 outputs per tile in registers, and stores them in the
// write part.  XOR instead of GF math: this measures the memory system, not
// a result.  Baseline in the same process: the one-workgroup-per-tile kernel
// of tools/membench.hip (8 in, 3 out, nt).
//
//   hipcc -O3 --offload-arch=gfx950 tools/phasebench.hip -o tools/_bin/phasebench
//   phasebench [blocks=512] [iters=20]
//
// One JSON line per configuration: TB/s of algorithmic bytes 11 * S * B and
// the fraction of the 8 TB/s peak.
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

constexpr int K = 8, R = 3;
constexpr uint64_t S = 524288;   // RS(8,3) 4 MiB blocks

__device__ __forceinline__ u32x4 ldnt(const uint8_t* p) {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}
__device__ __forceinline__ void stnt(uint8_t* p, u32x4 v) {
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
}

// Baseline: one workgroup per 4 KiB tile (membench kin_rout<8,3,1,nt>).
__global__ __launch_bounds__(256) void mixed(const uint8_t* __restrict__ in, uint8_t* __restrict__ out) {
    const uint64_t tpb = S / 4096;
    const uint64_t j = blockIdx.x / tpb;
    const uint64_t col = (blockIdx.x - j * tpb) * 4096 + threadIdx.x * 16;
    const uint8_t* ib = in + j * K * S + col;
    u32x4 acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = u32x4{blockIdx.x, uint32_t(r), 0, 0};
#pragma unroll
    for (int t = 0; t < K; ++t) {
        const u32x4 v = ldnt(ib + t * S);
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] ^= v + u32x4{uint32_t(r), 0, 0, 0};
    }
    uint8_t* ob = out + j * R * S + col;
#pragma unroll
    for (int r = 0; r < R; ++r) stnt(ob + r * S, acc[r]);
}

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }

// Persistent, time-phased.  Work unit = one wave-tile: 64 lanes x 16 B of one
// block's columns, all 8 inputs and 3 outputs.  Wave w takes units
// w*Q .. w*Q+Q-1, then w*Q + nwaves*Q, ...  Per period of P ticks the first
// Tr ticks are the read slot.  gate = 0 disables the gating (same schedule,
// no waiting) to separate the effect of gating from the persistent shape.
template <int Q>
__global__ __launch_bounds__(256) void phased(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                              uint64_t nunits, uint64_t P, uint64_t Tr, int gate) {
    const uint64_t upb = S / 1024;   // units per block
    const uint64_t wave = (uint64_t(blockIdx.x) * 256 + threadIdx.x) / 64;
    const uint64_t nwaves = uint64_t(gridDim.x) * 4;
    const uint32_t lane = threadIdx.x & 63;
    for (uint64_t base = wave * Q; base < nunits; base += nwaves * Q) {
        if (gate) {
            while (now() % P >= Tr) __builtin_amdgcn_s_sleep(2);
        }
        u32x4 acc[Q][R];
        u32x4 v[Q][K];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const uint64_t u = base + q < nunits ? base + q : nunits - 1;
            const uint64_t j = u / upb;
            const uint8_t* ib = in + j * K * S + (u - j * upb) * 1024 + lane * 16;
#pragma unroll
            for (int t = 0; t < K; ++t) v[q][t] = ldnt(ib + t * S);
        }
#pragma unroll
        for (int q = 0; q < Q; ++q)
#pragma unroll
            for (int r = 0; r < R; ++r) {
                acc[q][r] = u32x4{uint32_t(base + q), uint32_t(r), 0, 0};
#pragma unroll
                for (int t = 0; t < K; ++t) acc[q][r] ^= v[q][t] + u32x4{uint32_t(r), 0, 0, 0};
            }
        if (gate) {
            while (now() % P < Tr) __builtin_amdgcn_s_sleep(2);
        }
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const uint64_t u = base + q;
            if (u >= nunits) break;
            const uint64_t j = u / upb;
            uint8_t* ob = out + j * R * S + (u - j * upb) * 1024 + lane * 16;
#pragma unroll
            for (int r = 0; r < R; ++r) stnt(ob + r * S, acc[q][r]);
        }
    }
}

template <class F>
double time_ms(F launch, int iters) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int w = 0; w < 5; ++w) launch();
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return ms / iters;
}

void report(const char* name, int Q, int wgs, uint64_t P, uint64_t Tr, int gate, double ms, uint64_t B) {
    const double tbps = double(B) * (K + R) * S / (ms * 1e-3) / 1e12;
    std::printf("{\"kernel\": \"%s\", \"Q\": %d, \"workgroups\": %d, \"period_ticks\": %llu, \"read_ticks\": %llu, "
                "\"gate\": %d, \"ms\": %.4f, \"TBps\": %.3f, \"frac\": %.4f}\n",
                name, Q, wgs, (unsigned long long)P, (unsigned long long)Tr, gate, ms, tbps, tbps / 8.0);
    std::fflush(stdout);
}

template <int Q>
void sweep(const uint8_t* in, uint8_t* out, uint64_t B, int iters, int cus) {
    const uint64_t nunits = B * (S / 1024);
    for (int per_cu : {1, 2}) {
        const int wgs = cus * per_cu;
        // period sized so one round of every wave's Q units fits: reads at ~7 TB/s, writes at ~6.5
        const double rbytes = double(wgs) * 4 * Q * K * 1024, wbytes = double(wgs) * 4 * Q * R * 1024;
        const double tr_us = rbytes / 7.0e6, tw_us = wbytes / 6.5e6;   // bytes / (B/us)
        for (double scale : {1.0, 1.3}) {
            const uint64_t Tr = uint64_t(tr_us * scale * 100.0) + 1;   // 100 ticks per us
            const uint64_t P = Tr + uint64_t(tw_us * scale * 100.0) + 1;
            for (int gate : {0, 1}) {
                if (!gate && scale != 1.0) continue;
                const double ms = time_ms([&] { phased<Q><<<wgs, 256>>>(in, out, nunits, P, Tr, gate); }, iters);
                report("phased", Q, wgs, P, Tr, gate, ms, B);
            }
        }
    }
}

int main(int argc, char** argv) {
    const uint64_t B = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 512;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 20;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    int wall_khz = 0;
    CK(hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, 0));
    std::printf("{\"cus\": %d, \"realtime_khz\": %d}\n", cus, wall_khz);
    uint8_t *in, *out;
    CK(hipMalloc(&in, B * K * S));
    CK(hipMalloc(&out, B * R * S));
    CK(hipMemset(in, 0x5a, B * K * S));
    CK(hipMemset(out, 0, B * R * S));
    const uint32_t tiles = uint32_t(B * (S / 4096));
    for (int i = 0; i < 300; ++i) mixed<<<tiles, 256>>>(in, out);   // clock ramp
    CK(hipDeviceSynchronize());
    for (int rep = 0; rep < 2; ++rep) {
        report("mixed", 1, int(tiles), 0, 0, 0, time_ms([&] { mixed<<<tiles, 256>>>(in, out); }, iters), B);
        sweep<2>(in, out, B, iters, cus);
        sweep<4>(in, out, B, iters, cus);
    }
    CK(hipFree(in));
    CK(hipFree(out));
    return 0;
}
