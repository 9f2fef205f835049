// Cost of misaligned 16-byte vector accesses on the device, isolated from the
// erasure math: a streaming copy of N bytes from src + mi to dst + mo, one
// 16-byte chunk per lane (wave-contiguous), three load forms:
//   vec : one under-aligned dwordx4 load at src + mi (the product's path for
//         the reference's packed block buffer, shard i at i * S)
//   dw  : a dwordx4 load at the dword-aligned address below, the next lane's
//         first dword by a DPP wavefront shift (lane 63: one wave-uniform
//         dword load) and v_alignbyte per dword
//   x16 : a dwordx4 load at the 16-byte aligned address below, all four of the
//         next lane's dwords by DPP (the tools realign tile's form)
// and an under-aligned dwordx4 store at dst + mo (nontemporal); form
//   sts : an aligned load, then ALIGNED stores: lane L stores the 16-byte
//         output chunk made of lane L-1's last mo bytes and its own first
//         16-mo (previous lane by a DPP wavefront shift); lanes 0 and 63 store
//         the wave's two partial chunks with masked dword / short / byte stores.
//
//   hipcc -O3 --offload-arch=gfx950 tools/misalign_bench.hip -o tools/_bin/misalign_bench
//   misalign_bench [MiB=2048] [iters=20]
//
// Prints one JSON line per (form, mi, mo): GB/s of read + write bytes.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_u __attribute__((aligned(1)));

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            std::fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
            std::exit(1);                                                                    \
        }                                                                                    \
    } while (0)

constexpr int kVec = 0, kDw = 1, kX16 = 2, kSts = 3;

__device__ __forceinline__ u32x4 funnel16(const u32x4& lo, const u32x4& hi, uint32_t s) {
    const uint32_t r = s & 3u;
    auto ab = [r](uint32_t h, uint32_t l) { return __builtin_amdgcn_alignbyte(h, l, r); };
    switch (s >> 2) {
        case 0: return u32x4{ab(lo.y, lo.x), ab(lo.z, lo.y), ab(lo.w, lo.z), ab(hi.x, lo.w)};
        case 1: return u32x4{ab(lo.z, lo.y), ab(lo.w, lo.z), ab(hi.x, lo.w), ab(hi.y, hi.x)};
        case 2: return u32x4{ab(lo.w, lo.z), ab(hi.x, lo.w), ab(hi.y, hi.x), ab(hi.z, hi.y)};
        default: return u32x4{ab(hi.x, lo.w), ab(hi.y, hi.x), ab(hi.z, hi.y), ab(hi.w, hi.z)};
    }
}

__device__ __forceinline__ uint32_t shr1(uint32_t v) {
    return uint32_t(__builtin_amdgcn_update_dpp(int(v), int(v), 0x138, 0xf, 0xf, false));
}

// 64 consecutive 16-byte chunks of a wave at p (lane L at p + 16 L), p off
// 16-byte alignment by mo (wave-uniform): aligned full stores plus the two
// partial chunks at the wave's ends.
__device__ __forceinline__ void store_aligned_run(uint8_t* p, u32x4 v) {
    const uint32_t mo = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(uintptr_t(p)) & 15u)));
    if (mo == 0) {
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
        return;
    }
    const uint32_t lane = threadIdx.x & 63u;
    const u32x4 prev{shr1(v.x), shr1(v.y), shr1(v.z), shr1(v.w)};
    uint8_t* a = p - mo;   // the aligned chunk holding the lane's first byte
    if (lane != 0) __builtin_nontemporal_store(funnel16(prev, v, 16u - mo), reinterpret_cast<u32x4*>(a));
    // partial chunks: lane 0 the bytes [mo, 16) of chunk a, lane 63 the bytes
    // [0, mo) of chunk a + 16; both from the lane's value rotated into the
    // output chunk's frame
    const u32x4 rot = funnel16(v, v, 16u - mo);
    const bool head = lane == 0, tail = lane == 63;
    uint8_t* q = tail ? a + 16 : a;
    const uint32_t w[4] = {rot.x, rot.y, rot.z, rot.w};
#pragma unroll
    for (uint32_t d = 0; d < 4; ++d) {
        if ((head && 4 * d >= mo) || (tail && 4 * d + 4 <= mo))
            *reinterpret_cast<uint32_t*>(q + 4 * d) = w[d];
    }
    if (mo & 3u) {
        const uint32_t d = mo >> 2, x = w[d];
        if ((mo & 3u) == 2u) {   // the split dword's two halves
            if (head) *reinterpret_cast<uint16_t*>(q + 4 * d + 2) = uint16_t(x >> 16);
            if (tail) *reinterpret_cast<uint16_t*>(q + 4 * d) = uint16_t(x);
        } else {
#pragma unroll
            for (uint32_t b = 0; b < 4; ++b) {
                const uint32_t pos = 4 * d + b;
                if ((head && pos >= mo) || (tail && pos < mo)) q[pos] = uint8_t(x >> (8 * b));
            }
        }
    }
}

__device__ __forceinline__ uint32_t shl1(uint32_t edge, uint32_t v) {
    return uint32_t(__builtin_amdgcn_update_dpp(int(edge), int(v), 0x130, 0xf, 0xf, false));
}

template <int FORM>
__global__ __launch_bounds__(256) void copy_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                   uint64_t nchunks, uint32_t mi, uint32_t mo, uint32_t* sink) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t c0 = uint64_t(blockIdx.x) * blockDim.x; c0 < nchunks; c0 += stride) {
        const uint64_t c = c0 + threadIdx.x;   // nchunks is a multiple of the grid: no bounds check
        u32x4 v;
        if constexpr (FORM == kVec || FORM == kSts) {
            v = *reinterpret_cast<const u32x4_u*>(src + mi + c * 16);
        } else if constexpr (FORM == kDw) {
            const uint32_t r = mi & 3u;
            const uint8_t* p = src + (mi & ~3u) + c * 16;
            const u32x4 lo = *reinterpret_cast<const u32x4*>(__builtin_assume_aligned(p, 4));
            // the dword after this wave's run (one request: a wave-uniform address)
            const uint64_t wend = (c0 + (threadIdx.x & ~63u) + 64) * 16;
            const uint32_t e = *reinterpret_cast<const uint32_t*>(src + (mi & ~3u) + wend);
            const uint32_t nx = shl1(e, lo.x);
            v = u32x4{__builtin_amdgcn_alignbyte(lo.y, lo.x, r), __builtin_amdgcn_alignbyte(lo.z, lo.y, r),
                      __builtin_amdgcn_alignbyte(lo.w, lo.z, r), __builtin_amdgcn_alignbyte(nx, lo.w, r)};
        } else {
            const uint32_t m = mi & 15u;
            const uint8_t* p = src + (mi & ~15u) + c * 16;
            const u32x4 lo = *reinterpret_cast<const u32x4*>(p);
            const uint64_t wend = (c0 + (threadIdx.x & ~63u) + 64) * 16;
            const u32x4 e = *reinterpret_cast<const u32x4*>(src + (mi & ~15u) + wend);
            const u32x4 nx{shl1(e.x, lo.x), shl1(e.y, lo.y), shl1(e.z, lo.z), shl1(e.w, lo.w)};
            const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, nx.x, nx.y, nx.z, nx.w};
            const uint32_t q = m >> 2, r = m & 3u;
            uint32_t o[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                uint32_t a = w[0], b = w[1];
#pragma unroll
                for (int s = 1; s < 4; ++s)
                    if (q == uint32_t(s)) a = w[j + s], b = w[j + s + 1];
                if (q == 0) a = w[j], b = w[j + 1];
                o[j] = __builtin_amdgcn_alignbyte(b, a, r);
            }
            v = u32x4{o[0], o[1], o[2], o[3]};
        }
        if constexpr (FORM == kSts)
            store_aligned_run(dst + mo + c * 16, v);
        else
            __builtin_nontemporal_store(v, reinterpret_cast<u32x4_u*>(dst + mo + c * 16));
    }
    if (threadIdx.x == 0 && blockIdx.x == 0 && sink) sink[0] = 0u;
}

template <int FORM>
static float run(const uint8_t* src, uint8_t* dst, uint64_t nchunks, uint32_t mi, uint32_t mo, int iters, int grid) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) copy_kernel<FORM><<<grid, 256>>>(src, dst, nchunks, mi, mo, nullptr);
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) copy_kernel<FORM><<<grid, 256>>>(src, dst, nchunks, mi, mo, nullptr);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return ms / iters;
}

static bool check(const uint8_t* dsrc, uint8_t* ddst, uint64_t n, uint32_t mi, uint32_t mo) {
    const uint64_t probe = 1 << 20;
    uint8_t* a = static_cast<uint8_t*>(std::malloc(probe));
    uint8_t* b = static_cast<uint8_t*>(std::malloc(probe));
    bool ok = true;
    for (uint64_t off : {uint64_t(0), n / 2, n - probe}) {
        CK(hipMemcpy(a, dsrc + mi + off, probe, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b, ddst + mo + off, probe, hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < probe && ok; ++i) ok = a[i] == b[i];
    }
    std::free(a);
    std::free(b);
    return ok;
}

int main(int argc, char** argv) {
    const uint64_t mib = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 2048;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 20;
    const int grid = 256 * 8;
    const uint64_t n = (mib << 20) / (uint64_t(grid) * 256 * 16) * (uint64_t(grid) * 256 * 16);
    const uint64_t nchunks = n / 16;
    uint8_t *src, *dst;
    CK(hipMalloc(&src, n + 4096));   // slack: misaligned bases and the last wave's edge load
    CK(hipMalloc(&dst, n + 4096));
    {
        uint32_t* h = static_cast<uint32_t*>(std::malloc(n + 4096));
        uint32_t x = 2463534242u;
        for (uint64_t i = 0; i < (n + 4096) / 4; ++i) {
            x ^= x << 13;
            x ^= x >> 17;
            x ^= x << 5;
            h[i] = x;
        }
        CK(hipMemcpy(src, h, n + 4096, hipMemcpyHostToDevice));
        std::free(h);
    }
    const uint32_t offs[][2] = {{0, 0}, {10, 0}, {4, 0}, {2, 0}, {1, 0}, {0, 10}, {0, 4}, {0, 2}, {0, 1}, {0, 7}, {10, 4}, {4, 8}};
    const char* names[] = {"vec", "dw", "x16", "sts"};
    for (auto& o : offs) {
        for (int form = 0; form < 4; ++form) {
            float ms = 0.f;
            if (form == kVec) ms = run<kVec>(src, dst, nchunks, o[0], o[1], iters, grid);
            if (form == kDw) ms = run<kDw>(src, dst, nchunks, o[0], o[1], iters, grid);
            if (form == kX16) ms = run<kX16>(src, dst, nchunks, o[0], o[1], iters, grid);
            if (form == kSts) ms = run<kSts>(src, dst, nchunks, o[0], o[1], iters, grid);
            CK(hipDeviceSynchronize());
            const bool ok = check(src, dst, n, o[0], o[1]);
            std::printf("{\"form\": \"%s\", \"mi\": %u, \"mo\": %u, \"ms\": %.4f, \"GBps\": %.1f, \"ok\": %s}\n",
                        names[form], o[0], o[1], ms, 2.0 * double(n) / (ms * 1e6), ok ? "true" : "false");
            std::fflush(stdout);
        }
    }
    CK(hipFree(src));
    CK(hipFree(dst));
    return 0;
}
