// Lean GF(2^8) encode probe: is the product kernel's distance to the K -> R
// copy replica (tools/membench.hip) a property of the kernel framework (plan
// image, LDS staging, register ring, runtime k) or of the access pattern?
//
// Same dispatch and layout as membench (one workgroup per U x 4 KiB tile of a
// block, in [B][K][P], out [B][R][P], nontemporal loads and stores), but with
// the real GF math of gf_apply.hip (three v_perm_b32 lookups + v_bitop3 per
// row and dword) at compile-time K and R, the coefficient tables passed as a
// kernel argument (scalar loads, no LDS, no plan image) and the shard loop
// fully unrolled so the compiler schedules every load.  The XOR replica of the
// identical tiling runs in the same process.  Parity of block 0 / block B-1 is
// checked against a host GF multiply (RS(K, R) Vandermonde parity rows).
//
//   hipcc -O3 --offload-arch=gfx950 tools/gflean.hip -o tools/_probe/gflean
//   gflean [shard_bytes=1671168] [blocks=64] [iters=20] [pitch=shard_bytes]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            std::fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
            std::exit(1);                                                                    \
        }                                                                                    \
    } while (0)

// ---- host GF(2^8), polynomial 0x11D, generator 2 ---------------------------
static uint8_t g_exp[512], g_log[256];
static void gf_init() {
    int x = 1;
    for (int i = 0; i < 255; ++i) {
        g_exp[i] = uint8_t(x);
        g_log[x] = uint8_t(i);
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
    for (int i = 255; i < 512; ++i) g_exp[i] = g_exp[i - 255];
}
static uint8_t gmul(uint8_t a, uint8_t b) { return (a && b) ? g_exp[g_log[a] + g_log[b]] : 0; }
static uint8_t ginv(uint8_t a) { return g_exp[255 - g_log[a]]; }
static uint8_t gpow(uint8_t a, int n) {
    if (n == 0) return 1;
    if (a == 0) return 0;
    return g_exp[(g_log[a] * n) % 255];
}

// parity rows of the systematic code M = V * inv(V[0..k]), V[r][c] = r^c
static std::vector<uint8_t> parity_rows(int k, int p) {
    const int n = k + p;
    std::vector<uint8_t> V(n * k), top(k * k), inv(k * k, 0);
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < k; ++c) V[r * k + c] = gpow(uint8_t(r), c);
    top.assign(V.begin(), V.begin() + k * k);
    for (int i = 0; i < k; ++i) inv[i * k + i] = 1;
    for (int c = 0; c < k; ++c) {   // Gauss-Jordan
        int piv = c;
        while (top[piv * k + c] == 0) ++piv;
        for (int j = 0; j < k; ++j) {
            std::swap(top[c * k + j], top[piv * k + j]);
            std::swap(inv[c * k + j], inv[piv * k + j]);
        }
        const uint8_t s = ginv(top[c * k + c]);
        for (int j = 0; j < k; ++j) {
            top[c * k + j] = gmul(top[c * k + j], s);
            inv[c * k + j] = gmul(inv[c * k + j], s);
        }
        for (int r = 0; r < k; ++r)
            if (r != c && top[r * k + c]) {
                const uint8_t f = top[r * k + c];
                for (int j = 0; j < k; ++j) {
                    top[r * k + j] ^= gmul(f, top[c * k + j]);
                    inv[r * k + j] ^= gmul(f, inv[c * k + j]);
                }
            }
    }
    std::vector<uint8_t> P(p * k, 0);
    for (int r = 0; r < p; ++r)
        for (int c = 0; c < k; ++c) {
            uint8_t s = 0;
            for (int j = 0; j < k; ++j) s ^= gmul(V[(k + r) * k + j], inv[j * k + c]);
            P[r * k + c] = s;
        }
    return P;
}

// ---- device ----------------------------------------------------------------
constexpr int kMaxK = 16, kMaxR = 4;
struct Tabs {
    uint32_t w[kMaxK][kMaxR][5];   // t0lo t0hi t1lo t1hi t2 per (input, row)
};

__device__ __forceinline__ uint32_t gf_mac4(uint32_t acc, const uint32_t* t, uint32_t s0, uint32_t s1, uint32_t s2) {
    const uint32_t a = __builtin_amdgcn_perm(t[1], t[0], s0);
    const uint32_t b = __builtin_amdgcn_perm(t[3], t[2], s1);
    const uint32_t c = __builtin_amdgcn_perm(t[4], t[4], s2);
    return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(acc, a, b, 0x96), c, 0u, 0x96);
}

__device__ __forceinline__ u32x4 ldnt(const uint8_t* p) {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}
__device__ __forceinline__ void stnt(uint8_t* p, u32x4 v) {
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
}

// GF = false: the XOR replica (membench's kin_rout) of the same tiling.
template <int K, int R, int U, bool GF>
__global__ __launch_bounds__(256) void lean(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, uint64_t P,
                                            uint64_t tpb, const Tabs tabs) {
    const uint64_t tile = blockIdx.x;
    const uint64_t j = tile / tpb;
    const uint64_t col = (tile - j * tpb) * (4096ull * U) + threadIdx.x * 16;
    const uint8_t* ib = in + j * K * P + col;
    uint32_t acc[U][R][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int d = 0; d < 4; ++d) acc[u][r][d] = 0;
#pragma unroll
    for (int t = 0; t < K; ++t) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ldnt(ib + t * P + u * 4096);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                if constexpr (GF) {
                    const uint32_t s0 = w[d] & 0x07070707u, s1 = (w[d] >> 3) & 0x07070707u, s2 = (w[d] >> 6) & 0x03030303u;
#pragma unroll
                    for (int r = 0; r < R; ++r) acc[u][r][d] = gf_mac4(acc[u][r][d], tabs.w[t][r], s0, s1, s2);
                } else {
#pragma unroll
                    for (int r = 0; r < R; ++r) acc[u][r][d] ^= w[d] + uint32_t(r);
                }
            }
        }
    }
    uint8_t* ob = out + j * R * P + col;
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u)
            stnt(ob + r * P + u * 4096, u32x4{acc[u][r][0], acc[u][r][1], acc[u][r][2], acc[u][r][3]});
}

template <int K, int R, int U, bool GF>
double time_it(const uint8_t* in, uint8_t* out, uint64_t S, uint64_t P, uint64_t B, const Tabs& tb, int iters) {
    const uint64_t tpb = S / (4096ull * U);
    const uint32_t grid = uint32_t(tpb * B);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int w = 0; w < 5; ++w) lean<K, R, U, GF><<<grid, 256>>>(in, out, P, tpb, tb);
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) lean<K, R, U, GF><<<grid, 256>>>(in, out, P, tpb, tb);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return ms / iters;
}

template <int K, int R>
void pattern(uint8_t* in, uint8_t* out, uint64_t S, uint64_t P, uint64_t B, int iters, int rounds) {
    // tables of the RS(K, R) parity rows
    const std::vector<uint8_t> M = parity_rows(K, R);
    Tabs tb{};
    for (int t = 0; t < K; ++t)
        for (int r = 0; r < R; ++r) {
            const uint8_t c = M[r * K + t];
            uint8_t T0[8], T1[8], T2[4];
            for (int i = 0; i < 8; ++i) T0[i] = gmul(c, uint8_t(i)), T1[i] = gmul(c, uint8_t(i << 3));
            for (int i = 0; i < 4; ++i) T2[i] = gmul(c, uint8_t(i << 6));
            uint32_t* w = tb.w[t][r];
            std::memcpy(&w[0], T0, 4);
            std::memcpy(&w[1], T0 + 4, 4);
            std::memcpy(&w[2], T1, 4);
            std::memcpy(&w[3], T1 + 4, 4);
            std::memcpy(&w[4], T2, 4);
        }
    // correctness of the GF variant on the first and last block
    lean<K, R, 1, true><<<uint32_t(S / 4096 * B), 256>>>(in, out, P, S / 4096, tb);
    CK(hipDeviceSynchronize());
    bool ok = true;
    for (uint64_t b : {uint64_t(0), B - 1}) {
        std::vector<uint8_t> hin(K * P), hout(R * P);
        CK(hipMemcpy(hin.data(), in + b * K * P, K * P, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hout.data(), out + b * R * P, R * P, hipMemcpyDeviceToHost));
        for (uint64_t x = 0; x < S && ok; x += 4099)
            for (int r = 0; r < R; ++r) {
                uint8_t s = 0;
                for (int t = 0; t < K; ++t) s ^= gmul(M[r * K + t], hin[t * P + x]);
                if (s != hout[r * P + x]) ok = false;
            }
    }
    // interleaved rounds: XOR U=1, GF U=1, XOR U=2, GF U=2
    double best[4] = {1e9, 1e9, 1e9, 1e9};
    std::vector<double> med[4];
    for (int rnd = 0; rnd < rounds; ++rnd) {
        med[0].push_back(time_it<K, R, 1, false>(in, out, S, P, B, tb, iters));
        med[1].push_back(time_it<K, R, 1, true>(in, out, S, P, B, tb, iters));
        med[2].push_back(time_it<K, R, 2, false>(in, out, S, P, B, tb, iters));
        med[3].push_back(time_it<K, R, 2, true>(in, out, S, P, B, tb, iters));
    }
    const char* names[4] = {"xor_u1", "gf_u1", "xor_u2", "gf_u2"};
    for (int v = 0; v < 4; ++v) {
        std::vector<double> m = med[v];
        std::sort(m.begin(), m.end());
        const double ms = m[m.size() / 2];
        best[v] = m[0];
        const double tbps = double(B) * (K + R) * S / (ms * 1e-3) / 1e12;
        std::printf("{\"pattern\": \"%din%dout\", \"variant\": \"%s\", \"S\": %llu, \"pitch\": %llu, \"blocks\": %llu, "
                    "\"median_ms\": %.4f, \"min_ms\": %.4f, \"TBps\": %.3f, \"frac\": %.4f, \"gf_parity_ok\": %s}\n",
                    K, R, names[v], (unsigned long long)S, (unsigned long long)P, (unsigned long long)B, ms, best[v],
                    tbps, tbps / 8.0, ok ? "true" : "false");
    }
    std::fflush(stdout);
}

int main(int argc, char** argv) {
    gf_init();
    const uint64_t S = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1671168;
    const uint64_t B = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 64;
    const int iters = argc > 3 ? std::atoi(argv[3]) : 20;
    const uint64_t P = argc > 4 ? std::strtoull(argv[4], nullptr, 10) : S;
    const int rounds = argc > 5 ? std::atoi(argv[5]) : 7;
    const char* only = std::getenv("GFLEAN_ONLY");   // "83" / "104"
    if (S % 8192 != 0 || P < S || P % 16 != 0) {
        std::fprintf(stderr, "S must be a multiple of 8 KiB, pitch >= S and 16-byte aligned\n");
        return 2;
    }
    uint8_t *in, *out;
    CK(hipMalloc(&in, B * 10 * P));
    CK(hipMalloc(&out, B * 4 * P));
    {   // deterministic pseudo-random input
        std::vector<uint8_t> h(B * 10 * P);
        uint64_t x = 0x53484D52u;
        for (auto& c : h) {
            x ^= x << 13, x ^= x >> 7, x ^= x << 17;
            c = uint8_t(x >> 24);
        }
        CK(hipMemcpy(in, h.data(), h.size(), hipMemcpyHostToDevice));
    }
    Tabs z{};
    for (int i = 0; i < 300; ++i)   // clock ramp
        lean<10, 4, 1, false><<<uint32_t(S / 4096 * B), 256>>>(in, out, P, S / 4096, z);
    CK(hipDeviceSynchronize());
    if (!only || std::strcmp(only, "104") == 0) pattern<10, 4>(in, out, S, P, B, iters, rounds);
    if (!only || std::strcmp(only, "83") == 0) pattern<8, 3>(in, out, S, P, B, iters, rounds);
    CK(hipFree(in));
    CK(hipFree(out));
    return 0;
}
