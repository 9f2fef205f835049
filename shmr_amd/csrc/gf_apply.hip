// GF(2^8) matrix-apply kernel for gfx950 (MI355X / CDNA4).
//
//   out[r][col] = XOR_t  C[r][t] (x) in[t][col]        for every block of a batch
//
// Encode (reference: reed_solomon_erasure ReedSolomon::encode at
// src/vfs/block.rs:427) uses C = parity rows of the coding matrix; reconstruct
// (block.rs:560) uses the rows of the plan built in gf256.cpp.
//
// Design (see DESIGN.md "Kernel"):
//  * HBM-bound byte-field arithmetic, no MFMA.  Every input byte is read once,
//    every output byte written once: algorithmic traffic (k + R) * len per block.
//  * One workgroup = 256 lanes; a tile = 4 KiB * U of columns of one block;
//    each lane owns U 16-byte chunks per shard (global_load_dwordx4, 1 KiB per
//    wave instruction, fully coalesced).  Grid-strided over tiles so a launch
//    is a few thousand long-lived workgroups.
//  * Multiply by constant c via three 8-byte tables T0/T1/T2 (bits 0-2, 3-5,
//    6-7) held in LDS; v_perm_b32 looks up four byte lanes of a dword at once:
//    per input dword 5 VALU ops of nibble extraction shared by all rows, then
//    3 v_perm + ~2 xor per row.
//  * Tables are staged once per workgroup into LDS and read back with
//    wave-uniform (broadcast) ds_read_b128 per shard.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gf_apply.hpp"

namespace shmr {
namespace kern {

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct Tab {
    uint32_t t0lo, t0hi, t1lo, t1hi, t2;
};

__device__ __forceinline__ uint32_t gf_mul4(const Tab& t, uint32_t s0, uint32_t s1, uint32_t s2) {
    // v_perm_b32(src0=hi, src1=lo, sel): selector byte n picks byte n of {hi:lo}
    const uint32_t a = __builtin_amdgcn_perm(t.t0hi, t.t0lo, s0);
    const uint32_t b = __builtin_amdgcn_perm(t.t1hi, t.t1lo, s1);
    const uint32_t c = __builtin_amdgcn_perm(t.t2, t.t2, s2);
    return a ^ b ^ c;
}

template <bool NT>
__device__ __forceinline__ u32x4 load16(const uint8_t* p) {
    if constexpr (NT) {
        return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    } else {
        return *reinterpret_cast<const u32x4*>(p);
    }
}

template <bool NT>
__device__ __forceinline__ void store16(uint8_t* p, u32x4 v) {
    if constexpr (NT) {
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
    } else {
        *reinterpret_cast<u32x4*>(p) = v;
    }
}

// Byte-granular load of up to 16 bytes [p, p + n) (n may be <= 0).
__device__ __forceinline__ u32x4 load_bytes(const uint8_t* p, int64_t n) {
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int b = 0; b < 16; ++b)
        if (b < n) w[b >> 2] |= uint32_t(p[b]) << (8 * (b & 3));
    return u32x4{w[0], w[1], w[2], w[3]};
}

__device__ __forceinline__ void store_bytes(uint8_t* p, u32x4 v, int64_t n) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int b = 0; b < 16; ++b)
        if (b < n) p[b] = uint8_t(w[b >> 2] >> (8 * (b & 3)));
}

// MODE 0: full tile, aligned vector path.  MODE 1: partial tile (bounds per
// lane), aligned.  MODE 2: unaligned layout, byte-granular everything.
template <int MODE, bool NT>
__device__ __forceinline__ u32x4 ld(const uint8_t* base, uint64_t col, uint64_t len) {
    if constexpr (MODE == 0) {
        return load16<NT>(base + col);
    } else if constexpr (MODE == 1) {
        if (col + 16 <= len) return load16<NT>(base + col);
        return load_bytes(base + col, int64_t(len) - int64_t(col));
    } else {
        return load_bytes(base + col, int64_t(len) - int64_t(col));
    }
}

template <int MODE, bool NT>
__device__ __forceinline__ void st(uint8_t* base, uint64_t col, uint64_t len, u32x4 v) {
    if constexpr (MODE == 0) {
        store16<NT>(base + col, v);
    } else if constexpr (MODE == 1) {
        if (col + 16 <= len) store16<NT>(base + col, v);
        else store_bytes(base + col, v, int64_t(len) - int64_t(col));
    } else {
        store_bytes(base + col, v, int64_t(len) - int64_t(col));
    }
}

template <int R>
__device__ __forceinline__ void read_tabs(const u32x4* s_tab, uint32_t t, Tab (&tb)[R]) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const u32x4 a = s_tab[(size_t(t) * R + r) * 2];
        const uint32_t b = reinterpret_cast<const uint32_t*>(s_tab)[(size_t(t) * R + r) * 8 + 4];
        tb[r] = Tab{a.x, a.y, a.z, a.w, b};
    }
}

template <int R>
__device__ __forceinline__ void mac(uint32_t (&acc)[R][4], const u32x4& d, const Tab (&tb)[R]) {
    const uint32_t w[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t s0 = w[j] & 0x07070707u;
        const uint32_t s1 = (w[j] >> 3) & 0x07070707u;
        const uint32_t s2 = (w[j] >> 6) & 0x03030303u;
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r][j] ^= gf_mul4(tb[r], s0, s1, s2);
    }
}

// One tile: lanes own columns col0 + (u * 256 + tid) * 16, u < U.
//
// Shards rotate through three register buffers A/B/C (unrolled by 3 so the
// rotation is a renaming, never a register move that would force a vmcnt(0)):
// while shard t is multiplied, the loads of shards t+1 and t+2 are in flight
// (2 * U * 16 B per lane).  Loads past the last shard are clamped to shard
// k-1 (an L1/L2 hit of bytes just read) so every load is unconditional and the
// compiler's vmcnt bookkeeping stays exact.  KC > 0 fixes k at compile time.
template <int R, int U, int MODE, bool NT, int KC>
__device__ __forceinline__ void do_tile(const uint32_t k_rt, const uint64_t len, const uint8_t* ib,
                                        uint8_t* ob, uint64_t col0, const uint64_t* s_in_off,
                                        const uint64_t* s_out_off, const u32x4* s_tab) {
    const uint32_t k = KC > 0 ? uint32_t(KC) : k_rt;
    const uint32_t tid = threadIdx.x;
    uint32_t acc[U][R][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[u][r][j] = 0u;

    auto load = [&](u32x4 (&buf)[U], uint32_t t) {
        const uint32_t tt = t < k ? t : k - 1;
        const uint8_t* base = ib + s_in_off[tt];
#pragma unroll
        for (int u = 0; u < U; ++u) buf[u] = ld<MODE, NT>(base, col0 + (uint64_t(u) * kThreads + tid) * 16, len);
    };
    auto consume = [&](const u32x4 (&buf)[U], uint32_t t) {
        Tab tb[R];
        read_tabs<R>(s_tab, t, tb);
#pragma unroll
        for (int u = 0; u < U; ++u) mac<R>(acc[u], buf[u], tb);
    };

    u32x4 A[U], B[U], C[U];
    load(A, 0);
    load(B, 1);
    if constexpr (KC > 0) {
#pragma unroll
        for (uint32_t t = 0; t < uint32_t(KC); t += 3) {
            if (t + 2 < k) load(C, t + 2);
            consume(A, t);
            if (t + 3 < k) load(A, t + 3);
            if (t + 1 < k) consume(B, t + 1);
            if (t + 4 < k) load(B, t + 4);
            if (t + 2 < k) consume(C, t + 2);
        }
    } else {
        for (uint32_t t = 0; t < k; t += 3) {
            load(C, t + 2);
            consume(A, t);
            load(A, t + 3);
            if (t + 1 < k) consume(B, t + 1);
            load(B, t + 4);
            if (t + 2 < k) consume(C, t + 2);
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u)
            st<MODE, NT>(ob + s_out_off[r], col0 + (uint64_t(u) * kThreads + tid) * 16, len,
                         u32x4{acc[u][r][0], acc[u][r][1], acc[u][r][2], acc[u][r][3]});
}

// MODE 0: tiles lie fully inside [0, len) and every shard is 16-B aligned.
// MODE 1: the (single) partial tail tile of each block, aligned layout.
// MODE 2: arbitrary alignment, byte-granular (slow path for odd layouts).
template <int R, int U, int MODE, bool NT, int KC>
__global__ __launch_bounds__(kThreads) void gf_apply_kernel(const ApplyArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t k = a.k;
    // LDS carve: [tables k*R*32 B][in_off k*8 B][out_off R*8 B]
    u32x4* s_tab = reinterpret_cast<u32x4*>(smem);
    uint64_t* s_in_off = reinterpret_cast<uint64_t*>(smem + size_t(k) * R * 32);
    uint64_t* s_out_off = s_in_off + k;

    // Stage this launch's rows [row0, row0 + R) of the plan image into LDS.
    {
        const uint32_t m = a.m;
        const uint16_t* in_idx = reinterpret_cast<const uint16_t*>(a.plan + 8);
        const uint16_t* out_idx = in_idx + k;
        const u32x4* ptab = reinterpret_cast<const u32x4*>(a.plan + a.tab_off);
        const uint32_t n16 = k * R * 2;   // u32x4 count
        for (uint32_t i = threadIdx.x; i < n16; i += kThreads) {
            const uint32_t e = i >> 1, half = i & 1;
            const uint32_t t = e / R, r = e - t * R;
            s_tab[i] = ptab[(size_t(t) * m + a.row0 + r) * 2 + half];
        }
        for (uint32_t t = threadIdx.x; t < k; t += kThreads) s_in_off[t] = uint64_t(in_idx[t]) * a.in_spitch;
        for (uint32_t r = threadIdx.x; r < uint32_t(R); r += kThreads)
            s_out_off[r] = uint64_t(out_idx[a.row0 + r] - a.out_bias) * a.out_spitch;
    }
    __syncthreads();

    const uint32_t tpb = a.tiles_per_block;
    for (uint64_t tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
        const uint64_t j = tile / tpb;
        const uint64_t c = tile - j * tpb;
        const uint64_t blk = a.blk_list ? uint64_t(a.blk_list[j]) : a.blk_first + j * a.blk_stride;
        const uint8_t* ib = a.in_base + blk * a.in_bpitch;
        uint8_t* ob = a.out_base + blk * a.out_bpitch;
        const uint64_t col0 = a.col_base + c * uint64_t(kThreads * 16 * U);
        do_tile<R, U, MODE, NT, KC>(k, a.len, ib, ob, col0, s_in_off, s_out_off, s_tab);
    }
}

template <int R, int U, int MODE, bool NT, int KC>
hipError_t launch_one(const ApplyArgs& a, int grid_cap, hipStream_t stream) {
    auto kern = gf_apply_kernel<R, U, MODE, NT, KC>;
    const size_t lds = size_t(a.k) * R * 32 + size_t(a.k) * 8 + size_t(R) * 8;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
    }
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    static thread_local int cached_dev = -1;
    static thread_local int cus = 0;
    if (cached_dev != dev) {
        e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return e;
        cached_dev = dev;
    }
    int per_cu = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kThreads, lds);
    if (e != hipSuccess) return e;
    if (per_cu < 1) per_cu = 1;
    uint64_t grid = uint64_t(cus) * uint64_t(per_cu);
    if (grid_cap > 0 && uint64_t(grid_cap) < grid) grid = uint64_t(grid_cap);
    if (grid > a.ntiles) grid = a.ntiles;
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(kern, dim3(uint32_t(grid)), dim3(kThreads), lds, stream, a);
    return hipGetLastError();
}

template <int R, int U>
hipError_t dispatch(const ApplyArgs& a, int mode, bool nt, int grid_cap, hipStream_t s) {
    switch (mode) {
        case 0: return nt ? launch_one<R, U, 0, true, 0>(a, grid_cap, s) : launch_one<R, U, 0, false, 0>(a, grid_cap, s);
        case 1: return launch_one<R, U, 1, false, 0>(a, grid_cap, s);
        default: return launch_one<R, U, 2, false, 0>(a, grid_cap, s);
    }
}

template <int R>
hipError_t dispatch_u(const ApplyArgs& a, int u, int mode, bool nt, int grid_cap, hipStream_t s) {
    switch (u) {
        case 1: return dispatch<R, 1>(a, mode, nt, grid_cap, s);
        case 4: return dispatch<R, 4>(a, mode, nt, grid_cap, s);
        default: return dispatch<R, 2>(a, mode, nt, grid_cap, s);
    }
}

}  // namespace

hipError_t launch_apply(const ApplyArgs& a, unsigned rows, int u, int mode, bool nt, int grid_cap,
                        hipStream_t stream) {
    switch (rows) {
        case 1: return dispatch_u<1>(a, u, mode, nt, grid_cap, stream);
        case 2: return dispatch_u<2>(a, u, mode, nt, grid_cap, stream);
        case 3: return dispatch_u<3>(a, u, mode, nt, grid_cap, stream);
        case 4: return dispatch_u<4>(a, u, mode, nt, grid_cap, stream);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace kern
}  // namespace shmr
