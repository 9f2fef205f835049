// Device building blocks of the gfx950 GF(2^8) matrix-apply kernel
// (design: gf_apply.hip), shared by the product kernels (gf_apply.hip) and the
// tools-only measurement variants (gf_apply_tools.hip).  The tools-only tile
// forms are declared here and defined in gf_apply_tools.hip; the product TU
// never instantiates them.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "gf_apply.hpp"

namespace shmr {
namespace kern {

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// Shards may start at any byte address (the reference's packed block buffer,
// shard i at i * S): every 16-byte access goes through this under-aligned
// type, so a misaligned one is well-defined C++.  gfx950 still emits one
// global_load/store_dwordx4 for it (the memory system's unaligned access
// mode; checked on the product code object by tests/test_isa.py).
typedef u32x4 u32x4_u __attribute__((aligned(1)));

// Variant flags (kNtLoad ... kXcd, kOccShift): gf_apply.hpp.

template <int MODE, int F>
constexpr bool has_ptrs() {
    return MODE != 0 || (F & kPtrs) != 0;
}
template <int MODE, int F>
constexpr bool has_segs() {
    return MODE != 0 || (F & kSegs) != 0;
}
template <int F>
constexpr int occ_of() {
    return (F & kOcc8) ? 8 : ((F >> kOccShift) & 15);
}
template <int F>
constexpr int depth_of() {
    return (F & kDepth9) ? 9 : (F & kDepth5) ? 5 : (F & kDepth2) ? 2 : (F & kDepth1) ? 1 : 3;
}
template <int F>
constexpr int threads_of() {
    return (F & kTh128) ? 128 : (F & kTh512) ? 512 : kThreads;
}

struct Tab {
    uint32_t t0lo, t0hi, t1lo, t1hi, t2;
};

// Constant address space: wave-uniform loads through these are scalar
// (s_load, lgkmcnt) even though the kernel stores through other pointers --
// generic loads would be vector loads on the vmcnt queue of the data stream.
typedef __attribute__((address_space(4))) const uint32_t cu32;
typedef __attribute__((address_space(4))) const uint64_t cu64;
template <class T>
__device__ __forceinline__ const T* as_const(const void* p) {
    return (const T*)(uintptr_t)p;
}

// Element i of the plan's u16 index array (4-byte aligned base) via a scalar
// dword load (gfx9 has no 16-bit scalar loads).
__device__ __forceinline__ uint32_t plan_u16(const uint16_t* base, uint32_t i) {
    const uint32_t w = as_const<cu32>(base)[i >> 1];
    return (i & 1) ? (w >> 16) : (w & 0xffffu);
}

// acc ^= c (x) w for the four bytes of w, given w's three selector words.
// v_perm_b32(src0=hi, src1=lo, sel): selector byte n picks byte n of {hi:lo};
// v_bitop3_b32 with truth table 0x96 is a three-input XOR (gfx950).
__device__ __forceinline__ uint32_t gf_mac4(uint32_t acc, const Tab& t, uint32_t s0, uint32_t s1, uint32_t s2) {
    const uint32_t a = __builtin_amdgcn_perm(t.t0hi, t.t0lo, s0);
    const uint32_t b = __builtin_amdgcn_perm(t.t1hi, t.t1lo, s1);
    const uint32_t c = __builtin_amdgcn_perm(t.t2, t.t2, s2);
    return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(acc, a, b, 0x96), c, 0u, 0x96);
}

template <int F>
__device__ __forceinline__ u32x4 load16(const uint8_t* p) {
    if constexpr ((F & kNtLoad) != 0) {
        return __builtin_nontemporal_load(reinterpret_cast<const u32x4_u*>(p));
    } else {
        return *reinterpret_cast<const u32x4_u*>(p);
    }
}

template <int F>
__device__ __forceinline__ void store16(uint8_t* p, u32x4 v) {
    if constexpr ((F & kNtStore) != 0) {
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4_u*>(p));
    } else {
        *reinterpret_cast<u32x4_u*>(p) = v;
    }
}

// 16-byte store at column col of a wave-uniform output row.  kSc1Store: a raw
// buffer store with the sc1 cache-policy bit (aux 16; no global-store builtin
// takes policy bits, and an inline-asm store would hide the >8-byte store-data
// hazard from the compiler).  The resource covers 2 GiB from the row base:
// the policy keeps sc1 to shards shorter than that (ec_core launch_set).
template <int F>
__device__ __forceinline__ void store16_row(uint8_t* row, uint64_t col, u32x4 v) {
    if constexpr ((F & kSc1Store) != 0) {
        // (readfirstlane returns int: widen through uint32_t, never sign-extend)
        const uint64_t a = uint64_t(uintptr_t(row));
        const uint64_t ua = uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(a)))) |
                            (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(a >> 32)))) << 32);
        const __amdgpu_buffer_rsrc_t rsrc =
            __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(uintptr_t(ua)), 0, 0x7fffffff, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, uint32_t(col), 0, 16);
    } else {
        store16<F>(row + col, v);
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

// Bytes [s, s + 16) of the 32-byte window lo:hi, s in [0, 16) wave-uniform
// (the switch is a scalar branch; v_alignbyte_b32 takes the byte shift).
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

// MODE 0: full tile, vector path.  MODE 1: partial tail tile (bounds per
// lane).  MODE 2: byte-granular (any alignment, no vector access).  MODE 3:
// full tile over shards off 16-byte alignment without the device's unaligned
// access mode: aligned loads realigned in registers, stores realigned across
// lanes (st_shifted).  A shard's misalignment is uniform over the tile
// (lanes' columns are multiples of 16): it is read into a scalar register, so
// every branch on it is a scalar branch.
template <int MODE, int F>
__device__ __forceinline__ u32x4 ld(const uint8_t* base, uint64_t col, uint64_t len) {
    if constexpr (MODE == 0) {
        return load16<F>(base + col);
    } else if constexpr (MODE == 1) {
        if (col + 16 <= len) return load16<F>(base + col);
        return load_bytes(base + col, int64_t(len) - int64_t(col));
    } else {
        return load_bytes(base + col, int64_t(len) - int64_t(col));
    }
}

// MODE 3 store of one wave's contiguous 1 KiB run (lane L owns bytes
// [p_L, p_L + 16), p_L = p_0 + 16 L, p_0 misaligned by mo): lane L >= 1 writes
// the aligned chunk at p_L - mo, made of the last mo bytes of lane L-1's
// value and the first 16 - mo of its own; lane 0 writes its first 16 - mo
// bytes and lane 63 its last mo bytes with byte stores.  Every lane of the
// wave must call it (ds_bpermute).
template <int F>
__device__ __forceinline__ void st_shifted(uint8_t* p, u32x4 v) {
    const uint32_t mo = __builtin_amdgcn_readfirstlane(uint32_t(uintptr_t(p)) & 15u);
    if (mo == 0) {
        store16<F>(p, v);
        return;
    }
    const uint32_t lane = threadIdx.x & 63u;
    const int src = int(((lane + 63u) & 63u) << 2);   // lane - 1
    const u32x4 prev{uint32_t(__builtin_amdgcn_ds_bpermute(src, int(v.x))),
                     uint32_t(__builtin_amdgcn_ds_bpermute(src, int(v.y))),
                     uint32_t(__builtin_amdgcn_ds_bpermute(src, int(v.z))),
                     uint32_t(__builtin_amdgcn_ds_bpermute(src, int(v.w)))};
    if (lane != 0) store16<F>(p - mo, funnel16(prev, v, 16u - mo));
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    if (lane == 0) {
#pragma unroll
        for (uint32_t b = 0; b < 16; ++b)
            if (b < 16u - mo) p[b] = uint8_t(w[b >> 2] >> (8 * (b & 3)));
    } else if (lane == 63) {
#pragma unroll
        for (uint32_t b = 0; b < 16; ++b)
            if (b >= 16u - mo) p[b] = uint8_t(w[b >> 2] >> (8 * (b & 3)));
    }
}

template <int MODE, int F>
__device__ __forceinline__ void st(uint8_t* base, uint64_t col, uint64_t len, u32x4 v) {
    if constexpr (MODE == 0) {
        store16_row<F>(base, col, v);
    } else if constexpr (MODE == 3) {
        st_shifted<F>(base + col, v);
    } else if constexpr (MODE == 1) {
        if (col + 16 <= len) store16_row<F>(base, col, v);
        else store_bytes(base + col, v, int64_t(len) - int64_t(col));
    } else {
        store_bytes(base + col, v, int64_t(len) - int64_t(col));
    }
}

// Tools-only forms (gf_apply_tools.hip).
template <int U, int F>
__device__ __forceinline__ void store_run_aligned(uint8_t* p, const u32x4 (&v)[U]);
template <int R>
__device__ __forceinline__ void diag_mac(uint32_t (&acc)[R][4], const u32x4& d, const Tab (&tb)[R]);

template <int R, int F>
__device__ __forceinline__ void mac(uint32_t (&acc)[R][4], const u32x4& d, const Tab (&tb)[R]) {
    if constexpr ((F & kDiagXor) != 0) {
        diag_mac<R>(acc, d, tb);
        return;
    }
    uint32_t w[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t s0 = w[j] & 0x07070707u;
        const uint32_t s1 = (w[j] >> 3) & 0x07070707u;
        const uint32_t s2 = (w[j] >> 6) & 0x03030303u;
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r][j] = gf_mac4(acc[r][j], tb[r], s0, s1, s2);
        if constexpr ((F & kSerial) != 0) {
            // An empty asm that "writes" this dword's sums and the next input
            // dword: dword j+1's math can only start once dword j's is done.
            if (j < 3) {
#pragma unroll
                for (int r = 0; r < R; ++r) asm volatile("" : "+v"(acc[r][j]));
                asm volatile("" : "+v"(w[j + 1]));
            }
        }
    }
}

// Where a workgroup finds its shard offsets and coefficient tables (LDS).
struct Ctx {
    const uint64_t* s_in_off;   // k entries
    const uint64_t* s_out_off;  // R entries
    const u32x4* s_tab;         // [k][R][2] u32x4
    uint8_t* ring;              // tools (kGlds): LDS input ring behind the plan
};

template <int R>
__device__ __forceinline__ void read_tabs(const Ctx& c, uint32_t t, Tab (&tb)[R]) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const u32x4 v = c.s_tab[(size_t(t) * R + r) * 2];
        const uint32_t w = reinterpret_cast<const uint32_t*>(c.s_tab)[(size_t(t) * R + r) * 8 + 4];
        tb[r] = Tab{v.x, v.y, v.z, v.w, w};
    }
}

template <int R, int U, int F>
__device__ __forceinline__ void glds_tile(const ApplyArgs& a, const Ctx& c, const uint8_t* ib, uint8_t* ob, uint64_t col0);

template <int R, int U, int F>
__device__ __forceinline__ void realign_tile(const ApplyArgs& a, const Ctx& c, const uint8_t* ib, uint8_t* ob,
                                             uint64_t col0);

// Depth-2 ring with the tail peeled (kPeel): slot 0 holds shard 0 on entry;
// the loop body is unconditional (exact wait counts), and the one or two
// shards left after it are consumed with no load past shard k-1.  The branch
// between the two tails is uniform and nothing is pending after either.
template <class Load, class Consume, class Ring>
__device__ __forceinline__ void ring2_peeled(Load& load, Consume& consume, uint32_t k, Ring (&ring)[2]) {
    uint32_t t = 0;
    for (; t + 2 < k; t += 2) {
        load(ring[1], t + 1);
        __builtin_amdgcn_sched_barrier(0);
        consume(ring[0], t);
        __builtin_amdgcn_sched_barrier(0);
        load(ring[0], t + 2);
        __builtin_amdgcn_sched_barrier(0);
        consume(ring[1], t + 1);
        __builtin_amdgcn_sched_barrier(0);
    }
    if (t + 1 < k) {
        load(ring[1], t + 1);
        __builtin_amdgcn_sched_barrier(0);
        consume(ring[0], t);
        __builtin_amdgcn_sched_barrier(0);
        consume(ring[1], t + 1);
    } else {
        consume(ring[0], t);
    }
}

// Column chunk of a lane's slot u: workgroup-strided (u * TH + tid) or, with
// kWaveRun, the wave's contiguous run ((w * U + u) * 64 + lane).
template <int U, int TH, int F>
__device__ __forceinline__ uint64_t slot_chunk(int u, uint32_t tid) {
    if constexpr ((F & kWaveRun) != 0 && U > 1)
        return uint64_t((tid & ~63u) * U + uint32_t(u) * 64u + (tid & 63u));
    else
        return uint64_t(u) * TH + tid;
}

// The tile's R output rows from the accumulators.  kStAlign (tools), full
// tiles: one aligned-store run per wave and row -- the wave's U slots when
// they are contiguous (kWaveRun, or U = 1), else one run per slot.
template <int R, int U, int TH, int MODE, int F>
__device__ __forceinline__ void store_rows(uint8_t* ob, const Ctx& c, uint64_t col0, uint64_t len, uint32_t tid,
                                           const uint32_t (&acc)[U][R][4]) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
        uint8_t* o = ob + c.s_out_off[r];
        if constexpr ((F & kStAlign) != 0 && MODE == 0) {
            if constexpr (U == 1 || (F & kWaveRun) != 0) {
                u32x4 v[U];
#pragma unroll
                for (int u = 0; u < U; ++u) v[u] = u32x4{acc[u][r][0], acc[u][r][1], acc[u][r][2], acc[u][r][3]};
                store_run_aligned<U, F>(o + col0 + uint64_t((tid & ~63u) * U) * 16, v);
            } else {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const u32x4 v[1] = {u32x4{acc[u][r][0], acc[u][r][1], acc[u][r][2], acc[u][r][3]}};
                    store_run_aligned<1, F>(o + col0 + (uint64_t(u) * TH + (tid & ~63u)) * 16, v);
                }
            }
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u)
                st<MODE, F>(o, col0 + slot_chunk<U, TH, F>(u, tid) * 16, len,
                            u32x4{acc[u][r][0], acc[u][r][1], acc[u][r][2], acc[u][r][3]});
        }
    }
}

// One tile: lanes own columns col0 + slot_chunk(u, tid) * 16, u < U.
//
// sched_barrier(0) pins program order: without it the scheduler sinks the
// look-ahead loads next to their consumers and the wave drains vmcnt(0)
// every shard (no overlap of HBM latency with the GF math).
//
// Ring of NB register buffers, unrolled by NB so buffer indices are
// compile-time (the rotation is a renaming, never a register move that would
// force a vmcnt(0)): while shard t is multiplied the loads of shards
// t+1 .. t+NB-1 are in flight.  Every load is unconditional (a branch around
// a load makes the compiler's waitcnt merge fall back to vmcnt(0)): past the
// last shard it re-reads shard k-1, an L2 hit.
template <int R, int U, int MODE, int F>
__device__ __forceinline__ void do_tile(const ApplyArgs& a, const Ctx& c, const uint8_t* ib, uint8_t* ob,
                                        uint64_t col0) {
    if constexpr ((F & kGlds) != 0 && MODE == 0) {
        glds_tile<R, U, F>(a, c, ib, ob, col0);
        return;
    }
    if constexpr ((F & kRealign) != 0 && MODE == 0) {
        realign_tile<R, U, F>(a, c, ib, ob, col0);
        return;
    }
    constexpr int TH = threads_of<F>();
    const uint32_t k = a.k;
    const uint64_t len = a.len;
    const uint32_t tid = threadIdx.x;
    uint32_t acc[U][R][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[u][r][j] = 0u;

    if constexpr (MODE == 3) {
        // Misaligned shards: each ring slot holds the two aligned 16-byte
        // loads that cover the lane's 16 bytes and the shard's misalignment;
        // the realignment runs when the slot is consumed, so the look-ahead
        // loads stay in flight as in the aligned ring.  Both loads are 16-byte
        // aligned and each holds a byte the lane needs (with m == 0 the second
        // repeats the first), so neither leaves the shard's pages.
        static_assert(U == 1, "mode 3 tiles are 4 KiB");
        constexpr int NB = 2;
        u32x4 rlo[NB], rhi[NB];
        uint32_t rm[NB];
        auto load3 = [&](u32x4& lo, u32x4& hi, uint32_t& m, uint32_t t) {
            const uint32_t tt = t < k ? t : k - 1;
            const uint8_t* base = ib + c.s_in_off[tt] + col0;
            m = __builtin_amdgcn_readfirstlane(uint32_t(uintptr_t(base)) & 15u);
            const uint8_t* q = base - m + uint64_t(tid) * 16;
            lo = load16<F>(q);
            hi = load16<F>(q + (m ? 16 : 0));
        };
        load3(rlo[0], rhi[0], rm[0], 0);
        __builtin_amdgcn_sched_barrier(0);
        for (uint32_t t = 0; t < k; t += NB) {
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                const int nx = (i + 1) % NB;
                load3(rlo[nx], rhi[nx], rm[nx], t + i + 1);
                __builtin_amdgcn_sched_barrier(0);
                if (t + i < k) {
                    Tab tb[R];
                    read_tabs<R>(c, t + i, tb);
                    mac<R, F>(acc[0], funnel16(rlo[i], rhi[i], rm[i]), tb);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r)
            st_shifted<F>(ob + c.s_out_off[r] + col0 + uint64_t(tid) * 16,
                          u32x4{acc[0][r][0], acc[0][r][1], acc[0][r][2], acc[0][r][3]});
        return;
    }

    auto load = [&](u32x4 (&buf)[U], uint32_t t) {
        const uint32_t tt = t < k ? t : k - 1;
        const uint8_t* base = ib + c.s_in_off[tt];
#pragma unroll
        for (int u = 0; u < U; ++u) buf[u] = ld<MODE, F>(base, col0 + slot_chunk<U, TH, F>(u, tid) * 16, len);
    };
    auto consume = [&](const u32x4 (&buf)[U], uint32_t t) {
        Tab tb[R];
        read_tabs<R>(c, t, tb);
#pragma unroll
        for (int u = 0; u < U; ++u) mac<R, F>(acc[u], buf[u], tb);
    };
    // (the LDS-DMA tools kernels' bounds-checked tail tiles take depth 1)
    constexpr int NB = (F & kGlds) ? 1 : depth_of<F>();
    u32x4 ring[NB][U];
#pragma unroll
    for (int i = 0; i < NB - 1; ++i) load(ring[i], i);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr ((F & kPeel) != 0 && NB == 2) {
        ring2_peeled(load, consume, k, ring);
    } else {
        for (uint32_t t = 0; t < k; t += NB) {
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                load(ring[(i + NB - 1) % NB], t + i + NB - 1);
                __builtin_amdgcn_sched_barrier(0);
                if (t + i < k) consume(ring[i], t + i);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
    store_rows<R, U, TH, MODE, F>(ob, c, col0, len, tid, acc);
}

// Byte offset of the LDS input ring (tools, kGlds) behind the staged plan.
__host__ __device__ inline uint32_t glds_ring_off(uint32_t k, uint32_t R) {
    return (k * R * 32 + k * 8 + R * 8 + 255) & ~255u;
}

// Stages rows [row0, row0 + R) of a plan image into LDS:
// [tables k*R*32 B][in_off k*8 B][out_off R*8 B].
template <int R, int TH, bool PTRS>
__device__ __forceinline__ void stage_plan(const ApplyArgs& a, const uint8_t* plan, uint8_t* smem, Ctx& c,
                                           uint64_t blk) {
    const uint32_t k = a.k;
    const uint16_t* in_idx = reinterpret_cast<const uint16_t*>(plan + 8);
    const uint16_t* out_idx = in_idx + k;
    u32x4* s_tab = reinterpret_cast<u32x4*>(smem);
    uint64_t* s_in_off = reinterpret_cast<uint64_t*>(smem + size_t(k) * R * 32);
    uint64_t* s_out_off = s_in_off + k;
    const u32x4* ptab = reinterpret_cast<const u32x4*>(plan + a.tab_off);
    const uint32_t n16 = k * R * 2;   // u32x4 count
    for (uint32_t i = threadIdx.x; i < n16; i += TH) {
        const uint32_t e = i >> 1, half = i & 1;
        const uint32_t t = e / R, r = e - t * R;
        s_tab[i] = ptab[(size_t(t) * a.m + a.row0 + r) * 2 + half];
    }
    if (PTRS && a.shard_ptrs) {   // absolute shard addresses in plan order (in/out bases are 0)
        const uint64_t* bp = a.shard_ptrs + blk * a.total;
        for (uint32_t t = threadIdx.x; t < k; t += TH) s_in_off[t] = bp[t];
        for (uint32_t r = threadIdx.x; r < uint32_t(R); r += TH) s_out_off[r] = bp[k + a.row0 + r];
    } else {
        for (uint32_t t = threadIdx.x; t < k; t += TH) s_in_off[t] = uint64_t(in_idx[t]) * a.in_spitch;
        for (uint32_t r = threadIdx.x; r < uint32_t(R); r += TH)
            s_out_off[r] = uint64_t(out_idx[a.row0 + r] - a.out_bias) * a.out_spitch;
    }
    c.s_tab = s_tab;
    c.s_in_off = s_in_off;
    c.s_out_off = s_out_off;
    c.ring = smem + glds_ring_off(k, R);
}

// ---- early-prefetch tile (flag kEarly) -------------------------------------
// A workgroup lives for one tile, so its prologue matters: the plain path
// stages the plan into LDS (global loads -> ds_write -> barrier) before its
// first data load can issue.  Here the plan's first-pass loads go out first,
// then the first NB-1 data loads (their shard offsets come from scalar loads
// of the plan's in_idx), and only then are the plan registers written to LDS
// -- the compiler's wait for them is vmcnt(NB-1), which leaves the data loads
// in flight across the LDS barrier (a raw s_barrier: lgkmcnt(0) only).

__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0), vmcnt/expcnt untouched
    __builtin_amdgcn_s_barrier();
}

struct StageRegs {
    u32x4 tab;
    uint64_t in_off, out_off;
};

// First pass of stage_plan (entry threadIdx.x of each array), loaded into
// registers with clamped indices so every load is unconditional.  Global
// address space: vector loads on vmcnt only (a generic pointer would make
// them flat loads, which also count on lgkmcnt and serialise against the
// scalar loads of the prologue).
typedef __attribute__((address_space(1))) const u32x4 gu32x4;
typedef __attribute__((address_space(1))) const uint16_t gu16;
typedef __attribute__((address_space(1))) const uint64_t gu64;

// PTRS (kernels compiled with kPtrs): shard offsets are absolute addresses
// from block blk's row of the shard-pointer table (in/out bases are 0).
template <int R, bool PTRS>
__device__ __forceinline__ void stage_issue(const ApplyArgs& a, const uint8_t* plan, uint64_t blk, StageRegs& s) {
    const uint32_t k = a.k, i = threadIdx.x;
    const uint32_t n16 = k * R * 2;
    const uint32_t ic = i < n16 ? i : n16 - 1;
    const uint32_t e = ic >> 1, half = ic & 1;
    const uint32_t t = e / R, r = e - t * R;
    s.tab = ((const gu32x4*)(uintptr_t)(plan + a.tab_off))[(size_t(t) * a.m + a.row0 + r) * 2 + half];
    const uint32_t ii = i < k ? i : k - 1, ir = a.row0 + (i < uint32_t(R) ? i : R - 1);
    if constexpr (PTRS) {   // the block's row is in plan order: no index load in front
        const gu64* bp = (const gu64*)(uintptr_t)(a.shard_ptrs + blk * a.total);
        s.in_off = bp[ii];
        s.out_off = bp[k + ir];
    } else {
        const gu16* in_idx = (const gu16*)(uintptr_t)(plan + 8);
        const uint32_t ti = in_idx[ii];
        const uint32_t to = in_idx[k + ir];
        s.in_off = uint64_t(ti) * a.in_spitch;
        s.out_off = uint64_t(to - a.out_bias) * a.out_spitch;
    }
}

template <int R, int TH, bool PTRS>
__device__ __forceinline__ void stage_commit(const ApplyArgs& a, const uint8_t* plan, uint8_t* smem, Ctx& c,
                                             const StageRegs& s, uint64_t blk) {
    const uint32_t k = a.k, i = threadIdx.x;
    u32x4* s_tab = reinterpret_cast<u32x4*>(smem);
    uint64_t* s_in_off = reinterpret_cast<uint64_t*>(smem + size_t(k) * R * 32);
    uint64_t* s_out_off = s_in_off + k;
    const uint32_t n16 = k * R * 2;
    if (i < n16) s_tab[i] = s.tab;
    if (i < k) s_in_off[i] = s.in_off;
    if (i < uint32_t(R)) s_out_off[i] = s.out_off;
    // entries beyond the first TH (large k * R): plain staging
    const u32x4* ptab = reinterpret_cast<const u32x4*>(plan + a.tab_off);
    const uint16_t* in_idx = reinterpret_cast<const uint16_t*>(plan + 8);
    for (uint32_t j = i + TH; j < n16; j += TH) {
        const uint32_t e = j >> 1, half = j & 1;
        const uint32_t t = e / R, r = e - t * R;
        s_tab[j] = ptab[(size_t(t) * a.m + a.row0 + r) * 2 + half];
    }
    for (uint32_t t = i + TH; t < k; t += TH)
        s_in_off[t] = PTRS ? a.shard_ptrs[blk * a.total + t] : uint64_t(in_idx[t]) * a.in_spitch;
    c.s_tab = s_tab;
    c.s_in_off = s_in_off;
    c.s_out_off = s_out_off;
}

template <int R, int U, int MODE, int F>
__device__ __forceinline__ void early_tile(const ApplyArgs& a, const uint8_t* plan, uint8_t* smem, bool first,
                                           const uint8_t* ib, uint8_t* ob, uint64_t col0, uint64_t blk) {
    constexpr int TH = threads_of<F>();
    constexpr int NB = depth_of<F>();
    // shard-pointer tables (device memory): the first loads' addresses come
    // from scalar loads of the block's table row (plan order: entry t is input t)
    constexpr bool PTRS = (F & kPtrs) != 0;
    const uint32_t k = a.k;
    const uint64_t len = a.len;
    const uint32_t tid = threadIdx.x;
    const uint16_t* in_idx = reinterpret_cast<const uint16_t*>(plan + 8);
    StageRegs sr;
    stage_issue<R, PTRS>(a, plan, blk, sr);
    __builtin_amdgcn_sched_barrier(0);
    u32x4 ring[NB][U];
#pragma unroll
    for (int i = 0; i < NB - 1; ++i) {
        const uint32_t t = uint32_t(i) < k ? uint32_t(i) : k - 1;
        const uint8_t* base;
        if constexpr (PTRS)
            base = reinterpret_cast<const uint8_t*>(uintptr_t(as_const<cu64>(a.shard_ptrs + blk * a.total)[t]));
        else
            base = ib + uint64_t(plan_u16(in_idx, t)) * a.in_spitch;
#pragma unroll
        for (int u = 0; u < U; ++u) ring[i][u] = ld<MODE, F>(base, col0 + slot_chunk<U, TH, F>(u, tid) * 16, len);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (!first) lds_barrier();   // the previous tile's LDS readers are done
    Ctx c{};
    stage_commit<R, TH, PTRS>(a, plan, smem, c, sr, blk);
    lds_barrier();
    __builtin_amdgcn_sched_barrier(0);

    uint32_t acc[U][R][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[u][r][j] = 0u;
    auto load = [&](u32x4 (&buf)[U], uint32_t t) {
        const uint32_t tt = t < k ? t : k - 1;
        const uint8_t* base = ib + c.s_in_off[tt];
#pragma unroll
        for (int u = 0; u < U; ++u) buf[u] = ld<MODE, F>(base, col0 + slot_chunk<U, TH, F>(u, tid) * 16, len);
    };
    auto consume = [&](const u32x4 (&buf)[U], uint32_t t) {
        Tab tb[R];
        read_tabs<R>(c, t, tb);
#pragma unroll
        for (int u = 0; u < U; ++u) mac<R, F>(acc[u], buf[u], tb);
    };
    if constexpr ((F & kPeel) != 0 && NB == 2) {
        ring2_peeled(load, consume, k, ring);
    } else {
        for (uint32_t t = 0; t < k; t += NB) {
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                load(ring[(i + NB - 1) % NB], t + i + NB - 1);
                __builtin_amdgcn_sched_barrier(0);
                if (t + i < k) consume(ring[i], t + i);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
    store_rows<R, U, TH, MODE, F>(ob, c, col0, len, tid, acc);
}

template <int R, int U, int MODE, int F, bool IDENT>
__device__ __forceinline__ void spre_tile(const ApplyArgs& a, const uint8_t* plan, const uint8_t* ib, uint8_t* ob, uint64_t col0);

// Block index and plan of launch block j of a segment launch: binary search
// over the (kernel-argument, wave-uniform) segment table -- scalar loads.
__device__ __forceinline__ uint64_t seg_block(const ApplyArgs& a, uint64_t j, const uint8_t** plan) {
    uint32_t lo = 0, hi = a.nseg;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.segs[mid].start <= j) lo = mid;
        else hi = mid;
    }
    *plan = a.segs[lo].plan;
    return uint64_t(a.segs[lo].first) + (j - a.segs[lo].start) * uint64_t(a.segs[lo].stride);
}

// Block j and column tile cc of grid tile `tile` (see ApplyArgs::lead_tails).
struct TileRef {
    uint64_t j, cc;
    bool tail;
};
template <int F>
__device__ __forceinline__ TileRef tile_ref(const ApplyArgs& a, uint64_t tile) {
    const uint32_t tpb = a.tiles_per_block;
    if constexpr ((F & kFuse) != 0) {
        if (tile < a.lead_tails) return TileRef{tile, tpb, true};
        tile -= a.lead_tails;
    }
    const uint64_t j = tile / tpb;
    return TileRef{j, tile - j * tpb, false};
}

// Neighbouring tiles a workgroup takes per grid step (kPair: 2).
template <int F>
__device__ __host__ constexpr uint64_t tiles_per_wg() {
    return (F & kPair) != 0 ? 2 : 1;
}

// First grid tile of this workgroup (kXcd: XCD-grouped, one workgroup per
// tile; kPair: tile pairs 2w, 2w + 1, grid-strided over the pairs).
template <int F>
__device__ __forceinline__ uint64_t first_tile(const ApplyArgs& a) {
    uint64_t w = blockIdx.x;
    if constexpr ((F & kPair) != 0) return w * 2;
    if constexpr ((F & kXcd) != 0) {
        if (uint64_t(gridDim.x) == a.ntiles) {
            const uint64_t q = a.ntiles >> 3;
            if (w < (q << 3)) w = (w & 7u) * q + (w >> 3);
        }
    }
    return w;
}

template <int F>
__device__ __forceinline__ uint64_t next_tile(uint64_t tile) {
    if constexpr ((F & kPair) != 0) return (tile & 1) ? tile + uint64_t(gridDim.x) * 2 - 1 : tile + 1;
    return tile + gridDim.x;
}

// The second __launch_bounds__ argument is amdgpu_waves_per_eu (minimum).
template <int R, int U, int MODE, int F>
__global__ __launch_bounds__(threads_of<F>(), occ_of<F>() ? occ_of<F>() : 1) void gf_apply_kernel(const ApplyArgs a) {
    constexpr int TH = threads_of<F>();
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    // Multi-plan launches (reconstruct batches with several erasure patterns)
    // pick the plan per block; single-plan launches stage it once.
    const bool multi = a.plan_table != nullptr;
    if constexpr ((F & (kEarly | kSPre)) != 0) {
        const uint64_t tb = uint64_t(TH) * 16 * U;
        bool first = true;
        for (uint64_t tile = first_tile<F>(a); tile < a.ntiles; tile = next_tile<F>(tile)) {
            const TileRef tr = tile_ref<F>(a, tile);
            const uint64_t j = tr.j, cc = tr.cc;
            uint64_t blk;
            const uint8_t* plan = a.plan;
            if (has_segs<MODE, F>() && a.nseg) {
                blk = seg_block(a, j, &plan);
            } else {
                blk = a.blk_list ? uint64_t(as_const<cu32>(a.blk_list)[j]) : a.blk_first + j * a.blk_stride;
                if (multi) {   // plan_table[blk_plan[j]] through scalar loads
                    const uint32_t pi = plan_u16(a.blk_plan, uint32_t(j));
                    const cu32* pt = as_const<cu32>(a.plan_table);
                    plan = reinterpret_cast<const uint8_t*>(uint64_t(pt[2 * pi]) | (uint64_t(pt[2 * pi + 1]) << 32));
                }
            }
            const uint8_t* ib = a.in_base + blk * a.in_bpitch;
            uint8_t* ob = a.out_base + blk * a.out_bpitch;
            const uint64_t col = a.col_base + cc * tb;
            if constexpr ((F & kSPre) != 0) {
                if ((F & kFuse) != 0 && MODE == 0 && tr.tail) {
                    if (a.in_identity) spre_tile<R, U, 1, F, true>(a, plan, ib, ob, col);
                    else spre_tile<R, U, 1, F, false>(a, plan, ib, ob, col);
                } else if (a.in_identity) {
                    spre_tile<R, U, MODE, F, true>(a, plan, ib, ob, col);
                } else {
                    spre_tile<R, U, MODE, F, false>(a, plan, ib, ob, col);
                }
            } else if ((F & kFuse) != 0 && MODE == 0 && tr.tail) {
                early_tile<R, U, 1, F>(a, plan, smem, first, ib, ob, col, blk);
            } else {
                early_tile<R, U, MODE, F>(a, plan, smem, first, ib, ob, col, blk);
            }
            first = false;
        }
        return;
    }
    // Multi-plan, segment and shard-pointer launches restage per tile.
    constexpr bool PTRS = has_ptrs<MODE, F>(), SEGS = has_segs<MODE, F>();
    const bool restage = multi || (SEGS && a.nseg != 0) || (PTRS && a.shard_ptrs != nullptr);
    Ctx c{};
    if (!restage) {
        stage_plan<R, TH, PTRS>(a, a.plan, smem, c, 0);
        __syncthreads();
    }
    const uint64_t tb = uint64_t(TH) * 16 * U;
    for (uint64_t tile = first_tile<F>(a); tile < a.ntiles; tile = next_tile<F>(tile)) {
        const TileRef tr = tile_ref<F>(a, tile);
        const uint64_t j = tr.j, cc = tr.cc;
        const uint8_t* plan = a.plan;
        uint64_t blk;
        if (SEGS && a.nseg) {
            blk = seg_block(a, j, &plan);
        } else {
            blk = a.blk_list ? uint64_t(a.blk_list[j]) : a.blk_first + j * a.blk_stride;
            if (multi) plan = a.plan_table[a.blk_plan[j]];
        }
        if (restage) {
            __syncthreads();   // previous tile's LDS reads are done
            stage_plan<R, TH, PTRS>(a, plan, smem, c, blk);
            __syncthreads();
        }
        const uint8_t* ib = a.in_base + blk * a.in_bpitch;
        uint8_t* ob = a.out_base + blk * a.out_bpitch;
        if ((F & kFuse) != 0 && MODE == 0 && tr.tail) do_tile<R, U, 1, F>(a, c, ib, ob, a.col_base + cc * tb);
        else do_tile<R, U, MODE, F>(a, c, ib, ob, a.col_base + cc * tb);
    }
}

template <int R, int U, int MODE, int F>
hipError_t launch_one(const ApplyArgs& a, const Variant& v, int grid_cap, hipStream_t stream) {
    auto kern = gf_apply_kernel<R, U, MODE, F>;
    size_t lds = (F & kSPre) ? 0 : size_t(a.k) * R * 32 + size_t(a.k) * 8 + size_t(R) * 8;
    if constexpr ((F & kGlds) != 0)
        lds = glds_ring_off(a.k, R) + size_t(depth_of<F>()) * U * threads_of<F>() * 16;
    // Optional occupancy cap: pad the LDS allocation so at most wgs_per_cu
    // workgroups fit in a CU's 160 KiB.
    if (v.wgs_per_cu > 0) {
        const size_t cap = (160u * 1024u) / unsigned(v.wgs_per_cu) / 128u * 128u;
        if (cap > lds) lds = cap;
    }
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (e != hipSuccess) return e;
    }
    uint64_t grid;
    const uint64_t units = (a.ntiles + tiles_per_wg<F>() - 1) / tiles_per_wg<F>();   // kPair: tile pairs
    if (grid_cap < 0) {
        grid = units;                         // one workgroup per tile (pair)
        if (grid > 0x7fffffffull) grid = 0x7fffffffull;
    } else {
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        int cus = 0, per_cu = 0;
        e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return e;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads_of<F>(), lds);
        if (e != hipSuccess) return e;
        if (per_cu < 1) per_cu = 1;
        uint64_t maxg = uint64_t(cus) * uint64_t(per_cu);
        if (grid_cap > 0 && uint64_t(grid_cap) < maxg) maxg = uint64_t(grid_cap);
        // Balanced persistent grid: every workgroup gets ceil(ntiles / maxg)
        // or one fewer tile, so the launch has no straggler round.
        const uint64_t per = (units + maxg - 1) / maxg;
        grid = (units + per - 1) / per;
    }
    if (grid > units) grid = units;
    if (grid == 0) return hipSuccess;
    // Launched by name, never through the function-pointer variable `kern`: in
    // host code a kernel's "address" is its kernel handle (a data object), and
    // clang's -fsanitize=function (part of -fsanitize=undefined) instruments an
    // indirect kernel launch with a read of the 8 bytes in front of it --
    // out of bounds of the handle, which the optimizer then treats as
    // unreachable: the launch was deleted, leaving only
    // __hipPushCallConfiguration (no kernel ran, no sanitizer report; DESIGN.md
    // §3).  tests/test_isa.py checks every instantiation has its launch.
    hipLaunchKernelGGL((gf_apply_kernel<R, U, MODE, F>), dim3(uint32_t(grid)), dim3(threads_of<F>()), lds, stream, a);
    return hipGetLastError();
}

}  // namespace
}  // namespace kern
}  // namespace shmr
