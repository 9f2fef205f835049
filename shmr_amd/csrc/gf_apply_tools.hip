// Measurement-only variants of the gfx950 GF(2^8) matrix-apply kernel,
// linked into the tools build (libshmr_ec_tools.so, -DSHMR_EC_TOOLS) only.
// Each was measured against the product policy ("Kernel
// decisions at a glance") and kept as the record of that measurement:
//  * the LDS-DMA input ring (glds_tile): -1.2 to -9.6 points;
//  * scalar-loaded tables and offsets, no LDS (spre_tile): -1.0 to -6.5;
//  * the XOR-only diagnostic twin (diag_mac; WRONG results by design), the
//    ceiling of the kernel's own access pattern;
//  * the DPP realigning-load tile for misaligned shards (realign_tile):
//    -2.7 / -2.7 points against the unaligned vector path on
//    the reference's packed RS(10,4) buffer;
//  * tile pairs per workgroup on the table kernels (kPair: the second tile
//    finds its block's pointer-table row in the scalar cache): -2.0 to -10.3
//    points (profiles/r06/s39);
//  * ring depths 1/3/5/9, 128/512-lane workgroups, occupancy targets and the
//    other knob combinations of the instantiation list below.
#include <hip/hip_runtime.h>

#include "gf_tile.hpp"

namespace shmr {
namespace kern {

namespace {

template <int R>
__device__ __forceinline__ void diag_mac(uint32_t (&acc)[R][4], const u32x4& d, const Tab (&tb)[R]) {
    const uint32_t w[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r][j] ^= w[j] + tb[r].t2;
}

// LDS ring: slot s holds shard (t mod NB)'s U x 16 B per lane, lane-linear per
// wave (LDS-DMA writes wave base + lane * 16).  Each lane reads back only the
// bytes its own wave's DMA wrote, so the covering vmcnt orders the ds_read (no
// barrier); the slot a DMA refills was last read one step earlier, and those
// reads have returned (their values were used).
template <int R, int U, int F>
__device__ __forceinline__ void glds_tile(const ApplyArgs& a, const Ctx& c, const uint8_t* ib, uint8_t* ob, uint64_t col0) {
    constexpr int TH = threads_of<F>();
    constexpr int NB = depth_of<F>();
    constexpr int AUX = (F & kNtLoad) ? 2 : 0;   // nt
    const uint32_t k = a.k;
    const uint64_t len = a.len;
    const uint32_t tid = threadIdx.x;
    const uint32_t wave_base = (tid & ~63u) * 16;
    uint32_t acc[U][R][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[u][r][j] = 0u;
    auto gload = [&](int slot, uint32_t t) {
        const uint32_t tt = t < k ? t : k - 1;
        const uint8_t* base = ib + c.s_in_off[tt] + col0 + uint64_t(tid) * 16;
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_amdgcn_global_load_lds(
                (__attribute__((address_space(1))) void*)(uintptr_t)(base + uint64_t(u) * TH * 16),
                (__attribute__((address_space(3))) void*)(c.ring + (slot * U + u) * TH * 16 + wave_base), 16, 0, AUX);
    };
    auto consume_lds = [&](int slot, uint32_t t) {
        Tab tb[R];
        read_tabs<R>(c, t, tb);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u32x4 v = *reinterpret_cast<const u32x4*>(c.ring + ((slot * U + u) * TH + tid) * 16);
            mac<R, F>(acc[u], v, tb);
        }
    };
    // vmcnt(N) with expcnt / lgkmcnt left alone (gfx9 encoding)
    constexpr int VM = (NB - 1) * U;
    constexpr int WAIT = (VM & 15) | ((VM >> 4) << 14) | (7 << 4) | (15 << 8);
#pragma unroll
    for (int i = 0; i < NB - 1; ++i) gload(i, i);
    __builtin_amdgcn_sched_barrier(0);
    for (uint32_t t = 0; t < k; t += NB) {
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            gload((i + NB - 1) % NB, t + i + NB - 1);
            __builtin_amdgcn_s_waitcnt(WAIT);   // shard t+i has landed in slot i
            __builtin_amdgcn_sched_barrier(0);
            if (t + i < k) consume_lds(i, t + i);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0): no DMA into LDS outlives the tile
#pragma unroll
    for (int r = 0; r < R; ++r) {
        uint8_t* o = ob + c.s_out_off[r];
#pragma unroll
        for (int u = 0; u < U; ++u)
            st<0, F>(o, col0 + (uint64_t(u) * TH + tid) * 16, len,
                     u32x4{acc[u][r][0], acc[u][r][1], acc[u][r][2], acc[u][r][3]});
    }
}

// ---- scalar-table tile (flag kSPre) --------------------------------------
// No LDS: shard offsets (in_idx) and the coefficient tables are wave-uniform,
// so they come from the plan image by scalar loads (constant address space)
// into SGPRs; only the table words v_perm cannot take from an SGPR are copied
// to VGPRs.  Per step: issue the data load for shard t+NB-1 (its offset was
// fetched during the previous step), the scalar loads of shard t's tables and
// of the next offset, then multiply shard t.
template <int R>
__device__ __forceinline__ void s_tabs(const ApplyArgs& a, const uint8_t* plan, uint32_t t, Tab (&tb)[R]) {
    const cu32* e0 = as_const<cu32>(plan + a.tab_off) + (size_t(t) * a.m + a.row0) * 8;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const cu32* e = e0 + r * 8;
        tb[r] = Tab{e[0], e[1], e[2], e[3], e[4]};
    }
}

template <int R, int U, int MODE, int F, bool IDENT>
__device__ __forceinline__ void spre_tile(const ApplyArgs& a, const uint8_t* plan, const uint8_t* ib, uint8_t* ob, uint64_t col0) {
    constexpr int TH = threads_of<F>();
    constexpr int NB = depth_of<F>();
    const uint32_t k = a.k;
    const uint64_t len = a.len;
    const uint32_t tid = threadIdx.x;
    const uint16_t* in_idx = reinterpret_cast<const uint16_t*>(plan + 8);
    auto in_off = [&](uint32_t t) {
        const uint32_t tt = t < k ? t : k - 1;
        if constexpr (IDENT) return uint64_t(tt) * a.in_spitch;   // pure scalar arithmetic
        else return uint64_t(plan_u16(in_idx, tt)) * a.in_spitch;
    };
    uint32_t acc[U][R][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[u][r][j] = 0u;
    auto load = [&](u32x4 (&buf)[U], uint64_t off) {
        const uint8_t* base = ib + off;
#pragma unroll
        for (int u = 0; u < U; ++u) buf[u] = ld<MODE, F>(base, col0 + (uint64_t(u) * TH + tid) * 16, len);
    };
    u32x4 ring[NB][U];
#pragma unroll
    for (int i = 0; i < NB - 1; ++i) load(ring[i], in_off(i));
    uint64_t next_off = in_off(NB - 1);
    __builtin_amdgcn_sched_barrier(0);
    for (uint32_t t = 0; t < k; t += NB) {
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            load(ring[(i + NB - 1) % NB], next_off);   // shard t+i+NB-1
            __builtin_amdgcn_sched_barrier(0);
            next_off = in_off(t + i + NB);
            // Unconditional multiply (a branch here lets the compiler sink
            // the look-ahead load into it, collapsing the ring): past the
            // last shard the tables are zeroed, so the product is 0.
            {
                const bool live = t + i < k;
                Tab tb[R];
                s_tabs<R>(a, plan, live ? t + i : k - 1, tb);
                const uint32_t msk = live ? ~0u : 0u;
#pragma unroll
                for (int r = 0; r < R; ++r)
                    tb[r] = Tab{tb[r].t0lo & msk, tb[r].t0hi & msk, tb[r].t1lo & msk, tb[r].t1hi & msk, tb[r].t2 & msk};
#pragma unroll
                for (int u = 0; u < U; ++u) mac<R, F>(acc[u], ring[i][u], tb);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        uint8_t* o = ob + uint64_t(plan_u16(in_idx, k + a.row0 + r) - a.out_bias) * a.out_spitch;
#pragma unroll
        for (int u = 0; u < U; ++u)
            st<MODE, F>(o, col0 + (uint64_t(u) * TH + tid) * 16, len,
                        u32x4{acc[u][r][0], acc[u][r][1], acc[u][r][2], acc[u][r][3]});
    }
}

// Lane L's 16 bytes at byte offset m (1..15) of the 32-byte window formed by
// its own aligned chunk and lane L+1's; lane 63 supplies `edge` (the next
// wave's first chunk) as its neighbour.  wave_shl:1 moves lane L+1's dword
// to lane L; lane 63 has no source lane and keeps `edge`.
__device__ __forceinline__ u32x4 realign_lanes(const u32x4& lo, const u32x4& edge, uint32_t m) {
    const u32x4 nx{uint32_t(__builtin_amdgcn_update_dpp(int(edge.x), int(lo.x), 0x130, 0xf, 0xf, false)),
                   uint32_t(__builtin_amdgcn_update_dpp(int(edge.y), int(lo.y), 0x130, 0xf, 0xf, false)),
                   uint32_t(__builtin_amdgcn_update_dpp(int(edge.z), int(lo.z), 0x130, 0xf, 0xf, false)),
                   uint32_t(__builtin_amdgcn_update_dpp(int(edge.w), int(lo.w), 0x130, 0xf, 0xf, false))};
    return funnel16(lo, nx, m);
}

// ---- realigning-load tile (flag kRealign) --------------------------------
// Shards off 16-byte alignment (the reference's packed block buffer): every
// lane loads its ALIGNED 16-byte chunk, takes the next lane's leading bytes
// with a DPP wavefront shift (v_mov_b32_dpp wave_shl:1) and realigns in
// registers; lane 63's neighbour is the next wave's first chunk.  Stores stay
// unaligned 16-byte vector stores (probe-verified device only).  The depth-2
// register ring of do_tile, each slot holding the lane's aligned chunk(s),
// the edge chunk(s) and the shard's misalignment m (wave-uniform, a scalar).
// Why: a misaligned 16-byte vector load is split into several L1 (TCP)
// accesses -- 64 TCP cache accesses per KiB of RS(10,4) encode traffic on the
// packed buffer against 18 on aligned slots (profiles/r03/counters_encode104.md).
// The first form (lanes of instruction u over columns u * TH + tid, an edge
// load per instruction) measured -2.7 points against the unaligned vector
// path (profiles/r03/tune_*_packed_realign.txt).  Here each wave reads one
// contiguous U KiB run, so an edge load per run (a scalar load instead would
// share lgkmcnt with the LDS table reads and serialise the look-ahead).
template <int R, int U, int F>
__device__ __forceinline__ void realign_tile(const ApplyArgs& a, const Ctx& c, const uint8_t* ib, uint8_t* ob,
                                             uint64_t col0) {
    constexpr int NB = 2;
    const uint32_t k = a.k;
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t wave0 = tid - lane;
    // Wave-contiguous runs: chunk u of lane L in wave w covers column chunk
    // (w * U + u) * 64 + L, so a wave's U instructions read one contiguous
    // U KiB run and lane 63's neighbour in instruction u < U-1 is lane 0 of
    // instruction u+1 (readlane); only the run's end needs the edge load.
    auto chunk = [&](int u) { return uint64_t(wave0 * U + uint32_t(u) * 64u + lane); };
    uint32_t acc[U][R][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[u][r][j] = 0u;
    u32x4 rlo[NB][U], red[NB];
    uint32_t rm[NB];
    auto load = [&](int s, uint32_t t) {
        const uint32_t tt = t < k ? t : k - 1;
        const uint8_t* base = ib + c.s_in_off[tt] + col0;
        const uint32_t m = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(uintptr_t(base)) & 15u)));
        rm[s] = m;
        const uint8_t* al = base - m;
#pragma unroll
        for (int u = 0; u < U; ++u) rlo[s][u] = load16<F>(al + chunk(u) * 16);
        // the chunk after the run (wave-uniform address, one request; with
        // m == 0 it stays on the run's own last chunk, never past the buffer)
        red[s] = load16<F>(al + (uint64_t(wave0) * U + uint64_t(U) * 64u - (m ? 0u : 1u)) * 16);
    };
    auto neighbour = [&](const u32x4 (&lo)[U], const u32x4& edge, int u) -> u32x4 {
        if (u + 1 < U) {
            const u32x4& nx = lo[u + 1];
            return u32x4{uint32_t(__builtin_amdgcn_readlane(int(nx.x), 0)), uint32_t(__builtin_amdgcn_readlane(int(nx.y), 0)),
                         uint32_t(__builtin_amdgcn_readlane(int(nx.z), 0)), uint32_t(__builtin_amdgcn_readlane(int(nx.w), 0))};
        }
        return edge;
    };
    load(0, 0);
    __builtin_amdgcn_sched_barrier(0);
    for (uint32_t t = 0; t < k; t += NB) {
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            load((i + 1) % NB, t + i + 1);
            __builtin_amdgcn_sched_barrier(0);
            if (t + i < k) {
                Tab tb[R];
                read_tabs<R>(c, t + i, tb);
                const uint32_t m = rm[i];
#pragma unroll
                for (int u = 0; u < U; ++u)
                    mac<R, F>(acc[u], m ? realign_lanes(rlo[i][u], neighbour(rlo[i], red[i], u), m) : rlo[i][u], tb);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        uint8_t* o = ob + c.s_out_off[r];
#pragma unroll
        for (int u = 0; u < U; ++u)
            store16<F>(o + col0 + chunk(u) * 16, u32x4{acc[u][r][0], acc[u][r][1], acc[u][r][2], acc[u][r][3]});
    }
}

// ---- aligned-store runs (flag kStAlign) ------------------------------------
// An output row off 16-byte alignment by mo (wave-uniform): misaligned 16-byte
// vector stores cost ~18 % of a streaming copy's rate where misaligned loads
// cost nothing (profiles/r03/r03m/misalign_bench.jsonl).  The wave's U slots
// cover one contiguous run of U * 64 chunks at p; lane L of slot u stores the
// ALIGNED chunk made of its predecessor's last mo bytes and its own first
// 16 - mo (predecessor by DPP wave_shr:1; slot u > 0's lane 0 takes slot
// u-1's lane 63 by readlane).  The run's first chunk (lane 0 of slot 0: bytes
// [mo, 16) of the aligned chunk below p) and the chunk after its end (lane 63
// of slot U-1: bytes [0, mo)) are partial: masked dword stores plus the split
// dword's short / byte stores; the neighbouring run writes the complementary
// bytes.
__device__ __forceinline__ uint32_t dpp_shr1(uint32_t old, uint32_t v) {
    return uint32_t(__builtin_amdgcn_update_dpp(int(old), int(v), 0x138, 0xf, 0xf, false));
}

template <int U, int F>
__device__ __forceinline__ void store_run_aligned(uint8_t* p, const u32x4 (&v)[U]) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t mo = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(uintptr_t(p)) & 15u)));
    if (mo == 0) {
#pragma unroll
        for (int u = 0; u < U; ++u) store16<F>(p + (uint64_t(u) * 64 + lane) * 16, v[u]);
        return;
    }
    uint8_t* a = p - mo;   // the aligned chunk holding the run's first byte
#pragma unroll
    for (int u = 0; u < U; ++u) {
        u32x4 carry = v[u];
        if (u > 0)
            carry = u32x4{uint32_t(__builtin_amdgcn_readlane(int(v[u - 1].x), 63)),
                          uint32_t(__builtin_amdgcn_readlane(int(v[u - 1].y), 63)),
                          uint32_t(__builtin_amdgcn_readlane(int(v[u - 1].z), 63)),
                          uint32_t(__builtin_amdgcn_readlane(int(v[u - 1].w), 63))};
        const u32x4 prev{dpp_shr1(carry.x, v[u].x), dpp_shr1(carry.y, v[u].y), dpp_shr1(carry.z, v[u].z),
                         dpp_shr1(carry.w, v[u].w)};
        if (u > 0 || lane != 0)
            store16<F>(a + (uint64_t(u) * 64 + lane) * 16, funnel16(prev, v[u], 16u - mo));
    }
    const bool head = lane == 0, tail = lane == 63;
    const u32x4 src = tail ? v[U - 1] : v[0];
    const u32x4 rot = funnel16(src, src, 16u - mo);   // the lane's bytes in the output chunk's frame
    uint8_t* q = tail ? a + uint64_t(U) * 1024 : a;
    const uint32_t w[4] = {rot.x, rot.y, rot.z, rot.w};
#pragma unroll
    for (uint32_t d = 0; d < 4; ++d)
        if ((head && 4 * d >= mo) || (tail && 4 * d + 4 <= mo)) *reinterpret_cast<uint32_t*>(q + 4 * d) = w[d];
    if (mo & 3u) {
        const uint32_t d = mo >> 2;
        uint32_t x = w[0];
#pragma unroll
        for (uint32_t j = 1; j < 4; ++j)
            if (d == j) x = w[j];
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

#define SHMR_VARIANTS_TOOLS(X) \
    X(1, 0) \
    X(1, kNtLoad) \
    X(1, kNtStore) \
    X(1, kNtLoad | kNtStore) \
    X(1, kOcc8 | kNtLoad | kNtStore) \
    X(1, kDiagXor) \
    X(1, kDiagXor | kNtLoad | kNtStore) \
    X(2, 0) \
    X(2, kNtLoad | kNtStore) \
    X(4, kNtLoad | kNtStore) \
    X(1, kNtLoad | kNtStore | kTh128) \
    X(1, kNtLoad | kNtStore | kTh512) \
    X(1, kNtStore | kTh512) \
    X(2, kNtLoad | kNtStore | kTh128) \
    X(1, kNtLoad | kNtStore | kDepth5) \
    X(1, kNtLoad | kNtStore | kDepth9) \
    X(1, kNtLoad | kDepth5) \
    X(1, kNtLoad | kDepth9) \
    X(1, kNtLoad | kNtStore | kDepth1) \
    X(1, kNtLoad | kDepth2) \
    X(1, kNtLoad | kNtStore | kDepth2 | kTh512) \
    X(1, kNtLoad | kNtStore | kDepth2 | kTh128) \
    X(1, kNtLoad | kNtStore | kDepth2 | kOcc8) \
    X(1, kNtLoad | kNtStore | kDepth2 | (6 << kOccShift)) \
    X(1, kNtLoad | kNtStore | kDepth2 | (7 << kOccShift)) \
    X(1, kNtLoad | kNtStore | (6 << kOccShift)) \
    X(1, kNtLoad | kNtStore | (7 << kOccShift)) \
    X(2, kNtLoad | kNtStore | kDepth2 | (6 << kOccShift)) \
    X(1, kNtLoad | kNtStore | kEarly) \
    X(1, kNtLoad | kNtStore | kDepth2 | kEarly | (6 << kOccShift)) \
    X(1, kNtLoad | kNtStore | kDepth2 | kSPre) \
    X(2, kNtLoad | kNtStore | kDepth2 | kSPre) \
    X(1, kNtLoad | kNtStore | kSPre) \
    X(1, kNtLoad | kNtStore | kSegs) \
    X(1, kNtLoad | kNtStore | kSegs | kFuse) \
    X(1, kNtLoad | kNtStore | kDepth2 | kSegs | kTh512) \
    X(1, kNtLoad | kNtStore | kDepth2 | kSegs | kTh128) \
    X(2, kNtLoad | kNtStore | kFuse) \
    X(2, kNtLoad | kNtStore | kDepth2 | kFuse | kTh128) \
    X(1, kNtLoad | kNtStore | kDepth2 | kFuse | kTh512) \
    X(1, kNtLoad | kNtStore | kDepth2 | kSerial) \
    X(2, kNtLoad | kNtStore | kDepth2 | kSerial) \
    X(1, kNtLoad | kNtStore | kDepth2 | kFuse | kSerial) \
    X(2, kNtLoad | kNtStore | kDepth2 | kFuse | kSerial) \
    X(1, kNtLoad | kNtStore | kSerial) \
    X(1, kNtLoad | kNtStore | kFuse | kSerial) \
    X(1, kNtLoad | kNtStore | kDepth5 | kSerial) \
    X(1, kNtLoad | kNtStore | kDepth2 | kSegs | kSerial) \
    X(1, kNtLoad | kNtStore | kDepth2 | kSegs | kFuse | kSerial) \
    X(1, kNtLoad | kNtStore | kDepth2 | kEarly | kSerial) \
    X(1, kNtLoad | kNtStore | kDepth2 | kEarly | kFuse | kSerial) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kFuse | kSerial | (5 << kOccShift)) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kFuse | (5 << kOccShift)) \
    X(2, kNtLoad | kNtStore | kDepth2 | kFuse | (5 << kOccShift)) \
    X(1, kNtLoad | kNtStore | kDepth2 | kSegs | kEarly) \
    X(1, kNtLoad | kNtStore | kDepth2 | kSegs | kFuse | kEarly) \
    X(1, kDiagXor | kNtLoad | kNtStore | kDepth2) \
    X(2, kDiagXor | kNtLoad | kNtStore | kDepth2) \
    X(1, kDiagXor | kNtLoad | kNtStore | kDepth2 | kFuse) \
    X(2, kDiagXor | kNtLoad | kNtStore | kDepth2 | kFuse) \
    X(1, kDiagXor | kNtLoad | kNtStore | kDepth2 | kSegs) \
    X(1, kNtLoad | kNtStore | kGlds) \
    X(1, kNtLoad | kNtStore | kGlds | kDepth5) \
    X(1, kNtLoad | kNtStore | kGlds | kDepth9) \
    X(2, kNtLoad | kNtStore | kGlds) \
    X(2, kNtLoad | kNtStore | kGlds | kDepth5) \
    X(1, kNtLoad | kNtStore | kGlds | kFuse) \
    X(1, kNtLoad | kNtStore | kGlds | kDepth5 | kFuse) \
    X(1, kNtLoad | kNtStore | kGlds | kDepth9 | kFuse) \
    X(2, kNtLoad | kNtStore | kGlds | kFuse) \
    X(2, kNtLoad | kNtStore | kGlds | kDepth5 | kFuse) \
    X(1, kNtLoad | kNtStore | kGlds | kSegs) \
    X(1, kNtLoad | kNtStore | kGlds | kDepth5 | kSegs) \
    X(1, kNtLoad | kNtStore | kGlds | kSegs | kFuse) \
    X(1, kNtLoad | kNtStore | kGlds | kDepth5 | kSegs | kFuse) \
    X(2, kNtLoad | kNtStore | kDepth2 | kSPre | kFuse) \
    X(2, kNtLoad | kNtStore | kDepth2 | kSPre | kFuse | kSerial) \
    X(1, kNtLoad | kNtStore | kDepth2 | kSPre | kFuse) \
    X(1, kNtLoad | kNtStore | kDepth2 | kSPre | kFuse | kSerial) \
    X(1, kNtLoad | kDepth2 | kFuse) \
    X(1, kNtLoad | kDepth2 | kSegs) \
    X(1, kNtLoad | kDepth2 | kSegs | kFuse) \
    X(1, kNtLoad | kDepth2 | kPeel) \
    X(1, kNtLoad | kDepth2 | kFuse | kPeel) \
    X(1, kNtLoad | kDepth2 | kSegs | kPeel) \
    X(1, kNtLoad | kDepth2 | kSegs | kFuse | kPeel) \
    X(2, kNtLoad | kDepth2) \
    X(2, kNtLoad | kDepth2 | kSegs) \
    X(1, kNtLoad | kNtStore | kDepth2 | kRealign) \
    X(2, kNtLoad | kNtStore | kDepth2 | kRealign) \
    X(1, kNtLoad | kNtStore | kDepth2 | kFuse | kRealign) \
    X(2, kNtLoad | kNtStore | kDepth2 | kFuse | kRealign) \
    X(2, kNtLoad | kNtStore | kDepth2 | kFuse | kRealign | kSerial) \
    X(1, kNtLoad | kNtStore | kDepth2 | kSegs | kRealign) \
    X(1, kNtLoad | kNtStore | kDepth2 | kSegs | kFuse | kRealign) \
    X(2, kNtLoad | kNtStore | kDepth2 | kSegs | kFuse | kRealign) \
    X(2, kNtLoad | kNtStore | kDepth2 | kRealign | kSerial) \
    X(2, kNtLoad | kNtStore | kDepth2 | kSegs | kRealign) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kSegs | kRealign) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kSegs | kFuse | kRealign) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kRealign) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kFuse | kRealign) \
    X(2, kNtStore | kDepth2 | kEarly | kSerial | kFuse) \
    X(2, kNtLoad | kDepth2 | kEarly | kSerial | kFuse) \
    X(2, kDepth2 | kEarly | kSerial | kFuse) \
    X(1, kNtStore | kDepth2 | kSegs | kFuse) \
    X(1, kDepth2 | kSegs | kFuse) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kFuse | kSerial | kPeel) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kSerial | kPeel) \
    X(2, kNtLoad | kNtStore | kDepth2 | kFuse | kSerial | kWaveRun) \
    X(2, kNtLoad | kNtStore | kDepth2 | kSerial | kWaveRun) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kFuse | kSerial | kWaveRun | kStAlign) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kSerial | kWaveRun | kStAlign) \
    X(2, kNtLoad | kNtStore | kDepth2 | kFuse | kWaveRun | kStAlign) \
    X(2, kNtLoad | kNtStore | kDepth2 | kWaveRun | kStAlign) \
    X(1, kNtLoad | kNtStore | kDepth2 | kEarly | kFuse | kStAlign) \
    X(1, kNtLoad | kNtStore | kDepth2 | kEarly | kStAlign) \
    X(1, kNtLoad | kNtStore | kDepth2 | kSegs | kFuse | kPeel | kStAlign) \
    X(1, kNtLoad | kNtStore | kDepth2 | kSegs | kPeel | kStAlign) \
    X(1, kNtLoad | kNtStore | kDepth2 | kFuse | kPeel | kStAlign) \
    X(1, kNtLoad | kNtStore | kDepth2 | kPeel | kStAlign) \
    X(2, kNtLoad | kNtStore | kDepth2 | kSegs | kFuse | kPeel | kWaveRun | kStAlign) \
    X(2, kNtLoad | kNtStore | kDepth2 | kSegs | kPeel | kWaveRun | kStAlign) \
    X(2, kNtLoad | kNtStore | kDepth2 | kFuse | kPeel | kWaveRun | kStAlign) \
    X(2, kNtLoad | kNtStore | kDepth2 | kPeel | kWaveRun | kStAlign) \
    X(1, kNtLoad | kNtStore | kDepth2 | kSegs) \
    X(1, kNtLoad | kNtStore | kDepth2 | kSegs | kFuse) \
    X(2, kNtLoad | kNtStore | kDepth2 | kSegs) \
    X(2, kNtLoad | kNtStore | kDepth2 | kSegs | kFuse) \
    X(1, kNtLoad | kSc1Store | kDepth2) \
    X(2, kNtLoad | kSc1Store | kDepth2) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kFuse) \
    X(2, kNtLoad | kSc1Store | kDepth2 | kFuse) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kSegs) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kSegs | kFuse) \
    X(2, kNtLoad | kSc1Store | kDepth2 | kSegs) \
    X(2, kNtLoad | kSc1Store | kDepth2 | kSegs | kFuse) \
    X(2, kNtLoad | kNtStore | kDepth2) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly) \
    X(2, kNtLoad | kNtStore | kDepth2 | kFuse) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kFuse) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kSerial) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kFuse | kSerial) \
    X(2, kNtLoad | kNtStore | kDepth2 | kSegs | kPeel) \
    X(2, kNtLoad | kNtStore | kDepth2 | kSegs | kFuse | kPeel) \
    X(2, kNtLoad | kNtStore | kDepth2 | kPeel) \
    X(2, kNtLoad | kNtStore | kDepth2 | kFuse | kPeel) \
    X(2, kNtLoad | kNtStore | kDepth2 | kPtrs) \
    X(2, kNtLoad | kNtStore | kDepth2 | kPtrs | kPeel) \
    X(2, kNtLoad | kSc1Store | kDepth2 | kPeel) \
    X(2, kNtLoad | kSc1Store | kDepth2 | kFuse | kPeel) \
    X(2, kNtLoad | kSc1Store | kDepth2 | kSegs | kPeel) \
    X(2, kNtLoad | kSc1Store | kDepth2 | kSegs | kFuse | kPeel) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kFuse | kSerial | kWaveRun | kXcd) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kSerial | kWaveRun | kXcd) \
    X(1, kNtLoad | kNtStore | kDepth2 | kSegs | kFuse | kPeel | kXcd) \
    X(1, kNtLoad | kNtStore | kDepth2 | kSegs | kPeel | kXcd) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kSegs | kFuse | kPeel | kXcd) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kSegs | kPeel | kXcd) \
    X(1, kNtLoad | kNtStore | kDepth2 | kEarly | kFuse | kXcd) \
    X(1, kNtLoad | kNtStore | kDepth2 | kEarly | kXcd) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kPtrs | kPeel) \
    X(1, kNtLoad | kNtStore | kDepth2 | kFuse | kPtrs | kPeel) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kFuse | kPtrs | kPeel) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kEarly) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kEarly | kFuse) \
    X(2, kNtLoad | kSc1Store | kDepth2 | kEarly | kSerial | kWaveRun) \
    X(2, kNtLoad | kSc1Store | kDepth2 | kEarly | kFuse | kSerial | kWaveRun) \
    X(4, kNtLoad | kNtStore | kDepth2 | kEarly | kSerial | kWaveRun) \
    X(4, kNtLoad | kNtStore | kDepth2 | kEarly | kFuse | kSerial | kWaveRun) \
    X(4, kNtLoad | kNtStore | kDepth2 | kSegs | kFuse | kPeel | kWaveRun) \
    X(4, kNtLoad | kNtStore | kDepth2 | kSegs | kPeel | kWaveRun) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kSPre | kSegs) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kSPre | kSegs | kFuse) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kFuse | kSerial | kPeel | kWaveRun) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kSerial | kPeel | kWaveRun) \
    X(1, kNtLoad | kNtStore | kDepth2 | kEarly | kPtrs | kPair) \
    X(1, kNtLoad | kNtStore | kDepth2 | kEarly | kFuse | kPtrs | kPair) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kEarly | kPtrs | kPeel | kPair) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kEarly | kFuse | kPtrs | kPeel | kPair) \
    X(2, kNtLoad | kNtStore | kDepth2 | kPtrs | kWaveRun | kPair) \
    X(2, kNtLoad | kNtStore | kDepth2 | kFuse | kPtrs | kWaveRun | kPair)

// The round-3 product list (every row count), so the tools build can still
// A/B the r03 policy against the current one.
#define SHMR_VARIANTS_R03(X) \
    X(1, kNtLoad | kNtStore | kDepth2) \
    X(2, kNtLoad | kNtStore | kDepth2 | kWaveRun) \
    X(1, kNtStore | kDepth2) \
    X(2, kNtStore | kDepth2) \
    X(1, kNtLoad | kNtStore | kDepth2 | kEarly) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kWaveRun) \
    X(1, kNtLoad | kNtStore | kDepth2 | kFuse) \
    X(2, kNtLoad | kNtStore | kDepth2 | kFuse | kWaveRun) \
    X(1, kNtLoad | kNtStore | kDepth2 | kEarly | kFuse) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kFuse | kWaveRun) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kSerial | kWaveRun) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kFuse | kSerial | kWaveRun) \
    X(1, kNtLoad | kNtStore | kDepth2 | kSegs | kPeel) \
    X(1, kNtLoad | kNtStore | kDepth2 | kSegs | kFuse | kPeel) \
    X(2, kNtLoad | kNtStore | kDepth2 | kSegs | kPeel | kWaveRun) \
    X(2, kNtLoad | kNtStore | kDepth2 | kSegs | kFuse | kPeel | kWaveRun) \
    X(1, kNtLoad | kNtStore | kDepth2 | kPeel) \
    X(2, kNtLoad | kNtStore | kDepth2 | kPeel | kWaveRun) \
    X(1, kNtLoad | kNtStore | kDepth2 | kFuse | kPeel) \
    X(2, kNtLoad | kNtStore | kDepth2 | kFuse | kPeel | kWaveRun) \
    X(1, kNtStore | kDepth2 | kPtrs) \
    X(2, kNtStore | kDepth2 | kPtrs) \
    X(1, kNtStore | kDepth2 | kPtrs | kFuse) \
    X(2, kNtStore | kDepth2 | kPtrs | kFuse) \
    X(1, kNtStore | kDepth2 | kPtrs | kSegs) \
    X(1, kNtStore | kDepth2 | kPtrs | kSegs | kFuse) \
    X(2, kNtStore | kDepth2 | kPtrs | kSegs) \
    X(2, kNtStore | kDepth2 | kPtrs | kSegs | kFuse) \
    X(1, kNtLoad | kNtStore | kDepth2 | kPtrs) \
    X(2, kNtLoad | kNtStore | kDepth2 | kPtrs | kWaveRun) \
    X(1, kNtLoad | kNtStore | kDepth2 | kPtrs | kPeel) \
    X(1, kNtLoad | kNtStore | kDepth2 | kFuse | kPtrs) \
    X(2, kNtLoad | kNtStore | kDepth2 | kFuse | kPtrs | kWaveRun) \
    X(1, kNtLoad | kNtStore | kDepth2 | kEarly | kPtrs) \
    X(1, kNtLoad | kNtStore | kDepth2 | kEarly | kFuse | kPtrs) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kSerial | kWaveRun | kPtrs) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kFuse | kSerial | kWaveRun | kPtrs) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kEarly | kPtrs | kPeel) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kEarly | kFuse | kPtrs | kPeel) \
    X(2, kNtLoad | kSc1Store | kDepth2 | kEarly | kPtrs | kPeel | kWaveRun) \
    X(2, kNtLoad | kSc1Store | kDepth2 | kEarly | kFuse | kPtrs | kPeel | kWaveRun) \
    X(1, kNtLoad | kNtStore | kDepth2 | kEarly | kPtrs | kPeel) \
    X(1, kNtLoad | kNtStore | kDepth2 | kEarly | kFuse | kPtrs | kPeel) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kPtrs | kPeel | kWaveRun) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kFuse | kPtrs | kPeel | kWaveRun) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kEarly | kSegs | kPtrs | kPeel) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kEarly | kSegs | kFuse | kPtrs | kPeel) \
    X(2, kNtLoad | kSc1Store | kDepth2 | kEarly | kSegs | kPtrs | kPeel | kWaveRun) \
    X(2, kNtLoad | kSc1Store | kDepth2 | kEarly | kSegs | kFuse | kPtrs | kPeel | kWaveRun) \
    X(1, kNtLoad | kNtStore | kDepth2 | kEarly | kSegs | kPtrs | kPeel) \
    X(1, kNtLoad | kNtStore | kDepth2 | kEarly | kSegs | kFuse | kPtrs | kPeel) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kSegs | kPtrs | kPeel | kWaveRun) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kSegs | kFuse | kPtrs | kPeel | kWaveRun) \
    X(2, kNtLoad | kNtStore | kDepth2 | kPtrs | kPeel | kWaveRun) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kPeel) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kEarly | kPeel) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kEarly | kFuse | kPeel) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kEarly | kSegs | kPeel) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kEarly | kSegs | kFuse | kPeel) \
    X(1, kNtLoad | kNtStore | kDepth2 | kEarly | kPeel) \
    X(1, kNtLoad | kNtStore | kDepth2 | kEarly | kFuse | kPeel) \
    X(1, kNtLoad | kNtStore | kDepth2 | kEarly | kSegs | kPeel) \
    X(1, kNtLoad | kNtStore | kDepth2 | kEarly | kSegs | kFuse | kPeel) \
    X(2, kNtLoad | kSc1Store | kDepth2 | kEarly | kPeel | kWaveRun) \
    X(2, kNtLoad | kSc1Store | kDepth2 | kEarly | kFuse | kPeel | kWaveRun) \
    X(2, kNtLoad | kSc1Store | kDepth2 | kEarly | kSegs | kPeel | kWaveRun) \
    X(2, kNtLoad | kSc1Store | kDepth2 | kEarly | kSegs | kFuse | kPeel | kWaveRun) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kPeel | kWaveRun) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kFuse | kPeel | kWaveRun) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kSegs | kPeel | kWaveRun) \
    X(2, kNtLoad | kNtStore | kDepth2 | kEarly | kSegs | kFuse | kPeel | kWaveRun) \
    X(2, kNtLoad | kSc1Store | kDepth2 | kPeel | kWaveRun) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kFuse | kPeel) \
    X(2, kNtLoad | kSc1Store | kDepth2 | kFuse | kPeel | kWaveRun) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kSegs | kPeel) \
    X(1, kNtLoad | kSc1Store | kDepth2 | kSegs | kFuse | kPeel) \
    X(2, kNtLoad | kSc1Store | kDepth2 | kSegs | kPeel | kWaveRun) \
    X(2, kNtLoad | kSc1Store | kDepth2 | kSegs | kFuse | kPeel | kWaveRun)

template <int R>
hipError_t dispatch_tools(const ApplyArgs& a, const Variant& v, int grid_cap, hipStream_t s) {
    const int f = variant_flags(v);
#define SHMR_F(UU, FL) \
    if (v.u == UU && f == (FL)) return launch_one<R, UU, 0, FL>(a, v, grid_cap, s);
    SHMR_VARIANTS_TOOLS(SHMR_F)
    SHMR_VARIANTS_R03(SHMR_F)
#undef SHMR_F
    return hipErrorInvalidValue;
}

}  // namespace

hipError_t launch_full_tools(const ApplyArgs& a, unsigned rows, const Variant& v, int grid_cap, hipStream_t stream) {
    switch (rows) {
        case 1: return dispatch_tools<1>(a, v, grid_cap, stream);
        case 2: return dispatch_tools<2>(a, v, grid_cap, stream);
        case 3: return dispatch_tools<3>(a, v, grid_cap, stream);
        case 4: return dispatch_tools<4>(a, v, grid_cap, stream);
        default: return hipErrorInvalidValue;
    }
}

bool variant_compiled_tools(const Variant& v) {
    const int f = variant_flags(v);
#define SHMR_F(UU, FL) \
    if (v.u == UU && f == (FL)) return true;
    SHMR_VARIANTS_TOOLS(SHMR_F)
    SHMR_VARIANTS_R03(SHMR_F)
#undef SHMR_F
    return false;
}

}  // namespace kern
}  // namespace shmr
