// GF(2^8) matrix-apply kernels for gfx950 (MI355X / CDNA4): the product
// instantiations, their dispatch, and the unaligned-access probe.
//
//   out[r][col] = XOR_t  C[r][t] (x) in[t][col]        for every block of a batch
//
// Encode (reference: reed_solomon_erasure ReedSolomon::encode at
// src/vfs/block.rs:427) uses C = parity rows of the coding matrix; reconstruct
// (block.rs:560) uses the rows of the plan built in gf256.cpp.
//
// Design (device code in gf_tile.hpp):
//  * HBM-bound byte-field arithmetic, no MFMA.  Every input byte is read once,
//    every output byte written once: algorithmic traffic (k + R) * len per block.
//  * A tile = 256 lanes x U x 16 B of columns of one block, all k input shards
//    and R output rows.  Each lane owns U 16-byte chunks per shard
//    (global_load_dwordx4: 1 KiB per wave instruction, fully coalesced), one
//    workgroup per tile (~10^5 short workgroups; measured 7-10 % faster than a
//    persistent grid-stride loop).
//  * Multiply by constant c via three 8-byte tables T0/T1/T2 (bits 0-2, 3-5,
//    6-7); v_perm_b32 looks up four byte lanes of a dword at once:
//    per input dword 5 VALU ops of selector extraction shared by all rows, then
//    3 v_perm + 2 v_bitop3 (three-input XOR) per row.
//  * Tables are staged into LDS once per workgroup and read back with
//    wave-uniform (broadcast) ds_read_b128; shards rotate through a depth-2
//    register ring (one shard of loads in flight while the previous one is
//    multiplied).
//
// The measurement-only variants (LDS-DMA ring, scalar-loaded tables, ring
// depths 1/3/5/9, 128/512 lanes, occupancy targets, the XOR-only diagnostic)
// live in gf_apply_tools.hip, linked into the tools build only.
#include <hip/hip_runtime.h>

#include <array>
#include <atomic>
#include <cstring>
#include <utility>

#include "gf_tile.hpp"

namespace shmr {
namespace kern {

namespace {

// ---- the product instantiation list, derived from the launch policy --------
// Every valid LaunchShape (gf_apply.hpp) is mapped through policy_variant at
// compile time; the distinct (rows, U, flags) keys are the full-tile (MODE 0)
// kernels of the product library.  A kernel nothing can launch is therefore
// never compiled, and a shape's kernel always exists.  The tools build adds
// its measurement variants (gf_apply_tools.hip).
struct Key {
    int rows = 0, u = 0, flags = 0;
};
constexpr int kMaxKeys = 256;
struct KeyList {
    Key k[kMaxKeys] = {};
    int n = 0;
};

constexpr LaunchShape shape_at(unsigned i) {
    LaunchShape s;
    s.decode = i & 1;
    s.small_k = (i >> 1) & 1;
    s.host_mapped = (i >> 2) & 1;
    s.ptrs = (i >> 3) & 1;
    s.segs = (i >> 4) & 1;
    s.compact = (i >> 5) & 1;
    s.sc1_ok = (i >> 6) & 1;
    s.fused = (i >> 7) & 1;
    s.rows = 1 + (i >> 8);
    return s;
}
constexpr unsigned kShapes = 256 * kMaxRowsPerLaunch;

constexpr KeyList product_keys() {
    KeyList L;
    for (unsigned i = 0; i < kShapes; ++i) {
        const LaunchShape s = shape_at(i);
        if (!shape_valid(s)) continue;
        const Variant v = policy_variant(s);
        const Key key{int(s.rows), v.u, variant_flags(v)};
        bool seen = false;
        for (int j = 0; j < L.n && !seen; ++j)
            seen = L.k[j].rows == key.rows && L.k[j].u == key.u && L.k[j].flags == key.flags;
        if (!seen) L.k[L.n++] = key;   // (overflow: not a constant expression -> compile error)
    }
    return L;
}
constexpr KeyList kProduct = product_keys();
constexpr int kNumProduct = kProduct.n;
static_assert(kNumProduct > 0 && kNumProduct < kMaxKeys, "product kernel list");

using LaunchFn = hipError_t (*)(const ApplyArgs&, const Variant&, int, hipStream_t);
template <size_t... I>
constexpr std::array<LaunchFn, sizeof...(I)> product_fns(std::index_sequence<I...>) {
    return {{&launch_one<kProduct.k[I].rows, kProduct.k[I].u, 0, kProduct.k[I].flags>...}};
}
constexpr std::array<LaunchFn, kNumProduct> kProductFns = product_fns(std::make_index_sequence<kNumProduct>{});

// Launches served per kernel: [product list][MODE 1, 2, 3 x rows]
std::atomic<uint64_t> g_launches[kNumProduct + 3 * kMaxRowsPerLaunch];

int product_index(const Variant& v, unsigned rows) {
    const int f = variant_flags(v);
    for (int i = 0; i < kNumProduct; ++i)
        if (kProduct.k[i].rows == int(rows) && kProduct.k[i].u == v.u && kProduct.k[i].flags == f) return i;
    return -1;
}

hipError_t dispatch_full(const ApplyArgs& a, unsigned rows, const Variant& v, int grid_cap, hipStream_t s) {
    const int i = product_index(v, rows);
    if (i >= 0) {
        g_launches[i].fetch_add(1, std::memory_order_relaxed);
        return kProductFns[size_t(i)](a, v, grid_cap, s);
    }
#ifdef SHMR_EC_TOOLS
    return launch_full_tools(a, rows, v, grid_cap, s);
#else
    return hipErrorInvalidValue;
#endif
}

// MODE 1 (partial tail tiles), 2 (byte-granular) and 3 (realigning, for a
// device without the unaligned access mode): one kernel per row count.
template <int R>
hipError_t dispatch_mode(const ApplyArgs& a, const Variant& v, int mode, int grid_cap, hipStream_t s) {
    g_launches[kNumProduct + (mode - 1) * kMaxRowsPerLaunch + (R - 1)].fetch_add(1, std::memory_order_relaxed);
    switch (mode) {
        case 1: return launch_one<R, 1, 1, 0>(a, v, grid_cap, s);
        case 3: return launch_one<R, 1, 3, kNtLoad | kNtStore | kDepth2>(a, v, grid_cap, s);
        default: return launch_one<R, 1, 2, 0>(a, v, grid_cap, s);
    }
}
constexpr int kModeFlags[3] = {0, 0, kNtLoad | kNtStore | kDepth2};

}  // namespace

bool variant_compiled(const Variant& v, unsigned rows) {
    if (product_index(v, rows) >= 0) return true;
#ifdef SHMR_EC_TOOLS
    return variant_compiled_tools(v);
#else
    return false;
#endif
}

size_t kernel_inventory(KernelInfo* out, size_t cap) {
    const size_t n = size_t(kNumProduct) + 3 * kMaxRowsPerLaunch;
    for (size_t i = 0; i < n && out && i < cap; ++i) {
        KernelInfo& k = out[i];
        if (i < size_t(kNumProduct)) {
            k = KernelInfo{uint32_t(kProduct.k[i].rows), uint32_t(kProduct.k[i].u), 0u, uint32_t(kProduct.k[i].flags), 0};
        } else {
            const size_t j = i - size_t(kNumProduct);
            k = KernelInfo{uint32_t(j % kMaxRowsPerLaunch + 1), 1u, uint32_t(j / kMaxRowsPerLaunch + 1),
                           uint32_t(kModeFlags[j / kMaxRowsPerLaunch]), 0};
        }
        k.launches = g_launches[i].load(std::memory_order_relaxed);
    }
    return n;
}

namespace {
// 16-byte vector loads and stores at addresses off 16-byte alignment, with the
// plain and the nontemporal instructions the kernels use (see
// probe_unaligned_vector).  Lane-dependent addresses keep them vector memory
// instructions (a wave-uniform address from a read-only pointer may become a
// scalar load, which ignores the low address bits).
constexpr int kProbeLanes = 64, kProbeBytes = kProbeLanes * 16 + 64;
__global__ void unaligned_probe_kernel(const uint8_t* in, uint8_t* out) {
    const uint32_t l = threadIdx.x;
    store16<0>(out + 5 + 16 * l, load16<0>(in + 3 + 16 * l));
    store16<kNtStore>(out + kProbeBytes + 7 + 16 * l, load16<kNtLoad>(in + kProbeBytes + 9 + 16 * l));
}
}  // namespace

hipError_t probe_unaligned_vector(bool* ok, uint8_t* d_scratch, uint8_t* h_scratch, hipStream_t stream) {
    *ok = false;
    constexpr int N = 2 * kProbeBytes;
    static_assert(2 * N <= kProbeScratchBytes, "probe scratch");
    uint8_t* h_in = h_scratch;
    uint8_t* h_out = h_scratch + N;
    uint8_t want[N];
    for (int i = 0; i < N; ++i) h_in[i] = uint8_t(i * 37 + 11), want[i] = 0xA5;
    for (int i = 0; i < kProbeLanes * 16; ++i) {
        want[5 + i] = h_in[3 + i];
        want[kProbeBytes + 7 + i] = h_in[kProbeBytes + 9 + i];
    }
    uint8_t* d_in = d_scratch;
    uint8_t* d_out = d_scratch + N;
    hipError_t e = hipMemcpyAsync(d_in, h_in, N, hipMemcpyHostToDevice, stream);
    if (e == hipSuccess) e = hipMemsetAsync(d_out, 0xA5, N, stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(unaligned_probe_kernel, dim3(1), dim3(kProbeLanes), 0, stream, d_in, d_out);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(h_out, d_out, N, hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e == hipSuccess) *ok = std::memcmp(h_out, want, N) == 0;
    return e;
}

namespace {
// One lane stores: a vector memory (global) atomic store at system scope, so
// the host sees it only after every byte the batch's kernels wrote before it.
__global__ void queue_mark_kernel(uint64_t* word, uint64_t seq) {
    if (threadIdx.x == 0) __hip_atomic_store(word + threadIdx.x, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
}  // namespace

hipError_t launch_mark(uint64_t* word, uint64_t seq, hipStream_t stream) {
    hipLaunchKernelGGL(queue_mark_kernel, dim3(1), dim3(64), 0, stream, word, seq);
    return hipGetLastError();
}

hipError_t launch_apply(const ApplyArgs& a, unsigned rows, const Variant& v, int mode, int grid_cap,
                        hipStream_t stream) {
    if (rows < 1 || rows > kMaxRowsPerLaunch) return hipErrorInvalidValue;
    if (mode == 0) return dispatch_full(a, rows, v, grid_cap, stream);
    if (mode < 1 || mode > 3) return hipErrorInvalidValue;
    switch (rows) {
        case 1: return dispatch_mode<1>(a, v, mode, grid_cap, stream);
        case 2: return dispatch_mode<2>(a, v, mode, grid_cap, stream);
        case 3: return dispatch_mode<3>(a, v, mode, grid_cap, stream);
        default: return dispatch_mode<4>(a, v, mode, grid_cap, stream);
    }
}

}  // namespace kern
}  // namespace shmr
