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

#include <cstring>

#include "gf_tile.hpp"

namespace shmr {
namespace kern {

namespace {

// The variants the tuning policy (ec_core.cpp variant_policy / launch_variant)
// can select: depth-2 ring, nontemporal stores (sc1 for compact rebuilt-shard
// outputs), nontemporal loads unless the shards are mapped host memory, U = 1
// or 2, with the early prologue, fused tails, shard-pointer tables and segment
// launches as launch forms.  An unsupported combination returns
// hipErrorInvalidValue (the C ABI reports SHMR_EC_INVALID_ARGUMENT).
#define SHMR_VARIANTS_PRODUCT(X) \
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
hipError_t dispatch_full(const ApplyArgs& a, const Variant& v, int grid_cap, hipStream_t s) {
    const int f = variant_flags(v);
#define SHMR_F(UU, FL) \
    if (v.u == UU && f == (FL)) return launch_one<R, UU, 0, FL>(a, v, grid_cap, s);
    SHMR_VARIANTS_PRODUCT(SHMR_F)
#undef SHMR_F
#ifdef SHMR_EC_TOOLS
    return launch_full_tools(a, R, v, grid_cap, s);
#else
    return hipErrorInvalidValue;
#endif
}

template <int R>
hipError_t dispatch(const ApplyArgs& a, const Variant& v, int mode, int grid_cap, hipStream_t s) {
    switch (mode) {
        case 0: return dispatch_full<R>(a, v, grid_cap, s);
        case 1: return launch_one<R, 1, 1, 0>(a, v, grid_cap, s);
        case 3: return launch_one<R, 1, 3, kNtLoad | kNtStore | kDepth2>(a, v, grid_cap, s);
        default: return launch_one<R, 1, 2, 0>(a, v, grid_cap, s);
    }
}

}  // namespace

bool variant_compiled(const Variant& v) {
    const int f = variant_flags(v);
#define SHMR_F(UU, FL) \
    if (v.u == UU && f == (FL)) return true;
    SHMR_VARIANTS_PRODUCT(SHMR_F)
#undef SHMR_F
#ifdef SHMR_EC_TOOLS
    return variant_compiled_tools(v);
#else
    return false;
#endif
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

hipError_t launch_apply(const ApplyArgs& a, unsigned rows, const Variant& v, int mode, int grid_cap,
                        hipStream_t stream) {
    switch (rows) {
        case 1: return dispatch<1>(a, v, mode, grid_cap, stream);
        case 2: return dispatch<2>(a, v, mode, grid_cap, stream);
        case 3: return dispatch<3>(a, v, mode, grid_cap, stream);
        case 4: return dispatch<4>(a, v, mode, grid_cap, stream);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace kern
}  // namespace shmr
