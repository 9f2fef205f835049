// Launch interface of the gfx950 GF(2^8) matrix-apply kernel (gf_apply.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace shmr {
namespace kern {

constexpr int kThreads = 256;                          // lanes per workgroup (4 waves)
// A tile = kThreads * 16 * U bytes of columns of one block; U (16-byte chunks
// per lane per shard) is a launch parameter in {1, 2, 4}.
inline uint64_t tile_bytes(int u, int threads = kThreads) { return uint64_t(threads) * 16 * uint64_t(u); }
constexpr unsigned kMaxRowsPerLaunch = 4;

// Multi-plan launches described in the kernel arguments (no table upload):
// launch blocks j in [start, start + count) of a segment are blocks
// first + (j - start) * stride, all using `plan` (a device plan image).
#ifndef SHMR_MAX_SEGS
#define SHMR_MAX_SEGS 32
#endif
constexpr unsigned kMaxSegs = SHMR_MAX_SEGS;
struct Seg {
    uint32_t start;
    uint32_t first;
    uint32_t stride;
    uint32_t pad_;
    const uint8_t* plan;
};

// Shard t of block b lives at in_base + b * in_bpitch + in_idx[t] * in_spitch,
// output r of block b at out_base + b * out_bpitch + (out_idx[row0 + r] - out_bias) * out_spitch.
// Blocks of a launch: blk_list[j] if blk_list, else blk_first + j * blk_stride.
struct ApplyArgs {
    const uint8_t* in_base;
    uint8_t* out_base;
    uint64_t in_bpitch, in_spitch;
    uint64_t out_bpitch, out_spitch;
    const uint32_t* blk_list;
    uint64_t blk_first, blk_stride;
    uint64_t nblk;
    uint64_t len;            // shard length in bytes
    uint64_t col_base;       // column of tile 0 (tail launches start at the last partial tile)
    uint64_t ntiles;         // nblk * tiles_per_block
    uint32_t tiles_per_block;
    uint32_t k;              // inputs per block
    uint32_t m;              // rows in the plan image
    uint32_t row0;           // first plan row handled by this launch
    uint32_t out_bias;       // output r at (out_idx[row0 + r] - out_bias) * out_spitch
    const uint8_t* plan;     // device plan image (gf256.hpp Plan::image), single-plan launches
    // Multi-plan launches (plan_table != nullptr): block j uses plan
    // plan_table[blk_plan[j]]; every plan of a launch has the same k and m.
    const uint8_t* const* plan_table;
    const uint16_t* blk_plan;
    uint32_t tab_off;        // byte offset of the PermTab array in the image
    uint32_t in_identity;    // every plan of the launch reads input t from shard t (in_idx[t] == t)
    // Shard-pointer launches (shard_ptrs != nullptr; in/out bases and pitches
    // are then 0): block b's row shard_ptrs[b * total ..] is in PLAN ORDER --
    // input t at [t], output row r (plan row) at [k + r] -- so no address
    // depends on a load of the plan's in_idx / out_idx (the host permutes the
    // caller's shard-index table: ec_core permute_ptr_rows).  E.g. per-shard
    // device buffers, or Block-Cache buffers in mapped (pinned) host memory,
    // which the kernel reads and writes across PCIe without a staging copy.
    const uint64_t* shard_ptrs;
    uint32_t total;
    // Fused tails (kernels compiled with the fused-tail flag): the first
    // lead_tails tiles of the grid are the partial last tiles of blocks
    // j = 0 .. lead_tails-1 (column col_base + tiles_per_block * tile bytes),
    // run bounds-checked; tile lead_tails + t is full tile t.  Leading, so the
    // latency-bound partial tiles start first and finish under the full ones.
    uint64_t lead_tails;
    // Segment launches (nseg > 0; plan / plan_table / blk_list unused): block
    // j of the launch is found in segs[0 .. nseg) (ascending start, segs[0].start = 0).
    uint32_t nseg;
    Seg segs[kMaxSegs];
};

// Kernel variant flags (template parameter F of gf_apply_kernel).  The values
// are part of the kernels' mangled names: never renumber.
constexpr int kNtLoad = 1;       // nontemporal loads
constexpr int kNtStore = 2;      // nontemporal stores
constexpr int kOcc8 = 8;         // tools: ask for 8 waves / SIMD (<= 64 VGPRs)
constexpr int kDiagXor = 16;     // tools: XOR without GF multiply (wrong results)
constexpr int kTh128 = 32;       // tools: 128-lane workgroups (default 256)
constexpr int kTh512 = 64;       // tools: 512-lane workgroups
constexpr int kDepth5 = 128;     // tools: 4 shards of loads in flight (default 2)
constexpr int kDepth9 = 256;     // tools: 8 shards of loads in flight
constexpr int kDepth2 = 512;     // 1 shard of loads in flight
constexpr int kDepth1 = 1024;    // tools: no look-ahead (load, wait, multiply)
constexpr int kEarly = 1 << 16;  // first data loads issued before the plan's LDS staging completes
constexpr int kSPre = 1 << 17;   // tools: tables + offsets by scalar loads one shard ahead, no LDS
constexpr int kFuse = 1 << 18;   // leading partial tiles (ApplyArgs::lead_tails) in a MODE 0 launch; a
                                 // separate instantiation: the bounds-checked path costs 4-7 VGPRs
// Launch forms a full-tile (MODE 0) kernel supports only when compiled with
// the flag, so the lean encode kernel carries none of their code (measured:
// the runtime checks alone cost the RS(8,3) encode 1.3 %).  The tail and
// byte-granular kernels (MODE 1, 2) always support both.
constexpr int kPtrs = 1 << 19;   // shard-pointer tables (ApplyArgs::shard_ptrs)
constexpr int kSegs = 1 << 20;   // segment launches (ApplyArgs::segs)
constexpr int kGlds = 1 << 21;   // tools: input ring in LDS filled by LDS-DMA
// GF math one dword at a time: a scheduling fence after each of a lane's four
// dwords keeps the scheduler from computing every perm of a 16-byte chunk
// before the first XOR (48 live temporaries at R = 4), trading ILP inside a
// wave for registers (more waves per SIMD).
constexpr int kSerial = 1 << 22;
// Stores with the sc1 cache policy instead of nontemporal (compact rebuilt-
// shard outputs: a separate, densely written array; raw buffer stores)
constexpr int kSc1Store = 1 << 23;
constexpr int kRealign = 1 << 24;   // tools: misaligned shards by aligned loads realigned across lanes (DPP)
// The depth-2 ring with its tail peeled: no look-ahead load past the last
// shard (the plain ring re-reads shard k-1 there: one extra wave load per
// shard run, an L2 hit) and still no load behind a branch inside the loop
constexpr int kPeel = 1 << 25;
// U > 1 slots of a lane in wave-contiguous runs (chunk (w * U + u) * 64 +
// lane: each wave covers one contiguous U KiB run) instead of workgroup-
// strided slots (u * TH + tid)
constexpr int kWaveRun = 1 << 26;
constexpr int kStAlign = 1 << 27;   // tools: misaligned output rows stored aligned (DPP-shifted)
constexpr int kXcd = 1 << 28;       // tools: XCD-grouped tile order
// tools: two neighbouring tiles per workgroup (one workgroup per pair): the
// second tile of a block finds the block's pointer-table row in the scalar
// cache its first tile filled
constexpr int kPair = 1 << 29;
// Bits 12-15: occupancy target in waves per SIMD (0 = compiler's choice);
// the register allocator must then fit 512 / target VGPRs.
constexpr int kOccShift = 12;

// A full-tile kernel variant (MODE 0): the launch policy's choice (below), or
// a measurement variant of the tools build (knobs, ec_core.cpp).
struct Variant {
    int u = 1;               // 16-byte chunks per lane per shard (1, 2, 4)
    bool nt_load = false;    // nontemporal loads
    bool nt_store = false;   // nontemporal stores
    bool occ8 = false;       // __launch_bounds__ for 8 waves / SIMD
    bool diag = false;       // diagnostics: XOR-only (wrong results)
    int threads = kThreads;  // lanes per workgroup (128, 256, 512)
    int depth = 3;           // register ring depth: shards of loads in flight + 1 (1, 2, 3, 5, 9)
    int wgs_per_cu = 0;      // > 0: cap resident workgroups per CU (LDS padding; not a template flag)
    int occ = 0;             // > 0: register budget for this many waves per SIMD (6, 7)
    bool early = false;      // first data loads before the plan's LDS staging completes
    bool spre = false;       // tables/offsets by scalar loads one shard ahead (no LDS)
    bool fuse_tail = false;  // partial last tiles inside the full-tile launch (ApplyArgs::lead_tails)
    bool ptrs = false;       // full-tile kernel that reads shard-pointer tables
    bool segs = false;       // full-tile kernel that takes segment launches
    bool glds = false;       // input ring in LDS filled by LDS-DMA (depth = slots; full tiles only)
    bool serial = false;     // GF math one dword at a time (fewer live registers, more waves)
    bool sc1_store = false;  // stores with the sc1 cache policy instead of nontemporal
    bool realign = false;    // misaligned shards: aligned loads realigned across lanes (DPP), unaligned stores
    bool peel = false;       // depth-2 ring with the tail peeled (no look-ahead load past the last shard)
    bool wave_run = false;   // U > 1 slots in wave-contiguous runs
    bool st_align = false;   // misaligned output rows: aligned stores realigned across lanes (tools)
    bool xcd = false;        // XCD-grouped tile order: neighbouring tiles on one XCD's L2 (tools)
    bool pair = false;       // two neighbouring tiles per workgroup (tools)
};

// Template flags of a variant (its instantiation; wgs_per_cu is a launch
// parameter, not a flag).
constexpr int variant_flags(const Variant& v) {
    return (v.nt_load ? kNtLoad : 0) | (v.nt_store ? kNtStore : 0) | (v.occ8 ? kOcc8 : 0) |
           (v.diag ? kDiagXor : 0) | (v.threads == 128 ? kTh128 : 0) | (v.threads == 512 ? kTh512 : 0) |
           (v.depth == 5 ? kDepth5 : 0) | (v.depth == 9 ? kDepth9 : 0) | (v.depth == 2 ? kDepth2 : 0) |
           (v.depth == 1 ? kDepth1 : 0) | ((v.occ & 15) << kOccShift) | (v.early ? kEarly : 0) |
           (v.spre ? kSPre : 0) | (v.fuse_tail ? kFuse : 0) | (v.ptrs ? kPtrs : 0) | (v.segs ? kSegs : 0) |
           (v.glds ? kGlds : 0) | (v.serial ? kSerial : 0) | (v.sc1_store ? kSc1Store : 0) |
           (v.realign ? kRealign : 0) | (v.peel ? kPeel : 0) | (v.wave_run ? kWaveRun : 0) |
           (v.st_align ? kStAlign : 0) | (v.xcd ? kXcd : 0) | (v.pair ? kPair : 0);
}

// ---- launch policy -----------------------------------------------------------
// Everything a full-tile launch's kernel depends on.  ec_core.cpp launch_set
// fills it per launch group (<= 4 rows); gf_apply.hip derives the product
// library's instantiation list from policy_variant over every valid shape at
// compile time, so each compiled full-tile kernel is reachable and each
// reachable shape has its kernel (tests/test_gpu_kernel_sweep.py launches them
// all against the oracle).
struct LaunchShape {
    bool decode = false;       // reconstruct (else encode)
    bool small_k = false;      // k <= 8 data shards
    unsigned rows = 1;         // output rows of the launch, 1 .. kMaxRowsPerLaunch
    bool host_mapped = false;  // shards in mapped host memory (zero-copy across PCIe)
    bool ptrs = false;         // shards named by a pointer table (ApplyArgs::shard_ptrs)
    bool segs = false;         // segment launch (block runs, decode: their plans, in the kernel arguments)
    bool compact = false;      // decode into a compact output (shmr_ec_reconstruct_batch_dev_out)
    bool sc1_ok = false;       // outputs in device memory, 16-byte aligned, shorter than 2 GiB - 4 KiB
    bool fused = false;        // the shard length leaves a partial last tile after >= 1 full tile
};

// The shapes a call can produce: encodes take no compact output, and segment
// launches only over device pitch layouts (r06: the slot runs of a pool or of
// merged per-block calls, launch_slots); compact outputs are device pitch
// layouts; sc1 needs device memory.
constexpr bool shape_valid(const LaunchShape& s) {
    if (s.rows < 1 || s.rows > kMaxRowsPerLaunch) return false;
    if (!s.decode && (s.compact || (s.segs && (s.ptrs || s.host_mapped)))) return false;
    if (s.compact && (s.ptrs || s.host_mapped)) return false;
    if (s.sc1_ok && s.host_mapped) return false;
    return true;
}

// The measured policy (profiles/ and DESIGN.md §6; every adoption is an
// interleaved A/B in one process of >= 1 point of HBM peak, or repeated on
// three boxes).
constexpr Variant policy_variant(const LaunchShape& s) {
    Variant v;
    const bool dec = s.decode, hm = s.host_mapped;
    v.depth = 2;                        // one shard of loads in flight: beats depth 1/3/5/9 on every shape
    v.u = s.rows >= 4 ? 2 : 1;          // 8 KiB tiles for 4-row launches (encode and rebuild alike)
    v.nt_load = !hm;                    // temporal loads across PCIe: the look-ahead re-read hits L2
    v.nt_store = true;
    v.fuse_tail = s.fused;              // partial tiles at the head of the full-tile grid
    v.ptrs = s.ptrs;
    v.segs = s.segs;
    // early prologue: encodes with k <= 8 (short workgroups) and 4-row encodes
    // (with the per-dword math order, fewer live VGPRs at U = 2)
    v.early = !dec && (s.small_k || s.rows >= 4) && !hm;
    v.serial = !dec && s.rows >= 4 && !hm;
    v.peel = dec && !hm;                // reconstructs: no look-ahead load past the last input
    if (dec && s.rows == 1 && !hm) v.wgs_per_cu = 7;   // 1-row rebuilds in place: cap 7 WGs / CU
    // rebuilt shards into buffers of their own (compact output, device pointer
    // tables): sc1 stores, no residency cap; the early prologue pays for 4 rows
    if (dec && !hm && (s.compact || s.ptrs)) {
        v.sc1_store = true;
        v.nt_store = false;
        v.wgs_per_cu = 0;
        v.early = s.rows >= 4;
    }
    if (s.ptrs) {
        if (hm) {
            v.early = v.serial = false;   // the mapped policy: the plain LDS-staged tile
        } else {
            // first loads addressed from scalar loads of the block's table row:
            // RS(8,3) encode and every rebuild gain; RS(10,4) encode loses
            v.early = dec || s.small_k;
            if (!v.early) v.serial = false;
        }
    }
    v.wave_run = v.u > 1 && !hm;
    // sc1 stores are raw buffer stores: device memory, 16-byte aligned rows,
    // a 2 GiB resource per row
    if (v.sc1_store && !s.sc1_ok) {
        v.sc1_store = false;
        v.nt_store = true;
    }
    return v;
}

// rows in [1, kMaxRowsPerLaunch].  mode 0: full tiles, every shard base
// (base + b*bpitch + idx*spitch) 16-byte aligned (variant v); mode 1: one
// partial tail tile per block (aligned, U = 1); mode 2: any alignment,
// byte-granular (U = 1); mode 3: full 4 KiB tiles at any alignment, vector
// loads and stores realigned in registers (U = 1).  The variant only affects
// mode 0.  Modes 0 and 1 also run on misaligned shards where the device's
// unaligned vector access was verified (probe_unaligned_vector).
// grid_cap: -1 one workgroup per tile; 0 balanced persistent grid sized by
// occupancy; > 0 persistent grid capped at grid_cap.  hipErrorInvalidValue:
// the variant is not compiled into this library.
hipError_t launch_apply(const ApplyArgs& a, unsigned rows, const Variant& v, int mode, int grid_cap,
                        hipStream_t stream);

// Whether the full-tile kernel for variant v at `rows` rows is compiled into
// the library.
bool variant_compiled(const Variant& v, unsigned rows);

#ifdef SHMR_EC_TOOLS
// Full-tile measurement variants (gf_apply_tools.hip, tools build only):
// launch_apply / variant_compiled fall through to these for variants the
// product list does not carry.
hipError_t launch_full_tools(const ApplyArgs& a, unsigned rows, const Variant& v, int grid_cap, hipStream_t stream);
bool variant_compiled_tools(const Variant& v);
#endif

// Every gf_apply_kernel instantiation of the product list (gf_apply.hip) and
// the MODE 1-3 kernels, with the launches each has served in this process
// (shmr_ec_kernel_inventory).
struct KernelInfo {
    uint32_t rows, chunks, mode, flags;
    uint64_t launches;
};
size_t kernel_inventory(KernelInfo* out, size_t cap);

// The submission queue's completion mark (submit.cpp): a one-wave kernel on
// `stream` that stores `seq` to `word` -- pinned host memory, a system-scope
// release store -- once every earlier kernel of the stream has completed, so
// waiting callers poll a host word instead of the HIP runtime.
hipError_t launch_mark(uint64_t* word, uint64_t seq, hipStream_t stream);

// Runs a one-wave kernel on `stream` (current device) that loads and stores 16
// bytes at addresses off 16-byte alignment (plain and nontemporal), waits for
// it, and sets *ok if the bytes arrived where they belong: the memory
// system's unaligned access mode serves the vector kernels on misaligned
// shards (ec_core launch_set).  Scratch: kProbeScratchBytes of device memory
// and of pinned host memory.
constexpr int kProbeScratchBytes = 4 * (64 * 16 + 64);
hipError_t probe_unaligned_vector(bool* ok, uint8_t* d_scratch, uint8_t* h_scratch, hipStream_t stream);

}  // namespace kern
}  // namespace shmr
