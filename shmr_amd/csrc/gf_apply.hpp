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
    // are then 0): shard i of block b is at address shard_ptrs[b * total + i]
    // -- e.g. Block-Cache buffers in mapped (pinned) host memory, which the
    // kernel reads and writes across PCIe without a staging copy.  Only the
    // plain LDS-staged tile supports it (no early / spre).
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

// Compiled-in kernel variant for full tiles (see gf_apply.hip dispatch_full;
// measurement-only variants: gf_apply_tools.hip, tools build).
struct Variant {
    int u = 1;               // 16-byte chunks per lane per shard (1, 2, 4)
    bool nt_load = false;    // nontemporal loads
    bool nt_store = false;   // nontemporal stores
    bool occ8 = false;       // __launch_bounds__ for 8 waves / SIMD
    bool diag = false;       // diagnostics: XOR-only (wrong results)
    int threads = kThreads;  // lanes per workgroup (128, 256, 512)
    int depth = 3;           // register ring depth: shards of loads in flight + 1 (1, 2, 3, 5, 9)
    int wgs_per_cu = 0;      // > 0: cap resident workgroups per CU (LDS padding)
    int occ = 0;             // > 0: register budget for this many waves per SIMD (6, 7)
    bool early = false;      // first data loads before the plan's LDS staging completes
    bool spre = false;       // tables/offsets by scalar loads one shard ahead (no LDS)
    bool fuse_tail = false;  // partial last tiles inside the full-tile launch (ApplyArgs::lead_tails)
    bool ptrs = false;       // full-tile kernel that reads shard-pointer tables (set by launch_set)
    bool segs = false;       // full-tile kernel that takes segment launches (set by launch_set)
    bool glds = false;       // input ring in LDS filled by LDS-DMA (depth = slots; full tiles only)
    bool serial = false;     // GF math one dword at a time (fewer live registers, more waves)
    bool sc1_store = false;  // stores with the sc1 cache policy instead of nontemporal
    bool realign = false;    // misaligned shards: aligned loads realigned across lanes (DPP), unaligned stores
    bool peel = false;       // depth-2 ring with the tail peeled (no look-ahead load past the last shard)
    bool wave_run = false;   // U > 1 slots in wave-contiguous runs
    bool st_align = false;   // misaligned output rows: aligned stores realigned across lanes (tools)
    bool xcd = false;        // XCD-grouped tile order: neighbouring tiles on one XCD's L2 (tools)
};

// rows in [1, kMaxRowsPerLaunch].  mode 0: full tiles, every shard base
// (base + b*bpitch + idx*spitch) 16-byte aligned (variant v); mode 1: one
// partial tail tile per block (aligned, U = 1); mode 2: any alignment,
// byte-granular (U = 1); mode 3: full 4 KiB tiles at any alignment, vector
// loads and stores realigned in registers (U = 1).  The variant only affects
// mode 0.  Modes 0 and 1 also run on misaligned shards where the device's
// unaligned vector access was verified (probe_unaligned_vector).
// grid_cap: -1 one workgroup per tile; 0 balanced persistent grid sized by
// occupancy; > 0 persistent grid capped at grid_cap.
// Whether the full-tile kernel for variant v is compiled into the library.
bool variant_compiled(const Variant& v);

hipError_t launch_apply(const ApplyArgs& a, unsigned rows, const Variant& v, int mode, int grid_cap,
                        hipStream_t stream);

#ifdef SHMR_EC_TOOLS
// Full-tile measurement variants (gf_apply_tools.hip, tools build only):
// launch_apply / variant_compiled fall through to these for variants the
// product list does not carry.
hipError_t launch_full_tools(const ApplyArgs& a, unsigned rows, const Variant& v, int grid_cap, hipStream_t stream);
bool variant_compiled_tools(const Variant& v);
#endif

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
