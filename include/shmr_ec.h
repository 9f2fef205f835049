/*
 * shmr_ec.h -- C ABI of the MI355X-native Reed-Solomon erasure path for
 * shmr's StorageBlock (VirtualBlock) layer.
 *
 * Drop-in boundary: the reference binds reed_solomon_erasure::galois_8::
 * ReedSolomon (reference src/vfs/block.rs:10) and calls exactly three
 * entry points on the hot path:
 *
 *   ReedSolomon::new(data, parity)        src/vfs/block.rs:405, :531  -> shmr_ec_new
 *   r.encode(&mut Vec<Vec<u8>>)           src/vfs/block.rs:427        -> shmr_ec_encode
 *   r.reconstruct(&mut Vec<Option<..>>)   src/vfs/block.rs:560        -> shmr_ec_reconstruct
 *
 * plus the shard-size helper the callers use before every encode/decode
 * (calculate_shard_size, src/vfs/mod.rs:16-18) -> shmr_ec_shard_size.
 *
 * Everything runs on AMD Instinct MI355X (gfx950) through hand-written HIP
 * kernels.  There is no CPU compute fallback: without a usable GPU every
 * compute entry point returns SHMR_EC_NO_DEVICE / SHMR_EC_DEVICE_ERROR.
 *
 * Conventions: plain pointers and sizes, 0 on success, negative status on
 * failure, never aborts (an internal allocation failure returns
 * SHMR_EC_OUT_OF_MEMORY), never frees caller memory.  Thread-safe: contexts
 * may be shared across threads or created per call (the reference creates a
 * ReedSolomon per block from rayon workers, src/vfs/mod.rs:93-96).  Every
 * entry point runs under HIP's relaxed stream-capture mode (the calling
 * thread's mode is restored on return), so calls from other threads neither
 * fail nor break a graph capture in progress on some thread.
 */
#ifndef SHMR_EC_H
#define SHMR_EC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes.  -1..-13 are 1:1 with reed_solomon_erasure::Error (6.0.0),
 * which the reference wraps as ShmrError::EcError (src/config.rs:158,170-174). */
typedef enum shmr_ec_status {
    SHMR_EC_OK = 0,
    SHMR_EC_TOO_FEW_SHARDS = -1,
    SHMR_EC_TOO_MANY_SHARDS = -2,
    SHMR_EC_TOO_FEW_DATA_SHARDS = -3,
    SHMR_EC_TOO_MANY_DATA_SHARDS = -4,
    SHMR_EC_TOO_FEW_PARITY_SHARDS = -5,
    SHMR_EC_TOO_MANY_PARITY_SHARDS = -6,
    SHMR_EC_TOO_FEW_BUFFER_SHARDS = -7,
    SHMR_EC_TOO_MANY_BUFFER_SHARDS = -8,
    SHMR_EC_INCORRECT_SHARD_SIZE = -9,
    SHMR_EC_TOO_FEW_SHARDS_PRESENT = -10,
    SHMR_EC_EMPTY_SHARD = -11,
    SHMR_EC_INVALID_SHARD_FLAGS = -12,
    SHMR_EC_INVALID_INDEX = -13,
    /* library-level conditions (no crate equivalent) */
    SHMR_EC_INVALID_ARGUMENT = -100,
    SHMR_EC_NO_DEVICE = -101,
    SHMR_EC_DEVICE_ERROR = -102,
    SHMR_EC_OUT_OF_MEMORY = -103
} shmr_ec_status;

typedef struct shmr_ec shmr_ec_t;

/* Human-readable name of a status ("TooFewShardsPresent", ...). */
const char* shmr_ec_status_name(int status);

/* Library version string (names the flavour: "product" or "tools"). */
const char* shmr_ec_version(void);

/* Kernel build ID: hash of the kernel sources, device compile flags and
 * compiler version (12 hex digits).  Measurement records (PMC traffic) are
 * keyed by it, so they can be matched to the code that produced them. */
const char* shmr_ec_build_id(void);

/* 1 in the tools build (libshmr_ec_tools.so: measurement variants and kernel
 * knobs for tools/), 0 in the product library. */
int shmr_ec_is_tools_build(void);

/* ---- host logic (no GPU needed) ---------------------------------------- */

/* calculate_shard_size, src/vfs/mod.rs:16-18:
 * (length as f32 / data_shards as f32).ceil() as usize. 0 if data_shards==0. */
size_t shmr_ec_shard_size(uint64_t length, uint32_t data_shards);

/* ReedSolomon::new (src/vfs/block.rs:405,531).  Errors exactly as the crate:
 * data==0 -> TOO_FEW_DATA_SHARDS, parity==0 -> TOO_FEW_PARITY_SHARDS,
 * data+parity > 256 -> TOO_MANY_SHARDS.  Builds the (data+parity) x data
 * systematic Vandermonde matrix on the host; touches no GPU. */
int shmr_ec_new(uint32_t data_shards, uint32_t parity_shards, shmr_ec_t** out);
void shmr_ec_free(shmr_ec_t* rs);

uint32_t shmr_ec_data_shard_count(const shmr_ec_t* rs);
uint32_t shmr_ec_parity_shard_count(const shmr_ec_t* rs);
uint32_t shmr_ec_total_shard_count(const shmr_ec_t* rs);

/* Copies the (data+parity) x data coding matrix, row-major, into out
 * (out_len >= total*data). */
int shmr_ec_matrix(const shmr_ec_t* rs, uint8_t* out, size_t out_len);

/* Rows of the reconstruct plan the library would run for a presence
 * pattern: out_rows[m * data + t] (m < *n_out) applied to the shards listed in
 * in_idx[0..data) rebuilds shard out_idx[m].  Host only; for tests/tools. */
int shmr_ec_reconstruct_plan(shmr_ec_t* rs, const uint8_t* present, size_t nshards, int data_only,
                             uint16_t* in_idx, uint16_t* out_idx, uint8_t* out_rows,
                             size_t out_rows_len, uint32_t* n_out);

/* ---- host-buffer entry points (drop-in for the crate calls) ------------- */

/* ReedSolomon::encode (src/vfs/block.rs:427).  shards[0..data) are inputs,
 * shards[data..total) are overwritten with parity.  shard_lens[i] is the
 * length of shards[i]; the crate's checks run first and in its order
 * (count -> TOO_FEW/TOO_MANY_SHARDS, len 0 -> EMPTY_SHARD, unequal ->
 * INCORRECT_SHARD_SIZE).  Runs on the context's device: in place across
 * PCIe if the shards are mapped host memory (shmr_ec_host_alloc /
 * shmr_ec_host_register, zero-copy), else through a pooled mapped bounce
 * buffer (blocks up to "bounce_kib") or per-shard DMA staging. */
int shmr_ec_encode(shmr_ec_t* rs, uint8_t* const* shards, const size_t* shard_lens, size_t nshards);

/* ReedSolomon::reconstruct / reconstruct_data (src/vfs/block.rs:560).
 * present[i] != 0 marks shard i as Some(..); shard_lens[i] is only read for
 * present shards.  Absent shards must point at caller buffers of the common
 * shard length (the crate allocates them; the Rust shim allocates
 * vec![0; len] before calling).  data_only != 0: absent parity shards are left
 * untouched (and may be NULL).  All present -> no-op; fewer than data present
 * -> TOO_FEW_SHARDS_PRESENT. */
int shmr_ec_reconstruct(shmr_ec_t* rs, uint8_t* const* shards, const size_t* shard_lens,
                        const uint8_t* present, size_t nshards, int data_only);

/* Asynchronous forms of shmr_ec_encode / shmr_ec_reconstruct (same arguments,
 * validation and errors, returned by the start call), so a Block Cache can
 * overlap its file I/O or copies with the GPU: when every shard the call
 * touches lies in mapped memory, the kernels are enqueued and the start call
 * returns with *op pending; on every other path the work is complete when it
 * returns.  While *op is pending the caller may read -- not write -- the input
 * shards (encode: shards [0, data); reconstruct: the present ones) and must not
 * touch the output shards.  shmr_ec_op_wait(op) waits for the work, frees op
 * and returns SHMR_EC_OK or a device error; on a start error *op is NULL. */
typedef struct shmr_ec_op shmr_ec_op_t;
int shmr_ec_encode_start(shmr_ec_t* rs, uint8_t* const* shards, const size_t* shard_lens, size_t nshards,
                         shmr_ec_op_t** op);
int shmr_ec_reconstruct_start(shmr_ec_t* rs, uint8_t* const* shards, const size_t* shard_lens,
                              const uint8_t* present, size_t nshards, int data_only, shmr_ec_op_t** op);
int shmr_ec_op_wait(shmr_ec_op_t* op);

/* ---- one block per call on device buffers: the submission queue ----------- *
 * The crate's encode / reconstruct of ONE block (ReedSolomon::encode at
 * src/vfs/block.rs:427, reconstruct at :560) whose shards are device buffers
 * on `device`: the same arguments, checks and errors as shmr_ec_encode /
 * shmr_ec_reconstruct, with d_shards[i] device pointers.  The inputs must be
 * complete when the call is made (written by synchronous copies, or by work
 * the caller has waited for): these calls take no stream.
 *
 * The reference makes one such call per block from rayon workers
 * (src/vfs/mod.rs:91-97).  One launch per block leaves the GPU launch-bound,
 * so per device ID the library keeps a submission queue: a call's block is
 * launched at once when fewer than "coalesce_depth" (default 1) batches are in
 * flight on the queue's stream, and otherwise merges with every call that
 * arrives meanwhile (from any thread, any codec; knob "coalesce_us": an idle
 * queue waits that long for company) into the next launch, which the queue's
 * watcher thread issues "coalesce_lead_us" (default 30; 0: at completion)
 * before the running batch's estimated end, so it is queued behind it -- one pointer-
 * table call per (codec, operation, length, data_only) group, whose shards,
 * if they sit on a slot lattice (a slab, a shmr_ec_pool), run the strided
 * kernels over their slots.  The call returns when its own block is written,
 * with its own status (a group's device error is its members' status).
 * Completion is a word in pinned host memory that a one-wave kernel behind
 * every batch advances: a waiting caller spins on it for "coalesce_spin_us"
 * (default 30) and then sleeps until the queue's watcher thread (which
 * follows the oldest batch, asleep on its event after "coalesce_watch_us",
 * default 200) wakes it; a call waited for while still held back launches
 * everything pending at once.  "coalesce_target" (default 64): that many pending
 * calls launch even with "coalesce_depth" batches in flight.  The *_start forms return with the
 * block queued (*op); shmr_ec_op_wait completes it.  While pending, inputs
 * may be read, outputs must not be touched. */
int shmr_ec_encode_dev(shmr_ec_t* rs, uint8_t* const* d_shards, const size_t* shard_lens, size_t nshards,
                       int device);
int shmr_ec_reconstruct_dev(shmr_ec_t* rs, uint8_t* const* d_shards, const size_t* shard_lens, const uint8_t* present,
                            size_t nshards, int data_only, int device);
int shmr_ec_encode_dev_start(shmr_ec_t* rs, uint8_t* const* d_shards, const size_t* shard_lens, size_t nshards,
                             int device, shmr_ec_op_t** op);
int shmr_ec_reconstruct_dev_start(shmr_ec_t* rs, uint8_t* const* d_shards, const size_t* shard_lens,
                                  const uint8_t* present, size_t nshards, int data_only, int device,
                                  shmr_ec_op_t** op);

/* Submission-queue counters of a device ID since load: out[i] for i < n in
 * the order below. */
enum {
    SHMR_EC_Q_REQUESTS = 0,   /* blocks submitted (device calls, and mapped host calls under "coalesce") */
    SHMR_EC_Q_BATCHES = 1,    /* launch groups taken from the queue */
    SHMR_EC_Q_MAX_BATCH = 2,  /* the most blocks one launch group merged */
    SHMR_EC_Q_SLEEPS = 3,     /* waits that ended in a blocking event synchronize */
    SHMR_EC_Q_EARLY = 4,      /* batches launched behind a running one before its end (knob coalesce_lead_us) */
    SHMR_EC_Q_COUNTERS = 5
};
int shmr_ec_queue_stats(int device, uint64_t* out, size_t n);

/* ---- device-resident batched entry points ------------------------------ *
 * All pointers are device pointers on `device`; `stream` is a hipStream_t
 * (NULL = the null stream).  Block b's shard i lives at
 *     base + b * block_pitch + i * shard_pitch,
 * at any byte alignment (the reference's packed block buffer, shard i at
 * i * S, included).
 *
 * Stream-ordered: after the device's one-time initialisation (the first call
 * that touches the device, or shmr_ec_device_init) these calls make no
 * blocking HIP call -- they enqueue kernels (and, for an erasure pattern not
 * seen before on the device, one hipMemcpyAsync of its coefficient plan from
 * a permanent pinned slot) on `stream` and return.  They can be captured into
 * a HIP graph (e.g. torch.cuda.graph) once the device is initialised; a
 * capture that would need the initialisation returns INVALID_ARGUMENT with
 * nothing enqueued, and so does one whose stream state cannot be read (the
 * legacy null stream while another thread captures in global mode).
 * SHMR_EC_DEV_BLOCKING_CALLS counts the exceptions.
 *
 * Cross-stream coupling: the readiness of an upload (a plan image, an upload-
 * ring slot, a table-cache entry) that a call enqueued on a caller stream is
 * tracked by an event mirrored onto the device's one private stream, which
 * waits for the caller stream's events in the order they were recorded.  A
 * later call on ANOTHER stream that needs such an upload (or a busy ring
 * slot) may therefore wait for work queued earlier on unrelated caller
 * streams.  A stream held back by something outside the library (a host
 * function, a stream wait on a value, a collective) can delay, and with a
 * full ring block, another thread's call until it progresses.  Streams that
 * only reuse plans and tables already uploaded are not affected. */

/* One-time per-device initialisation (probe of the memory system's unaligned
 * access mode on a private stream, the plan arena and a 4 MiB capture reserve
 * in pinned and device memory).  Optional: the first device call does it
 * implicitly.  Blocking. */
int shmr_ec_device_init(int device);

/* Captured calls keep their tables in the device's capture reserve, which a
 * capture never grows: a captured *_ptrs_dev call needs nblocks * total * 8
 * bytes, a captured reconstruct of several erasure patterns in more than 32
 * block runs about 6 bytes per block plus 8 per pattern (each rounded up to
 * 256 bytes).  A captured call that does not fit returns OUT_OF_MEMORY with
 * nothing enqueued.  This makes sure one free range of `bytes` exists
 * (initialising the device if needed; blocking, not inside a capture).  A
 * captured call's block returns to the reserve when its graph and every
 * executable graph instantiated from it have been destroyed. */
int shmr_ec_capture_reserve(int device, size_t bytes);

/* Encode nblocks blocks: data shard i of block b at
 * d_data + b*data_block_pitch + i*data_shard_pitch; parity shard r at
 * d_parity + b*parity_block_pitch + r*parity_shard_pitch. */
int shmr_ec_encode_batch_dev(shmr_ec_t* rs, const uint8_t* d_data, size_t data_shard_pitch,
                             size_t data_block_pitch, uint8_t* d_parity, size_t parity_shard_pitch,
                             size_t parity_block_pitch, size_t nblocks, size_t shard_len,
                             int device, void* stream);

/* Reconstruct nblocks blocks in place.  All total shards of block b live at
 * d_shards + b*block_pitch + i*shard_pitch.  present is HOST memory,
 * nblocks x total flags (row-major).  Blocks may have different presence
 * patterns; validation of every block precedes any launch. */
int shmr_ec_reconstruct_batch_dev(shmr_ec_t* rs, uint8_t* d_shards, size_t shard_pitch,
                                  size_t block_pitch, const uint8_t* present, size_t nblocks,
                                  size_t shard_len, int data_only, int device, void* stream);

/* Reconstruct with the crate's memory semantics: every absent shard is
 * rebuilt into a buffer of its own (reed_solomon_erasure allocates
 * vec![0; len] for each None, called at src/vfs/block.rs:556-565; load_block
 * then concatenates them, :567-576), not into the block's slot.  Present
 * shards of block b are read in place at d_shards + b*block_pitch +
 * i*shard_pitch (absent slots are neither read nor written); block b's
 * rebuilt shards, in ascending shard index, are written to
 *     d_out + b*out_block_pitch + j*out_shard_pitch,  j = 0 .. rebuilt-1
 * (data_only != 0: the absent data shards only).  d_out must hold the largest
 * rebuilt count of the batch per block and must not overlap a present shard.
 * Blocks with every shard present write nothing.  Validation and errors as
 * shmr_ec_reconstruct_batch_dev. */
int shmr_ec_reconstruct_batch_dev_out(shmr_ec_t* rs, const uint8_t* d_shards, size_t shard_pitch,
                                      size_t block_pitch, const uint8_t* present, size_t nblocks,
                                      size_t shard_len, int data_only, uint8_t* d_out,
                                      size_t out_shard_pitch, size_t out_block_pitch, int device,
                                      void* stream);

/* Device-resident shards that live anywhere -- the crate's own argument shape
 * (ReedSolomon::encode(&mut [Vec<u8>]) at block.rs:427 over shards that
 * block.rs:408-419 copies into a Vec each; reconstruct(&mut [Option<Vec<u8>>])
 * at block.rs:560, every None rebuilt into a fresh buffer, :556-565), batched.
 * d_shards is a HOST array of nblocks x total DEVICE pointers:
 * d_shards[b*total + i] is shard i of block b, shard_len bytes, any alignment
 * (16-byte aligned shards take the vector kernels; otherwise the device's
 * verified unaligned access mode, else byte-granular).  The table is copied
 * before the call returns (the caller may reuse it) and uploaded on `stream`;
 * stream-ordered and graph-capturable as the calls above.
 * encode: shards [0, data) in, [data, total) overwritten with parity; every
 * pointer non-NULL.
 * reconstruct: present = nblocks x total host flags; absent shards point at
 * caller buffers that receive the rebuilt bytes (absent parity may be NULL
 * with data_only != 0); validation and errors as shmr_ec_reconstruct_batch_dev. */
int shmr_ec_encode_ptrs_dev(shmr_ec_t* rs, uint8_t* const* d_shards, size_t nblocks, size_t shard_len,
                            int device, void* stream);
int shmr_ec_reconstruct_ptrs_dev(shmr_ec_t* rs, uint8_t* const* d_shards, const uint8_t* present,
                                 size_t nblocks, size_t shard_len, int data_only, int device, void* stream);

/* ---- host-buffer batches over one or more GPUs ---------------------------- *
 * Blocks held in HOST memory (the Block Cache / shard file buffers), whole
 * blocks round-robin across `devices` (block b -> devices[b % ndev]); per
 * device the H2D copy, the kernel and the D2H copy of successive chunks
 * overlap on separate streams.  host_shards[b * total + i] points at shard i
 * of block b, each shard_len bytes.  Mapped buffers (shmr_ec_host_alloc /
 * shmr_ec_host_register) are coded in place across PCIe (zero-copy); other
 * pinned buffers are DMA'd; pageable ones are gathered into a mapped pinned
 * mirror by a crew of copy threads and coded there ("mirror_zc").
 * Synchronous; every block is validated before device work. */
int shmr_ec_encode_blocks_host(shmr_ec_t* rs, uint8_t* const* host_shards, size_t nblocks,
                               size_t shard_len, const int* devices, int ndev);

/* Reconstruct host-resident blocks: present = nblocks x total flags; absent
 * shards are written (absent parity only when data_only == 0) and need a
 * buffer; semantics per block as shmr_ec_reconstruct. */
int shmr_ec_reconstruct_blocks_host(shmr_ec_t* rs, uint8_t* const* host_shards, const uint8_t* present,
                                    size_t nblocks, size_t shard_len, int data_only,
                                    const int* devices, int ndev);

/* Mapped (page-locked, device-visible from every GPU) host memory for Block
 * Cache buffers.  When every shard a host-buffer call touches (shmr_ec_encode,
 * shmr_ec_reconstruct, the *_blocks_host batches) lies in memory from
 * shmr_ec_host_alloc or a range given to shmr_ec_host_register, the kernels
 * read and write those buffers in place across PCIe (zero-copy: no staging
 * copies, no device buffers); otherwise the call stages through device memory. */
int shmr_ec_host_alloc(size_t bytes, void** out);
void shmr_ec_host_free(void* p);

/* Page-locks and maps an existing host range (e.g. a Rust Vec<u8> Block Cache
 * buffer) for zero-copy use; shmr_ec_host_unregister(p) with the same p undoes
 * it.  The range must stay allocated while registered. */
int shmr_ec_host_register(void* p, size_t bytes);
int shmr_ec_host_unregister(void* p);

/* Device memory for block batches (the *_batch_dev entry points), so a caller
 * (e.g. the Rust shim) needs no HIP bindings of its own.  contiguous == 0 is a
 * plain hipMalloc; contiguous != 0 asks for physically contiguous VRAM
 * (hipDeviceMallocContiguous, mapped with large page fragments) and fails
 * with OUT_OF_MEMORY if the driver cannot supply it (no silent fallback).
 * Measured on MI355X: contiguous VRAM lifts the XOR-only replica of the
 * RS(8,3) access pattern over 2,048 blocks (11 GiB) from 76 % to 78.5 % of
 * HBM peak, but the GF kernel itself runs the same on both (78.8 % at 2,048
 * blocks, 79.7 % at 512).  Free with shmr_ec_device_free on the same device.
 * The frees here (shmr_ec_device_free, shmr_ec_device_free_shards,
 * shmr_ec_pool_destroy, shmr_ec_host_free) are hipFree / hipHostFree: each
 * waits for the work of every stream of the device, a caller stream held by a
 * wait included.  The compute calls grow their own scratch without a free
 * (r06 s40); only the pinned bounce pool of pageable host calls frees, and only
 * a buffer returned while 32 others lie idle. */
int shmr_ec_device_alloc(int device, size_t bytes, int contiguous, void** out);
int shmr_ec_device_free(int device, void* p);

/* Shard buffers for the *_ptrs_dev calls with the slot placement of the
 * device-resident batches: nblocks x shards_per_block buffers of shard_len
 * bytes carved from one device slab (256-byte aligned base), each at the slot
 * pitch P = shard_len rounded up to 4 KiB, plus one 4 KiB page when that is a
 * multiple of 64 KiB:
 *     out_ptrs[b * shards_per_block + i] = slab + (b * shards_per_block + i) * P.
 * The crate keeps every shard in a Vec<u8> of its own (reference
 * src/vfs/block.rs:408-419, :556-565); a device Block Cache that takes its
 * shard buffers from here -- all total shards of its blocks in one call, and
 * the buffers for rebuilt shards (one per absent shard) in another -- hands
 * the *_ptrs_dev calls tables that form a slot grid, which run through the
 * strided kernels (knob "ptrs_grid").  The bytes are not initialised.  Free
 * with shmr_ec_device_free_shards(device, out_ptrs[0]); any other pointer
 * returns INVALID_ARGUMENT (shmr_ec_device_free(device, out_ptrs[0]) frees
 * it too). */
int shmr_ec_device_alloc_shards(int device, size_t nblocks, size_t shards_per_block, size_t shard_len,
                                uint8_t** out_ptrs);
int shmr_ec_device_free_shards(int device, uint8_t* first);

/* A device Block Cache of per-block slots (r06).  The reference's Block Cache
 * takes and drops one block's buffers at a time (src/vfs/block.rs:148-152,
 * :586-608); a shmr_ec_device_alloc_shards slab is freed only whole.  A pool
 * carves block slots -- shards_per_block shard buffers of shard_len bytes at
 * the slot pitch P of the device-resident batches (shard_len rounded up to 4
 * KiB, one page more for a multiple of 64 KiB) -- from device slabs of
 * slots_per_slab slots (allocated on demand, blocking), and hands them out one
 * block at a time, the lowest free slot first:
 *     out_ptrs[i] = slab + slot * shards_per_block * P + i * P.
 * Pointer tables over pool blocks, in any order and with holes, lie on the
 * slab's slot lattice: the *_ptrs_dev calls and the submission queue run them
 * through the strided kernels over their slots.  shmr_ec_pool_free takes
 * out_ptrs[0] of an alloc (anything else, or a second free: INVALID_ARGUMENT);
 * shmr_ec_pool_destroy frees every slab (no kernel may still use them).  The
 * bytes are not initialised. */
typedef struct shmr_ec_pool shmr_ec_pool_t;
int shmr_ec_pool_new(int device, size_t shards_per_block, size_t shard_len, size_t slots_per_slab,
                     shmr_ec_pool_t** out);
int shmr_ec_pool_alloc(shmr_ec_pool_t* pool, uint8_t** out_ptrs);
int shmr_ec_pool_free(shmr_ec_pool_t* pool, uint8_t* first);
int shmr_ec_pool_destroy(shmr_ec_pool_t* pool);
int shmr_ec_pool_stats(shmr_ec_pool_t* pool, uint64_t* slabs, uint64_t* slots, uint64_t* in_use);

/* ---- configuration -------------------------------------------------------- */

/* Device used by the host-buffer entry points (default 0; negative ->
 * SHMR_EC_INVALID_ARGUMENT).  Device IDs are checked at every compute call:
 * an ID >= the number of GPUs returns SHMR_EC_INVALID_ARGUMENT
 * (SHMR_EC_NO_DEVICE without a GPU); the *_blocks_host calls check every
 * entry of their device list the same way, and a NULL list or ndev <= 0 is
 * INVALID_ARGUMENT -- all before any buffer is touched.  A device listed
 * twice gets two shares of the blocks. */
int shmr_ec_set_device(shmr_ec_t* rs, int device);

/* Tuning knobs (process-wide).
 *
 * Host-path knobs (both flavours; they choose how bytes move, never what
 * the kernels compute): "coalesce" (0/1, default 0 -- measured no faster on
 * PCIe-bound mapped blocks): shmr_ec_encode /
 * shmr_ec_reconstruct (and *_start) whose shards all lie in mapped memory go
 * through the device's submission queue (above), merged with concurrent
 * calls, instead of one zero-copy launch per call; "coalesce_depth",
 * "coalesce_target", "coalesce_us", "coalesce_max" (blocks per launch, default
 * 1024), "coalesce_spin_us", "coalesce_watch_us", "coalesce_lead_us" and "coalesce_idle_us" (default 1000:
 * the watcher spins this long for calls after the queue goes idle, then sleeps): the queue (above).  "bounce_kib": pageable single-block calls whose
 * (k+p) x shard bytes fit in this many KiB go through one mapped bounce
 * buffer and a single zero-copy launch instead of per-shard DMA copies
 * (default 8192; 0 disables).  "mirror_zc" (0/1, default 1): pageable host
 * batches are gathered into a pinned mirror that the kernel codes in place
 * across PCIe (zero-copy) instead of DMA-ing it to device staging.
 * "ptrs_grid" (0/1, default 1): a *_ptrs_dev table whose shards form a slot
 * grid -- entry (b, i) at base + b * block_pitch + i * shard_pitch for the
 * inputs, and for the outputs (encode: parity rows; reconstruct: the absent
 * shards in place, or rebuilt shard j of block b at out + b * out_block_pitch +
 * j * out_shard_pitch) -- runs through the strided kernels of the *_batch_dev
 * calls with no table (same bytes; SHMR_EC_DEV_PTR_TABLE_GRIDS counts them);
 * 0 always takes the table kernels.  A table whose blocks sit on a slot
 * lattice (a slab or a pool, in any order, with holes) runs the strided
 * kernels over its slots when they form one arithmetic run or up to 32 runs
 * (segment launches); beyond that the table kernels run, measured faster than
 * an uploaded slot list ("lattice_list" (0/1, default 0): 1 takes the list).
 * Rebuilds with several erasure patterns in more runs than that take the
 * table kernels too.
 * "ptrs_direct" (default 16): zero-copy launches of at most this many 4 KiB
 * tiles read their shard-pointer table from pinned host memory in place
 * instead of uploading it first (0: always upload).  "sync_spin_us"
 * (default 0): the single-call and zero-copy paths poll their stream this
 * long before a blocking synchronize.
 *
 * Kernel knobs select a measurement variant of the kernel.  In the product
 * library (libshmr_ec.so) every launch uses the measured per-shape policy and
 * a kernel knob can only be set to its default (anything else returns
 * SHMR_EC_INVALID_ARGUMENT); the tools build (libshmr_ec_tools.so) takes:
 * "chunks" (16-B chunks per lane per tile: 1, 2, 4), "nt_load", "nt_store"
 * (nontemporal 0/1), "occ8" (0/1), "grid" (-1 one
 * workgroup per tile, 0 balanced persistent grid, >0 capped persistent
 * grid), "threads" (lanes per workgroup: 128, 256, 512), "depth" (register
 * ring depth = shards of loads in flight + 1: 1, 2, 3, 5, 9), "wgs_per_cu"
 * (0 = no cap, else the most workgroups resident per CU, enforced by LDS
 * padding; auto: 7 for single-row reconstructs, else no cap), "occ" (0, 5, 6, 7: register budget for that many waves per SIMD),
 * "early" (0/1: issue the first data loads before the plan's LDS staging
 * completes; auto: encodes with fewer than 8 data shards or 4 output rows),
 * "spre" (0/1: coefficient tables and shard offsets by scalar
 * loads one shard ahead, no LDS), "fuse_tail" (0/1: a shard length that is
 * not a multiple of the tile runs the partial last tile of every block at the
 * head of the full-tile launch instead of in a second launch), "glds" (0/1:
 * input ring in LDS filled by global_load_lds_dwordx4, depth = ring slots),
 * "serial" (0/1: GF math ordered one dword at a time, fewer VGPRs; auto:
 * encodes of 4 output rows), "sc1_store" (0/1: stores with the sc1 cache
 * policy instead of nontemporal; auto: reconstructs into a compact output),
 * "diag"
 * (0/1: XOR-only diagnostic kernel, WRONG results, for ceiling measurements).
 * Prefix "encode." or "decode." to set one operation class only.
 * "chunks", "nt_load", "nt_store", "depth", "wgs_per_cu", "occ", "early",
 * "spre", "fuse_tail", "glds", "serial" and "sc1_store" default to -2 (auto): the per-shape policy; any other value pins
 * the knob, and setting -2 returns it to the policy. */
int shmr_ec_set_tuning(const char* key, int value);
int shmr_ec_get_tuning(const char* key);

/* Writes the kernel variant that a launch of `rows` output rows over
 * `data_shards` inputs would use (encode: decode=0, reconstruct in place:
 * decode=1, reconstruct into a compact output: decode=2; over 16-byte aligned
 * device shard-pointer tables, *_ptrs_dev: encode 3, reconstruct 4). */
int shmr_ec_describe_variant(int decode, uint32_t data_shards, uint32_t rows, char* buf, size_t len);

/* Kernel inventory: every gf_apply kernel instantiation compiled into this
 * library -- the full-tile kernels the launch policy can select (mode 0, one
 * per reachable (rows, chunks, flags); the product list is derived from the
 * policy at compile time) and the partial-tile (mode 1), byte-granular (mode 2)
 * and realigning (mode 3) kernels per row count -- with the launches each has
 * served in this process.  Writes min(cap, count) entries and returns the
 * count (out may be NULL to query it).  flags are the kernel's template flags
 * (the F of gf_apply_kernel<R, U, MODE, F> in the code object's symbol). */
typedef struct shmr_ec_kernel_info {
    uint32_t rows, chunks, mode, flags;
    uint64_t launches;
} shmr_ec_kernel_info;
size_t shmr_ec_kernel_inventory(shmr_ec_kernel_info* out, size_t cap);

/* Decode-matrix LRU statistics of the (data, parity) codec (crate cache
 * semantics, capacity 254). */
int shmr_ec_cache_stats(const shmr_ec_t* rs, uint64_t* hits, uint64_t* misses);

/* Number of visible GPUs (0 when none; never fails). */
int shmr_ec_device_count(void);

/* Blocks the host-buffer entry points served zero-copy (mapped memory) and
 * through device staging since the library was loaded.  Either may be NULL. */
int shmr_ec_path_stats(uint64_t* zero_copy_blocks, uint64_t* staged_blocks);

/* Per-device counters since the library was loaded, for the device ID the
 * caller passed (blocks b -> devices[b % ndev] of the *_blocks_host calls, the
 * context's device, or a *_batch_dev call's device): out[i] for i < n in the
 * order below.  Every per-device object (plan images, upload rings, staging
 * streams) is created per device ID, so N GPUs show N sets.  In the tools
 * build, tuning key "alias_devices" = a adds IDs n .. n+a-1 that run on
 * physical GPU (id mod n) with their own per-device state (a one-GPU
 * rehearsal of multi-device bookkeeping); the product library has none. */
enum {
    SHMR_EC_DEV_BLOCKS_ENCODED = 0,
    SHMR_EC_DEV_BLOCKS_RECONSTRUCTED = 1, /* blocks with at least one absent shard */
    SHMR_EC_DEV_LAUNCHES = 2,             /* full-tile launch groups (<= 4 rows each) */
    SHMR_EC_DEV_PLAN_IMAGES = 3,          /* coefficient plans uploaded to this device */
    SHMR_EC_DEV_UPLOAD_RINGS = 4,         /* pinned upload rings created for this device */
    SHMR_EC_DEV_STAGING_STREAMS = 5,      /* staging / pipeline streams created for this device */
    SHMR_EC_DEV_BLOCKING_CALLS = 6,       /* blocking HIP calls the library made on its own: device
                                             init, plan-arena growth, upload-ring creation and waits
                                             for a ring slot (not the host-buffer calls' final sync) */
    SHMR_EC_DEV_PTR_TABLE_HITS = 7,       /* *_ptrs_dev tables reused from the device's table cache
                                             (no upload) */
    SHMR_EC_DEV_CAPTURE_TABLES = 8,       /* capture-reserve blocks taken by captured calls */
    SHMR_EC_DEV_CAPTURE_RELEASED = 9,     /* ... and returned when their graph was destroyed */
    SHMR_EC_DEV_PTR_TABLE_GRIDS = 10,     /* *_ptrs_dev calls whose table named a slot grid and ran
                                             through the strided kernels (no table) */
    SHMR_EC_DEV_COUNTERS = 11
};
int shmr_ec_device_stats(int device, uint64_t* out, size_t n);

#ifdef __cplusplus
}
#endif

#endif /* SHMR_EC_H */
