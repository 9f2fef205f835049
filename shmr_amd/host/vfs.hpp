// C++ host mirror of the reference's StorageBlock layer (src/vfs/{block,mod,path}.rs,
// src/config.rs) around the MI355X codec.  Same types, method names and error
// behaviour as the reference; the Erasure arms call shmr::ReedSolomon (GPU).
//
// Block Cache layout: an Erasure block's buffer is one
// allocation of (k+p)*S bytes -- the data shards are already contiguous at i*S
// in the reference's buffer, so sync encodes and writes the shard files
// straight from it (no chunks().to_vec() copies), and load reads every shard
// file into its slot and reconstructs in place.  With VfsOptions::pinned_buffers
// the allocation is mapped host memory (shmr_ec_host_alloc) that the GPU kernels
// read and write in place across PCIe (zero-copy, no staging).
// VirtualFile::sync_data / read fan the work out over a persistent worker pool:
// with mapped buffers one task per block (zero-copy encode / reconstruct on
// GPU devices[i % n] plus its shard-file I/O); with pageable buffers the Erasure
// blocks go into pipelined multi-GPU batch calls (shmr_ec_encode_blocks_host /
// shmr_ec_reconstruct_blocks_host) against parallel pwrite+fsync / reads
// (row 3).  Deviations from the reference are opt-in (VfsOptions).
#pragma once

#include <cstdint>
#include <filesystem>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <string>
#include <utility>
#include <vector>

#include "reed_solomon.hpp"

namespace shmr {

namespace fs = std::filesystem;

constexpr uint64_t VIRTUAL_BLOCK_DEFAULT_SIZE = 1024 * 1024;   // src/vfs/path.rs:12
constexpr uint64_t VFS_DEFAULT_BLOCK_SIZE = 4096;              // src/lib.rs:22 (the chunk size)
constexpr const char* VP_DEFAULT_FILE_EXT = "bin";             // src/vfs/path.rs:14

// ShmrError (src/config.rs:151-164).  FsError carries errno, EcError the crate code.
struct ShmrError {
    enum Kind {
        InvalidPoolId,
        InvalidBucketId,
        OutOfSpace,
        EndOfFile,
        FsError,
        EcError,
        ShardOpened,
        ShardMissing,
        InvalidInodeType,
        InodeNotExist,
        BlockIndexOutOfBounds,
    } kind;
    int code = 0;   // errno for FsError, shmr_ec status for EcError
    std::string what() const;
};
using Status = std::optional<ShmrError>;   // std::nullopt == Ok(())

// BlockTopology (src/vfs/block.rs:22-98)
struct BlockTopology {
    enum Kind { Single, Mirror, Erasure } kind = Single;
    uint8_t n = 0;                              // Mirror(n)
    uint8_t version = 0, data = 0, parity = 0;  // Erasure(version, data, parity)
    static BlockTopology single() { return {}; }
    static BlockTopology mirror(uint8_t n) { return {Mirror, n, 0, 0, 0}; }
    static BlockTopology erasure(uint8_t v, uint8_t d, uint8_t p) { return {Erasure, 0, v, d, p}; }
    // BlockTopology::try_from(String); error text as the reference's.
    static std::optional<BlockTopology> try_from(const std::string& value, std::string* err = nullptr);
    std::string to_string() const;   // Display
};

// Bucket / ShmrFsConfig (src/config.rs:17-39, 100-139)
enum class BucketPriority { Evacuate = 0, Ignore = 1, Deprioritize = 2, Normal = 3, Prioritize = 4 };
struct Bucket {
    fs::path path;
    uint64_t capacity = 0;
    uint64_t available = 0;
    BucketPriority priority = BucketPriority::Normal;
};
struct ShmrFsConfig {
    std::map<std::string, std::map<std::string, Bucket>> pools;   // pool -> bucket name -> bucket
    std::string write_pool;
    uint64_t block_size = VIRTUAL_BLOCK_DEFAULT_SIZE;
    // select_buckets (src/config.rs:46-85): buckets above Ignore, sorted by
    // (priority, available) ascending, repeated until `count`, first `count`.
    // (The reference iterates a HashMap, so ties are unordered there; here
    // ties keep bucket-name order.)
    Status select_buckets(const std::string& pool, size_t count, std::vector<std::string>* out) const;
};

// VirtualPath (src/vfs/path.rs:20-83)
struct VirtualPath {
    std::string pool, bucket, filename;
    // (file path, directory) -- the directory is the unused <bucket>/fn[0..2]/fn[2..4]
    Status resolve(const ShmrFsConfig& cfg, fs::path* file, fs::path* dir) const;
    Status create(const ShmrFsConfig& cfg) const;   // mkdir -p dir; create+truncate file
    std::string to_string() const;
};

// Opt-in deviations from the reference (all off = reference behaviour).
struct VfsOptions {
    // load_block: a shard file that cannot be opened is an erasure (the
    // reference fails in open_handles, block.rs:481-487).
    bool missing_shard_is_erasure = false;
    // load_block: read shards with pread at offset 0 (the reference reads from
    // the handle's current cursor, so a second load after drop_buffer without
    // drop_handles reads 0 bytes, block.rs:544).
    bool pread_from_start = false;
    // load_block: a shard whose length is not S is an erasure (the reference
    // zero-pads it and keeps it present, block.rs:548-551).
    bool short_shard_is_erasure = false;
    // load_block with pread_from_start: read only the shard files a load
    // needs -- the first k files of exactly S bytes (the reconstruct's
    // inputs, the crate's first-k-present rule); other intact shards count as
    // present unread.  Reads 8 of 11 RS(8,3) shards instead of 10-11; the
    // loaded data is byte-identical (the unread parity slots are never
    // returned, and every flush re-encodes parity).  Falls back to reading
    // everything where the reference's short-shard rule needs the bytes.
    bool read_needed_shards = false;
    // Block Cache buffers in mapped host memory (shmr_ec_host_alloc: the codec
    // runs zero-copy on them); falls back to pageable memory when no device is
    // present.
    bool pinned_buffers = false;
    // sync_data of a buffer longer than k*S (calculate_shard_size's f32
    // hazard, e.g. 16,777,217 B at Erasure(1,8,3)): off = refuse with
    // EcError(TooManyDataShards) before any write (the default: the
    // reference silently loses data there); on = the reference's release
    // build bit for bit (block.rs:421's u8 arithmetic wraps, parity row 0
    // overwrites data chunk k in the shard files; Cargo.toml:10-13).
    bool release_u8_wrap = false;
    // fsync every shard file after writing it (write_path, block.rs:633).
    // Benchmarks may turn it off to separate the device path from the disk.
    bool fsync_shards = true;
    // Test hook: a per-block Erasure flush reports a device error at the
    // encode's wait, after the data shard files went out (the failure path
    // that truncates the parity files and keeps the block dirty).
    bool fault_encode_wait = false;
    // Shard files read into and written from the Block-Cache slots with
    // O_DIRECT (no page-cache copy; raw S bytes at offset 0, the same files).
    // Applies to slots that are whole 4 KiB-aligned pages (S a multiple of
    // 4096) and reads from offset 0 (pread_from_start); a file system that
    // refuses O_DIRECT (tmpfs, overlay) and any other slot take the buffered
    // path (direct_io_stats() counts both).  Reads of hot files then come
    // from the disk instead of the page cache.
    bool direct_io = false;
};

// What VfsOptions::direct_io did since the library was loaded: shard files
// read / written with O_DIRECT, shard I/O under direct_io that went buffered
// (a slot that is not whole pages, a refused open, a failed O_DIRECT call, or
// a file that is not exactly S bytes), refused opens, the first refusal's
// errno and file system, and the first O_DIRECT I/O error.
struct DirectIoStats {
    uint64_t reads = 0, writes = 0, fallbacks = 0, refusals = 0;
    int refused_errno = 0;
    std::string refused_fs;
    int io_errno = 0;   // first O_DIRECT read/write error (the shard then went buffered)
};
DirectIoStats direct_io_stats();

// Where a VirtualFile flush / batched load spent its time (last call).
// The codec and I/O phases of a batch are pipelined (batch b+1's codec call
// overlaps batch b's file I/O), so codec_s + io_s can exceed total_s.
struct IoStats {
    double prepare_s = 0;   // opening handles, padding buffers
    double codec_s = 0;     // batched GPU encode / reconstruct calls (PCIe included)
    double io_s = 0;        // shard-file reads or writes (+ fsync), busy time
    double total_s = 0;     // codec + I/O phase, wall
    size_t blocks = 0;      // Erasure blocks coded
    // Per-block task mode (mapped Block-Cache buffers with the auto batch: one
    // task per block on the worker pool, VirtualBlock::sync_data / load_block
    // each): thread time summed over the tasks.  Tasks run concurrently, so the
    // sums exceed total_s; their ratios say where a task's time goes.
    double task_read_s = 0;    // load: shard-file reads into the block's slots
    double task_write_s = 0;   // flush: shard-file writes (+ fsync)
    double task_codec_s = 0;   // the block's zero-copy GPU call, PCIe included
    double task_copy_s = 0;    // VirtualFile::read: copy-out into the caller's buffer (after the load)
    double task_overlap_s = 0; // VirtualFile::read: copy-out of present shards while the GPU rebuilds
    double task_total_s = 0;   // whole tasks (the rest: locks, handles, buffer set-up)
    size_t tasks = 0;
};

// Phase times of one VirtualBlock::sync_data / load_block call (seconds).
struct PhaseTimes {
    double io_s = 0;        // shard-file reads or writes (flush: those not overlapped with the encode)
    double codec_s = 0;     // the GPU encode / reconstruct call, minus work overlapped with it
    double overlap_s = 0;   // load: the during-rebuild callback (copies overlapping the GPU work)
};

// VirtualBlock (src/vfs/block.rs:119-634).  Copies share state, like the
// reference's Arc<Mutex<..>> fields.
class VirtualBlock {
public:
    uint64_t ino = 0;
    uint64_t idx = 0;
    uint64_t size = 0;
    BlockTopology topology;
    std::vector<VirtualPath> shards;

    VirtualBlock();
    static Status create(uint64_t ino, uint64_t idx, std::shared_ptr<const ShmrFsConfig> cfg, uint64_t size,
                         BlockTopology topology, VirtualBlock* out);
    static Status create_with_pool(uint64_t ino, uint64_t idx, const std::string& pool,
                                   std::shared_ptr<const ShmrFsConfig> cfg, uint64_t size, BlockTopology topology,
                                   VirtualBlock* out);
    void populate(std::shared_ptr<const ShmrFsConfig> cfg) { cfg_ = std::move(cfg); }
    void set_options(const VfsOptions& o);

    Status read(uint64_t pos, uint8_t* buf, size_t len, size_t* nread) const;
    Status write(uint64_t pos, const uint8_t* buf, size_t len, size_t* nwritten) const;
    Status sync_data(bool force) const { return sync_data(force, 0); }
    Status sync_data(bool force, int device, PhaseTimes* times = nullptr) const;   // Erasure encode on that GPU
    Status drop_buffer() const;
    Status drop_handles() const;

    // Test hooks (the reference's tests read these fields directly).
    std::vector<uint8_t> buffer_snapshot() const;
    bool buffer_loaded() const;
    bool buffer_pinned() const;
    size_t buffered_len() const;   // the buffer's current length

private:
    friend class VirtualFile;
    struct State;
    Status open_handles() const;
    Status load_block() const { return load_block(nullptr, 0); }
    // *reconstructed (if set): an Erasure block needed a reconstruct (on `device`)
    // during (if set): called while the block's reconstruct runs, with the
    // presence flags (mapped buffers: the kernel is still running; otherwise
    // after it finished)
    Status load_block(bool* reconstructed, int device, PhaseTimes* times = nullptr,
                      const std::function<void(const uint8_t*)>* during = nullptr) const;
    size_t shard_size() const;   // S of an Erasure block (mod.rs:16-18)
    std::shared_ptr<State> st_;
    std::shared_ptr<const ShmrFsConfig> cfg_;
    VfsOptions opt_;
};

// Frees the Block Cache allocations kept for reuse (dropped buffers are pooled
// by capacity, up to 16 GiB, because pinning memory costs more than filling
// it).  Returns the bytes freed.
size_t block_cache_trim();

// Shard files read by Erasure-block loads since the library was loaded.
uint64_t shard_reads_total();

// VirtualFile (src/vfs/mod.rs:35-272)
class VirtualFile {
public:
    uint64_t ino = 0;
    uint64_t size = 0;
    uint64_t chunk_size = VFS_DEFAULT_BLOCK_SIZE;
    std::vector<VirtualBlock> blocks;
    uint64_t block_size = VIRTUAL_BLOCK_DEFAULT_SIZE;

    static VirtualFile new_with(uint64_t ino, uint64_t size);
    void populate(std::shared_ptr<const ShmrFsConfig> cfg);
    void set_options(const VfsOptions& o);   // this file's blocks, present and future

    std::vector<int> devices = {0};   // GPUs for the batched calls (blocks round-robin)
    IoStats last_sync, last_load;     // instrumentation of the last batched flush / load
    // Data bytes per pipelined batch of a flush / load (the codec call of one
    // batch overlaps the shard-file I/O of the previous one); 0 = one batch.
    // Auto (the default): with mapped Block-Cache buffers flushes pipeline in
    // 128 MiB batches and loads in 64 MiB batches; pageable buffers run as one
    // batch -- there the codec's copies and the file I/O compete for host
    // memory bandwidth and pipelining measured slower.
    static constexpr size_t kAutoBatch = ~size_t(0);
    size_t pipeline_batch_bytes = kAutoBatch;
    // Concurrent per-block tasks of the mapped-buffer flush and load (the
    // reference's rayon fan-out, mod.rs:93-96; the worker pool has 32 threads).
    // Loads run 24: +13 %, +14 % and +10-13 % read with erasure on three boxes
    // (-1 % on a fourth; profiles/r04/s2, s9, s10, profiles/r05/s11); flushes
    // stay at 16 (24 was no faster, and slower with fsync on one box).
    size_t per_block_tasks = 16;
    size_t per_block_read_tasks = 24;

    // read (mod.rs:137-180): the blocks the range touches are loaded in one
    // batched call (load_blocks) and copied out as the reference's chunk loop
    // would; runs of Erasure blocks are copied while later batches still load.
    Status read(uint64_t pos, uint8_t* buf, size_t len, size_t* nread);
    Status write(uint64_t pos, const uint8_t* buf, size_t len, size_t* nwritten);
    // sync_data (mod.rs:91-103): every block is flushed, errors reported after
    // all were attempted.  Mapped Block-Cache buffers (auto batching): one
    // flush task per block on the worker pool, as the reference's rayon
    // fan-out, each a zero-copy encode on GPU devices[i % n] plus its shard
    // writes -- fine-grained overlap of encodes and writes (40 vs 34 GiB/s
    // batched).  Otherwise Erasure blocks with the same (k, p, S) are encoded
    // in pipelined batched GPU calls, their k+p shard files written in parallel.
    Status sync_data(bool force);
    // Loads every listed block that is not buffered.  Mapped Block-Cache
    // buffers (auto batching): one load task per block on the worker pool
    // (shard reads, then a zero-copy reconstruct on devices[i % n] if needed).
    // Otherwise Erasure blocks with erasures are reconstructed in batched GPU
    // calls per (k, p, S), pipelined against the shard-file reads.
    // on_batch, if set, is called on a helper thread with the Erasure blocks of
    // each pipeline batch as soon as they are loaded (while later batches load);
    // it may read those blocks' buffers without locking -- load_blocks holds
    // their locks until every on_batch call has returned.
    // during_rebuild (per-block tasks only), if set, is called by a block's load
    // task while its zero-copy reconstruct runs on the GPU, with the block
    // index and the shard presence flags: the present shards' bytes in the
    // buffer are final then (the kernel only reads them) and may be copied.
    using DuringRebuild = std::function<void(size_t blk, const uint8_t* present)>;
    Status load_blocks(const std::vector<size_t>& block_indices,
                       const std::function<void(const std::vector<size_t>&)>& on_batch = {},
                       const DuringRebuild& during_rebuild = {});
    Status drop_buffers() const;
    Status drop_handles() const;
    Status replace_block(size_t block_idx, VirtualBlock new_block);
    // Rewrites every block that is not Erasure(1, k, p) into a new Erasure
    // block (the file-level form of replace_block; the reference's D-Bus
    // RewriteFile is todo!(), dbus.rs:46): batched load, batched encode.
    Status rewrite_erasure(uint8_t data, uint8_t parity);

    // Durable record of the file: ino, size, chunk_size, every block's ino,
    // idx, size, BlockTopology and shard paths, block_size -- the fields the
    // reference's serde derives persist in the superblock as serde_yaml
    // (src/vfs/mod.rs:35-56, block.rs:22-30,119-158, path.rs:20-28,
    // databunny.rs:297-327; record.cpp).  A loaded file needs populate(cfg).
    std::string to_yaml() const;
    static Status from_yaml(const std::string& text, VirtualFile* out, std::string* err = nullptr);
    Status save_record(const fs::path& path) const;   // write + fsync a temp file, rename over path
    static Status load_record(const fs::path& path, VirtualFile* out, std::string* err = nullptr);

private:
    Status allocate_block();
    size_t batch_bytes(bool load) const;
    std::vector<size_t> blocks_for_range(uint64_t pos, size_t len) const;
    std::shared_ptr<const ShmrFsConfig> cfg_;
    VfsOptions opt_;
};

}  // namespace shmr
