// Host-buffer batch engine (host_engine.cpp): encode / reconstruct StorageBlocks
// whose shards live in host memory, pipelined over one or more devices.
#pragma once

#include <cstdint>
#include <vector>

#include "ec_core.hpp"

namespace shmr {
namespace core {

struct HostJob {
    Codec& codec;
    OpClass op;
    bool data_only;
    uint8_t* const* host_shards;   // [nblocks * total]: shard i of block b at [b * total + i]
    const uint8_t* present;        // kDecode: host flags [nblocks * total]; kEncode: unused
    uint64_t nblocks;
    uint64_t len;                  // shard length
    uint64_t chunk_bytes;          // device staging per pipeline stage (per staging set)
    int copy_threads;              // pageable mode: memcpy crew size
};

int copy_threads_default();

// Synchronous.  Validates every block before any device work.  When every
// shard the job touches lies in mapped host memory (below), the kernels read
// and write the host buffers directly across PCIe (zero-copy, no staging);
// otherwise blocks are staged through device memory in pipelined chunks.
int run_host_job(const HostJob& job, const int* devices, int ndev);

// Zero-copy only: *handled = false (and nothing runs) unless every shard the
// job touches is mapped.  Used by the single-block entry points.
// async (one device only): the kernels are enqueued and *async receives the
// staging stream they run on, not synchronised -- the caller waits on it and
// releases it (finish_async); nothing is kept when the job is not handled.
int run_mapped_job(const HostJob& job, const int* devices, int ndev, bool* handled, bool count = true,
                   Staging** async = nullptr);
// Device addresses of every shard the job touches (0 for the others), if every
// one of them lies in mapped host memory (the zero-copy precondition).
bool map_rows(const HostJob& job, std::vector<uint64_t>* dptrs);
// Waits for an async mapped job's stream and returns it to the pool.
int finish_async(Staging* s);

// Pageable single-block job through a pooled mapped bounce buffer: the input
// shards are memcpy'd in, the kernel runs zero-copy on the bounce buffer, the
// outputs are memcpy'd back -- one launch instead of one DMA per shard.
int run_bounced_job(const HostJob& job, int device);

// Registry of mapped (page-locked, device-visible) host memory: allocations of
// shmr_ec_host_alloc and ranges given to shmr_ec_host_register.
void mapped_add(const void* host, size_t bytes, const void* dev);
bool mapped_remove(const void* host);
// Device address of [p, p + len) if the whole range lies in one mapped range.
bool mapped_translate(const void* p, size_t len, uint64_t* dev);

// Blocks served by each host-buffer path since load (introspection/tests).
void count_blocks(bool zero_copy, uint64_t nblocks);
void path_stats(uint64_t* zero_copy_blocks, uint64_t* staged_blocks);

}  // namespace core
}  // namespace shmr
