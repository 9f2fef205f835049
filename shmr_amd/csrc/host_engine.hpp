// Host-buffer batch engine (host_engine.cpp): encode / reconstruct StorageBlocks
// whose shards live in host memory, pipelined over one or more devices.
#pragma once

#include <cstdint>

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

// Synchronous.  Validates every block before any device work.
int run_host_job(const HostJob& job, const int* devices, int ndev);

}  // namespace core
}  // namespace shmr
