// C++ host mirror of reed_solomon_erasure::galois_8::ReedSolomon over the C ABI
// (include/shmr_ec.h).  Same names and argument meaning as the crate calls the
// reference makes (src/vfs/block.rs:405,427,531,560); errors are the crate's
// variants as status codes.  Header-only.
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <optional>
#include <string>
#include <vector>

#include "shmr_ec.h"

namespace shmr {

// A reed_solomon_erasure::Error (codes -1..-13) or a device condition.
struct EcStatus {
    int code = SHMR_EC_OK;
    bool ok() const { return code == SHMR_EC_OK; }
    const char* name() const { return shmr_ec_status_name(code); }
};

// A pending shmr_ec_encode_start / shmr_ec_reconstruct_start; waits on
// destruction if wait() was not called.
class EcOp {
public:
    EcOp() = default;
    EcOp(const EcOp&) = delete;
    EcOp& operator=(const EcOp&) = delete;
    ~EcOp() {
        if (op_) (void)shmr_ec_op_wait(op_);
    }
    // The op's status; a device error of an earlier op that out() had to wait
    // for is reported here (once) if this op itself succeeded.
    EcStatus wait() {
        shmr_ec_op_t* o = op_;
        op_ = nullptr;
        int rc = o ? shmr_ec_op_wait(o) : SHMR_EC_OK;
        if (rc == SHMR_EC_OK) rc = carried_;
        carried_ = SHMR_EC_OK;
        return EcStatus{rc};
    }
    // For a *_start call: an op still pending from an earlier start is waited
    // for first (its kernels may still use that call's buffers; handing out
    // &op_ would make the C call overwrite it with NULL and lose it).  Its
    // status is kept for the next wait(), not dropped.
    shmr_ec_op_t** out() {
        if (op_) {
            const int rc = shmr_ec_op_wait(op_);
            op_ = nullptr;
            if (carried_ == SHMR_EC_OK) carried_ = rc;
        }
        return &op_;
    }

private:
    shmr_ec_op_t* op_ = nullptr;
    int carried_ = SHMR_EC_OK;
};

class ReedSolomon {
public:
    // ReedSolomon::new(data_shards, parity_shards)
    static std::unique_ptr<ReedSolomon> create(size_t data_shards, size_t parity_shards, EcStatus* st) {
        shmr_ec_t* h = nullptr;
        st->code = shmr_ec_new(uint32_t(data_shards), uint32_t(parity_shards), &h);
        if (!st->ok()) return nullptr;
        return std::unique_ptr<ReedSolomon>(new ReedSolomon(h));
    }
    ~ReedSolomon() { shmr_ec_free(h_); }
    ReedSolomon(const ReedSolomon&) = delete;
    ReedSolomon& operator=(const ReedSolomon&) = delete;

    size_t data_shard_count() const { return shmr_ec_data_shard_count(h_); }
    size_t parity_shard_count() const { return shmr_ec_parity_shard_count(h_); }
    size_t total_shard_count() const { return shmr_ec_total_shard_count(h_); }
    shmr_ec_t* handle() const { return h_; }

    // encode(&mut Vec<Vec<u8>>): shards[k..] overwritten with parity.
    EcStatus encode(std::vector<std::vector<uint8_t>>& shards) const {
        std::vector<uint8_t*> ptrs;
        std::vector<size_t> lens;
        for (auto& s : shards) {
            ptrs.push_back(s.data());
            lens.push_back(s.size());
        }
        return EcStatus{shmr_ec_encode(h_, ptrs.data(), lens.data(), ptrs.size())};
    }

    // reconstruct(&mut Vec<Option<Vec<u8>>>): None entries are allocated and filled.
    EcStatus reconstruct(std::vector<std::optional<std::vector<uint8_t>>>& shards) const {
        return reconstruct_inner(shards, false);
    }
    // reconstruct_data: only absent data shards are rebuilt; absent parity stays None.
    EcStatus reconstruct_data(std::vector<std::optional<std::vector<uint8_t>>>& shards) const {
        return reconstruct_inner(shards, true);
    }

    // In-place forms over caller buffers (the Block Cache layout: shard i at
    // shards[i], all `len` bytes).  encode writes shards[k..]; reconstruct
    // writes the absent shards (present[i] == 0) and needs every pointer valid.
    EcStatus encode_in_place(uint8_t* const* shards, size_t n, size_t len) const {
        std::vector<size_t> lens(n, len);
        return EcStatus{shmr_ec_encode(h_, shards, lens.data(), n)};
    }
    EcStatus reconstruct_in_place(uint8_t* const* shards, const uint8_t* present, size_t n, size_t len,
                                  bool data_only) const {
        std::vector<size_t> lens(n);
        for (size_t i = 0; i < n; ++i) lens[i] = present[i] ? len : 0;
        return EcStatus{shmr_ec_reconstruct(h_, shards, lens.data(), present, n, data_only)};
    }
    // The same, started: the GPU work may still run when they return (mapped
    // shards); op->wait() completes it.  Inputs may be read meanwhile.
    EcStatus encode_start(uint8_t* const* shards, size_t n, size_t len, EcOp* op) const {
        std::vector<size_t> lens(n, len);
        return EcStatus{shmr_ec_encode_start(h_, shards, lens.data(), n, op->out())};
    }
    EcStatus reconstruct_start(uint8_t* const* shards, const uint8_t* present, size_t n, size_t len, bool data_only,
                               EcOp* op) const {
        std::vector<size_t> lens(n);
        for (size_t i = 0; i < n; ++i) lens[i] = present[i] ? len : 0;
        return EcStatus{shmr_ec_reconstruct_start(h_, shards, lens.data(), present, n, data_only, op->out())};
    }

private:
    explicit ReedSolomon(shmr_ec_t* h) : h_(h) {}

    EcStatus reconstruct_inner(std::vector<std::optional<std::vector<uint8_t>>>& shards, bool data_only) const {
        const size_t k = data_shard_count();
        size_t len = 0;
        for (auto& s : shards)
            if (s && !s->empty()) {
                len = s->size();
                break;
            }
        std::vector<uint8_t> present(shards.size());
        std::vector<size_t> lens(shards.size(), 0);
        std::vector<std::vector<uint8_t>> scratch(shards.size());
        std::vector<uint8_t*> ptrs(shards.size(), nullptr);
        for (size_t i = 0; i < shards.size(); ++i) {
            if (shards[i]) {
                present[i] = 1;
                lens[i] = shards[i]->size();
                ptrs[i] = shards[i]->data();
            } else if (!(data_only && i >= k)) {
                scratch[i].assign(len, 0);   // the crate's get_or_initialize
                ptrs[i] = scratch[i].data();
            }
        }
        EcStatus st{shmr_ec_reconstruct(h_, ptrs.data(), lens.data(), present.data(), shards.size(), data_only)};
        if (!st.ok()) return st;
        bool any_absent = false;
        for (size_t i = 0; i < shards.size(); ++i) any_absent |= !present[i];
        if (!any_absent) return st;
        for (size_t i = 0; i < shards.size(); ++i)
            if (!present[i] && !(data_only && i >= k)) shards[i] = std::move(scratch[i]);
        return st;
    }

    shmr_ec_t* h_;
};

// calculate_shard_size (src/vfs/mod.rs:16-18)
inline size_t calculate_shard_size(uint64_t length, uint8_t data_shards) {
    return shmr_ec_shard_size(length, data_shards);
}

}  // namespace shmr
