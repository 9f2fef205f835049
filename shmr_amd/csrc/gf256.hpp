// GF(2^8) field, coding matrices and decode plans -- host side of the
// MI355X erasure path.
//
// Semantics follow the arithmetic that the reference delegates to
// reed-solomon-erasure 6.0.0 (reference Cargo.toml:16, Cargo.lock:1577-1589),
// called from src/vfs/block.rs:405,427 (new/encode) and :531,560
// (new/reconstruct).  Restated, not vendored: the crate is not in the
// reference tree.
#pragma once

#include <cstddef>
#include <cstdint>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace shmr {
namespace gf {

// x^8 + x^4 + x^3 + x^2 + 1 (the crate's GENERATING_POLYNOMIAL 29), generator 2.
constexpr unsigned kPoly = 29;

struct Tables {
    uint8_t log[256];
    uint8_t exp[510];
    uint8_t mul[256][256];
};
const Tables& tables();

inline uint8_t mul(uint8_t a, uint8_t b) { return tables().mul[a][b]; }
uint8_t div(uint8_t a, uint8_t b);      // b != 0
uint8_t exp(uint8_t a, unsigned n);     // a^n, 0^0 == 1

// Row-major dense matrix over GF(2^8).
struct Matrix {
    unsigned rows = 0, cols = 0;
    std::vector<uint8_t> d;
    Matrix() = default;
    Matrix(unsigned r, unsigned c) : rows(r), cols(c), d(size_t(r) * c, 0) {}
    uint8_t& at(unsigned r, unsigned c) { return d[size_t(r) * cols + c]; }
    uint8_t at(unsigned r, unsigned c) const { return d[size_t(r) * cols + c]; }
    const uint8_t* row(unsigned r) const { return d.data() + size_t(r) * cols; }
};

Matrix multiply(const Matrix& a, const Matrix& b);
bool invert(const Matrix& m, Matrix* out);          // false when singular
Matrix vandermonde(unsigned rows, unsigned cols);    // V[r][c] = r^c
Matrix build_matrix(unsigned k, unsigned total);     // V * inv(V[0..k])

// ---------------------------------------------------------------------------
// Kernel coefficient tables.  GF multiplication by a constant is linear over
// GF(2), so c (x) b = T0[b & 7] ^ T1[(b >> 3) & 7] ^ T2[b >> 6].  Each table
// fits the 8-byte source window of one v_perm_b32, so a byte lookup for four
// byte lanes costs one VALU op per table.  One entry = 8 dwords (padded for
// two ds_read_b128):
//   w[0] = T0[0..3]  w[1] = T0[4..7]
//   w[2] = T1[0..3]  w[3] = T1[4..7]
//   w[4] = T2[0..3]  w[5..7] = 0
// ---------------------------------------------------------------------------
struct alignas(32) PermTab {
    uint32_t w[8];
};
PermTab perm_table(uint8_t c);

// A decode/encode "plan": out[m] = XOR_t rows[m][t] (x) in[t], where in[t] is
// shard in_idx[t] of the block and out[m] is shard out_idx[m].
struct Plan {
    unsigned k = 0;                 // inputs
    unsigned m = 0;                 // outputs
    std::vector<uint16_t> in_idx;   // size k
    std::vector<uint16_t> out_idx;  // size m
    Matrix rows;                    // m x k
    // Device image: [u32 k][u32 m][u16 in_idx[k]][u16 out_idx[m]] padded to
    // 32 B, then PermTab[k][m] (input-major so one shard's rows are contiguous
    // for the kernel).  compact: out_idx[j] = j, i.e. output j goes to slot j
    // of a separate output array (the rebuilt shards in index order) instead
    // of its shard's own slot.
    std::vector<uint8_t> image(bool compact = false) const;
    // Per (device ID, compact) the core's upload record (ec_core PlanDev,
    // arena memory that lives as long as the process: in-flight kernels).
    std::mutex dev_mu;
    std::map<int, void*> dev_image;
};

// One codec per (k, p): matrix, encode plan and the crate's decode-matrix LRU.
class Codec {
public:
    Codec(unsigned k, unsigned p);
    ~Codec();
    unsigned k() const { return k_; }
    unsigned p() const { return p_; }
    const Matrix& matrix() const { return matrix_; }
    std::shared_ptr<Plan> encode_plan() const { return encode_plan_; }

    // Crate get_data_decode_matrix: inverse of the rows of `valid`,
    // LRU-cached (capacity 254) keyed by `invalid`.
    std::shared_ptr<const Matrix> data_decode_matrix(const std::vector<uint16_t>& valid,
                                                     const std::vector<uint16_t>& invalid);

    // Full reconstruct plan for a presence pattern (present.size() == k+p,
    // at least k present, not all present).  Missing data rows are
    // Dec[j]; missing parity rows are M[k+r] * Dec (identical to the crate's
    // "rebuild data, then re-encode parity" for any input, because Dec
    // maps the sub-shards to the data shards exactly).  Cached per pattern.
    std::shared_ptr<Plan> reconstruct_plan(const std::vector<uint8_t>& present, bool data_only);

    uint64_t decode_cache_hits() const { return hits_; }
    uint64_t decode_cache_misses() const { return misses_; }

private:
    unsigned k_, p_;
    Matrix matrix_;
    std::shared_ptr<Plan> encode_plan_;

    std::mutex mu_;
    // LRU of decode matrices (crate semantics), key = invalid indices.
    using Key = std::vector<uint16_t>;
    std::list<std::pair<Key, std::shared_ptr<const Matrix>>> lru_;
    std::map<Key, decltype(lru_)::iterator> lru_index_;
    // Plans keyed by (presence bitmap, data_only).  Plans own device images,
    // so they are kept for the codec lifetime.
    std::map<std::vector<uint8_t>, std::shared_ptr<Plan>> plans_;
    uint64_t hits_ = 0, misses_ = 0;
};

// Process-wide codec registry: codecs are immutable apart from their caches
// and are shared by every shmr_ec_t of the same (k, p).
std::shared_ptr<Codec> get_codec(unsigned k, unsigned p);

}  // namespace gf
}  // namespace shmr
