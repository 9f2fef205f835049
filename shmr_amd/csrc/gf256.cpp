// Host-side GF(2^8) math for the MI355X erasure path.  See gf256.hpp.
#include "gf256.hpp"

#include <algorithm>
#include <cstring>


namespace shmr {
namespace gf {

namespace {
Tables make_tables() {
    Tables t{};
    unsigned b = 1;
    for (unsigned lg = 0; lg < 255; ++lg) {   // log table: successive powers of 2
        t.log[b] = uint8_t(lg);
        b <<= 1;
        if (b >= 256) b = (b - 256) ^ kPoly;
    }
    for (unsigned i = 1; i < 256; ++i) {      // exp table, doubled so log a + log b indexes directly
        t.exp[t.log[i]] = uint8_t(i);
        t.exp[t.log[i] + 255] = uint8_t(i);
    }
    for (unsigned a = 0; a < 256; ++a)
        for (unsigned c = 0; c < 256; ++c)
            t.mul[a][c] = (a && c) ? t.exp[t.log[a] + t.log[c]] : 0;
    return t;
}
}  // namespace

const Tables& tables() {
    static const Tables t = make_tables();
    return t;
}

uint8_t div(uint8_t a, uint8_t b) {
    if (a == 0) return 0;
    const Tables& t = tables();
    int lr = int(t.log[a]) - int(t.log[b]);
    if (lr < 0) lr += 255;
    return t.exp[lr];
}

uint8_t exp(uint8_t a, unsigned n) {
    if (n == 0) return 1;
    if (a == 0) return 0;
    unsigned lr = unsigned(tables().log[a]) * n;
    return tables().exp[lr % 255];
}

Matrix multiply(const Matrix& a, const Matrix& b) {
    Matrix out(a.rows, b.cols);
    for (unsigned r = 0; r < a.rows; ++r)
        for (unsigned i = 0; i < a.cols; ++i) {
            const uint8_t f = a.at(r, i);
            if (!f) continue;
            const uint8_t* mt = tables().mul[f];
            for (unsigned c = 0; c < b.cols; ++c) out.at(r, c) ^= mt[b.at(i, c)];
        }
    return out;
}

bool invert(const Matrix& m, Matrix* out) {
    const unsigned n = m.rows;
    Matrix w(n, 2 * n);
    for (unsigned r = 0; r < n; ++r) {
        std::memcpy(&w.at(r, 0), m.row(r), n);
        w.at(r, n + r) = 1;
    }
    for (unsigned r = 0; r < n; ++r) {
        if (w.at(r, r) == 0) {
            for (unsigned b = r + 1; b < n; ++b)
                if (w.at(b, r)) {
                    std::swap_ranges(&w.at(r, 0), &w.at(r, 0) + 2 * n, &w.at(b, 0));
                    break;
                }
        }
        if (w.at(r, r) == 0) return false;
        if (w.at(r, r) != 1) {
            const uint8_t* mt = tables().mul[div(1, w.at(r, r))];
            for (unsigned c = 0; c < 2 * n; ++c) w.at(r, c) = mt[w.at(r, c)];
        }
        for (unsigned o = 0; o < n; ++o) {
            if (o == r || !w.at(o, r)) continue;
            const uint8_t* mt = tables().mul[w.at(o, r)];
            for (unsigned c = 0; c < 2 * n; ++c) w.at(o, c) ^= mt[w.at(r, c)];
        }
    }
    *out = Matrix(n, n);
    for (unsigned r = 0; r < n; ++r) std::memcpy(&out->at(r, 0), &w.at(r, n), n);
    return true;
}

Matrix vandermonde(unsigned rows, unsigned cols) {
    Matrix v(rows, cols);
    for (unsigned r = 0; r < rows; ++r)
        for (unsigned c = 0; c < cols; ++c) v.at(r, c) = exp(uint8_t(r), c);
    return v;
}

Matrix build_matrix(unsigned k, unsigned total) {
    Matrix v = vandermonde(total, k);
    Matrix top(k, k);
    std::memcpy(top.d.data(), v.d.data(), size_t(k) * k);
    Matrix top_inv;
    invert(top, &top_inv);   // a Vandermonde top block with distinct nodes is invertible
    return multiply(v, top_inv);
}

PermTab perm_table(uint8_t c) {
    PermTab t{};
    const uint8_t* mt = tables().mul[c];
    uint8_t b[20];
    for (int x = 0; x < 8; ++x) b[x] = mt[x];
    for (int x = 0; x < 8; ++x) b[8 + x] = mt[x << 3];
    for (int x = 0; x < 4; ++x) b[16 + x] = mt[x << 6];
    std::memcpy(t.w, b, 20);
    return t;
}

std::vector<uint8_t> Plan::image(bool compact) const {
    // header: u32 k, u32 m, u16 in_idx[k], u16 out_idx[m], pad to 32 B
    size_t hdr = 8 + 2 * size_t(k) + 2 * size_t(m);
    hdr = (hdr + 31) & ~size_t(31);
    std::vector<uint8_t> img(hdr + sizeof(PermTab) * size_t(k) * m, 0);
    uint32_t km[2] = {k, m};
    std::memcpy(img.data(), km, 8);
    std::memcpy(img.data() + 8, in_idx.data(), 2 * size_t(k));
    std::vector<uint16_t> oi = out_idx;
    if (compact)
        for (unsigned j = 0; j < m; ++j) oi[j] = uint16_t(j);
    std::memcpy(img.data() + 8 + 2 * size_t(k), oi.data(), 2 * size_t(m));
    PermTab* tabs = reinterpret_cast<PermTab*>(img.data() + hdr);
    for (unsigned t = 0; t < k; ++t)
        for (unsigned r = 0; r < m; ++r) tabs[size_t(t) * m + r] = perm_table(rows.at(r, t));
    return img;
}

Codec::Codec(unsigned k, unsigned p) : k_(k), p_(p), matrix_(build_matrix(k, k + p)) {
    auto plan = std::make_shared<Plan>();
    plan->k = k;
    plan->m = p;
    plan->rows = Matrix(p, k);
    std::memcpy(plan->rows.d.data(), matrix_.row(k), size_t(p) * k);
    for (unsigned i = 0; i < k; ++i) plan->in_idx.push_back(uint16_t(i));
    for (unsigned r = 0; r < p; ++r) plan->out_idx.push_back(uint16_t(k + r));
    encode_plan_ = plan;
}

// Device plan images live in the per-device arenas of ec_core (process
// lifetime: a kernel may still read them when the last handle goes).
Codec::~Codec() = default;

std::shared_ptr<const Matrix> Codec::data_decode_matrix(const std::vector<uint16_t>& valid,
                                                        const std::vector<uint16_t>& invalid) {
    // caller holds mu_
    auto it = lru_index_.find(invalid);
    if (it != lru_index_.end()) {
        ++hits_;
        lru_.splice(lru_.begin(), lru_, it->second);
        return it->second->second;
    }
    ++misses_;
    Matrix sub(k_, k_);
    for (unsigned r = 0; r < k_; ++r) std::memcpy(&sub.at(r, 0), matrix_.row(valid[r]), k_);
    auto dec = std::make_shared<Matrix>();
    invert(sub, dec.get());   // rows of a systematic MDS matrix: always invertible
    lru_.emplace_front(invalid, dec);
    lru_index_[invalid] = lru_.begin();
    constexpr size_t kCap = 254;   // crate DATA_DECODE_MATRIX_CACHE_CAPACITY
    if (lru_.size() > kCap) {
        lru_index_.erase(lru_.back().first);
        lru_.pop_back();
    }
    return dec;
}

std::shared_ptr<Plan> Codec::reconstruct_plan(const std::vector<uint8_t>& present, bool data_only) {
    std::vector<uint8_t> key(present.size() + 1);
    for (size_t i = 0; i < present.size(); ++i) key[i] = present[i] ? 1 : 0;
    key.back() = data_only ? 1 : 0;
    std::lock_guard<std::mutex> lock(mu_);
    // valid = first k present shards in index order; invalid = all absent.
    std::vector<uint16_t> valid, invalid;
    for (unsigned i = 0; i < k_ + p_; ++i) {
        if (key[i]) {
            if (valid.size() < k_) valid.push_back(uint16_t(i));
        } else {
            invalid.push_back(uint16_t(i));
        }
    }
    // The LRU is consulted on every reconstruct, as in the crate.
    auto dec = data_decode_matrix(valid, invalid);
    auto found = plans_.find(key);
    if (found != plans_.end()) return found->second;

    auto plan = std::make_shared<Plan>();
    plan->k = k_;
    plan->in_idx = valid;
    std::vector<std::vector<uint8_t>> rows;
    for (uint16_t j : invalid) {
        if (j < k_) {
            plan->out_idx.push_back(j);
            rows.emplace_back(dec->row(j), dec->row(j) + k_);
        }
    }
    if (!data_only) {
        for (uint16_t j : invalid) {
            if (j < k_) continue;
            // parity row r applied to the rebuilt data = (M[j] * Dec) . sub_shards
            std::vector<uint8_t> row(k_, 0);
            for (unsigned d = 0; d < k_; ++d) {
                const uint8_t f = matrix_.at(j, d);
                if (!f) continue;
                for (unsigned t = 0; t < k_; ++t) row[t] ^= mul(f, dec->at(d, t));
            }
            plan->out_idx.push_back(j);
            rows.push_back(std::move(row));
        }
    }
    plan->m = unsigned(rows.size());
    plan->rows = Matrix(plan->m, k_);
    for (unsigned r = 0; r < plan->m; ++r) std::memcpy(&plan->rows.at(r, 0), rows[r].data(), k_);
    plans_[key] = plan;
    return plan;
}

std::shared_ptr<Codec> get_codec(unsigned k, unsigned p) {
    // Leaked on purpose: codecs own device images that must outlive every
    // in-flight kernel, and HIP may already be torn down at static exit.
    static std::mutex* mu = new std::mutex;
    static auto* reg = new std::map<std::pair<unsigned, unsigned>, std::shared_ptr<Codec>>;
    std::lock_guard<std::mutex> lock(*mu);
    auto& slot = (*reg)[{k, p}];
    if (!slot) slot = std::make_shared<Codec>(k, p);
    return slot;
}

}  // namespace gf
}  // namespace shmr
