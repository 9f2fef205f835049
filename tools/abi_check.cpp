// Stand-alone C-ABI round trip over mapped Block-Cache buffers (the shape of
// VirtualFile's batched load): encode B blocks, erase shards (one lost file
// and, every third block, one short file), reconstruct in batches of 3, check
// every shard.  Used to compare library builds (e.g. the host-sanitized one of
// tools/asan_host.sh) without the StorageBlock layer on top.
//
// Then the same blocks in device memory from shmr_ec_device_alloc_shards
// through pointer tables on a slot grid (encode; rebuild into a second slab).
//
//   hipcc -O1 -g -std=c++17 -Iinclude tools/abi_check.cpp -Lshmr_amd/_lib -lshmr_ec -o tools/_bin/abi_check
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "shmr_ec.h"

// GF(2^8), polynomial 0x11D (the crate's field): parity check of the encode.
static uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t r = 0;
    while (b) {
        if (b & 1) r ^= a;
        a = uint8_t((a << 1) ^ ((a & 0x80) ? 0x1D : 0));
        b >>= 1;
    }
    return r;
}

static size_t parity_errors(const std::vector<uint8_t>& M, unsigned k, unsigned p, uint8_t* const* sh, size_t S) {
    size_t bad = 0;
    for (unsigned r = 0; r < p; ++r)
        for (size_t o = 0; o < S; ++o) {
            uint8_t v = 0;
            for (unsigned i = 0; i < k; ++i) v ^= gmul(M[(k + r) * k + i], sh[i][o]);
            bad += v != sh[k + r][o];
        }
    return bad;
}

int main(int argc, char** argv) {
    const unsigned k = 8, p = 3, t = k + p;
    const size_t S = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 131072;
    const size_t B = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 12;
    shmr_ec_t* rs = nullptr;
    if (shmr_ec_new(k, p, &rs)) return 2;
    std::vector<uint8_t*> bufs(B);
    for (size_t b = 0; b < B; ++b) {
        void* q = nullptr;
        int rc = shmr_ec_host_alloc(t * S, &q);
        if (rc) {
            std::printf("host_alloc: %s\n", shmr_ec_status_name(rc));
            return 1;
        }
        bufs[b] = static_cast<uint8_t*>(q);
    }
    std::mt19937_64 rng(7);
    std::vector<uint8_t*> ptrs(B * t);
    for (size_t b = 0; b < B; ++b)
        for (unsigned i = 0; i < t; ++i) {
            ptrs[b * t + i] = bufs[b] + i * S;
            if (i < k)
                for (size_t o = 0; o < S; ++o) ptrs[b * t + i][o] = uint8_t(rng());
        }
    int dev = 0;
    int rc = shmr_ec_encode_blocks_host(rs, ptrs.data(), B, S, &dev, 1);
    uint64_t zc = 0, st = 0;
    shmr_ec_path_stats(&zc, &st);
    std::printf("encode: %s (zero_copy %llu staged %llu)\n", shmr_ec_status_name(rc), (unsigned long long)zc,
                (unsigned long long)st);
    std::vector<uint8_t> M(size_t(t) * k);
    shmr_ec_matrix(rs, M.data(), M.size());
    size_t pbad = 0;
    for (size_t b = 0; b < B; ++b) pbad += parity_errors(M, k, p, ptrs.data() + b * t, S);
    std::printf("encode parity vs CPU field arithmetic: %zu bytes wrong\n", pbad);
    {   // pageable single block (bounce path) and device-resident check of the same block
        std::vector<std::vector<uint8_t>> pg(t, std::vector<uint8_t>(S, 0));
        std::vector<uint8_t*> pp(t);
        std::vector<size_t> lens(t, S);
        for (unsigned i = 0; i < t; ++i) {
            if (i < k) std::memcpy(pg[i].data(), ptrs[i], S);
            pp[i] = pg[i].data();
        }
        rc = shmr_ec_encode(rs, pp.data(), lens.data(), t);
        std::printf("pageable shmr_ec_encode: %s, parity wrong bytes %zu\n", shmr_ec_status_name(rc),
                    parity_errors(M, k, p, pp.data(), S));
    }
    std::vector<std::vector<uint8_t>> want(B * t);
    for (size_t q = 0; q < B * t; ++q) want[q].assign(ptrs[q], ptrs[q] + S);
    std::vector<uint8_t> present(B * t, 1);
    for (size_t b = 0; b < B; ++b) {
        const unsigned lost = unsigned(b % t);
        present[b * t + lost] = 0;
        std::memset(ptrs[b * t + lost], 0, S);
        if (b % 3 == 0) {
            const unsigned sh = unsigned((b + 5) % t);
            present[b * t + sh] = 0;
            std::memset(ptrs[b * t + sh] + 100, 0, S - 100);
        }
    }
    int bad = pbad ? 1 : 0;
    for (size_t b0 = 0; b0 < B; b0 += 3) {
        const size_t n = std::min<size_t>(3, B - b0);
        rc = shmr_ec_reconstruct_blocks_host(rs, ptrs.data() + b0 * t, present.data() + b0 * t, n, S, 0, &dev, 1);
        if (rc) std::printf("reconstruct [%zu, %zu): %s\n", b0, b0 + n, shmr_ec_status_name(rc));
    }
    shmr_ec_path_stats(&zc, &st);
    std::printf("after reconstruct: zero_copy %llu staged %llu\n", (unsigned long long)zc, (unsigned long long)st);
    for (size_t q = 0; q < B * t; ++q)
        if (std::memcmp(ptrs[q], want[q].data(), S) != 0) {
            std::printf("MISMATCH block %zu shard %zu (present %d)\n", q / t, q % t, int(present[q]));
            ++bad;
        }
    {   // device-resident slab buffers, pointer tables on a slot grid
        std::vector<uint8_t*> dp(B * t), outs(B * 2);
        rc = shmr_ec_device_alloc_shards(0, B, t, S, dp.data());
        if (!rc) rc = shmr_ec_device_alloc_shards(0, B, 2, S, outs.data());
        if (rc) {
            std::printf("device_alloc_shards: %s\n", shmr_ec_status_name(rc));
            return 1;
        }
        for (size_t q = 0; q < B * t; ++q)
            if (hipMemcpy(dp[q], want[q].data(), (q % t) < k ? S : 0, hipMemcpyHostToDevice) != hipSuccess) return 1;
        uint64_t g0[SHMR_EC_DEV_COUNTERS] = {}, g1[SHMR_EC_DEV_COUNTERS] = {};
        shmr_ec_device_stats(0, g0, SHMR_EC_DEV_COUNTERS);
        rc = shmr_ec_encode_ptrs_dev(rs, dp.data(), B, S, 0, nullptr);
        std::vector<uint8_t*> tab(dp);
        for (size_t b = 0; b < B; ++b) {   // absent shards -> the b-th row of the output slab
            unsigned j = 0;
            for (unsigned i = 0; i < t; ++i)
                if (!present[b * t + i]) tab[b * t + i] = outs[b * 2 + j++];
        }
        if (!rc) rc = shmr_ec_reconstruct_ptrs_dev(rs, tab.data(), present.data(), B, S, 0, 0, nullptr);
        if (hipDeviceSynchronize() != hipSuccess) return 1;
        shmr_ec_device_stats(0, g1, SHMR_EC_DEV_COUNTERS);
        std::printf("slab grid calls: %s, grid calls %llu\n", shmr_ec_status_name(rc),
                    (unsigned long long)(g1[SHMR_EC_DEV_PTR_TABLE_GRIDS] - g0[SHMR_EC_DEV_PTR_TABLE_GRIDS]));
        if (rc || g1[SHMR_EC_DEV_PTR_TABLE_GRIDS] - g0[SHMR_EC_DEV_PTR_TABLE_GRIDS] != 2) ++bad;
        std::vector<uint8_t> h(S);
        for (size_t q = 0; q < B * t; ++q) {
            if (hipMemcpy(h.data(), tab[q], S, hipMemcpyDeviceToHost) != hipSuccess) return 1;
            if (std::memcmp(h.data(), want[q].data(), S) != 0) {
                std::printf("SLAB MISMATCH block %zu shard %zu (present %d)\n", q / t, q % t, int(present[q]));
                ++bad;
            }
        }
        if (shmr_ec_device_free_shards(0, dp[1]) != SHMR_EC_INVALID_ARGUMENT) ++bad;   // not a slab base
        if (shmr_ec_device_free_shards(0, dp[0]) || shmr_ec_device_free_shards(0, outs[0])) ++bad;
    }
    for (auto* q : bufs) shmr_ec_host_free(q);
    shmr_ec_free(rs);
    std::printf(bad ? "FAIL\n" : "PASS\n");
    return bad ? 1 : 0;
}
