// Test driver for the C++ StorageBlock mirror (vfs.hpp).  Each case mirrors a
// test of the reference (src/vfs/block.rs:647-812, src/vfs/mod.rs:322-370) or
// exercises the MI355X Erasure arms.  Run by tests/test_host_cpp.py:
//
//   shmr_vfs_test <case> <bucket_dir> [input_file]
//
// Prints "PASS" and exits 0, or prints "FAIL: ..." and exits 1.  Erasure cases
// also print one "SHARDS <block> <path>..." line per block so the Python side
// can compare the shard files with the CPU oracle.
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <random>

#include "vfs.hpp"

using namespace shmr;

namespace {

struct Failure {
    std::string msg;
};

static std::string diff_report(const std::vector<uint8_t>& a, const std::vector<uint8_t>& b, size_t bs, size_t S) {
    std::string r;
    if (a.size() != b.size()) return ": sizes " + std::to_string(a.size()) + " vs " + std::to_string(b.size());
    for (size_t blk = 0; blk * bs < a.size(); ++blk) {
        size_t nd = 0, first = SIZE_MAX;
        for (size_t o = blk * bs; o < std::min(a.size(), (blk + 1) * bs); ++o)
            if (a[o] != b[o]) {
                ++nd;
                if (first == SIZE_MAX) first = o - blk * bs;
            }
        if (nd)
            r += "\n  block " + std::to_string(blk) + ": " + std::to_string(nd) + " bytes differ, first at " +
                 std::to_string(first) + " (shard " + std::to_string(first / S) + " + " + std::to_string(first % S) + ")";
    }
    return r;
}

#define CHECK(cond)                                                                     \
    do {                                                                                \
        if (!(cond)) throw Failure{std::string(#cond) + " (line " + std::to_string(__LINE__) + ")"}; \
    } while (0)
// Equality with a diagnostic: per block of bs bytes, the number of differing
// bytes and the first differing offset (and its shard of size S).
#define CHECK_SAME(a, b, bs, S)                                                          \
    do {                                                                                \
        if ((a) != (b)) throw Failure{std::string(#a " == " #b) + " (line " + std::to_string(__LINE__) + ")" + \
                                      diff_report(a, b, bs, S)};                       \
    } while (0)
#define CHECK_OK(st)                                                                    \
    do {                                                                                \
        Status _s = (st);                                                               \
        if (_s) throw Failure{std::string(#st) + " -> " + _s->what() + " (line " + std::to_string(__LINE__) + ")"}; \
    } while (0)

std::string g_bucket;
std::string g_input;
std::mt19937_64 g_rng(0x53484D52);

// get_shmr_config (src/lib.rs tests): one bucket "bucket1" in pool "test_pool".
std::shared_ptr<const ShmrFsConfig> test_config() {
    auto cfg = std::make_shared<ShmrFsConfig>();
    Bucket b;
    b.path = g_bucket;
    b.capacity = 999;
    b.available = 999;
    cfg->pools["test_pool"]["bucket1"] = b;
    cfg->write_pool = "test_pool";
    return cfg;
}

std::vector<uint8_t> random_data(size_t n) {   // config.rs random_data
    std::vector<uint8_t> v(n);
    for (auto& x : v) x = uint8_t(g_rng());
    return v;
}

std::vector<uint8_t> read_input() {
    std::ifstream f(g_input, std::ios::binary);
    return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

fs::path shard_file(const ShmrFsConfig& cfg, const VirtualBlock& b, size_t i) {
    fs::path p;
    CHECK_OK(b.shards[i].resolve(cfg, &p, nullptr));
    return p;
}

uint64_t fsize(const fs::path& p) { return fs::file_size(p); }

std::vector<uint8_t> read_file(const fs::path& p, size_t n) {
    std::vector<uint8_t> v(n);
    FILE* f = std::fopen(p.c_str(), "rb");
    CHECK(f != nullptr);
    const size_t got = std::fread(v.data(), 1, n, f);
    std::fclose(f);
    CHECK(got == n);   // read_exact
    return v;
}

void print_shards(const ShmrFsConfig& cfg, size_t idx, const VirtualBlock& b) {
    std::printf("SHARDS %zu", idx);
    for (size_t i = 0; i < b.shards.size(); ++i) std::printf(" %s", shard_file(cfg, b, i).c_str());
    std::printf("\n");
}

// ---- reference tests -------------------------------------------------------

void test_block_topology_try_from() {   // block.rs:647-659
    auto t = BlockTopology::try_from("Erasure(1, 3, 2)");
    CHECK(t && t->kind == BlockTopology::Erasure && t->version == 1 && t->data == 3 && t->parity == 2);
    auto m = BlockTopology::try_from("Mirror(3)");
    CHECK(m && m->kind == BlockTopology::Mirror && m->n == 3);
    auto s = BlockTopology::try_from("Single()");
    CHECK(s && s->kind == BlockTopology::Single);
    std::string err;
    CHECK(!BlockTopology::try_from("Single", &err) && err == "'Single' does not have '('");
    CHECK(!BlockTopology::try_from("Erasure(1, x, 2)", &err) && err == "Unable to parse data shards");
    CHECK(!BlockTopology::try_from("Raid(5)", &err));
    CHECK(BlockTopology::erasure(1, 8, 3).to_string() == "Erasure(1, 8, 3)");
    auto rt = BlockTopology::try_from(BlockTopology::erasure(1, 8, 3).to_string());
    CHECK(rt && rt->data == 8 && rt->parity == 3);
    auto e104 = BlockTopology::try_from("Erasure(1,10,4)");
    CHECK(e104 && e104->kind == BlockTopology::Erasure && e104->data == 10 && e104->parity == 4);
    CHECK(BlockTopology::mirror(2).to_string() == "Mirror(2)" && BlockTopology::single().to_string() == "Single");
    auto m3 = BlockTopology::try_from(BlockTopology::mirror(3).to_string());
    CHECK(m3 && m3->kind == BlockTopology::Mirror && m3->n == 3);
    // Display "Single" does not parse back (block.rs:57-59); missing or non-u8 fields fail
    for (const char* bad : {"Single", "Erasure(1, 8)", "Erasure(x, 8, 3)", "Erasure(1, 8, 300)", "Mirror(a)"})
        CHECK(!BlockTopology::try_from(bad));
    // random strings from the parser's alphabet: no crash, and whatever
    // parses (other than Single) re-parses from its Display form unchanged
    std::mt19937_64 rng(77);
    const std::string al = "SingleMirorEasu(), 0123456789 -+x";
    for (int it = 0; it < 20000; ++it) {
        std::string t;
        const size_t n = rng() % 24;
        for (size_t i = 0; i < n; ++i) t += al[rng() % al.size()];
        if (rng() % 3 == 0) t = std::string(rng() % 2 ? "Erasure(" : "Mirror(") + t;
        auto r = BlockTopology::try_from(t);
        if (r && r->kind != BlockTopology::Single) {
            auto again = BlockTopology::try_from(r->to_string());
            CHECK(again && again->to_string() == r->to_string());
        }
    }
}

void test_virtual_block_new_block() {   // block.rs:661-675
    auto cfg = test_config();
    VirtualBlock b;
    CHECK_OK(VirtualBlock::create(1, 0, cfg, 1024, BlockTopology::single(), &b));
    for (size_t i = 0; i < b.shards.size(); ++i) CHECK(fs::exists(shard_file(*cfg, b, i)));
    CHECK(b.shards[0].filename == "1:0_single_0.bin");
    fs::path dir;
    CHECK_OK(b.shards[0].resolve(*cfg, nullptr, &dir));
    CHECK(fs::is_directory(dir));   // <bucket>/1:/0_ is created (unused by the file)
}

void unbuffered_common(bool read_back) {   // block.rs:677-744
    auto cfg = test_config();
    VirtualBlock b;
    CHECK_OK(VirtualBlock::create(3, 0, cfg, 1024, BlockTopology::single(), &b));
    const fs::path sp = shard_file(*cfg, b, 0);
    auto data = random_data(500);
    size_t n = 0;
    CHECK_OK(b.write(0, data.data(), data.size(), &n));
    CHECK(n == 500);
    CHECK_OK(b.sync_data(true));
    CHECK(fsize(sp) == data.size());
    CHECK_OK(b.drop_buffer());
    CHECK(!b.buffer_loaded());
    CHECK(b.buffer_snapshot().empty());
    if (!read_back) {
        CHECK(read_file(sp, 500) == data);
        return;
    }
    std::vector<uint8_t> rb(500);
    CHECK_OK(b.read(0, rb.data(), rb.size(), &n));
    CHECK(n == 500);
    CHECK(rb == data);
}

void test_virtual_block_unbuffered_backing() { unbuffered_common(false); }
void test_virtual_block_unbuffered() { unbuffered_common(true); }

void test_virtual_block_buffered() {   // block.rs:746-797
    auto cfg = test_config();
    VirtualBlock b;
    CHECK_OK(VirtualBlock::create(5, 0, cfg, 1024, BlockTopology::single(), &b));
    const fs::path sp = shard_file(*cfg, b, 0);
    auto data = random_data(420);
    size_t n = 0;
    CHECK_OK(b.write(0, data.data(), data.size(), &n));
    CHECK(fsize(sp) == 0);
    {
        auto buf = b.buffer_snapshot();
        CHECK(buf.size() == data.size());
        CHECK(std::equal(data.begin(), data.end(), buf.begin()));
    }
    std::vector<uint8_t> rb(data.size());
    CHECK_OK(b.read(0, rb.data(), rb.size(), &n));
    CHECK(n == data.size());
    auto data2 = random_data(420);
    CHECK_OK(b.write(0, data2.data(), data2.size(), &n));
    CHECK_OK(b.read(0, rb.data(), rb.size(), &n));
    CHECK(rb == data2);
    CHECK(fsize(sp) == 0);
    CHECK_OK(b.sync_data(true));
    CHECK(read_file(sp, 420) == data2);
    CHECK(fsize(sp) == 1024);   // load_block grew the buffer to `size` before the flush
}

void test_virtual_block_erasure_buffered() {   // block.rs:799-811 (a Single block there too)
    auto cfg = test_config();
    VirtualBlock b;
    CHECK_OK(VirtualBlock::create(7, 0, cfg, 1024, BlockTopology::single(), &b));
    auto data = random_data(500);
    size_t n = 0;
    CHECK_OK(b.write(0, data.data(), data.size(), &n));
    std::vector<uint8_t> rb(250);
    CHECK_OK(b.read(0, rb.data(), rb.size(), &n));
    CHECK(std::equal(rb.begin(), rb.end(), data.begin()));
}

void test_block_errors() {
    auto cfg = test_config();
    VirtualBlock b;
    CHECK_OK(VirtualBlock::create(9, 0, cfg, 1024, BlockTopology::single(), &b));
    std::vector<uint8_t> buf(2048);
    size_t n = 0;
    Status st = b.write(1000, buf.data(), 100, &n);   // pos + len > size
    CHECK(st && st->kind == ShmrError::OutOfSpace);
    CHECK_OK(b.read(0, buf.data(), 0, &n));            // zero-length read: Ok(0), nothing loaded
    CHECK(n == 0 && !b.buffer_loaded());
    Status sp = VirtualBlock::create(9, 1, cfg, 1024, BlockTopology::single(), &b);
    CHECK(!sp);
    VirtualBlock bad;
    st = VirtualBlock::create_with_pool(9, 2, "nope", cfg, 1024, BlockTopology::single(), &bad);
    CHECK(st && st->kind == ShmrError::InvalidPoolId);
    // select_buckets repeats the single bucket for every shard
    VirtualBlock ec;
    CHECK_OK(VirtualBlock::create(9, 3, cfg, 1024, BlockTopology::erasure(1, 4, 2), &ec));
    CHECK(ec.shards.size() == 6 && ec.shards[5].filename == "9:3_ec42_5.bin");
    // no GPU work: an Erasure block with an empty buffer flushes nothing
    CHECK_OK(ec.sync_data(true));
    CHECK(fsize(shard_file(*cfg, ec, 0)) == 0);
}

// calculate_shard_size's f32 hazard (mod.rs:16-18): 16,777,217 / 8 rounds to
// S = 2,097,152, so a full buffer splits into 9 chunks and block.rs:421's
// `data - nchunks` underflows u8 (panic in debug, a data chunk overwritten by
// parity in release).  The mirror refuses before any GPU work or shard write.
void test_erasure_f32_hazard() {
    auto cfg = test_config();
    const uint64_t size = 16777217;
    VirtualBlock b;
    CHECK_OK(VirtualBlock::create(11, 0, cfg, size, BlockTopology::erasure(1, 8, 3), &b));
    CHECK(calculate_shard_size(size, 8) == 2097152 && calculate_shard_size(size, 8) * 8 < size);
    std::vector<uint8_t> buf(size, 0x5a);
    size_t n = 0;
    CHECK_OK(b.write(0, buf.data(), buf.size(), &n));
    CHECK(n == size);
    Status st = b.sync_data(true);
    CHECK(st && st->kind == ShmrError::EcError && st->code == SHMR_EC_TOO_MANY_DATA_SHARDS);
    CHECK(fsize(shard_file(*cfg, b, 0)) == 0 && fsize(shard_file(*cfg, b, 10)) == 0);
}

// VfsOptions::release_u8_wrap: the same hazard with the reference's release
// build reproduced (block.rs:421 wraps, Cargo.toml:10-13) on both flush paths
// -- VirtualBlock::sync_data (block 0) and a batched VirtualFile::sync_data
// (block 1).  Shard files and the reloaded block are compared with the oracle
// (sync_data_erasure / load_block_erasure, mode "release") by the Python side;
// here: the Block Cache buffer still holds the caller's data after the flush
// (the reference encoded chunks().to_vec() copies).
void test_erasure_f32_hazard_release() {
    auto cfg = test_config();
    auto in = read_input();
    const uint64_t size = 16777217;
    CHECK(in.size() == size);
    VfsOptions o;
    o.release_u8_wrap = true;
    o.fsync_shards = false;
    VirtualBlock b;
    CHECK_OK(VirtualBlock::create(15, 0, cfg, size, BlockTopology::erasure(1, 8, 3), &b));
    b.set_options(o);
    size_t n = 0;
    CHECK_OK(b.write(0, in.data(), in.size(), &n));
    CHECK_OK(b.sync_data(true));
    CHECK(b.buffer_snapshot() == in);
    print_shards(*cfg, 0, b);
    CHECK_OK(b.drop_buffer());
    CHECK_OK(b.drop_handles());
    std::vector<uint8_t> rb(size);
    CHECK_OK(b.read(0, rb.data(), rb.size(), &n));
    CHECK(n == size);
    FILE* f = std::fopen((g_bucket + "/loaded_release.bin").c_str(), "wb");
    std::fwrite(rb.data(), 1, rb.size(), f);
    std::fclose(f);

    VirtualFile vf = VirtualFile::new_with(16, 0);
    vf.populate(cfg);
    vf.pipeline_batch_bytes = 0;   // the batched (shmr_ec_encode_blocks_host) flush
    VirtualBlock c;
    CHECK_OK(VirtualBlock::create(16, 0, cfg, size, BlockTopology::erasure(1, 8, 3), &c));
    vf.blocks.push_back(c);
    vf.set_options(o);
    CHECK_OK(vf.blocks[0].write(0, in.data(), in.size(), &n));
    CHECK_OK(vf.sync_data(true));
    CHECK(vf.last_sync.blocks == 1);
    CHECK(vf.blocks[0].buffer_snapshot() == in);
    print_shards(*cfg, 1, vf.blocks[0]);
}

void test_virtual_file_1() {   // mod.rs:322-349
    auto cfg = test_config();
    VirtualFile vf = VirtualFile::new_with(g_rng() >> 16, 0);
    vf.populate(cfg);
    auto data = random_data(7000);
    size_t n = 0;
    CHECK_OK(vf.write(0, data.data(), data.size(), &n));
    CHECK(n == 7000);
    CHECK(vf.size == 7000);
    CHECK(vf.blocks.size() == 1);
    for (size_t i = 0; i < vf.blocks.size(); ++i) {
        std::vector<uint8_t> buf(vf.chunk_size);
        CHECK_OK(vf.blocks[i].read(0, buf.data(), buf.size(), &n));
        CHECK(n == vf.chunk_size);
        const size_t s = i * vf.chunk_size, e = std::min<size_t>(s + vf.chunk_size, data.size());
        CHECK(std::equal(buf.begin(), buf.end(), data.begin() + s) && e - s == buf.size());
    }
    std::vector<uint8_t> buf(7000);
    CHECK_OK(vf.read(0, buf.data(), buf.size(), &n));
    CHECK(n == 7000);
    CHECK(buf == data);
}

void test_virtual_file_2_4_mb() {   // mod.rs:351-370
    auto cfg = test_config();
    VirtualFile vf = VirtualFile::new_with(g_rng() >> 16, 0);
    vf.populate(cfg);
    auto data = random_data(2 * 1024 * 1024);
    size_t n = 0;
    CHECK_OK(vf.write(0, data.data(), data.size(), &n));
    CHECK(vf.size == 2 * 1024 * 1024);
    CHECK(vf.blocks.size() == 3);   // the trailing empty chunk allocates a third block
    CHECK_OK(vf.sync_data(true));
    auto f = read_file(shard_file(*cfg, vf.blocks[0], 0), 1024 * 1024);
    CHECK(std::equal(f.begin(), f.end(), data.begin()));
}

// The reference's chunk loops (mod.rs:137-242), restated literally over a
// plain model of Single blocks that are never flushed: random writes and reads
// (unaligned positions, partial buffers, short reads) must leave the same
// bytes and return the same counts as VirtualFile's merged-run copies.
struct ChunkModel {
    uint64_t chunk = VFS_DEFAULT_BLOCK_SIZE, bs;
    std::vector<std::vector<uint8_t>> buf;
    std::vector<bool> loaded;
    uint64_t size = 0;
    explicit ChunkModel(uint64_t block_size) : bs(block_size) {}
    bool write(uint64_t pos, const uint8_t* d, size_t len, size_t* out) {
        *out = 0;
        if (len == 0) return true;
        const uint64_t sc = pos / chunk, ec = len / chunk + sc, per = bs / chunk;
        size_t w = 0;
        for (uint64_t c = sc; c <= ec; ++c) {
            while (buf.size() * per <= c) {
                buf.emplace_back();
                loaded.push_back(false);
            }
            const uint64_t b = c * chunk / bs, bp = c * chunk % bs;
            const size_t end = size_t(std::min<uint64_t>(w + chunk, len));
            if (bp + (end - w) > bs) return false;   // OutOfSpace
            if (buf[b].size() < bp + (end - w)) buf[b].resize(bp + (end - w), 0);
            std::memcpy(buf[b].data() + bp, d + w, end - w);
            w = end;
        }
        size = std::max<uint64_t>(size, pos + len);
        *out = w;
        return true;
    }
    bool read(uint64_t pos, uint8_t* d, size_t len, size_t* out) {
        *out = 0;
        if (len == 0 || size == 0) return true;
        if (pos > size) return false;   // EndOfFile
        const uint64_t sc = pos / chunk, ec = len / chunk + sc;
        size_t r = 0;
        for (uint64_t c = sc; c <= ec; ++c) {
            const uint64_t b = c * chunk / bs, bp = c * chunk % bs;
            const size_t end = size_t(std::min<uint64_t>(r + chunk, len));
            if (b >= buf.size()) return false;
            if (end == r) continue;   // VirtualBlock::read of 0 bytes: Ok(0), no load
            if (!loaded[b]) {   // load_block: resize to size; the empty shard file reads 0 bytes
                if (buf[b].size() < bs) buf[b].resize(bs, 0);
                loaded[b] = true;
            }
            if (buf[b].size() < bp) return false;   // OutOfSpace
            const size_t n = std::min<size_t>(buf[b].size() - bp, end - r);
            std::memcpy(d + r, buf[b].data() + bp, n);
            r += n;
        }
        *out = r;
        return true;
    }
};

void test_virtual_file_chunk_model() {
    auto cfg = test_config();
    for (int trial = 0; trial < 6; ++trial) {
        // trials 4-5: 4 MiB blocks and multi-MiB copies at odd offsets
        const bool big = trial >= 4;
        const uint64_t bs = big ? 4 << 20 : trial % 2 ? 64 * 1024 : 16 * 1024;
        VirtualFile vf = VirtualFile::new_with(40 + trial, 0);
        vf.populate(cfg);
        vf.block_size = bs;
        ChunkModel m(bs);
        std::mt19937_64 rng(777 + trial);
        for (int op = 0; op < (big ? 24 : 300); ++op) {
            const bool is_write = vf.blocks.empty() || rng() % 3 != 0;
            const uint64_t span = vf.blocks.size() * bs + 2 * bs;
            uint64_t pos = rng() % span;
            if (rng() % 4 == 0) pos -= pos % VFS_DEFAULT_BLOCK_SIZE;
            size_t len = size_t(rng() % (3 * bs));
            if (rng() % 5 == 0) len = size_t(rng() % 5000);
            if (is_write) {
                auto d = random_data(len);
                size_t a = 0, b = 0;
                const bool okm = m.write(pos, d.data(), len, &b);
                Status st = vf.write(pos, d.data(), len, &a);
                CHECK(okm == !st);
                if (!okm) break;   // both stopped mid-file; states may differ only past the failure
                CHECK(a == b && vf.size == m.size && vf.blocks.size() == m.buf.size());
            } else {
                std::vector<uint8_t> x(len, 0xEE), y(len, 0xEE);
                size_t a = 0, b = 0;
                const bool okm = m.read(pos, y.data(), len, &b);
                Status st = vf.read(pos, x.data(), len, &a);
                CHECK(okm == !st);
                if (okm) CHECK(a == b && x == y);
            }
        }
        for (size_t i = 0; i < m.buf.size(); ++i) CHECK(vf.blocks[i].buffer_snapshot() == m.buf[i]);
    }
}

void test_virtual_file_errors() {
    auto cfg = test_config();
    VirtualFile vf = VirtualFile::new_with(77, 0);
    size_t n = 0;
    std::vector<uint8_t> buf(16);
    Status st = vf.write(0, buf.data(), buf.size(), &n);
    CHECK(st && st->kind == ShmrError::FsError);   // config not populated (a panic in the reference)
    vf.populate(cfg);
    CHECK_OK(vf.read(0, buf.data(), buf.size(), &n));   // size 0: Ok(0)
    CHECK(n == 0);
    CHECK_OK(vf.write(0, buf.data(), buf.size(), &n));
    st = vf.read(100, buf.data(), buf.size(), &n);
    CHECK(st && st->kind == ShmrError::EndOfFile);
    st = vf.replace_block(5, VirtualBlock());
    CHECK(st && st->kind == ShmrError::BlockIndexOutOfBounds);
}

// ---- MI355X Erasure arms (GPU) ---------------------------------------------

// Erasure(1, k, p) block: write the input, sync (GPU encode), print the shard
// files; then drop and load it back, with erasures per the reference's rules
// (a shard truncated to 0 bytes is zero-padded and kept present).
void test_erasure_block_sync_load() {
    auto cfg = test_config();
    auto in = read_input();
    VirtualBlock b;
    const uint64_t size = 1024 * 1024;
    CHECK_OK(VirtualBlock::create(11, 0, cfg, size, BlockTopology::erasure(1, 8, 3), &b));
    size_t n = 0;
    CHECK(in.size() <= size);
    CHECK_OK(b.write(0, in.data(), in.size(), &n));
    CHECK_OK(b.sync_data(true));
    print_shards(*cfg, 0, b);
    CHECK_OK(b.drop_buffer());
    CHECK_OK(b.drop_handles());
    // intact load
    std::vector<uint8_t> rb(size);
    CHECK_OK(b.read(0, rb.data(), rb.size(), &n));
    CHECK(n == size);
    CHECK(std::equal(in.begin(), in.end(), rb.begin()));
    for (size_t i = in.size(); i < size; ++i) CHECK(rb[i] == 0);
    // reference rule: truncate data shard 1 -> zero-padded, present
    CHECK_OK(b.drop_buffer());
    CHECK_OK(b.drop_handles());
    fs::resize_file(shard_file(*cfg, b, 1), 0);
    CHECK_OK(b.read(0, rb.data(), rb.size(), &n));
    auto snap = b.buffer_snapshot();
    std::printf("LOADED_TRUNCATED %zu\n", snap.size());
    FILE* f = std::fopen((g_bucket + "/loaded_truncated.bin").c_str(), "wb");
    std::fwrite(snap.data(), 1, snap.size(), f);
    std::fclose(f);
}

// Opt-in rule: missing shard files are erasures; 3 of 11 removed -> exact data.
void test_erasure_block_missing_shards() {
    auto cfg = test_config();
    auto in = read_input();
    const uint64_t size = 1024 * 1024;
    VirtualBlock b;
    CHECK_OK(VirtualBlock::create(12, 0, cfg, size, BlockTopology::erasure(1, 8, 3), &b));
    VfsOptions o;
    o.missing_shard_is_erasure = true;
    o.short_shard_is_erasure = true;
    o.pread_from_start = true;
    b.set_options(o);
    size_t n = 0;
    CHECK_OK(b.write(0, in.data(), in.size(), &n));
    CHECK_OK(b.sync_data(true));
    const fs::path keep0 = shard_file(*cfg, b, 0);
    CHECK_OK(b.drop_buffer());
    CHECK_OK(b.drop_handles());
    fs::remove(shard_file(*cfg, b, 0));
    fs::remove(shard_file(*cfg, b, 5));
    fs::resize_file(shard_file(*cfg, b, 9), 17);   // short -> erasure
    std::vector<uint8_t> rb(size);
    CHECK_OK(b.read(0, rb.data(), rb.size(), &n));
    CHECK(std::equal(in.begin(), in.end(), rb.begin()));
    // the flush rewrote (repaired) every shard; now lose one more than parity
    CHECK_OK(b.drop_buffer());
    CHECK_OK(b.drop_handles());
    CHECK(fs::exists(keep0) && fsize(keep0) == calculate_shard_size(size, 8));
    for (size_t i : {1, 2, 3, 4}) fs::remove(shard_file(*cfg, b, i));
    // without the option a missing file fails in open_handles (block.rs:481-487)
    VirtualBlock strict;
    strict.ino = b.ino;
    strict.idx = b.idx;
    strict.size = b.size;
    strict.topology = b.topology;
    strict.shards = b.shards;
    strict.populate(cfg);
    Status st = strict.read(0, rb.data(), rb.size(), &n);
    CHECK(st && st->kind == ShmrError::FsError && st->code == ENOENT);
    // with it, 4 erasures > 3 parity: the crate's TooFewShardsPresent
    st = b.read(0, rb.data(), rb.size(), &n);
    CHECK(st && st->kind == ShmrError::EcError && st->code == SHMR_EC_TOO_FEW_SHARDS_PRESENT);
}

// A per-block flush whose encode fails at the wait, after the data shard
// files went out (mapped Block Cache: started encode): the parity files are
// unlinked (the stripe is detectably no codeword), the block stays dirty,
// and the next flush -- forced or not -- re-encodes and rewrites the stripe.
void test_erasure_flush_encode_failure() {
    auto cfg = test_config();
    auto in = read_input();
    const uint64_t size = 1024 * 1024;
    CHECK(in.size() >= 2 * size);
    const size_t S = calculate_shard_size(size, 8);
    VirtualBlock b;
    CHECK_OK(VirtualBlock::create(19, 0, cfg, size, BlockTopology::erasure(1, 8, 3), &b));
    VfsOptions o;
    o.missing_shard_is_erasure = true;
    o.short_shard_is_erasure = true;
    o.pread_from_start = true;
    o.pinned_buffers = true;
    b.set_options(o);
    size_t n = 0;
    CHECK_OK(b.write(0, in.data(), size, &n));
    CHECK_OK(b.sync_data(true));
    for (size_t i = 0; i < 11; ++i) CHECK(fsize(shard_file(*cfg, b, i)) == S);
    // new bytes; the flush's encode fails at the wait
    CHECK_OK(b.write(0, in.data() + size, size, &n));
    o.fault_encode_wait = true;
    b.set_options(o);
    Status st = b.sync_data(true);
    CHECK(st && st->kind == ShmrError::EcError && st->code == SHMR_EC_DEVICE_ERROR);
    for (size_t i = 0; i < 8; ++i) {   // the data shards went out
        std::ifstream f(shard_file(*cfg, b, i), std::ios::binary);
        std::vector<uint8_t> got(S);
        f.read(reinterpret_cast<char*>(got.data()), std::streamsize(S));
        CHECK(std::equal(got.begin(), got.end(), in.begin() + size + i * S));
    }
    for (size_t i = 8; i < 11; ++i) CHECK(!fs::exists(shard_file(*cfg, b, i)));   // no stale parity
    {   // a crash here, then a lost data shard, under the reference's short-
        // shard rule (zero-padded and kept present, block.rs:548-551): the
        // unlinked parity counts as missing -- never rebuilt from zeros
        VirtualBlock crashed;
        crashed.size = b.size;
        crashed.topology = b.topology;
        crashed.shards = b.shards;
        crashed.populate(cfg);
        VfsOptions lax;
        lax.missing_shard_is_erasure = true;
        lax.short_shard_is_erasure = false;
        crashed.set_options(lax);
        const fs::path lost = shard_file(*cfg, b, 3);
        const fs::path saved = lost.string() + ".saved";
        fs::rename(lost, saved);
        std::vector<uint8_t> rb(size);
        Status cs = crashed.read(0, rb.data(), rb.size(), &n);
        CHECK(cs && cs->kind == ShmrError::EcError && cs->code == SHMR_EC_TOO_FEW_SHARDS_PRESENT);
        VirtualBlock strict;   // the reference's rule: a missing shard file fails the open
        strict.size = b.size;
        strict.topology = b.topology;
        strict.shards = b.shards;
        strict.populate(cfg);
        fs::rename(saved, lost);
        cs = strict.read(0, rb.data(), rb.size(), &n);
        CHECK(cs && cs->kind == ShmrError::FsError && cs->code == ENOENT);
    }
    // the block is still dirty: an unforced flush re-encodes
    o.fault_encode_wait = false;
    b.set_options(o);
    CHECK_OK(b.sync_data(false));
    for (size_t i = 8; i < 11; ++i) CHECK(fsize(shard_file(*cfg, b, i)) == S);
    CHECK_OK(b.drop_buffer());
    CHECK_OK(b.drop_handles());
    fs::remove(shard_file(*cfg, b, 2));
    fs::remove(shard_file(*cfg, b, 6));
    std::vector<uint8_t> rb(size);
    CHECK_OK(b.read(0, rb.data(), rb.size(), &n));
    CHECK(std::equal(rb.begin(), rb.end(), in.begin() + size));
    print_shards(*cfg, 0, b);
}

// VfsOptions::direct_io: shard files written and read with O_DIRECT into and
// out of the Block-Cache slots (or, where the file system refuses O_DIRECT,
// through the buffered path -- counted either way).  A file of Erasure(1, 8,
// 3) 1 MiB blocks (S = 131,072: whole pages) through write -> sync -> lose
// a shard per block -> read; then one Erasure(1, 10, 4) block, whose S =
// 104,858 is not a whole page and must take the buffered path.
void direct_io_roundtrip(bool pinned) {
    auto cfg = test_config();
    auto in = read_input();
    const uint64_t bs = 1024 * 1024;
    const size_t nblk = in.size() / bs;
    CHECK(nblk * bs == in.size() && nblk > 1);
    VfsOptions o;
    o.missing_shard_is_erasure = true;
    o.short_shard_is_erasure = true;
    o.pread_from_start = true;
    o.pinned_buffers = pinned;
    o.direct_io = true;
    VirtualFile vf = VirtualFile::new_with(pinned ? 21 : 22, 0);
    vf.populate(cfg);
    for (size_t i = 0; i < nblk; ++i) {
        VirtualBlock b;
        CHECK_OK(VirtualBlock::create(vf.ino, i + 1, cfg, bs, BlockTopology::erasure(1, 8, 3), &b));
        vf.blocks.push_back(b);
    }
    vf.set_options(o);
    const DirectIoStats d0 = direct_io_stats();
    size_t n = 0;
    CHECK_OK(vf.write(0, in.data(), in.size(), &n));
    CHECK_OK(vf.sync_data(true));
    for (size_t i = 0; i < nblk; ++i) print_shards(*cfg, i, vf.blocks[i]);
    CHECK_OK(vf.drop_buffers());
    CHECK_OK(vf.drop_handles());
    for (size_t i = 0; i < nblk; ++i) fs::remove(shard_file(*cfg, vf.blocks[i], (i * 3) % 11));
    std::vector<uint8_t> rb(in.size());
    CHECK_OK(vf.read(0, rb.data(), rb.size(), &n));
    CHECK(n == in.size() && rb == in);
    const DirectIoStats d1 = direct_io_stats();
    const uint64_t used = (d1.reads - d0.reads) + (d1.writes - d0.writes);
    const uint64_t fell = d1.fallbacks - d0.fallbacks;
    // shard writes and reads went direct, or fell back (a refusal names its file system)
    CHECK(used + fell > 0);
    if (d1.refusals > d0.refusals) CHECK(!d1.refused_fs.empty() && d1.refused_errno != 0);
    std::printf("DIRECT reads=%llu writes=%llu fallbacks=%llu refusals=%llu fs=%s errno=%d io_errno=%d\n",
                (unsigned long long)(d1.reads - d0.reads), (unsigned long long)(d1.writes - d0.writes),
                (unsigned long long)fell, (unsigned long long)(d1.refusals - d0.refusals),
                d1.refused_fs.empty() ? "-" : d1.refused_fs.c_str(), d1.refused_errno, d1.io_errno);
    // a block whose shards are not whole pages: buffered, same bytes
    VirtualBlock odd;
    CHECK_OK(VirtualBlock::create(vf.ino + 100, 0, cfg, bs, BlockTopology::erasure(1, 10, 4), &odd));
    odd.set_options(o);
    CHECK_OK(odd.write(0, in.data(), bs, &n));
    const DirectIoStats d2 = direct_io_stats();
    CHECK_OK(odd.sync_data(true));
    CHECK_OK(odd.drop_buffer());
    CHECK_OK(odd.drop_handles());
    fs::remove(shard_file(*cfg, odd, 4));
    std::vector<uint8_t> ob(bs);
    CHECK_OK(odd.read(0, ob.data(), ob.size(), &n));
    CHECK(std::equal(ob.begin(), ob.end(), in.begin()));
    const DirectIoStats d3 = direct_io_stats();
    CHECK(d3.reads == d2.reads && d3.writes == d2.writes && d3.fallbacks > d2.fallbacks);
}
void test_direct_io_mapped() { direct_io_roundtrip(true); }
void test_direct_io_pageable() { direct_io_roundtrip(false); }

// VirtualFile with Erasure blocks: one batched GPU encode per flush.
void test_virtual_file_erasure_batch() {
    auto cfg = test_config();
    auto in = read_input();
    const uint64_t bs = 1024 * 1024;
    const size_t nblk = in.size() / bs;
    CHECK(nblk * bs == in.size() && nblk > 0);
    VirtualFile vf = VirtualFile::new_with(13, 0);
    vf.populate(cfg);
    for (size_t i = 0; i < nblk; ++i) {
        VirtualBlock b;
        CHECK_OK(VirtualBlock::create(13, i + 1, cfg, bs, BlockTopology::erasure(1, 8, 3), &b));
        vf.blocks.push_back(b);
    }
    size_t n = 0;
    CHECK_OK(vf.write(0, in.data(), in.size(), &n));
    CHECK(n == in.size());
    CHECK(vf.blocks.size() == nblk + 1);   // trailing empty chunk -> one Single block
    CHECK_OK(vf.sync_data(true));
    for (size_t i = 0; i < nblk; ++i) print_shards(*cfg, i, vf.blocks[i]);
    CHECK_OK(vf.drop_buffers());
    for (auto& b : vf.blocks) CHECK_OK(b.drop_handles());
    std::vector<uint8_t> rb(in.size());
    CHECK_OK(vf.read(0, rb.data(), rb.size(), &n));
    CHECK(rb == in);
}

// replace_block: Single -> Erasure(1, 4, 2) migration (mod.rs:244-271)
void test_replace_block_erasure() {
    auto cfg = test_config();
    VirtualFile vf = VirtualFile::new_with(14, 0);
    vf.populate(cfg);
    auto data = read_input();
    size_t n = 0;
    CHECK(data.size() < vf.block_size);
    CHECK_OK(vf.write(0, data.data(), data.size(), &n));
    VirtualBlock ec;
    CHECK_OK(VirtualBlock::create(14, 99, cfg, vf.block_size, BlockTopology::erasure(1, 4, 2), &ec));
    CHECK_OK(vf.replace_block(0, ec));
    print_shards(*cfg, 0, vf.blocks[0]);
    CHECK_OK(vf.blocks[0].drop_buffer());
    CHECK_OK(vf.blocks[0].drop_handles());
    std::vector<uint8_t> rb(data.size());
    CHECK_OK(vf.read(0, rb.data(), rb.size(), &n));
    CHECK(rb == data);
}

// Batched load with erasures: one shard file per block removed (data and
// parity positions), pinned Block-Cache buffers; one reconstruct call.
void test_virtual_file_batched_reconstruct() {
    auto cfg = test_config();
    auto in = read_input();
    const uint64_t bs = 1024 * 1024;
    const size_t nblk = in.size() / bs;
    CHECK(nblk * bs == in.size() && nblk > 0);
    VirtualFile vf = VirtualFile::new_with(15, 0);
    vf.populate(cfg);
    VfsOptions o;
    o.missing_shard_is_erasure = true;
    o.pread_from_start = true;
    o.short_shard_is_erasure = true;
    o.pinned_buffers = true;
    for (size_t i = 0; i < nblk; ++i) {
        VirtualBlock b;
        CHECK_OK(VirtualBlock::create(15, i + 1, cfg, bs, BlockTopology::erasure(1, 8, 3), &b));
        vf.blocks.push_back(b);
    }
    vf.set_options(o);
    vf.pipeline_batch_bytes = 3 * 1024 * 1024;   // 3 blocks per batch: exercises the pipelined batches
    size_t n = 0;
    CHECK_OK(vf.write(0, in.data(), in.size(), &n));
    CHECK(vf.blocks[0].buffer_pinned());
    CHECK_OK(vf.sync_data(true));
    CHECK(vf.last_sync.blocks == nblk);
    for (size_t i = 0; i < nblk; ++i) print_shards(*cfg, i, vf.blocks[i]);
    CHECK_OK(vf.drop_buffers());
    CHECK_OK(vf.drop_handles());
    for (size_t i = 0; i < nblk; ++i) {
        fs::remove(shard_file(*cfg, vf.blocks[i], i % 11));
        if (i % 3 == 0) fs::resize_file(shard_file(*cfg, vf.blocks[i], (i + 5) % 11), 100);   // short -> erasure
    }
    std::vector<uint8_t> rb(in.size());
    CHECK_OK(vf.read(0, rb.data(), rb.size(), &n));
    CHECK(n == in.size());
    CHECK(vf.last_load.blocks == nblk);   // every block needed a reconstruct, one batch
    CHECK_SAME(rb, in, bs, calculate_shard_size(bs, 8));
    // the flush after the repair rewrites the lost shard files
    CHECK_OK(vf.drop_buffers());
    for (size_t i = 0; i < nblk; ++i)
        CHECK(fs::exists(shard_file(*cfg, vf.blocks[i], i % 11)) &&
              fsize(shard_file(*cfg, vf.blocks[i], i % 11)) == calculate_shard_size(bs, 8));
}

// Mapped Block Cache with auto batching: sync_data flushes block by block on
// the worker pool (zero-copy encodes, blocks round-robin over a device list),
// then a pipelined load rebuilds a lost shard of every block.
void test_virtual_file_mapped_per_block_flush() {
    auto cfg = test_config();
    auto in = read_input();
    const uint64_t bs = 1024 * 1024;
    const size_t nblk = in.size() / bs;
    CHECK(nblk * bs == in.size() && nblk > 0);
    VirtualFile vf = VirtualFile::new_with(17, 0);
    vf.populate(cfg);
    VfsOptions o;
    o.missing_shard_is_erasure = true;
    o.pread_from_start = true;
    o.pinned_buffers = true;
    for (size_t i = 0; i < nblk; ++i) {
        VirtualBlock b;
        CHECK_OK(VirtualBlock::create(17, i + 1, cfg, bs, BlockTopology::erasure(1, 8, 3), &b));
        vf.blocks.push_back(b);
    }
    vf.set_options(o);
    vf.devices = {0, 0};   // round-robin over a device list (one GPU on the test box)
    uint64_t zc0 = 0, st0 = 0, zc1 = 0, st1 = 0;
    shmr_ec_path_stats(&zc0, &st0);
    size_t n = 0;
    CHECK_OK(vf.write(0, in.data(), in.size(), &n));
    CHECK(vf.blocks[0].buffer_pinned());
    CHECK_OK(vf.sync_data(true));
    CHECK(vf.last_sync.blocks == nblk);
    shmr_ec_path_stats(&zc1, &st1);
    CHECK(zc1 - zc0 == nblk && st1 == st0);   // every block encoded zero-copy
    for (size_t i = 0; i < nblk; ++i) print_shards(*cfg, i, vf.blocks[i]);
    CHECK_OK(vf.drop_buffers());
    CHECK_OK(vf.drop_handles());
    for (size_t i = 0; i < nblk; ++i) fs::remove(shard_file(*cfg, vf.blocks[i], (i * 5) % 11));
    std::vector<uint8_t> rb(in.size());
    CHECK_OK(vf.read(0, rb.data(), rb.size(), &n));
    CHECK(n == in.size());
    CHECK(vf.last_load.blocks == nblk);
    CHECK(rb == in);
    // a clean flush writes nothing; a forced one rewrites every shard
    CHECK_OK(vf.sync_data(false));
    CHECK_OK(vf.sync_data(true));
    for (size_t i = 0; i < nblk; ++i)
        CHECK(fsize(shard_file(*cfg, vf.blocks[i], (i * 5) % 11)) == calculate_shard_size(bs, 8));
}

// rewrite_erasure: Single blocks -> Erasure(1, 4, 2), batched.
void test_rewrite_erasure() {
    auto cfg = test_config();
    auto in = read_input();
    VirtualFile vf = VirtualFile::new_with(16, 0);
    vf.populate(cfg);
    size_t n = 0;
    CHECK_OK(vf.write(0, in.data(), in.size(), &n));
    const size_t nblk = vf.blocks.size();
    CHECK_OK(vf.sync_data(true));
    CHECK_OK(vf.rewrite_erasure(4, 2));
    CHECK(vf.blocks.size() == nblk);
    for (size_t i = 0; i < nblk; ++i) {
        CHECK(vf.blocks[i].topology.kind == BlockTopology::Erasure && vf.blocks[i].topology.data == 4);
        print_shards(*cfg, i, vf.blocks[i]);
    }
    CHECK(vf.last_sync.blocks == nblk);
    CHECK_OK(vf.drop_buffers());
    CHECK_OK(vf.drop_handles());
    std::vector<uint8_t> rb(in.size());
    CHECK_OK(vf.read(0, rb.data(), rb.size(), &n));
    CHECK(rb == in);
    CHECK_OK(vf.rewrite_erasure(4, 2));   // already Erasure(1, 4, 2): no-op
}

// The durable VirtualFile record (record.cpp; the reference's serde_yaml
// superblock value): every topology and awkward strings round-trip, the text
// has the serde shape, hand-written flow/quoted forms parse, bad records fail.
void test_virtual_file_record_roundtrip() {
    auto cfg = std::make_shared<ShmrFsConfig>(*test_config());
    cfg->pools["test_pool"]["b: #2"] = Bucket{g_bucket, 999, 998, BucketPriority::Normal};
    VirtualFile vf = VirtualFile::new_with(21, 4242);
    vf.populate(cfg);
    vf.block_size = 1 << 20;
    VirtualBlock s, m, e;
    CHECK_OK(VirtualBlock::create(21, 1, cfg, 1 << 20, BlockTopology::single(), &s));
    CHECK_OK(VirtualBlock::create(21, 2, cfg, 1 << 20, BlockTopology::mirror(3), &m));
    CHECK_OK(VirtualBlock::create(21, 3, cfg, 4 << 20, BlockTopology::erasure(1, 8, 3), &e));
    m.shards[1].pool = "-odd";
    m.shards[2].filename = "it's";
    e.shards[4].bucket = "true";
    vf.blocks = {s, m, e};
    const std::string text = vf.to_yaml();
    CHECK(text.rfind("ino: 21\nsize: 4242\nchunk_size: 4096\nblocks:\n- ino: 21\n  idx: 1\n  size: 1048576\n"
                     "  topology: Single\n  shards:\n  - pool: test_pool\n    bucket: ", 0) == 0);
    CHECK(text.find("  topology: !Mirror 3\n") != std::string::npos);
    CHECK(text.find("  topology: !Erasure\n  - 1\n  - 8\n  - 3\n  shards:\n") != std::string::npos);
    CHECK(text.find("filename: 21:3_ec83_10.bin\n") != std::string::npos);
    CHECK(text.find("pool: '-odd'") != std::string::npos && text.find("filename: it's\n") != std::string::npos &&
          text.find("bucket: 'true'") != std::string::npos);
    CHECK(text.size() > 13 && text.compare(text.size() - 20, 20, "block_size: 1048576\n") == 0);
    VirtualFile back;
    std::string err;
    CHECK_OK(VirtualFile::from_yaml(text, &back, &err));
    CHECK(back.ino == 21 && back.size == 4242 && back.chunk_size == 4096 && back.block_size == (1u << 20));
    CHECK(back.blocks.size() == 3);
    for (size_t i = 0; i < 3; ++i) {
        const auto &a = vf.blocks[i], &b = back.blocks[i];
        CHECK(a.ino == b.ino && a.idx == b.idx && a.size == b.size);
        CHECK(a.topology.to_string() == b.topology.to_string());
        CHECK(a.shards.size() == b.shards.size());
        for (size_t j = 0; j < a.shards.size(); ++j)
            CHECK(a.shards[j].pool == b.shards[j].pool && a.shards[j].bucket == b.shards[j].bucket &&
                  a.shards[j].filename == b.shards[j].filename);
    }
    CHECK(back.to_yaml() == text);
    // serde_yaml's other spellings: flow sequence, quoted scalars, document marker
    const std::string hand =
        "---\nino: 5\nsize: 10\nchunk_size: 4096\nblocks:\n  - ino: 5\n    idx: 1\n    size: 100\n"
        "    topology: !Erasure [1, 2, 1]\n    shards:\n      - {pool: x, bucket: y, filename: a}\n";
    CHECK(VirtualFile::from_yaml(hand, &back, &err));   // flow mappings are not part of the subset
    const std::string hand2 =
        "---\nino: 5\nsize: 10\nchunk_size: 4096\nblocks:\n  - ino: 5\n    idx: 1\n    size: 100\n"
        "    topology: !Erasure [1, 2, 1]   # comment\n    shards:\n      - pool: \"x\"\n        bucket: 'y'\n"
        "        filename: a\n      - pool: x\n        bucket: y\n        filename: b\n      - pool: x\n"
        "        bucket: y\n        filename: \"c\\x41\"\nblock_size: 7\n";
    CHECK_OK(VirtualFile::from_yaml(hand2, &back, &err));
    CHECK(back.blocks.size() == 1 && back.blocks[0].topology.to_string() == "Erasure(1, 2, 1)");
    CHECK(back.blocks[0].shards[2].filename == "cA" && back.blocks[0].shards[0].bucket == "y" && back.block_size == 7);
    CHECK_OK(VirtualFile::from_yaml("ino: 1\nsize: 0\nchunk_size: 4096\nblocks: []\nblock_size: 9\n", &back, &err));
    CHECK(back.blocks.empty() && back.block_size == 9);
    // malformed records: FsError(EINVAL) with a reason
    for (const char* bad : {"ino: 1\n", "ino: x\nsize: 0\nchunk_size: 1\nblocks: []\nblock_size: 1\n",
                            "ino: 1\nsize: 0\nchunk_size: 1\nblocks:\n- ino: 1\n  idx: 0\n  size: 1\n"
                            "  topology: !Raid 5\n  shards: []\nblock_size: 1\n",
                            "ino: 1\nsize: 0\nchunk_size: 1\nblocks:\n- ino: 1\n  idx: 0\n  size: 1\n"
                            "  topology: !Erasure [1, 300, 1]\n  shards: []\nblock_size: 1\n",
                            "ino: 1\nsize: 0\nchunk_size: 1\nblocks:\n- ino: 1\n  idx: 0\n  size: 1\n"
                            "  topology: !Erasure [1, 2, 1]\n  shards: []\nblock_size: 1\n"}) {
        err.clear();
        Status st = VirtualFile::from_yaml(bad, &back, &err);
        CHECK(st && st->kind == ShmrError::FsError && st->code == EINVAL && !err.empty());
    }
    {   // pathological nesting is refused, not recursed into
        std::string deep = "ino: 1\nsize: 0\nchunk_size: 1\nblock_size: 1\nblocks:\n";
        for (int d = 0; d < 5000; ++d) deep += std::string(size_t(d), ' ') + "-\n";
        err.clear();
        Status st = VirtualFile::from_yaml(deep, &back, &err);
        CHECK(st && st->code == EINVAL && err.find("nesting") != std::string::npos);
    }
    // save / load through the file system (temp file + rename)
    const fs::path rec = fs::path(g_bucket) / "vf21.yaml";
    CHECK_OK(vf.save_record(rec));
    CHECK(!fs::exists(rec.string() + ".tmp"));
    CHECK_OK(VirtualFile::load_record(rec, &back, &err));
    CHECK(back.to_yaml() == text);
    Status st = VirtualFile::load_record(fs::path(g_bucket) / "missing.yaml", &back, &err);
    CHECK(st && st->kind == ShmrError::FsError && st->code == ENOENT);
}

// Record fuzz: random files (every topology, random shard strings drawn from
// printable ASCII, YAML indicators, quotes, '#', ': ' and control bytes)
// round-trip exactly; random truncations and byte flips of valid records
// either parse or fail with FsError(EINVAL) -- never crash or hang.
void test_virtual_file_record_fuzz() {
    std::mt19937_64 rng(0x5EC0DE);
    auto rnd = [&](uint64_t n) { return uint64_t(rng() % n); };
    const std::string alphabet =
        "abcXYZ019_-.:/ #'\"!&*[]{},|>%@`?~\t\x01\x7f";
    auto rstr = [&]() {
        std::string t;
        const size_t n = rnd(12);
        for (size_t i = 0; i < n; ++i) t += alphabet[rnd(alphabet.size())];
        if (rnd(8) == 0) t = "true";
        if (rnd(8) == 0) t = "0x1F";
        return t;
    };
    for (int it = 0; it < 400; ++it) {
        VirtualFile vf = VirtualFile::new_with(rng(), rng() >> rnd(64));
        vf.chunk_size = 1 + rnd(1 << 20);
        vf.block_size = rng() >> rnd(64);
        const size_t nb = rnd(5);
        for (size_t b = 0; b < nb; ++b) {
            VirtualBlock blk;
            blk.ino = rng();
            blk.idx = rnd(1000);
            blk.size = rng() >> rnd(64);
            const uint64_t kind = rnd(3);
            size_t n = 1;
            if (kind == 1) {
                blk.topology = BlockTopology::mirror(uint8_t(rnd(256)));
                n = blk.topology.n;
            } else if (kind == 2) {
                blk.topology = BlockTopology::erasure(uint8_t(rnd(256)), uint8_t(rnd(20)), uint8_t(rnd(20)));
                n = size_t(blk.topology.data) + blk.topology.parity;
            }
            for (size_t i = 0; i < n; ++i) blk.shards.push_back({rstr(), rstr(), rstr()});
            vf.blocks.push_back(blk);
        }
        const std::string text = vf.to_yaml();
        VirtualFile back;
        std::string err;
        Status st = VirtualFile::from_yaml(text, &back, &err);
        if (st) throw Failure{"round trip failed: " + err + "\n" + text};
        if (back.to_yaml() != text) throw Failure{"round trip changed the record:\n" + text + "\n---\n" + back.to_yaml()};
        for (int m = 0; m < 8; ++m) {   // mutations: parse or EINVAL, nothing else
            std::string bad = text;
            if (m % 2 == 0 && !bad.empty()) bad.resize(rnd(bad.size()));
            else if (!bad.empty()) bad[rnd(bad.size())] = alphabet[rnd(alphabet.size())];
            Status ms = VirtualFile::from_yaml(bad, &back, &err);
            CHECK(!ms || (ms->kind == ShmrError::FsError && ms->code == EINVAL));
        }
    }
}

// a file rewritten to Erasure(1, 8, 3) survives a restart
// through its record alone -- everything in memory is dropped, the record is
// reloaded, one shard file of every block is lost, and the file reads back
// bit-exact (reconstructed on the GPU).
void test_rewrite_erasure_record_reload() {
    auto cfg = test_config();
    auto in = read_input();
    const fs::path rec = fs::path(g_bucket) / "vf17.yaml";
    size_t nblk = 0;
    {
        VirtualFile vf = VirtualFile::new_with(17, 0);
        vf.populate(cfg);
        size_t n = 0;
        CHECK_OK(vf.write(0, in.data(), in.size(), &n));
        CHECK_OK(vf.sync_data(true));
        CHECK_OK(vf.rewrite_erasure(8, 3));
        nblk = vf.blocks.size();
        CHECK_OK(vf.save_record(rec));
        for (size_t i = 0; i < nblk; ++i) print_shards(*cfg, i, vf.blocks[i]);
        CHECK_OK(vf.drop_buffers());
        CHECK_OK(vf.drop_handles());
    }   // the process's view of the file is gone; only the record and the shard files remain
    VirtualFile vf;
    std::string err;
    CHECK_OK(VirtualFile::load_record(rec, &vf, &err));
    vf.populate(cfg);
    CHECK(vf.size == in.size() && vf.blocks.size() == nblk);
    VfsOptions o;
    o.missing_shard_is_erasure = true;
    o.pread_from_start = true;
    vf.set_options(o);
    for (size_t i = 0; i < nblk; ++i) {
        CHECK(vf.blocks[i].topology.to_string() == "Erasure(1, 8, 3)");
        fs::remove(shard_file(*cfg, vf.blocks[i], (3 * i) % 11));
    }
    std::vector<uint8_t> rb(in.size());
    size_t n = 0;
    CHECK_OK(vf.read(0, rb.data(), rb.size(), &n));
    CHECK(n == in.size());
    CHECK_SAME(rb, in, vf.block_size, calculate_shard_size(vf.block_size, 8));
}

// VfsOptions::read_needed_shards: a load reads only the first k intact shard
// files (per-block and batched paths) and returns the same bytes as the
// read-everything load; a shard of another length without
// short_shard_is_erasure falls back to reading all of them (reference rule).
void test_read_needed_shards() {
    auto cfg = test_config();
    auto in = read_input();
    const uint64_t bs = 1024 * 1024;
    const size_t nblk = in.size() / bs;
    CHECK(nblk * bs == in.size() && nblk >= 2);
    VirtualFile vf = VirtualFile::new_with(18, 0);
    vf.populate(cfg);
    for (size_t i = 0; i < nblk; ++i) {
        VirtualBlock b;
        CHECK_OK(VirtualBlock::create(18, i + 1, cfg, bs, BlockTopology::erasure(1, 8, 3), &b));
        vf.blocks.push_back(b);
    }
    size_t n = 0;
    CHECK_OK(vf.write(0, in.data(), in.size(), &n));
    CHECK_OK(vf.sync_data(true));
    CHECK_OK(vf.drop_buffers());
    CHECK_OK(vf.drop_handles());
    VfsOptions o;
    o.missing_shard_is_erasure = true;
    o.pread_from_start = true;
    o.read_needed_shards = true;
    vf.set_options(o);
    const size_t S = calculate_shard_size(bs, 8);
    std::vector<uint8_t> rb(in.size());
    auto load_all = [&](size_t* reads) {
        const uint64_t r0 = shard_reads_total();
        std::fill(rb.begin(), rb.end(), 0xEE);
        CHECK_OK(vf.read(0, rb.data(), rb.size(), &n));
        CHECK(n == in.size());
        *reads = size_t(shard_reads_total() - r0);
        CHECK_OK(vf.drop_buffers());
    };
    size_t reads = 0;
    load_all(&reads);   // batched path, all intact
    CHECK_SAME(rb, in, bs, S);
    CHECK(reads == 8 * nblk);
    // lose data shard (i % 8) and parity shard 9 of every block: still 8 reads each
    CHECK_OK(vf.drop_handles());
    for (size_t i = 0; i < nblk; ++i) {
        fs::remove(shard_file(*cfg, vf.blocks[i], i % 8));
        fs::remove(shard_file(*cfg, vf.blocks[i], 9));
    }
    load_all(&reads);   // the flush in drop_buffers repairs the files
    CHECK_SAME(rb, in, bs, S);
    CHECK(reads == 8 * nblk);
    CHECK(fsize(shard_file(*cfg, vf.blocks[0], 0)) == S && fsize(shard_file(*cfg, vf.blocks[0], 9)) == S);
    // per-block path (VirtualBlock::read)
    CHECK_OK(vf.drop_handles());
    VirtualBlock& b = vf.blocks[1];
    fs::remove(shard_file(*cfg, b, 3));
    std::vector<uint8_t> one(bs);
    uint64_t r0 = shard_reads_total();
    CHECK_OK(b.read(0, one.data(), one.size(), &n));
    CHECK(shard_reads_total() - r0 == 8);
    CHECK(std::equal(one.begin(), one.end(), in.begin() + bs));
    CHECK_OK(b.drop_buffer());
    CHECK_OK(b.drop_handles());
    // a truncated data shard (reference rule: zero-padded and kept): every file
    // is read, and the load equals the read-everything load.  Fresh views of
    // the block, so no flush repairs the file between the two loads.
    fs::resize_file(shard_file(*cfg, b, 2), 100);
    auto view = [&](bool needed) {
        VirtualBlock v;
        v.ino = b.ino;
        v.idx = b.idx;
        v.size = b.size;
        v.topology = b.topology;
        v.shards = b.shards;
        v.populate(cfg);
        VfsOptions vo = o;
        vo.read_needed_shards = needed;
        v.set_options(vo);
        const uint64_t r = shard_reads_total();
        CHECK_OK(v.read(0, one.data(), one.size(), &n));
        CHECK(shard_reads_total() - r == 11);
        return v.buffer_snapshot();
    };
    const auto planned = view(true);
    CHECK(fsize(shard_file(*cfg, b, 2)) == 100);
    CHECK(planned == view(false));
}

// CPU-only view of the same plan: shard files written directly (no encode), all
// present, so a load needs no codec call.  With the option the load reads the 8
// data shard files; without it all 11; the loaded bytes are the data shards.
void test_read_needed_shards_plan() {
    auto cfg = test_config();
    const uint64_t size = 1024 * 1024 - 4096;   // partial last data shard
    VirtualBlock b;
    CHECK_OK(VirtualBlock::create(19, 0, cfg, size, BlockTopology::erasure(1, 8, 3), &b));
    const size_t S = calculate_shard_size(size, 8);
    std::vector<uint8_t> want;
    for (size_t i = 0; i < 11; ++i) {
        const auto bytes = random_data(S);   // parity files hold noise: never read, never returned
        if (i < 8) want.insert(want.end(), bytes.begin(), bytes.end());
        FILE* f = std::fopen(shard_file(*cfg, b, i).c_str(), "wb");
        CHECK(f != nullptr);
        CHECK(std::fwrite(bytes.data(), 1, S, f) == S);
        std::fclose(f);
    }
    want.resize(size);
    for (bool needed : {true, false}) {
        VirtualBlock v;
        v.ino = b.ino;
        v.idx = b.idx;
        v.size = b.size;
        v.topology = b.topology;
        v.shards = b.shards;
        v.populate(cfg);
        VfsOptions o;
        o.pread_from_start = true;
        o.read_needed_shards = needed;
        v.set_options(o);
        std::vector<uint8_t> rb(size);
        size_t n = 0;
        const uint64_t r0 = shard_reads_total();
        CHECK_OK(v.read(0, rb.data(), rb.size(), &n));
        CHECK(n == size);
        CHECK(shard_reads_total() - r0 == (needed ? 8u : 11u));
        CHECK(rb == want);
    }
}

// Randomised Erasure-block round trips against a byte model: random (k, p) and
// block sizes, random writes, flush, lose up to p shard files (and sometimes
// truncate one, an erasure under short_shard_is_erasure), reload, compare;
// then more writes into the loaded block and another round.  Options (mapped
// Block Cache, needed-shards reads) vary per block.
void test_virtual_block_erasure_fuzz() {
    auto cfg = test_config();
    const std::pair<int, int> codes[] = {{4, 2}, {8, 3}, {10, 4}, {5, 5}, {3, 1}, {6, 3}};
    for (int it = 0; it < 120; ++it) {
        const auto [k, p] = codes[g_rng() % 6];
        const uint64_t size = 1 + g_rng() % (3 << 20);
        VirtualBlock b;
        CHECK_OK(VirtualBlock::create(20, it, cfg, size, BlockTopology::erasure(1, k, p), &b));
        VfsOptions o;
        o.missing_shard_is_erasure = true;
        o.short_shard_is_erasure = true;
        o.pread_from_start = true;
        o.pinned_buffers = g_rng() % 2;
        o.read_needed_shards = g_rng() % 2;
        b.set_options(o);
        std::vector<uint8_t> model(size, 0);
        for (int round = 0; round < 2; ++round) {
            const int writes = 1 + int(g_rng() % 5);
            for (int w = 0; w < writes; ++w) {
                const uint64_t pos = g_rng() % size;
                const size_t len = size_t(1 + g_rng() % std::min<uint64_t>(size - pos, 1 << 20));
                const auto bytes = random_data(len);
                size_t n = 0;
                CHECK_OK(b.write(pos, bytes.data(), len, &n));
                CHECK(n == len);
                std::memcpy(model.data() + pos, bytes.data(), len);
            }
            CHECK_OK(b.sync_data(true));
            CHECK_OK(b.drop_buffer());
            CHECK_OK(b.drop_handles());
            const size_t lose = g_rng() % (p + 1);
            std::vector<size_t> idx(k + p);
            for (size_t i = 0; i < idx.size(); ++i) idx[i] = i;
            std::shuffle(idx.begin(), idx.end(), g_rng);
            for (size_t i = 0; i < lose; ++i) {
                if (i == 0 && g_rng() % 3 == 0) fs::resize_file(shard_file(*cfg, b, idx[i]), g_rng() % 4096);
                else fs::remove(shard_file(*cfg, b, idx[i]));
            }
            std::vector<uint8_t> rb(size);
            size_t n = 0;
            CHECK_OK(b.read(0, rb.data(), rb.size(), &n));
            CHECK(n == size);
            if (rb != model)
                throw Failure{"iteration " + std::to_string(it) + " round " + std::to_string(round) + " RS(" +
                              std::to_string(k) + "," + std::to_string(p) + ") size " + std::to_string(size) +
                              diff_report(rb, model, size, calculate_shard_size(size, k))};
        }
        CHECK_OK(b.drop_buffer());   // repairs the lost files
        CHECK_OK(b.drop_handles());
        for (size_t i = 0; i < size_t(k + p); ++i) CHECK(fsize(shard_file(*cfg, b, i)) == calculate_shard_size(size, k));
    }
}

// File-level twin of the Erasure-block fuzz: random codes, block counts,
// Block-Cache kinds, batch sizes and needed-shards reads; whole-file batched
// flushes and loads with shard files lost or truncated in random blocks, and
// block-level rewrites in between, against a byte model of the file.
void test_virtual_file_erasure_fuzz() {
    auto cfg = test_config();
    const std::pair<int, int> codes[] = {{4, 2}, {8, 3}, {10, 4}, {5, 5}, {3, 1}};
    const size_t batches[] = {VirtualFile::kAutoBatch, 0, 1 << 20, 3 << 20};
    for (int it = 0; it < 16; ++it) {
        const auto [k, p] = codes[g_rng() % 5];
        const uint64_t bs = uint64_t(1 + g_rng() % 2) << 20;
        const size_t nblk = 2 + g_rng() % 9;
        VirtualFile vf = VirtualFile::new_with(30 + it, 0);
        vf.populate(cfg);
        vf.block_size = bs;
        vf.pipeline_batch_bytes = batches[g_rng() % 4];
        for (size_t i = 0; i < nblk; ++i) {
            VirtualBlock b;
            CHECK_OK(VirtualBlock::create(30 + it, i + 1, cfg, bs, BlockTopology::erasure(1, k, p), &b));
            vf.blocks.push_back(b);
        }
        VfsOptions o;
        o.missing_shard_is_erasure = true;
        o.short_shard_is_erasure = true;
        o.pread_from_start = true;
        o.pinned_buffers = g_rng() % 2;
        o.read_needed_shards = g_rng() % 2;
        vf.set_options(o);
        std::vector<uint8_t> model = random_data(nblk * bs);
        size_t n = 0;
        CHECK_OK(vf.write(0, model.data(), model.size(), &n));
        CHECK(n == model.size());
        const size_t S = calculate_shard_size(bs, k);
        for (int round = 0; round < 3; ++round) {
            CHECK_OK(vf.sync_data(true));
            CHECK_OK(vf.drop_buffers());
            CHECK_OK(vf.drop_handles());
            for (size_t i = 0; i < nblk; ++i) {
                const size_t lose = g_rng() % (p + 1);
                std::vector<size_t> idx(k + p);
                for (size_t j = 0; j < idx.size(); ++j) idx[j] = j;
                std::shuffle(idx.begin(), idx.end(), g_rng);
                for (size_t j = 0; j < lose; ++j) {
                    if (j == 0 && g_rng() % 3 == 0) fs::resize_file(shard_file(*cfg, vf.blocks[i], idx[j]), g_rng() % S);
                    else fs::remove(shard_file(*cfg, vf.blocks[i], idx[j]));
                }
            }
            std::vector<uint8_t> rb(model.size());
            CHECK_OK(vf.read(0, rb.data(), rb.size(), &n));
            CHECK(n == model.size());
            if (rb != model)
                throw Failure{"iteration " + std::to_string(it) + " round " + std::to_string(round) + " RS(" +
                              std::to_string(k) + "," + std::to_string(p) + ") " + std::to_string(nblk) + " x " +
                              std::to_string(bs) + diff_report(rb, model, bs, S)};
            // block-level rewrites into the loaded blocks
            for (int w = int(g_rng() % 4); w > 0; --w) {
                const size_t i = g_rng() % nblk;
                const uint64_t pos = g_rng() % bs;
                const size_t len = size_t(1 + g_rng() % (bs - pos));
                const auto bytes = random_data(len);
                CHECK_OK(vf.blocks[i].write(pos, bytes.data(), len, &n));
                std::memcpy(model.data() + i * bs + pos, bytes.data(), len);
            }
        }
        CHECK_OK(vf.sync_data(true));
        CHECK_OK(vf.drop_buffers());
        CHECK_OK(vf.drop_handles());
    }
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s <case> <bucket_dir> [input]\n", argv[0]);
        return 2;
    }
    const std::string name = argv[1];
    g_bucket = argv[2];
    if (argc > 3) g_input = argv[3];
    static const std::map<std::string, std::function<void()>> cases = {
        {"block_topology_try_from", test_block_topology_try_from},
        {"virtual_block_new_block", test_virtual_block_new_block},
        {"virtual_block_unbuffered_backing", test_virtual_block_unbuffered_backing},
        {"virtual_block_unbuffered", test_virtual_block_unbuffered},
        {"virtual_block_buffered", test_virtual_block_buffered},
        {"virtual_block_erasure_buffered", test_virtual_block_erasure_buffered},
        {"block_errors", test_block_errors},
        {"erasure_f32_hazard", test_erasure_f32_hazard},
        {"erasure_f32_hazard_release", test_erasure_f32_hazard_release},
        {"virtual_file_1", test_virtual_file_1},
        {"virtual_file_2_4_mb", test_virtual_file_2_4_mb},
        {"virtual_file_errors", test_virtual_file_errors},
        {"virtual_file_chunk_model", test_virtual_file_chunk_model},
        {"erasure_block_sync_load", test_erasure_block_sync_load},
        {"erasure_block_missing_shards", test_erasure_block_missing_shards},
        {"erasure_flush_encode_failure", test_erasure_flush_encode_failure},
        {"direct_io_mapped", test_direct_io_mapped},
        {"direct_io_pageable", test_direct_io_pageable},
        {"virtual_file_erasure_batch", test_virtual_file_erasure_batch},
        {"replace_block_erasure", test_replace_block_erasure},
        {"virtual_file_batched_reconstruct", test_virtual_file_batched_reconstruct},
        {"rewrite_erasure", test_rewrite_erasure},
        {"virtual_file_mapped_per_block_flush", test_virtual_file_mapped_per_block_flush},
        {"virtual_file_record_roundtrip", test_virtual_file_record_roundtrip},
        {"virtual_file_record_fuzz", test_virtual_file_record_fuzz},
        {"rewrite_erasure_record_reload", test_rewrite_erasure_record_reload},
        {"read_needed_shards", test_read_needed_shards},
        {"read_needed_shards_plan", test_read_needed_shards_plan},
        {"virtual_block_erasure_fuzz", test_virtual_block_erasure_fuzz},
        {"virtual_file_erasure_fuzz", test_virtual_file_erasure_fuzz},
    };
    auto it = cases.find(name);
    if (it == cases.end()) {
        std::printf("FAIL: unknown case %s\n", name.c_str());
        return 1;
    }
    try {
        it->second();
    } catch (const Failure& f) {
        std::printf("FAIL: %s\n", f.msg.c_str());
        return 1;
    } catch (const std::exception& e) {
        std::printf("FAIL: exception %s\n", e.what());
        return 1;
    }
    std::printf("PASS\n");
    return 0;
}
