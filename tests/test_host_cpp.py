"""C++ host mirror of the reference's StorageBlock layer (shmr_amd/host/vfs.{hpp,cpp}).

Drives shmr_amd/_lib/shmr_vfs_test, whose cases mirror the reference's Rust tests
(src/vfs/block.rs:647-812, src/vfs/mod.rs:322-370).  Single-topology cases do no
GPU work and run on CPU; the Erasure cases encode/reconstruct on the MI355X and
their shard files are compared here, byte for byte, with the CPU oracle's
restatement of the Erasure arms (oracle.rs_oracle.sync_data_erasure /
load_block_erasure, block.rs:404-440 / :529-579).
"""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

from oracle import rs_oracle as O

KAT = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "kat.json")))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "shmr_amd", "_lib", "shmr_vfs_test")
MiB = 1 << 20


def run_case(name, bucket, data=None, timeout=300):
    if not os.path.exists(BIN):
        pytest.fail(f"{BIN} not built (run __graft_entry__.build())")
    args = [BIN, name, str(bucket)]
    if data is not None:
        path = os.path.join(str(bucket), "input.bin")
        with open(path, "wb") as f:
            f.write(np.asarray(data, np.uint8).tobytes())
        args.append(path)
    p = subprocess.run(args, capture_output=True, text=True, timeout=timeout)
    out = p.stdout.strip().splitlines()
    assert p.returncode == 0 and out and out[-1] == "PASS", f"{name}: rc={p.returncode}\n{p.stdout}\n{p.stderr}"
    shards = {}
    for line in out:
        if line.startswith("SHARDS "):
            parts = line.split()
            shards[int(parts[1])] = parts[2:]
    return shards


def read(path):
    with open(path, "rb") as f:
        return np.frombuffer(f.read(), np.uint8)


CPU_CASES = [
    "block_topology_try_from",
    "virtual_block_new_block",
    "virtual_block_unbuffered_backing",
    "virtual_block_unbuffered",
    "virtual_block_buffered",
    "virtual_block_erasure_buffered",
    "block_errors",
    "erasure_f32_hazard",
    "virtual_file_1",
    "virtual_file_2_4_mb",
    "virtual_file_errors",
    "virtual_file_chunk_model",
    "virtual_file_record_roundtrip",
    "virtual_file_record_fuzz",
    "read_needed_shards_plan",
]


@pytest.mark.parametrize("case", CPU_CASES)
def test_reference_case(case, tmp_path):
    run_case(case, tmp_path)


def test_library_exports():
    """libshmr_vfs.so links the codec through the C ABI only."""
    lib = os.path.join(ROOT, "shmr_amd", "_lib", "libshmr_vfs.so")
    assert os.path.exists(lib)
    nm = subprocess.run(["nm", "-D", "--undefined-only", lib], capture_output=True, text=True, check=True).stdout
    used = {l.split()[-1] for l in nm.splitlines() if "shmr_ec_" in l}
    # VirtualBlock::sync_data starts the encode and writes the data shard files
    # while it runs (shmr_ec_encode_start / shmr_ec_op_wait); load_block
    # reconstructs synchronously, or started when a copy-out overlaps it
    assert {"shmr_ec_new", "shmr_ec_encode_start", "shmr_ec_op_wait", "shmr_ec_reconstruct",
            "shmr_ec_reconstruct_start", "shmr_ec_encode_blocks_host"} <= used


# --------------------------------------------------------------------------- GPU

@pytest.mark.gpu
def test_erasure_block_sync_and_load(tmp_path, gpu):
    size, k, p = MiB, 8, 3
    data = O.seeded_block(O.BENCH_SEED, 101, 700_001)   # partial block: 6 chunks + 2 zero data shards
    files = run_case("erasure_block_sync_load", tmp_path, data)[0]
    want = O.sync_data_erasure(data.tobytes(), size, k, p)
    S = O.calculate_shard_size(size, k)
    assert len(files) == k + p
    for i, f in enumerate(files):
        if i == 1:
            assert os.path.getsize(f) == 0   # truncated by the test
            continue
        got = read(f)
        assert len(got) == S and np.array_equal(got, want[i]), f"shard {i}"
    # load with shard 1 truncated: zero-padded and kept present (reference rule)
    raw = [read(f).tobytes() for f in files]
    expect = O.load_block_erasure(raw, size, k, p)
    got = read(os.path.join(str(tmp_path), "loaded_truncated.bin"))
    assert np.array_equal(got, expect)


@pytest.mark.gpu
def test_erasure_block_missing_shards(tmp_path, gpu):
    data = O.seeded_block(O.BENCH_SEED, 102, MiB)
    run_case("erasure_block_missing_shards", tmp_path, data)


@pytest.mark.gpu
def test_erasure_flush_encode_failure(tmp_path, gpu):
    """A per-block flush (mapped Block Cache: started encode, data shard files
    written while the GPU runs) whose encode fails at the wait (test hook
    VfsOptions::fault_encode_wait): the parity files are unlinked (a reload
    that then loses a data shard fails -- TooFewShardsPresent under
    missing_shard_is_erasure with the reference's zero-pad rule for short
    shards, ENOENT without it -- instead of rebuilding from stale or zero
    parity), the block stays dirty, and the next unforced flush writes the
    oracle's stripe."""
    k, p = 8, 3
    data = np.concatenate([O.seeded_block(O.BENCH_SEED, 150 + i, MiB) for i in range(2)])
    files = run_case("erasure_flush_encode_failure", tmp_path, data)[0]
    want = O.sync_data_erasure(data[MiB:].tobytes(), MiB, k, p)
    for i, f in enumerate(files):
        if i in (2, 6):
            continue                      # removed by the test, rebuilt into the read
        assert np.array_equal(read(f), want[i]), f"shard {i}"


@pytest.mark.gpu
@pytest.mark.parametrize("buffers", ["mapped", "pageable"])
def test_direct_io_shard_files(tmp_path, gpu, buffers):
    """VfsOptions::direct_io: shard files written and read
    with O_DIRECT, or -- where the file system refuses it -- through the
    buffered path, counted (the case prints which); the shard files are the
    oracle's either way, and the read rebuilds a lost shard per block."""
    nblk, k, p = 4, 8, 3
    data = np.concatenate([O.seeded_block(O.BENCH_SEED, 700 + i, MiB) for i in range(nblk)])
    args = [BIN, "direct_io_" + buffers, str(tmp_path)]
    path = os.path.join(str(tmp_path), "input.bin")
    with open(path, "wb") as f:
        f.write(data.tobytes())
    out = subprocess.run(args + [path], capture_output=True, text=True, timeout=300)
    lines = out.stdout.strip().splitlines()
    assert out.returncode == 0 and lines and lines[-1] == "PASS", out.stdout + out.stderr
    direct = [l for l in lines if l.startswith("DIRECT ")]
    assert len(direct) == 1
    print(direct[0])
    shards = {}
    for line in lines:
        if line.startswith("SHARDS "):
            parts = line.split()
            shards[int(parts[1])] = parts[2:]
    for b in range(nblk):
        want = O.sync_data_erasure(data[b * MiB:(b + 1) * MiB].tobytes(), MiB, k, p)
        for i, fpath in enumerate(shards[b]):
            if i == (b * 3) % 11:
                continue                  # removed by the case (rebuilt into the read, rewritten by the flush)
            assert np.array_equal(read(fpath), want[i]), f"block {b} shard {i}"


@pytest.mark.gpu
def test_virtual_file_erasure_batch(tmp_path, gpu):
    nblk, k, p = 6, 8, 3
    data = np.concatenate([O.seeded_block(O.BENCH_SEED, 200 + i, MiB) for i in range(nblk)])
    shards = run_case("virtual_file_erasure_batch", tmp_path, data)
    assert sorted(shards) == list(range(nblk))
    for b in range(nblk):
        want = O.sync_data_erasure(data[b * MiB:(b + 1) * MiB].tobytes(), MiB, k, p)
        for i, f in enumerate(shards[b]):
            assert np.array_equal(read(f), want[i]), f"block {b} shard {i}"


@pytest.mark.gpu
def test_replace_block_erasure(tmp_path, gpu):
    data = O.seeded_block(O.BENCH_SEED, 300, 300_000)
    files = run_case("replace_block_erasure", tmp_path, data)[0]
    buf = np.zeros(MiB, np.uint8)   # the old Single block loads as a full 1 MiB buffer
    buf[:len(data)] = data
    want = O.sync_data_erasure(buf.tobytes(), MiB, 4, 2)
    assert len(files) == 6
    for i, f in enumerate(files):
        assert np.array_equal(read(f), want[i]), f"shard {i}"


@pytest.mark.gpu
def test_virtual_file_batched_reconstruct(tmp_path, gpu):
    nblk, k, p = 12, 8, 3
    data = np.concatenate([O.seeded_block(O.BENCH_SEED, 400 + i, MiB) for i in range(nblk)])
    shards = run_case("virtual_file_batched_reconstruct", tmp_path, data)
    assert sorted(shards) == list(range(nblk))
    # after the read the repair flush rewrote every shard: all must equal the oracle's
    for b in range(nblk):
        want = O.sync_data_erasure(data[b * MiB:(b + 1) * MiB].tobytes(), MiB, k, p)
        for i, f in enumerate(shards[b]):
            assert np.array_equal(read(f), want[i]), f"block {b} shard {i}"


@pytest.mark.gpu
def test_rewrite_erasure(tmp_path, gpu):
    data = O.seeded_block(O.BENCH_SEED, 500, 2 * MiB + 12345)
    shards = run_case("rewrite_erasure", tmp_path, data)
    for b, files in sorted(shards.items()):
        buf = np.zeros(MiB, np.uint8)   # each old Single block loads as a full 1 MiB buffer
        part = data[b * MiB:(b + 1) * MiB]
        buf[:len(part)] = part
        want = O.sync_data_erasure(buf.tobytes(), MiB, 4, 2)
        assert len(files) == 6
        for i, f in enumerate(files):
            assert np.array_equal(read(f), want[i]), f"block {b} shard {i}"


@pytest.mark.gpu
def test_virtual_file_mapped_per_block_flush(tmp_path, gpu):
    """Mapped Block Cache, auto batching: per-block zero-copy flushes on the
    worker pool (devices round-robin), then a pipelined load with one lost
    shard per block -- shard files equal the oracle's sync_data Erasure arm."""
    nblk, k, p = 10, 8, 3
    data = np.concatenate([O.seeded_block(O.BENCH_SEED, 600 + i, MiB) for i in range(nblk)])
    shards = run_case("virtual_file_mapped_per_block_flush", tmp_path, data)
    assert sorted(shards) == list(range(nblk))
    for b in range(nblk):
        want = O.sync_data_erasure(data[b * MiB:(b + 1) * MiB].tobytes(), MiB, k, p)
        for i, f in enumerate(shards[b]):
            assert np.array_equal(read(f), want[i]), f"block {b} shard {i}"


@pytest.mark.gpu
def test_erasure_f32_hazard_release(tmp_path, gpu):
    """VfsOptions::release_u8_wrap reproduces the reference's release build at
    block.rs:421 (u8 wrap: 9 chunks of a 16,777,217 B Erasure(1,8,3) buffer,
    chunk 8 overwritten by parity row 0 in the shard files) bit for bit, on
    the per-block and the batched flush; the default refuses (CPU case
    erasure_f32_hazard)."""
    size, k, p = 16777217, 8, 3
    case = KAT["f32_hazard_release"]
    data = O.seeded_block(*case["seed"], size)
    shards = run_case("erasure_f32_hazard_release", tmp_path, data)
    want = O.sync_data_erasure(data.tobytes(), size, k, p, mode="release")
    assert [sha(w) for w in want] == case["shard_sha256"]
    assert sorted(shards) == [0, 1]
    for blk in (0, 1):
        assert len(shards[blk]) == k + p
        for i, f in enumerate(shards[blk]):
            assert np.array_equal(read(f), want[i]), f"block {blk} shard {i}"
    loaded = read(os.path.join(str(tmp_path), "loaded_release.bin"))
    assert sha(loaded) == case["load_block_sha256"]
    assert np.array_equal(loaded, O.load_block_erasure([w.tobytes() for w in want], size, k, p))


@pytest.mark.gpu
def test_read_needed_shards(tmp_path, gpu):
    """VfsOptions::read_needed_shards: intact and degraded loads read 8 of 11
    RS(8,3) shard files per block (batched and per-block paths) and return the
    written bytes; a truncated shard under the reference's zero-pad rule reads
    all 11 and loads the same buffer as the read-everything path (checked in
    C++)."""
    data = O.seeded_block(O.BENCH_SEED, 701, 4 * MiB)
    run_case("read_needed_shards", tmp_path, data)


@pytest.mark.gpu
def test_virtual_block_erasure_fuzz(tmp_path, gpu):
    """120 random Erasure blocks (RS(3,1) .. RS(10,4), 1 B .. 3 MiB): random
    writes, flush, up to p shard files lost or truncated, reload, compare with
    a byte model -- twice per block, with mapped Block Cache and needed-shards
    reads chosen at random (checked in C++)."""
    run_case("virtual_block_erasure_fuzz", tmp_path, timeout=300)


@pytest.mark.gpu
def test_virtual_file_erasure_fuzz(tmp_path, gpu):
    """16 random files of 2-10 Erasure blocks (RS(3,1) .. RS(10,4), 1-2 MiB):
    three rounds of batched flush, random shard files lost or truncated in
    every block, batched load compared with a byte model, block-level
    rewrites; Block-Cache kind, batch size and needed-shards reads at random
    (checked in C++)."""
    run_case("virtual_file_erasure_fuzz", tmp_path, timeout=300)


@pytest.mark.gpu
def test_rewrite_erasure_record_reload(tmp_path, gpu):
    """a file rewritten to Erasure(1,8,3) reloads from its
    durable record (the reference's serde_yaml VirtualFile value) after
    everything in memory is dropped, loses one shard per block, and reads back
    bit-exact (checked in C++); the shard files equal the oracle's."""
    data = O.seeded_block(O.BENCH_SEED, 700, 2 * MiB + 12345)
    shards = run_case("rewrite_erasure_record_reload", tmp_path, data)
    assert sorted(shards) == [0, 1, 2]
    for b, files in sorted(shards.items()):
        buf = np.zeros(MiB, np.uint8)   # each old Single block loads as a full 1 MiB buffer
        part = data[b * MiB:(b + 1) * MiB]
        buf[:len(part)] = part
        want = O.sync_data_erasure(buf.tobytes(), MiB, 8, 3)
        assert len(files) == 11
        for i, f in enumerate(files):
            if i == (3 * b) % 11:
                assert not os.path.exists(f) or read(f).size == O.calculate_shard_size(MiB, 8)
                continue
            assert np.array_equal(read(f), want[i]), f"block {b} shard {i}"
    rec = open(os.path.join(str(tmp_path), "vf17.yaml")).read()
    assert rec.count("topology: !Erasure\n  - 1\n  - 8\n  - 3\n") == 3
