"""GPU tests of the zero-copy host path: shards in mapped host memory
(shmr_ec_host_alloc / shmr_ec_host_register) are encoded and rebuilt in place
by the kernel across PCIe through a device table of shard pointers.  Every
case checks the path that ran (shmr_ec_path_stats) and the bytes against the
CPU oracle, bit-exact.

Reference call sites: ReedSolomon::encode (src/vfs/block.rs:427) and
ReedSolomon::reconstruct (src/vfs/block.rs:560) on Block Cache buffers
(VirtualBlock::sync_data / load_block, block.rs:404-440, 529-579).
"""
import numpy as np
import pytest

import shmr_amd
from oracle import c_oracle

pytestmark = pytest.mark.gpu


def oracle_parity(k, p, data):
    L = len(data[0])
    sh = [np.ascontiguousarray(d).copy() for d in data] + [np.zeros(L, np.uint8) for _ in range(p)]
    c_oracle.encode(k, p, sh)
    return sh[k:]


class Delta:
    """Blocks each path served during a with-block."""

    def __enter__(self):
        self.z0, self.s0 = shmr_amd.path_stats()
        return self

    def __exit__(self, *exc):
        z, s = shmr_amd.path_stats()
        self.zero_copy, self.staged = z - self.z0, s - self.s0


def pinned_blocks(rng, k, p, S, B, offset=0, gap=0):
    """B blocks in one mapped buffer; shard i of block b at
    offset + b*((k+p)*(S+gap)) + i*(S+gap) (offset/gap de-align on purpose)."""
    stride = S + gap
    buf = shmr_amd.PinnedBuffer(offset + B * (k + p) * stride + 16)
    a = buf.array
    a[:] = 0x5A
    blocks = []
    for b in range(B):
        base = offset + b * (k + p) * stride
        blk = [a[base + i * stride: base + i * stride + S] for i in range(k + p)]
        for i in range(k):
            blk[i][:] = rng.integers(0, 256, S, dtype=np.uint8)
        blocks.append(blk)
    return buf, blocks


@pytest.mark.parametrize("k,p,S,B,offset,gap", [
    (8, 3, 524288, 24, 0, 0),        # BASELINE config 2 shape, Block-Cache layout
    (10, 4, 1677722, 3, 0, 0),       # config 4: S = 2 mod 4, so shards 1.. are unaligned
    (4, 2, 262144, 9, 0, 0),         # config 1 shape
    (8, 3, 4096 * 3 + 48, 5, 16, 16),  # tail tile, aligned
    (5, 3, 1001, 7, 3, 5),           # every shard unaligned: byte-granular kernel
    (1, 1, 1, 4, 0, 0),
    (17, 7, 8192, 3, 0, 0),          # 7 parity rows: two launches (4 + 3)
])
def test_encode_blocks_zero_copy(gpu, k, p, S, B, offset, gap):
    rng = np.random.default_rng([k, p, S, B])
    buf, blocks = pinned_blocks(rng, k, p, S, B, offset, gap)
    with Delta() as d:
        shmr_amd.ReedSolomon(k, p).encode_blocks_host(blocks, devices=[0])
    assert (d.zero_copy, d.staged) == (B, 0)
    for blk in blocks:
        for got, want in zip(blk[k:], oracle_parity(k, p, blk[:k])):
            assert np.array_equal(got, want)
    if gap:   # bytes between shards untouched
        a = buf.array
        stride = S + gap
        for b in range(B):
            for i in range(k + p):
                end = offset + b * (k + p) * stride + i * stride + S
                assert (a[end:end + gap] == 0x5A).all()


@pytest.mark.parametrize("data_only", [False, True])
@pytest.mark.parametrize("k,p,S", [(8, 3, 524288 + 100), (10, 4, 1677722), (6, 6, 777)])
def test_reconstruct_blocks_zero_copy_mixed(gpu, k, p, S, data_only):
    B = 12
    rng = np.random.default_rng([k, p, S, int(data_only)])
    buf, blocks = pinned_blocks(rng, k, p, S, B)
    shmr_amd.ReedSolomon(k, p).encode_blocks_host(blocks, devices=[0])
    full = [[x.copy() for x in blk] for blk in blocks]
    present = np.ones((B, k + p), np.uint8)
    for b in range(B):
        if b == 0:
            continue   # one block with nothing missing (crate no-op)
        present[b, rng.choice(k + p, size=int(rng.integers(1, p + 1)), replace=False)] = 0
    for b in range(B):
        for i in range(k + p):
            if not present[b, i]:
                blocks[b][i][:] = 0
    with Delta() as d:
        shmr_amd.ReedSolomon(k, p).reconstruct_blocks_host(blocks, present, data_only=data_only, devices=[0])
    assert (d.zero_copy, d.staged) == (B, 0)
    for b in range(B):
        for i in range(k + p):
            if data_only and i >= k and not present[b, i]:
                assert not blocks[b][i].any()
            else:
                assert np.array_equal(blocks[b][i], full[b][i]), (b, i)


@pytest.mark.parametrize("direct", [0, 1 << 20])
@pytest.mark.parametrize("k,p,S,B", [(8, 3, 4096, 1), (8, 3, 12288 + 48, 3), (10, 4, 1677722, 2)])
def test_pointer_table_in_place_or_uploaded(gpu, direct, k, p, S, B):
    """Shard-pointer tables read in place from the pinned ring slot (ptrs_direct
    large) or uploaded first (ptrs_direct 0): same bytes either way."""
    rng = np.random.default_rng([k, S, B, direct])
    buf, blocks = pinned_blocks(rng, k, p, S, B)
    rs = shmr_amd.ReedSolomon(k, p)
    try:
        shmr_amd.set_tuning(ptrs_direct=direct)
        with Delta() as d:
            rs.encode_blocks_host(blocks, devices=[0])
        assert (d.zero_copy, d.staged) == (B, 0)
        for blk in blocks:
            for got, want in zip(blk[k:], oracle_parity(k, p, blk[:k])):
                assert np.array_equal(got, want)
        full = [[x.copy() for x in blk] for blk in blocks]
        present = np.ones((B, k + p), np.uint8)
        for b in range(B):
            present[b, [b % k, k + (b % p)]] = 0
            blocks[b][b % k][:] = 0
            blocks[b][k + (b % p)][:] = 0
        rs.reconstruct_blocks_host(blocks, present, devices=[0])
        for b in range(B):
            for i in range(k + p):
                assert np.array_equal(blocks[b][i], full[b][i]), (b, i)
    finally:
        shmr_amd.set_tuning(ptrs_direct=-2)


def test_single_block_calls_zero_copy(gpu):
    """The drop-in per-block calls (shmr_ec_encode / shmr_ec_reconstruct) on
    mapped shards: in place, no staging."""
    k, p, S = 8, 3, 524288
    rng = np.random.default_rng(5)
    buf, (blk,) = pinned_blocks(rng, k, p, S, 1)
    rs = shmr_amd.ReedSolomon(k, p)
    with Delta() as d:
        rs.encode(blk)
    assert (d.zero_copy, d.staged) == (1, 0)
    want = oracle_parity(k, p, blk[:k])
    for got, w in zip(blk[k:], want):
        assert np.array_equal(got, w)
    full = [x.copy() for x in blk]
    blk[2][:] = 0
    blk[k + 1][:] = 0
    # reconstruct() takes buffers for absent shards as None -> the shim allocates
    # pageable ones, so drive the C ABI with mapped buffers for every shard.
    import ctypes
    from shmr_amd._native import _u8p, lib
    present = np.ones(k + p, np.uint8)
    present[[2, k + 1]] = 0
    ptrs = (_u8p * (k + p))(*[x.ctypes.data_as(_u8p) for x in blk])
    lens = (ctypes.c_size_t * (k + p))(*([S] * (k + p)))
    with Delta() as d:
        rc = lib().shmr_ec_reconstruct(rs._h, ptrs, lens, present.ctypes.data_as(_u8p), k + p, 0)
    assert rc == 0
    assert (d.zero_copy, d.staged) == (1, 0)
    for got, w in zip(blk, full):
        assert np.array_equal(got, w)


def test_registered_numpy_buffers(gpu):
    """shmr_ec_host_register on plain numpy memory (a Vec<u8> Block Cache
    buffer in the reference) makes it zero-copy; after unregister the same
    buffers take the staged path with identical results."""
    k, p, S, B = 8, 3, 65536 + 32, 6
    rng = np.random.default_rng(9)
    big = np.zeros(B * (k + p) * S, np.uint8)
    blocks = [[big[(b * (k + p) + i) * S:(b * (k + p) + i + 1) * S] for i in range(k + p)] for b in range(B)]
    for blk in blocks:
        for i in range(k):
            blk[i][:] = rng.integers(0, 256, S, dtype=np.uint8)
    rs = shmr_amd.ReedSolomon(k, p)
    shmr_amd.host_register(big)
    try:
        with Delta() as d:
            rs.encode_blocks_host(blocks, devices=[0])
        assert (d.zero_copy, d.staged) == (B, 0)
        zc = [[x.copy() for x in blk[k:]] for blk in blocks]
    finally:
        shmr_amd.host_unregister(big)
    for blk in blocks:
        for i in range(k, k + p):
            blk[i][:] = 0
    with Delta() as d:
        rs.encode_blocks_host(blocks, devices=[0])
    assert (d.zero_copy, d.staged) == (0, B)
    for b, blk in enumerate(blocks):
        want = oracle_parity(k, p, blk[:k])
        for r in range(p):
            assert np.array_equal(blk[k + r], want[r])
            assert np.array_equal(zc[b][r], want[r])


def test_partly_mapped_batch_is_staged(gpu):
    """One pageable shard in the batch: the whole call stages (the kernel
    never touches unmapped host memory)."""
    k, p, S, B = 4, 2, 8192, 3
    rng = np.random.default_rng(11)
    buf, blocks = pinned_blocks(rng, k, p, S, B)
    blocks[1][k + 1] = np.zeros(S, np.uint8)     # pageable parity buffer
    with Delta() as d:
        shmr_amd.ReedSolomon(k, p).encode_blocks_host(blocks, devices=[0])
    assert (d.zero_copy, d.staged) == (0, B)
    for blk in blocks:
        for got, want in zip(blk[k:], oracle_parity(k, p, blk[:k])):
            assert np.array_equal(got, want)


def test_register_errors(gpu):
    from shmr_amd._native import lib
    import ctypes
    assert lib().shmr_ec_host_unregister(ctypes.c_void_p(12345)) == -100   # never registered
    assert lib().shmr_ec_host_register(None, 10) == -100


def _start(rs, fn, shards, present=None, data_only=False):
    """shmr_ec_encode_start / shmr_ec_reconstruct_start through ctypes: (rc, op)."""
    import ctypes
    from shmr_amd.reed_solomon import _ptr, _u8p
    n = len(shards)
    L = next(len(s) for s in shards if s is not None)
    ptrs = (_u8p * n)(*[(_ptr(s) if s is not None else _u8p()) for s in shards])
    lens = (ctypes.c_size_t * n)(*[(L if s is not None and (present is None or present[i]) else 0)
                                   for i, s in enumerate(shards)])
    op = ctypes.c_void_p()
    if fn == "encode":
        rc = rs._L.shmr_ec_encode_start(rs._h, ptrs, lens, n, ctypes.byref(op))
    else:
        pr = np.ascontiguousarray(present, dtype=np.uint8)
        rc = rs._L.shmr_ec_reconstruct_start(rs._h, ptrs, lens, _ptr(pr), n, int(data_only), ctypes.byref(op))
    return rc, op


@pytest.mark.parametrize("mapped", [True, False])
def test_started_encode_and_reconstruct(gpu, mapped):
    """shmr_ec_encode_start / shmr_ec_reconstruct_start + shmr_ec_op_wait (the
    Block Cache's overlap of shard-file writes and copy-outs with the GPU
    work): mapped shards run zero-copy and the inputs may be read while the
    op is pending; pageable shards finish inside the start call.  Bytes equal
    the oracle's; validation errors come from the start call with no op."""
    k, p, S = 8, 3, 3 * 4096 + 100
    rng = np.random.default_rng(31 + int(mapped))
    rs = shmr_amd.ReedSolomon(k, p)
    if mapped:
        keep, blocks = pinned_blocks(rng, k, p, S, 1)
        sh = blocks[0]
    else:
        sh = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + [np.zeros(S, np.uint8) for _ in range(p)]
    want = oracle_parity(k, p, sh[:k])
    with Delta() as d:
        rc, op = _start(rs, "encode", sh)
        assert rc == 0 and op.value
        snapshot = [s.copy() for s in sh[:k]]          # reading the inputs meanwhile is allowed
        assert rs._L.shmr_ec_op_wait(op) == 0
    assert (d.zero_copy, d.staged) == ((1, 0) if mapped else (0, 1))
    assert all(np.array_equal(a, b) for a, b in zip(snapshot, sh[:k]))
    for r in range(p):
        assert np.array_equal(sh[k + r], want[r]), r
    full = [s.copy() for s in sh]
    present = np.ones(k + p, np.uint8)
    present[[1, 6, 9]] = 0
    for i in (1, 6, 9):
        sh[i][:] = 0xEE
    rc, op = _start(rs, "reconstruct", sh, present)
    assert rc == 0 and op.value
    assert rs._L.shmr_ec_op_wait(op) == 0
    for i in range(k + p):
        assert np.array_equal(sh[i], full[i]), i
    # all present: a completed op; too few present: the crate's error, no op
    rc, op = _start(rs, "reconstruct", sh, np.ones(k + p, np.uint8))
    assert rc == 0 and rs._L.shmr_ec_op_wait(op) == 0
    few = np.ones(k + p, np.uint8)
    few[:4] = 0
    rc, op = _start(rs, "reconstruct", sh, few)
    assert shmr_amd.Error(rc).name == "TooFewShardsPresent" and not op.value
    assert shmr_amd.Error(rs._L.shmr_ec_op_wait(None)).name == "InvalidArgument"
