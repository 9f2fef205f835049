"""Large address ranges and long shards, vs the CPU oracle, bit-exact.

The rest of the suite stays under ~3 GB per call, so no launch there puts a
shard more than 4 GiB past its base, and no shard is longer than 2 GiB.  A
device Block Cache sized for 288 GB of HBM does both.  These cases check that
the strided kernels' 64-bit address arithmetic holds past 4 GiB of block
offsets, against the table kernels (whose addresses are whole 64-bit pointers
from the table) and the oracle, and that shards longer than 2 GiB (the compact
rebuild's sc1 stores have a 2 GiB buffer resource per row: the policy switches
them off from 2 GiB - 4 KiB) encode and rebuild exactly.
"""
import ctypes

import numpy as np
import pytest

import shmr_amd
from oracle import c_oracle
from shmr_amd.reed_solomon import _u8p

pytestmark = pytest.mark.gpu

K, P = 8, 3
S = 512 << 10
PITCH = S + 4096          # the slot rule
B_BIG = 1100              # 1100 x 11 x 516 KiB = 6.2 GiB: offsets well past 4 GiB


def _stream():
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(0).cuda_stream)


def _oracle_parity(data):
    """data: host uint8 [n, k, S] -> [n, p, S]."""
    n, k, L = data.shape
    par = np.zeros((n, P, L), np.uint8)
    c_oracle.encode_batch(k, P, np.ascontiguousarray(data), par, n, L, 8)
    return par


def _sc1_launches():
    """Launches served so far by kernels with sc1 stores (flag kSc1Store)."""
    return sum(e["launches"] for e in shmr_amd.kernel_inventory() if e["flags"] & (1 << 23))


@pytest.fixture(scope="module")
def big(gpu):
    import torch
    g = torch.Generator(device=gpu).manual_seed(0x53484D52)
    t = torch.randint(0, 256, (B_BIG, K + P, PITCH), dtype=torch.uint8, device=gpu, generator=g)
    t[:, K:] = 0
    yield t
    del t
    torch.cuda.empty_cache()


def test_encode_beyond_4gib_of_offsets(gpu, big):
    """One strided encode over 6.2 GiB of slots: every block's parity equals the
    table kernels' (64-bit pointers, knob ptrs_grid=0) and, for blocks at the
    start, middle and end of the range, the oracle's."""
    import torch
    rs = shmr_amd.ReedSolomon(K, P)
    assert big.stride(0) * (B_BIG - 1) > (1 << 32)
    rs.encode_batch_dev(big[:, :K], big[:, K:], shard_len=S)
    torch.cuda.synchronize()
    # the same blocks through the table kernels, into a parity buffer of their own
    par = torch.zeros((B_BIG, P, S), dtype=torch.uint8, device=gpu)
    base, pbase = big.data_ptr(), par.data_ptr()
    tab = np.empty((B_BIG, K + P), np.uint64)
    tab[:, :K] = base + np.arange(B_BIG, dtype=np.uint64)[:, None] * np.uint64(big.stride(0)) + \
        np.arange(K, dtype=np.uint64)[None, :] * np.uint64(PITCH)
    tab[:, K:] = pbase + np.arange(B_BIG, dtype=np.uint64)[:, None] * np.uint64(P * S) + \
        np.arange(P, dtype=np.uint64)[None, :] * np.uint64(S)
    tab = np.ascontiguousarray(tab.reshape(-1))
    shmr_amd.set_tuning(ptrs_grid=0)
    try:
        assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab.ctypes.data_as(ctypes.POINTER(_u8p)), B_BIG, S, 0,
                                             _stream()) == 0
        torch.cuda.synchronize()
    finally:
        shmr_amd.set_tuning(ptrs_grid=-2)
    assert torch.equal(big[:, K:, :S], par)
    assert (big[:, K:, S:] == 0).all()                      # slot tails untouched
    for b in (0, 1, B_BIG // 2, B_BIG - 2, B_BIG - 1):
        data = big[b:b + 1, :K, :S].cpu().numpy()
        assert np.array_equal(big[b, K:, :S].cpu().numpy(), _oracle_parity(data)[0]), b


def test_reconstruct_beyond_4gib_of_offsets(gpu, big):
    """In-place rebuild of one or two lost shards per block over the same 6.2
    GiB range (patterns vary by block, so the launch carries a block/plan
    table): the lost bytes come back exactly."""
    import torch
    rs = shmr_amd.ReedSolomon(K, P)
    rs.encode_batch_dev(big[:, :K], big[:, K:], shard_len=S)
    torch.cuda.synchronize()
    present = np.ones((B_BIG, K + P), np.uint8)
    lost = list(range(B_BIG - 64, B_BIG)) + [0, 3, 700]     # the far end, and a few near the base
    for b in lost:
        present[b, b % K] = 0
        if b % 3 == 0:
            present[b, K + b % P] = 0
    keep = {b: big[b].clone() for b in lost}
    for b in lost:
        for i in np.flatnonzero(present[b] == 0):
            big[b, int(i)].fill_(0xEE)
    torch.cuda.synchronize()
    rs.reconstruct_batch_dev(big, present, shard_len=S)
    torch.cuda.synchronize()
    for b in lost:
        assert torch.equal(big[b, :, :S], keep[b][:, :S]), b


@pytest.mark.parametrize("L", [(1 << 31) + 4096 + 37, (1 << 31) - 4096 - 16, (1 << 31) - 4096])
def test_shards_around_and_past_2gib(gpu, L):
    """RS(2,1) with shards of 2 GiB - 4 KiB - 16 B (compact rebuild with sc1
    stores), exactly 2 GiB - 4 KiB (the first length without them) and 2 GiB +
    4 KiB + 37 B (the partial last tile more than 2 GiB into every shard):
    encode equals the oracle; a lost data shard rebuilt into a separate compact
    output equals the original."""
    import torch
    k, p = 2, 1
    pitch = (L + 4095) // 4096 * 4096
    g = torch.Generator(device=gpu).manual_seed(L)
    sh = torch.randint(0, 256, (1, k + p, pitch), dtype=torch.uint8, device=gpu, generator=g)
    sh[:, k:] = 0
    rs = shmr_amd.ReedSolomon(k, p)
    rs.encode_batch_dev(sh[:, :k], sh[:, k:], shard_len=L)
    torch.cuda.synchronize()
    host = [sh[0, i, :L].cpu().numpy() for i in range(k)] + [np.zeros(L, np.uint8)]
    c_oracle.encode(k, p, host)
    assert np.array_equal(sh[0, k, :L].cpu().numpy(), host[k])
    del host
    out = torch.full((1, 1, pitch), 0xA5, dtype=torch.uint8, device=gpu)
    present = np.array([[0, 1, 1]], np.uint8)
    sc1_before = _sc1_launches()
    rs.reconstruct_batch_dev_out(sh, present, out, shard_len=L)
    torch.cuda.synchronize()
    assert (_sc1_launches() > sc1_before) == (L < (1 << 31) - 4096)   # the policy's switch
    assert torch.equal(out[0, 0, :L], sh[0, 0, :L])
    assert (out[0, 0, L:] == 0xA5).all()
    del sh, out
    torch.cuda.empty_cache()
