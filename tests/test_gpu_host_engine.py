"""GPU tests of the pipelined host-buffer batch engine (shmr_ec_encode_blocks_host /
shmr_ec_reconstruct_blocks_host): pageable and pinned buffers, several chunks
per device, mixed erasure patterns, bit-exact vs the CPU oracle."""
import numpy as np
import pytest

import shmr_amd
from oracle import c_oracle

pytestmark = pytest.mark.gpu


def oracle_parity(k, p, data):
    L = len(data[0])
    sh = [d.copy() for d in data] + [np.zeros(L, np.uint8) for _ in range(p)]
    c_oracle.encode(k, p, sh)
    return sh[k:]


@pytest.mark.parametrize("k,p,S,B", [(8, 3, 524288, 40), (4, 2, 262144, 7), (10, 4, 1677722, 6), (3, 2, 1000, 5)])
def test_encode_blocks_host_pageable(gpu, k, p, S, B):
    rng = np.random.default_rng([k, p, B])
    blocks = [[rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + [np.full(S, 7, np.uint8) for _ in range(p)]
              for _ in range(B)]
    shmr_amd.ReedSolomon(k, p).encode_blocks_host(blocks, devices=[0])
    for blk in blocks:
        ref = oracle_parity(k, p, blk[:k])
        for r in range(p):
            assert np.array_equal(blk[k + r], ref[r])


def test_encode_blocks_host_pinned(gpu):
    k, p, S, B = 8, 3, 524288, 20
    rng = np.random.default_rng(1)
    bufs = [shmr_amd.PinnedBuffer((k + p) * S) for _ in range(B)]
    blocks = []
    for buf in bufs:
        a = buf.array
        a[:k * S] = rng.integers(0, 256, k * S, dtype=np.uint8)
        blocks.append([a[i * S:(i + 1) * S] for i in range(k + p)])
    shmr_amd.ReedSolomon(k, p).encode_blocks_host(blocks, devices=[0])
    for blk in blocks:
        ref = oracle_parity(k, p, [x.copy() for x in blk[:k]])
        for r in range(p):
            assert np.array_equal(blk[k + r], ref[r])


@pytest.mark.parametrize("data_only", [False, True])
def test_reconstruct_blocks_host_mixed(gpu, data_only):
    k, p, S, B = 8, 3, 524288 + 100, 30
    rng = np.random.default_rng(2)
    full = []
    for _ in range(B):
        d = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
        full.append(d + oracle_parity(k, p, d))
    present = np.ones((B, k + p), np.uint8)
    for b in range(B):
        present[b, rng.choice(k + p, size=int(rng.integers(0, p + 1)), replace=False)] = 0
    blocks = [[full[b][i].copy() if present[b, i] else np.zeros(S, np.uint8) for i in range(k + p)]
              for b in range(B)]
    shmr_amd.ReedSolomon(k, p).reconstruct_blocks_host(blocks, present, data_only=data_only, devices=[0])
    for b in range(B):
        for i in range(k + p):
            if data_only and i >= k and not present[b, i]:
                assert not blocks[b][i].any()           # untouched
            else:
                assert np.array_equal(blocks[b][i], full[b][i]), (b, i)


def test_reconstruct_blocks_host_validates_first(gpu):
    k, p, S = 4, 2, 4096
    blocks = [[np.zeros(S, np.uint8) for _ in range(k + p)] for _ in range(3)]
    present = np.ones((3, k + p), np.uint8)
    present[2, :3] = 0                          # block 2 has only 3 of 4 needed shards
    with pytest.raises(shmr_amd.Error) as e:
        shmr_amd.ReedSolomon(k, p).reconstruct_blocks_host(blocks, present, devices=[0])
    assert e.value.name == "TooFewShardsPresent"


@pytest.mark.parametrize("mapped", [False, True])
def test_blocks_host_array_form(gpu, mapped):
    """encode/reconstruct_blocks_host on one [B, total, S] array (vectorised
    pointer marshalling), pageable and mapped, bit-exact vs the oracle."""
    k, p, S, B = 8, 3, 65536 + 4, 7
    rng = np.random.default_rng(31)
    keep = None
    if mapped:
        keep = shmr_amd.PinnedBuffer(B * (k + p) * S)
        arr = keep.array.reshape(B, k + p, S)
    else:
        arr = np.zeros((B, k + p, S), np.uint8)
    arr[:, :k] = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    rs = shmr_amd.ReedSolomon(k, p)
    z0, s0 = shmr_amd.path_stats()
    rs.encode_blocks_host(arr)
    z1, s1 = shmr_amd.path_stats()
    assert (z1 - z0, s1 - s0) == ((B, 0) if mapped else (0, B))
    for b in range(B):
        want = oracle_parity(k, p, [arr[b, i].copy() for i in range(k)])
        for r in range(p):
            assert np.array_equal(arr[b, k + r], want[r])
    full = arr.copy()
    present = np.ones((B, k + p), np.uint8)
    for b in range(B):
        present[b, [b % k, k + (b % p)]] = 0
        arr[b, b % k] = 0
        arr[b, k + b % p] = 0
    rs.reconstruct_blocks_host(arr, present)
    assert np.array_equal(arr, full)
    with pytest.raises(TypeError):
        rs.encode_blocks_host(arr[:, :, ::2])     # shard bytes not contiguous


@pytest.mark.parametrize("mirror_zc", [0, 1])
def test_pageable_batch_mirror_modes(gpu, mirror_zc):
    """Pageable host batches: the pinned mirror coded in place (zero-copy) or
    DMA'd to device staging -- identical, oracle-exact results."""
    saved = shmr_amd.get_tuning("mirror_zc")
    shmr_amd.set_tuning(mirror_zc=mirror_zc)
    try:
        k, p, S, B = 10, 4, 1677722, 5
        rng = np.random.default_rng([mirror_zc, 5])
        arr = np.zeros((B, k + p, S), np.uint8)
        arr[:, :k] = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
        rs = shmr_amd.ReedSolomon(k, p)
        rs.encode_blocks_host(arr)
        for b in range(B):
            want = oracle_parity(k, p, [arr[b, i].copy() for i in range(k)])
            for r in range(p):
                assert np.array_equal(arr[b, k + r], want[r])
        full = arr.copy()
        present = np.ones((B, k + p), np.uint8)
        for b in range(B):
            present[b, [b % k, (b + 3) % k, k + b % p]] = 0
            arr[b, [b % k, (b + 3) % k, k + b % p]] = 0
        rs.reconstruct_blocks_host(arr, present)
        assert np.array_equal(arr, full)
    finally:
        shmr_amd.set_tuning(mirror_zc=saved)
