"""Device-resident shards that live anywhere (shmr_ec_encode_ptrs_dev /
shmr_ec_reconstruct_ptrs_dev) vs the CPU oracle, bit-exact.

This is the crate's own argument shape on device memory: the reference copies
every S-byte chunk of the block buffer into a Vec<u8> of its own before
``encode`` (src/vfs/block.rs:408-427), and ``reconstruct`` turns every ``None``
shard into a fresh buffer (block.rs:556-565).  Here each shard is a separate
GPU buffer named by a pointer table: separate torch allocations, or slices of
one guarded arena at aligned and odd offsets (guards checked).
"""
import numpy as np
import pytest

import shmr_amd
from oracle import c_oracle

pytestmark = pytest.mark.gpu

GUARD = 0x5A


def _parity(k, p, data):
    B, _, S = data.shape
    par = np.zeros((B, p, S), np.uint8)
    c_oracle.encode_batch(k, p, np.ascontiguousarray(data), par, B, S, 8)
    return par


def _arena_shards(gpu, B, t, S, misalign, seed):
    """B x t shard views into one guarded arena; shard starts 16-byte aligned
    or (misalign) at scattered odd offsets, in shuffled order."""
    import torch
    rng = np.random.default_rng(seed)
    slot = (S + 64 + 255) // 256 * 256
    arena = torch.full((B * t * slot + 256,), GUARD, dtype=torch.uint8, device=gpu)
    order = rng.permutation(B * t)
    views = []
    for b in range(B):
        row = []
        for i in range(t):
            off = int(order[b * t + i]) * slot + 32 + (int(rng.integers(1, 16)) if misalign else 0)
            row.append(arena[off:off + S])
        views.append(row)
    return arena, views


def _guards_intact(arena, views):
    import torch
    mask = torch.ones(arena.numel(), dtype=torch.bool, device=arena.device)
    base = arena.data_ptr()
    for row in views:
        for v in row:
            o = v.data_ptr() - base
            mask[o:o + v.numel()] = False
    return bool((arena[mask] == GUARD).all())


@pytest.mark.parametrize("k,p,S,B", [(8, 3, 65536 + 12, 7), (10, 4, 3 * 8192 + 2458, 5), (4, 2, 4096, 9),
                                     (1, 1, 17, 3)])
@pytest.mark.parametrize("misalign", [False, True])
def test_encode_ptrs_matches_oracle(gpu, k, p, S, B, misalign):
    import torch
    t = k + p
    arena, views = _arena_shards(gpu, B, t, S, misalign, seed=k * 100 + S)
    rng = np.random.default_rng(S)
    data = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    for b in range(B):
        for i in range(k):
            views[b][i].copy_(torch.from_numpy(data[b, i]))
    shmr_amd.ReedSolomon(k, p).encode_ptrs_dev(views)
    torch.cuda.synchronize()
    want = _parity(k, p, data)
    for b in range(B):
        for r in range(p):
            assert np.array_equal(views[b][k + r].cpu().numpy(), want[b, r]), (b, r)
        for i in range(k):
            assert np.array_equal(views[b][i].cpu().numpy(), data[b, i]), ("data shard modified", b, i)
    assert _guards_intact(arena, views), "bytes outside the shards written"


def test_encode_ptrs_full_size_separate_allocations(gpu):
    """BASELINE configs 2 and 4 with every shard its own torch allocation (the
    crate's Vec<u8> per shard): RS(8,3) 4 MiB and RS(10,4) 16 MiB blocks."""
    import torch
    for k, p, size, B in ((8, 3, 4 << 20, 6), (10, 4, 16 << 20, 3)):
        S = shmr_amd.calculate_shard_size(size, k)
        g = torch.Generator(device=gpu).manual_seed(size)
        blocks = [[torch.randint(0, 256, (S,), dtype=torch.uint8, device=gpu, generator=g) for _ in range(k)]
                  + [torch.zeros(S, dtype=torch.uint8, device=gpu) for _ in range(p)] for _ in range(B)]
        shmr_amd.ReedSolomon(k, p).encode_ptrs_dev(blocks)
        torch.cuda.synchronize()
        data = np.stack([np.stack([s.cpu().numpy() for s in blk[:k]]) for blk in blocks])
        want = _parity(k, p, data)
        for b in range(B):
            for r in range(p):
                assert np.array_equal(blocks[b][k + r].cpu().numpy(), want[b, r]), (size, b, r)


def _codeword_blocks(gpu, k, p, S, B, seed):
    import torch
    rng = np.random.default_rng(seed)
    host = np.zeros((B, k + p, S), np.uint8)
    host[:, :k] = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    host[:, k:] = _parity(k, p, host[:, :k])
    return host, [[torch.from_numpy(host[b, i].copy()).to(gpu) for i in range(k + p)] for b in range(B)]


@pytest.mark.parametrize("k,p,erasures,B", [(8, 3, 1, 12), (8, 3, 3, 12), (10, 4, 2, 40), (10, 4, 4, 8)])
@pytest.mark.parametrize("data_only", [False, True])
def test_reconstruct_ptrs_none_become_fresh_buffers(gpu, k, p, erasures, B, data_only):
    """Mixed erasure patterns (40 blocks of random 2-erasure patterns: more
    than 32 runs, the uploaded table launch); None entries come back as fresh
    GPU buffers holding the crate's rebuilt shard; absent parity stays None
    under data_only; present shards are untouched; an all-present block is left
    alone."""
    import torch
    S = 2 * 4096 + 777
    t = k + p
    host, blocks = _codeword_blocks(gpu, k, p, S, B, seed=k * 7 + erasures)
    rng = np.random.default_rng([k, erasures, B])
    lost = []
    for b in range(B):
        m = [] if b == 2 else sorted(rng.choice(t, size=erasures, replace=False).tolist())
        lost.append(m)
        for i in m:
            blocks[b][i] = None
    keep = [[s for s in blk] for blk in blocks]
    shmr_amd.ReedSolomon(k, p).reconstruct_ptrs_dev(blocks, data_only=data_only)
    torch.cuda.synchronize()
    for b in range(B):
        for i in range(t):
            if i in lost[b]:
                if data_only and i >= k:
                    assert blocks[b][i] is None, ("absent parity filled under data_only", b, i)
                    continue
                assert blocks[b][i] is not None and blocks[b][i].numel() == S
                assert np.array_equal(blocks[b][i].cpu().numpy(), host[b, i]), (b, i)
            else:
                assert blocks[b][i] is keep[b][i]
                assert np.array_equal(blocks[b][i].cpu().numpy(), host[b, i]), ("present shard modified", b, i)


def test_reconstruct_ptrs_misaligned_buffers(gpu):
    """Present shards and output buffers at odd offsets of one guarded arena
    (the device's unaligned access mode), RS(10,4), 2 erasures per block."""
    import torch
    k, p, S, B = 10, 4, 3 * 8192 + 2458, 6
    t = k + p
    host, _ = _codeword_blocks(gpu, k, p, S, B, seed=3)
    arena, views = _arena_shards(gpu, B, t, S, True, seed=4)
    present = np.ones((B, t), np.uint8)
    for b in range(B):
        present[b, [b % t, (b + 5) % t]] = 0
        for i in range(t):
            if present[b, i]:
                views[b][i].copy_(torch.from_numpy(host[b, i]))
    rs = shmr_amd.ReedSolomon(k, p)
    ptrs = (shmr_amd.reed_solomon._u8p * (B * t))(*[shmr_amd.reed_solomon.ctypes.cast(
        views[b][i].data_ptr(), shmr_amd.reed_solomon._u8p) for b in range(B) for i in range(t)])
    import ctypes
    stream = ctypes.c_void_p(torch.cuda.current_stream(0).cuda_stream)
    pr = np.ascontiguousarray(present)
    rc = rs._L.shmr_ec_reconstruct_ptrs_dev(rs._h, ptrs, pr.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), B, S, 0,
                                            0, stream)
    assert rc == 0, shmr_amd.reed_solomon.lib().shmr_ec_status_name(rc)
    torch.cuda.synchronize()
    for b in range(B):
        for i in range(t):
            assert np.array_equal(views[b][i].cpu().numpy(), host[b, i]), (b, i)
    assert _guards_intact(arena, views)


def test_ptrs_graph_capture(gpu):
    """Pointer-table calls are stream-ordered: an encode and a reconstruct with
    an unseen pattern captured into a graph, replayed twice, bit-exact, and no
    blocking HIP call inside the capture."""
    import torch
    k, p, S, B = 6, 5, 8192 + 100, 4
    t = k + p
    rs = shmr_amd.ReedSolomon(k, p)
    shmr_amd.device_init(0)
    base = shmr_amd.device_stats(0)["blocking_calls"]
    g = torch.Generator(device=gpu).manual_seed(77)
    enc = [[torch.empty(S, dtype=torch.uint8, device=gpu) for _ in range(t)] for _ in range(B)]
    host, dec = _codeword_blocks(gpu, k, p, S, B, seed=78)
    lost = [[0, 7], [3], [1, 2, 9], [10]]
    outs = [[torch.empty(S, dtype=torch.uint8, device=gpu) if i in lost[b] else dec[b][i] for i in range(t)]
            for b in range(B)]
    present = np.array([[i not in lost[b] for i in range(t)] for b in range(B)], np.uint8)
    import ctypes
    from shmr_amd.reed_solomon import _u8p
    tab = (_u8p * (B * t))(*[ctypes.cast(outs[b][i].data_ptr(), _u8p) for b in range(B) for i in range(t)])
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    stream = torch.cuda.Stream()
    with torch.cuda.graph(graph, stream=stream):
        rs.encode_ptrs_dev(enc)
        rc = rs._L.shmr_ec_reconstruct_ptrs_dev(rs._h, tab, np.ascontiguousarray(present).ctypes.data_as(
            ctypes.POINTER(ctypes.c_uint8)), B, S, 0, 0, ctypes.c_void_p(stream.cuda_stream))
    assert rc == 0
    assert shmr_amd.device_stats(0)["blocking_calls"] == base, "a blocking HIP call inside the capture"
    for rep in range(2):
        for b in range(B):
            for i in range(k):
                enc[b][i].copy_(torch.randint(0, 256, (S,), dtype=torch.uint8, device=gpu, generator=g))
            for i in lost[b]:
                outs[b][i].fill_(0xEE)
        torch.cuda.synchronize()
        graph.replay()
        torch.cuda.synchronize()
        data = np.stack([np.stack([s.cpu().numpy() for s in blk[:k]]) for blk in enc])
        want = _parity(k, p, data)
        for b in range(B):
            for r in range(p):
                assert np.array_equal(enc[b][k + r].cpu().numpy(), want[b, r]), (rep, b, r)
            for i in lost[b]:
                assert np.array_equal(outs[b][i].cpu().numpy(), host[b, i]), (rep, b, i)


def test_ptrs_validation(gpu):
    """Crate error order in the shim (shard count, EmptyShard,
    IncorrectShardSize, TooFewShardsPresent) before any launch; the library
    refuses NULL shards that a call would touch."""
    import ctypes
    import torch
    rs = shmr_amd.ReedSolomon(4, 2)
    z = lambda n=64: torch.zeros(n, dtype=torch.uint8, device=gpu)  # noqa: E731
    with pytest.raises(shmr_amd.Error) as e:
        rs.encode_ptrs_dev([[z() for _ in range(5)]])
    assert e.value.name == "TooFewShards"
    with pytest.raises(shmr_amd.Error) as e:
        rs.encode_ptrs_dev([[z() for _ in range(7)]])
    assert e.value.name == "TooManyShards"
    with pytest.raises(shmr_amd.Error) as e:
        rs.encode_ptrs_dev([[z(0) for _ in range(6)]])
    assert e.value.name == "EmptyShard"
    with pytest.raises(shmr_amd.Error) as e:
        rs.encode_ptrs_dev([[z() for _ in range(5)] + [z(65)]])
    assert e.value.name == "IncorrectShardSize"
    with pytest.raises(shmr_amd.Error) as e:
        rs.reconstruct_ptrs_dev([[None, None, None, z(), z(), z()]])
    assert e.value.name == "TooFewShardsPresent"
    from shmr_amd.reed_solomon import _u8p
    tab = (_u8p * 6)(*([ctypes.cast(z().data_ptr(), _u8p) for _ in range(5)] + [_u8p()]))
    assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab, 1, 64, 0, None) == -100    # InvalidArgument
    # data_only: an absent parity shard may be NULL
    host, blocks = _codeword_blocks(gpu, 4, 2, 64, 1, seed=1)
    pres = np.array([1, 0, 1, 1, 1, 0], np.uint8)
    out1 = z()
    tab = (_u8p * 6)(*[ctypes.cast((out1 if i == 1 else blocks[0][i]).data_ptr(), _u8p) if i != 5 else _u8p()
                       for i in range(6)])
    rc = rs._L.shmr_ec_reconstruct_ptrs_dev(rs._h, tab, pres.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), 1, 64,
                                            1, 0, None)
    assert rc == 0
    torch.cuda.synchronize()
    assert np.array_equal(out1.cpu().numpy(), host[0, 1])
    assert rs._L.shmr_ec_reconstruct_ptrs_dev(rs._h, tab, pres.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), 1,
                                              64, 0, 0, None) == -100      # the same without data_only


def test_ptrs_table_cache(gpu, table_kernels):
    """A table passed again on the same stream is reused from the device's
    table cache (no upload; counter ptr_table_hits), and stays exact when the
    shards' bytes change between calls; a changed table, or the same table on
    another stream, is uploaded again; more distinct tables than cache entries
    cycle through it (and through the ring when busy) without a mismatch."""
    import torch
    k, p, S, B = 8, 3, 4096 * 3 + 100, 5
    t = k + p
    rs = shmr_amd.ReedSolomon(k, p)
    shmr_amd.device_init(0)
    g = torch.Generator(device=gpu).manual_seed(3)
    sets = [[[torch.empty(S, dtype=torch.uint8, device=gpu) for _ in range(t)] for _ in range(B)] for _ in range(11)]

    def check(blocks):
        data = np.stack([np.stack([s.cpu().numpy() for s in blk[:k]]) for blk in blocks])
        want = _parity(k, p, data)
        for b in range(B):
            for r in range(p):
                assert np.array_equal(blocks[b][k + r].cpu().numpy(), want[b, r]), (b, r)

    def fill(blocks):
        for blk in blocks:
            for s in blk[:k]:
                s.copy_(torch.randint(0, 256, (S,), dtype=torch.uint8, device=gpu, generator=g))

    hits = lambda: shmr_amd.device_stats(0)["ptr_table_hits"]  # noqa: E731
    fill(sets[0])
    rs.encode_ptrs_dev(sets[0])
    torch.cuda.synchronize()
    check(sets[0])
    h0 = hits()
    fill(sets[0])                       # same table, new bytes
    rs.encode_ptrs_dev(sets[0])
    torch.cuda.synchronize()
    assert hits() == h0 + 1
    check(sets[0])
    fill(sets[1])                       # another table: uploaded
    rs.encode_ptrs_dev(sets[1])
    torch.cuda.synchronize()
    assert hits() == h0 + 1
    check(sets[1])
    side = torch.cuda.Stream()
    fill(sets[0])
    with torch.cuda.stream(side):      # same table, other stream: its own upload
        rs.encode_ptrs_dev(sets[0])
    torch.cuda.synchronize()
    assert hits() == h0 + 1
    check(sets[0])
    for rep in range(3):                # 11 tables > 8 entries, back to back without a sync
        for s in sets:
            fill(s)
            rs.encode_ptrs_dev(s)
        torch.cuda.synchronize()
        for s in sets:
            check(s)


def test_ptrs_many_shards_and_chunks(gpu, table_kernels):
    """RS(200,55) (255 shards, the crate's maximum total) over 130 blocks: the
    pointer table spans two upload chunks (128 blocks per 256 KiB slot); encode,
    then a reconstruct with random erasures (up to 55 per block, mixed patterns),
    run twice so the second pass reads both chunks from the table cache."""
    import ctypes
    import torch
    from shmr_amd.reed_solomon import _u8p
    k, p, S, B = 200, 55, 48, 130
    t = k + p
    slot = 64
    rng = np.random.default_rng(255)
    arena = torch.zeros(B * t * slot + 64, dtype=torch.uint8, device=gpu)
    base = arena.data_ptr()
    addr = np.array([base + (b * t + i) * slot for b in range(B) for i in range(t)], dtype=np.uint64)
    tab = addr.ctypes.data_as(ctypes.POINTER(_u8p))
    rs = shmr_amd.ReedSolomon(k, p)
    stream = ctypes.c_void_p(torch.cuda.current_stream(0).cuda_stream)
    view = arena[:B * t * slot].view(B, t, slot)
    for rep in range(2):
        data = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
        view[:, :k, :S] = torch.from_numpy(data).to(gpu)
        hits0 = shmr_amd.device_stats(0)["ptr_table_hits"]
        assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab, B, S, 0, stream) == 0
        torch.cuda.synchronize()
        if rep:
            assert shmr_amd.device_stats(0)["ptr_table_hits"] == hits0 + 2
        got = view[:, :, :S].cpu().numpy()
        want = _parity(k, p, data)
        assert np.array_equal(got[:, k:], want)
        present = np.ones((B, t), np.uint8)
        for b in range(B):
            present[b, rng.choice(t, size=int(rng.integers(1, p + 1)), replace=False)] = 0
        erased = torch.from_numpy(present == 0).to(gpu)
        shard_bytes = view[:, :, :S]
        shard_bytes[erased] = 0xEE            # absent shards' bytes (the slot tails stay 0)
        rc = rs._L.shmr_ec_reconstruct_ptrs_dev(rs._h, tab, present.ctypes.data_as(_u8p), B, S, 0, 0, stream)
        assert rc == 0
        torch.cuda.synchronize()
        assert np.array_equal(view[:, :, :S].cpu().numpy(), got)
        assert (view[:, :, S:].cpu().numpy() == 0).all(), "bytes past the shards written"
