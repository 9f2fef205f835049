"""Shard buffers in slot placement (shmr_ec_device_alloc_shards) and pointer
tables that name a slot grid (knob ptrs_grid), vs the CPU oracle, bit-exact.

The crate keeps every shard in a Vec<u8> of its own (reference
src/vfs/block.rs:408-419) and rebuilds every ``None`` shard into a fresh buffer
(block.rs:556-565).  A device Block Cache that takes those buffers from the
library's slab allocator hands *_ptrs_dev a table whose shards sit on a grid;
the library then runs the strided kernels of the *_batch_dev calls (counter
``ptr_table_grids``).  These tests check the allocator's placement, that grid
tables (encode; in-place and fresh-buffer rebuilds; data_only) give the
oracle's bytes, that a table off the grid still takes the table kernels, and
that both paths write the same bytes.
"""
import ctypes

import numpy as np
import pytest

import shmr_amd
from oracle import c_oracle
from shmr_amd.reed_solomon import _u8p

pytestmark = pytest.mark.gpu


def _parity(k, p, data):
    B, _, S = data.shape
    par = np.zeros((B, p, S), np.uint8)
    c_oracle.encode_batch(k, p, np.ascontiguousarray(data), par, B, S, 8)
    return par


def _stream():
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(0).cuda_stream)


def _tab(addrs):
    a = np.ascontiguousarray(addrs, dtype=np.uint64)
    return a, a.ctypes.data_as(ctypes.POINTER(_u8p))


def _stats():
    return shmr_amd.device_stats(0)


def _slot_pitch(S):
    p = (S + 4095) // 4096 * 4096
    return p + 4096 if p % 65536 == 0 else p


def test_alloc_shards_placement_and_free(gpu):
    """Slot pitch = S rounded up to 4 KiB, one page more for a power-of-two
    stride; buffers in table order, 256-byte aligned; only the slab base frees
    it, on its own device."""
    L = shmr_amd.reed_solomon.lib()
    for S, pitch in ((524288, 528384), (1677722, 1679360), (262144, 266240), (17, 4096), (4096 * 3 + 5, 16384)):
        assert _slot_pitch(S) == pitch
        slab = shmr_amd.ShardSlab(3, 11, S)
        assert slab.pitch == pitch
        assert int(slab.ptrs[0]) % 256 == 0
        assert np.array_equal(np.diff(slab.ptrs.astype(np.int64)), np.full(32, pitch))
        del slab
    assert shmr_amd.ShardSlab(1, 1, 65536).pitch == 69632          # one buffer: the same rule
    arr = (_u8p * 4)()
    assert L.shmr_ec_device_alloc_shards(0, 0, 4, 64, arr) == -100
    assert L.shmr_ec_device_alloc_shards(0, 1, 0, 64, arr) == -100
    assert L.shmr_ec_device_alloc_shards(0, 1, 4, 0, arr) == -100
    assert L.shmr_ec_device_alloc_shards(0, 1, 4, 64, None) == -100
    assert L.shmr_ec_device_alloc_shards(0, 1, 4, 64, arr) == 0
    assert L.shmr_ec_device_free_shards(0, arr[1]) == -100          # not a slab base
    assert L.shmr_ec_device_free_shards(1, arr[0]) in (-100,)       # another device ID
    assert L.shmr_ec_device_free_shards(0, arr[0]) == 0
    assert L.shmr_ec_device_free_shards(0, arr[0]) == -100          # freed already
    assert L.shmr_ec_device_free_shards(0, None) == 0
    # freed the plain way, a slab leaves no registry entry behind
    assert L.shmr_ec_device_alloc_shards(0, 1, 4, 64, arr) == 0
    assert L.shmr_ec_device_free(0, arr[0]) == 0
    assert L.shmr_ec_device_free_shards(0, arr[0]) == -100


def _needs_plan_list(present, k_max_segs=32):
    """Mirror of ptrs.cpp lattice_needs_plan_list for blocks on slots 0..B-1:
    several erasure patterns of one absent count whose blocks fall into more
    arithmetic runs than the kernel arguments hold send a rebuild to the table
    kernels (no grid call counted)."""
    by_pattern = {}
    for b, row in enumerate(np.asarray(present)):
        by_pattern.setdefault(bytes(row), []).append(b)
    by_m = {}
    for pat, slots in by_pattern.items():
        m = sum(1 for x in pat if not x)
        runs, i = 0, 0
        while i < len(slots):
            e = i + 1
            st = slots[e] - slots[i] if e < len(slots) else 1
            while e < len(slots) and slots[e] - slots[e - 1] == st:
                e += 1
            runs += 1
            i = e
        c = by_m.setdefault(m, [0, 0])
        c[0] += 1
        c[1] += runs
    return any(n > 1 and r > k_max_segs for n, r in by_m.values())


@pytest.mark.parametrize("k,p,S,B", [(8, 3, 65536, 9), (10, 4, 3 * 8192 + 2458, 5), (4, 2, 4096 * 5, 33),
                                     (1, 1, 17, 4)])
@pytest.mark.parametrize("joint", [True, False])
def test_grid_encode(gpu, k, p, S, B, joint):
    """Encode over slab buffers: all total shards of a block in one slab
    (joint), or data and parity in slabs of their own; the parity rows equal
    the oracle's, data untouched, slot tails untouched, one grid call and no
    table upload."""
    import torch
    t = k + p
    rng = np.random.default_rng([k, S, B, joint])
    data = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    if joint:
        slab = shmr_amd.ShardSlab(B, t, S)
        view = slab.tensor()
        view.fill_(0x5A)
        view[:, :k, :S] = torch.from_numpy(data).to(gpu)
        addrs = slab.ptrs
        dview, pview = view[:, :k], view[:, k:]
    else:
        ds, ps = shmr_amd.ShardSlab(B, k, S), shmr_amd.ShardSlab(B, p, S)
        dview, pview = ds.tensor(), ps.tensor()
        dview.fill_(0x5A)
        pview.fill_(0x5A)
        dview[:, :, :S] = torch.from_numpy(data).to(gpu)
        addrs = np.concatenate([ds.ptrs.reshape(B, k), ps.ptrs.reshape(B, p)], axis=1).reshape(-1)
    torch.cuda.synchronize()
    st0 = _stats()
    rs = shmr_amd.ReedSolomon(k, p)
    keep, tab = _tab(addrs)
    assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab, B, S, 0, _stream()) == 0
    torch.cuda.synchronize()
    st1 = _stats()
    assert st1["ptr_table_grids"] == st0["ptr_table_grids"] + 1
    assert st1["ptr_table_hits"] == st0["ptr_table_hits"]
    assert np.array_equal(pview[:, :, :S].cpu().numpy(), _parity(k, p, data))
    assert np.array_equal(dview[:, :, :S].cpu().numpy(), data)
    assert (dview[:, :, S:].cpu().numpy() == 0x5A).all() and (pview[:, :, S:].cpu().numpy() == 0x5A).all()


def _codeword(k, p, S, B, rng):
    cw = np.zeros((B, k + p, S), np.uint8)
    cw[:, :k] = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    cw[:, k:] = _parity(k, p, cw[:, :k])
    return cw


def _patterns(rng, B, t, k, p, mixed):
    present = np.ones((B, t), np.uint8)
    for b in range(B):
        if b % 7 == 3:
            continue                          # every shard present: left alone
        if mixed:
            present[b, rng.choice(t, size=int(rng.integers(1, p + 1)), replace=False)] = 0
        else:
            present[b, [b % k, (b + 3) % t][:min(p, 2)]] = 0
    return present


@pytest.mark.parametrize("k,p,S,B,mixed", [(8, 3, 65536, 16, False), (10, 4, 3 * 8192 + 2458, 40, True),
                                           (4, 2, 4096 * 2 + 100, 9, True)])
@pytest.mark.parametrize("data_only", [False, True])
def test_grid_reconstruct_in_place(gpu, k, p, S, B, mixed, data_only):
    """Every shard of the block (present and rebuilt) in one joint slab: the
    in-place strided rebuild (mixed patterns in more than 32 block runs take
    the uploaded block/plan tables); absent parity stays untouched under
    data_only."""
    import torch
    t = k + p
    rng = np.random.default_rng([k, B, int(mixed), int(data_only)])
    cw = _codeword(k, p, S, B, rng)
    present = _patterns(rng, B, t, k, p, mixed)
    slab = shmr_amd.ShardSlab(B, t, S)
    view = slab.tensor()
    start = cw.copy()
    start[present == 0] = 0xEE
    view[:, :, :S] = torch.from_numpy(start).to(gpu)
    torch.cuda.synchronize()
    st0 = _stats()
    rs = shmr_amd.ReedSolomon(k, p)
    keep, tab = _tab(slab.ptrs)
    pr = np.ascontiguousarray(present)
    rc = rs._L.shmr_ec_reconstruct_ptrs_dev(rs._h, tab, pr.ctypes.data_as(_u8p), B, S, int(data_only), 0, _stream())
    assert rc == 0, shmr_amd.Error(rc).name
    torch.cuda.synchronize()
    assert _stats()["ptr_table_grids"] == st0["ptr_table_grids"] + (0 if _needs_plan_list(present) else 1)
    want = cw.copy()
    if data_only:
        keep_parity = (present == 0)
        keep_parity[:, :k] = False
        want[keep_parity] = 0xEE
    assert np.array_equal(view[:, :, :S].cpu().numpy(), want)


@pytest.mark.parametrize("k,p,S,B,erasures", [(8, 3, 65536, 16, 1), (10, 4, 3 * 8192 + 2458, 12, 2),
                                              (10, 4, 4096, 40, 4)])
@pytest.mark.parametrize("data_only", [False, True])
def test_grid_reconstruct_fresh_buffers(gpu, k, p, S, B, erasures, data_only):
    """Present shards in one slab, each rebuilt shard in a buffer of its own
    from a second slab (the crate's fresh buffer per None): the compact-output
    kernels; absent parity NULL under data_only."""
    import torch
    t = k + p
    rng = np.random.default_rng([k, B, erasures, int(data_only)])
    cw = _codeword(k, p, S, B, rng)
    present = np.ones((B, t), np.uint8)
    for b in range(B):
        present[b, rng.choice(t, size=erasures, replace=False)] = 0
    written = (present == 0)
    if data_only:
        written[:, k:] = False
    nout = int(written.sum(axis=1).max())
    shards = shmr_amd.ShardSlab(B, t, S)
    sview = shards.tensor()
    sview[:, :, :S] = torch.from_numpy(np.where(present[:, :, None] == 1, cw, 0xEE).astype(np.uint8)).to(gpu)
    outs = shmr_amd.ShardSlab(B, max(nout, 1), S)
    oview = outs.tensor()
    oview.fill_(0x77)
    addrs = shards.ptrs.reshape(B, t).copy()
    for b in range(B):
        j = 0
        for i in range(t):
            if present[b, i]:
                continue
            if written[b, i]:
                addrs[b, i] = outs.ptrs[b * max(nout, 1) + j]
                j += 1
            else:
                addrs[b, i] = 0
    torch.cuda.synchronize()
    st0 = _stats()
    rs = shmr_amd.ReedSolomon(k, p)
    keep, tab = _tab(addrs.reshape(-1))
    pr = np.ascontiguousarray(present)
    rc = rs._L.shmr_ec_reconstruct_ptrs_dev(rs._h, tab, pr.ctypes.data_as(_u8p), B, S, int(data_only), 0, _stream())
    assert rc == 0, shmr_amd.Error(rc).name
    torch.cuda.synchronize()
    # (mixed patterns in more runs than the kernel arguments hold: the table kernels)
    assert _stats()["ptr_table_grids"] == st0["ptr_table_grids"] + (0 if _needs_plan_list(present) else 1)
    o = oview.cpu().numpy()
    for b in range(B):
        idx = np.flatnonzero(written[b])
        for j, i in enumerate(idx):
            assert np.array_equal(o[b, j, :S], cw[b, i]), (b, i)
        assert (o[b, len(idx):] == 0x77).all() and (o[b, :len(idx), S:] == 0x77).all()
    got = sview[:, :, :S].cpu().numpy()
    assert np.array_equal(got[present == 1], cw[present == 1]), "a present shard was written"
    assert (got[present == 0] == 0xEE).all(), "an absent slot of the shard slab was written"


def test_grid_and_table_kernels_write_the_same_bytes(gpu):
    """One slab table through both paths (knob ptrs_grid): identical parity and
    rebuilt bytes; a table with two entries swapped is off the grid and takes
    the table kernels with the default knob."""
    import torch
    k, p, S, B = 8, 3, 8192 * 3 + 48, 24
    t = k + p
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    slab = shmr_amd.ShardSlab(B, t, S)
    view = slab.tensor()
    rs = shmr_amd.ReedSolomon(k, p)
    keep, tab = _tab(slab.ptrs)
    results = []
    try:
        for grid in (1, 0):
            shmr_amd.set_tuning(ptrs_grid=grid)
            view.zero_()
            view[:, :k, :S] = torch.from_numpy(data).to(gpu)
            st0 = _stats()
            assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab, B, S, 0, _stream()) == 0
            present = np.ones((B, t), np.uint8)
            present[np.arange(B), np.arange(B) % t] = 0
            present[np.arange(B), (np.arange(B) + 5) % t] = 0
            torch.cuda.synchronize()
            snap = view.clone()
            view[:, :, :S][torch.from_numpy(present == 0).to(gpu)] = 0
            rc = rs._L.shmr_ec_reconstruct_ptrs_dev(rs._h, tab, present.ctypes.data_as(_u8p), B, S, 0, 0, _stream())
            assert rc == 0
            torch.cuda.synchronize()
            assert torch.equal(view, snap)
            assert _stats()["ptr_table_grids"] - st0["ptr_table_grids"] == (2 if grid else 0)
            results.append(view.cpu().numpy())
    finally:
        shmr_amd.set_tuning(ptrs_grid=-2)
    assert np.array_equal(results[0], results[1])
    assert np.array_equal(results[0][:, k:, :S], _parity(k, p, data))
    # off the grid: blocks 3 and 4 swap their parity shard 1
    swapped = slab.ptrs.reshape(B, t).copy()
    swapped[[3, 4], k + 1] = swapped[[4, 3], k + 1]
    keep2, tab2 = _tab(swapped.reshape(-1))
    view[:, k:] = 0
    st0 = _stats()
    assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab2, B, S, 0, _stream()) == 0
    torch.cuda.synchronize()
    assert _stats()["ptr_table_grids"] == st0["ptr_table_grids"]
    want = _parity(k, p, data)
    want[[3, 4], 1] = want[[4, 3], 1]      # each block's parity row 1 landed in the other's slot
    assert np.array_equal(view[:, k:, :S].cpu().numpy(), want)


def test_grid_table_capture(gpu):
    """A grid table inside a graph capture needs no capture-reserve block (no
    table): the captured encode and rebuild replay bit-exact."""
    import torch
    k, p, S, B = 6, 3, 4096 * 4, 10
    t = k + p
    shmr_amd.device_init(0)
    rs = shmr_amd.ReedSolomon(k, p)
    slab = shmr_amd.ShardSlab(B, t, S)
    view = slab.tensor()
    keep, tab = _tab(slab.ptrs)
    present = np.ones((B, t), np.uint8)
    present[np.arange(B), np.arange(B) % k] = 0
    rng = np.random.default_rng(9)
    stream = torch.cuda.Stream()
    sp = ctypes.c_void_p(stream.cuda_stream)
    torch.cuda.synchronize()
    st0 = _stats()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=stream):
        assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab, B, S, 0, sp) == 0
    graph2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph2, stream=stream):
        assert rs._L.shmr_ec_reconstruct_ptrs_dev(rs._h, tab, present.ctypes.data_as(_u8p), B, S, 0, 0, sp) == 0
    assert _stats()["capture_tables"] == st0["capture_tables"]
    for rep in range(2):
        data = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
        view.zero_()
        view[:, :k, :S] = torch.from_numpy(data).to(gpu)
        torch.cuda.synchronize()
        graph.replay()
        torch.cuda.synchronize()
        full = view[:, :, :S].cpu().numpy().copy()
        assert np.array_equal(full[:, k:], _parity(k, p, data)), rep
        view[:, :, :S][torch.from_numpy(present == 0).to(gpu)] = 0
        torch.cuda.synchronize()
        graph2.replay()
        torch.cuda.synchronize()
        assert np.array_equal(view[:, :, :S].cpu().numpy(), full), rep


@pytest.mark.parametrize("k,p,size,B,erasures", [(8, 3, 4 << 20, 8, 1), (10, 4, 16 << 20, 3, 2)])
def test_grid_full_size(gpu, k, p, size, B, erasures):
    """BASELINE configs 2-4 on slab buffers: RS(8,3) 4 MiB and RS(10,4) 16 MiB
    blocks (S = 1,677,722: 2 mod 4), encode then rebuild into fresh slab
    buffers, against the oracle."""
    import torch
    S = shmr_amd.calculate_shard_size(size, k)
    t = k + p
    g = torch.Generator(device=gpu).manual_seed(size + B)
    slab = shmr_amd.ShardSlab(B, t, S)
    view = slab.tensor()
    view[:, :k, :S] = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device=gpu, generator=g)
    rs = shmr_amd.ReedSolomon(k, p)
    keep, tab = _tab(slab.ptrs)
    assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab, B, S, 0, _stream()) == 0
    torch.cuda.synchronize()
    full = view[:, :, :S].cpu().numpy()
    assert np.array_equal(full[:, k:], _parity(k, p, full[:, :k]))
    present = np.ones((B, t), np.uint8)
    for b in range(B):
        present[b, [(b + 3 * j) % 10 for j in range(erasures)]] = 0
    outs = shmr_amd.ShardSlab(B, erasures, S)
    addrs = slab.ptrs.reshape(B, t).copy()
    for b in range(B):
        for j, i in enumerate(np.flatnonzero(present[b] == 0)):
            addrs[b, i] = outs.ptrs[b * erasures + j]
    keep2, tab2 = _tab(addrs.reshape(-1))
    st0 = _stats()
    rc = rs._L.shmr_ec_reconstruct_ptrs_dev(rs._h, tab2, present.ctypes.data_as(_u8p), B, S, 0, 0, _stream())
    assert rc == 0
    torch.cuda.synchronize()
    assert _stats()["ptr_table_grids"] == st0["ptr_table_grids"] + 1
    o = outs.tensor()[:, :, :S].cpu().numpy()
    for b in range(B):
        for j, i in enumerate(np.flatnonzero(present[b] == 0)):
            assert np.array_equal(o[b, j], full[b, i]), (b, i)
