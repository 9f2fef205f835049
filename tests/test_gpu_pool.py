"""Device Block Cache slots (include/shmr_ec.h shmr_ec_pool_*) vs the CPU
oracle, bit-exact.

The reference's Block Cache takes and drops one block's buffers at a time
(src/vfs/block.rs:148-152, :586-608).  A pool hands out block slots of one
slab and takes them back singly; after churn the live blocks of a flush sit in
any order with holes.  Their pointer tables lie on the slab's slot lattice
(ptr_grid.hpp), so *_ptrs_dev and the submission queue run the strided
kernels over the slots (counter ptr_table_grids): one run or up to 32
segment runs; beyond that the table kernels (measured faster than an uploaded
slot list; knob lattice_list).  Every byte must equal the oracle's and nothing
outside the blocks' shards may change."""
import ctypes

import numpy as np
import pytest

import shmr_amd
from shmr_amd.reed_solomon import _ptr, _u8p
from oracle import c_oracle

pytestmark = pytest.mark.gpu


def _parity(k, p, data):
    B, _, S = data.shape
    par = np.zeros((B, p, S), np.uint8)
    c_oracle.encode_batch(k, p, np.ascontiguousarray(data), par, B, S, 8)
    return par


def _tab(rows):
    arr = np.ascontiguousarray(np.asarray(rows, dtype=np.uint64).reshape(-1))
    return arr, arr.ctypes.data_as(ctypes.POINTER(_u8p))


def _fits_args(slots):
    """Mirror of ec_core slots_launch_fits on device pitch layouts: the slots
    (ascending) form at most 32 arithmetic runs -- otherwise the table kernels
    run (knob lattice_list, default 0)."""
    slots = sorted(int(x) for x in slots)
    runs, i = 0, 0
    while i < len(slots):
        e = i + 1
        st = slots[e] - slots[i] if e < len(slots) else 1
        while e < len(slots) and slots[e] - slots[e - 1] == st:
            e += 1
        runs += 1
        i = e
    return runs <= 32


def _stream():
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def test_pool_alloc_free_rules(gpu):
    pool = shmr_amd.ShardPool(11, 4096 * 3 + 5, 4)
    a = [pool.alloc() for _ in range(5)]                   # the fifth opens a second slab
    assert pool.stats() == {"slabs": 2, "slots": 8, "in_use": 5}
    P = int(a[0][1] - a[0][0])
    assert P == 16384 and int(a[1][0] - a[0][0]) == 11 * P   # slot pitch, joint block slots
    pool.free(a[1])
    again = pool.alloc()                                    # the lowest free slot comes back
    assert int(again[0]) == int(a[1][0])
    with pytest.raises(shmr_amd.Error) as e:
        pool.free(np.array([int(a[0][1])], np.uint64))      # not a block's first shard
    assert e.value.code == -100
    pool.free(a[2])
    with pytest.raises(shmr_amd.Error):
        pool.free(a[2])                                     # twice
    assert pool.stats()["in_use"] == 4
    with pytest.raises(shmr_amd.Error):
        shmr_amd.ShardPool(0, 4096, 4)


@pytest.mark.parametrize("k,p,S", [(8, 3, 65536), (10, 4, 12345 * 4 + 2), (4, 2, 4096 * 2)])
def test_pool_churn_encode_and_rebuild(gpu, k, p, S):
    """Rounds of churn (random frees and allocs), then an encode and an
    in-place rebuild of every live block (random erasures, mixed patterns) in
    shuffled table order: the oracle's bytes, the encode on the lattice path,
    and free slots untouched."""
    import torch
    t = k + p
    rng = np.random.default_rng(k * 10 + p)
    rs = shmr_amd.ReedSolomon(k, p)
    nslots = 96
    pool = shmr_amd.ShardPool(t, S, nslots)
    live = [pool.alloc() for _ in range(nslots)]
    P = int(live[0][1] - live[0][0])
    base = min(int(b[0]) for b in live)
    slab = torch.as_tensor(shmr_amd.reed_solomon._RawView(pool, base, (nslots * t * P,)), device=gpu)
    for rnd in range(4):
        for _ in range(int(rng.integers(8, 40))):           # churn
            if live and rng.integers(0, 3):
                pool.free(live.pop(int(rng.integers(0, len(live)))))
            elif pool.stats()["in_use"] < nslots:
                live.append(pool.alloc())
        assert pool.stats()["slabs"] == 1
        slab.fill_(0xC3)                                     # free slots must keep this
        torch.cuda.synchronize()
        order = rng.permutation(len(live))
        rows = np.stack([live[int(j)] for j in order])
        B = len(rows)
        data = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
        for b in range(B):
            for i in range(k):
                pool.shard(rows[b], i).copy_(torch.from_numpy(data[b, i]).to(gpu))
        torch.cuda.synchronize()
        g0 = shmr_amd.device_stats(0)["ptr_table_grids"]
        keep, tab = _tab(rows)
        assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab, B, S, 0, _stream()) == 0
        torch.cuda.synchronize()
        enc = 1 if _fits_args([(int(r[0]) - base) // (t * P) for r in rows]) else 0
        assert shmr_amd.device_stats(0)["ptr_table_grids"] == g0 + enc
        want = _parity(k, p, data)
        full = np.concatenate([data, want], axis=1)
        for b in range(B):
            for r in range(p):
                assert np.array_equal(pool.shard(rows[b], k + r).cpu().numpy(), want[b, r]), (rnd, b, r)
        present = np.ones((B, t), np.uint8)
        for b in range(B):
            present[b, rng.choice(t, size=int(rng.integers(1, p + 1)), replace=False)] = 0
            for i in np.flatnonzero(present[b] == 0):
                pool.shard(rows[b], int(i)).fill_(0xEE)
        torch.cuda.synchronize()
        assert rs._L.shmr_ec_reconstruct_ptrs_dev(rs._h, tab, _ptr(present), B, S, 0, 0, _stream()) == 0
        torch.cuda.synchronize()
        # (mixed patterns in more runs than the kernel arguments hold take the
        # table kernels: ptrs.cpp lattice_needs_plan_list, slots_launch_fits)
        assert shmr_amd.device_stats(0)["ptr_table_grids"] in (g0 + enc, g0 + enc + 1)
        for b in range(B):
            for i in range(t):
                assert np.array_equal(pool.shard(rows[b], i).cpu().numpy(), full[b, i]), (rnd, b, i)
        # slot tails and free slots untouched
        used = torch.zeros(nslots * t * P, dtype=torch.bool, device=gpu)
        for r in rows:
            for i in range(t):
                o = int(r[i]) - base
                used[o:o + S] = True
        assert bool((slab[~used] == 0xC3).all()), rnd


def test_pool_blocks_through_the_queue(gpu):
    """Per-block calls (shmr_ec_encode_dev, started) over pool blocks in
    shuffled order: the merged launches take the lattice path; exact."""
    import torch
    k, p, S, n = 8, 3, 131072, 48
    t = k + p
    rs = shmr_amd.ReedSolomon(k, p)
    pool = shmr_amd.ShardPool(t, S, 64)
    blocks = [pool.alloc() for _ in range(64)]
    rng = np.random.default_rng(4)
    for j in sorted(rng.choice(64, size=16, replace=False).tolist(), reverse=True):
        pool.free(blocks.pop(j))
    data = rng.integers(0, 256, (n, k, S), dtype=np.uint8)
    for b in range(n):
        for i in range(k):
            pool.shard(blocks[b], i).copy_(torch.from_numpy(data[b, i]).to(gpu))
    torch.cuda.synchronize()
    g0 = shmr_amd.device_stats(0)["ptr_table_grids"]
    ops = [rs.encode_dev([(int(a), S) for a in blocks[int(b)]], start=True) for b in rng.permutation(n)]
    for op in ops:
        op.wait()
    assert shmr_amd.device_stats(0)["ptr_table_grids"] > g0
    want = _parity(k, p, data)
    for b in range(n):
        for r in range(p):
            assert np.array_equal(pool.shard(blocks[b], k + r).cpu().numpy(), want[b, r])


def test_pool_failed_disk_rebuild_on_the_lattice(gpu):
    """A failed disk: every live block of a holed pool lost the same shard --
    one pattern, rebuilt in place over the slots (lattice path: a run list or
    segment runs), exact, nothing else written."""
    import torch
    k, p, S = 8, 3, 65536
    t = k + p
    rs = shmr_amd.ReedSolomon(k, p)
    pool = shmr_amd.ShardPool(t, S, 80)
    live = [pool.alloc() for _ in range(80)]
    rng = np.random.default_rng(8)
    for j in sorted(rng.choice(80, size=20, replace=False).tolist(), reverse=True):
        pool.free(live.pop(j))
    rows = np.stack([live[int(j)] for j in rng.permutation(len(live))])
    B = len(rows)
    data = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    full = np.concatenate([data, _parity(k, p, data)], axis=1)
    for b in range(B):
        for i in range(t):
            pool.shard(rows[b], i).copy_(torch.from_numpy(full[b, i]).to(gpu))
        pool.shard(rows[b], 5).fill_(0xEE)
    torch.cuda.synchronize()
    present = np.ones((B, t), np.uint8)
    present[:, 5] = 0
    g0 = shmr_amd.device_stats(0)["ptr_table_grids"]
    keep, tab = _tab(rows)
    assert rs._L.shmr_ec_reconstruct_ptrs_dev(rs._h, tab, _ptr(present), B, S, 0, 0, _stream()) == 0
    torch.cuda.synchronize()
    assert shmr_amd.device_stats(0)["ptr_table_grids"] == g0 + 1
    for b in range(B):
        for i in range(t):
            assert np.array_equal(pool.shard(rows[b], i).cpu().numpy(), full[b, i]), (b, i)


def test_pool_lattice_encode_as_first_call(gpu):
    """A process whose first compute call is a pool encode over segment runs
    (r06 s30: the segment launch uploaded its plan before the device state
    existed and returned INVALID_ARGUMENT)."""
    import os
    import subprocess
    import sys
    code = r'''
import ctypes, numpy as np, torch, shmr_amd
from shmr_amd.reed_solomon import _u8p
k, p, S = 8, 3, 65536
rs = shmr_amd.ReedSolomon(k, p)
pool = shmr_amd.ShardPool(k + p, S, 16)
blocks = [pool.alloc() for _ in range(16)]
for j in (13, 9, 4, 1):
    pool.free(blocks.pop(j))
tab = np.ascontiguousarray(np.stack(blocks).reshape(-1))
sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
g0 = shmr_amd.device_stats(0)["ptr_table_grids"]
rc = rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab.ctypes.data_as(ctypes.POINTER(_u8p)), len(blocks), S, 0, sp)
torch.cuda.synchronize()
print(rc, shmr_amd.device_stats(0)["ptr_table_grids"] - g0)
'''
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, env=env,
                         cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.split()[-2:] == ["0", "1"], out.stdout
