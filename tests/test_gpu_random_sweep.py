"""Seeded random sweep of the device-resident entry points against the CPU
oracle: random (k, p), shard lengths (tiny, around tile boundaries, odd),
batch sizes, shard/block pitches and base offsets (aligned and not), erasure
patterns (mixed per block, all-present blocks, up to p losses) and data_only.
Every byte of every output is checked, and bytes outside the shards must stay
untouched.

Reference call sites: ReedSolomon::encode (src/vfs/block.rs:427) and
ReedSolomon::reconstruct / reconstruct_data (block.rs:560).
"""
import ctypes
import os

import numpy as np
import pytest

import shmr_amd
from oracle import c_oracle
from shmr_amd._native import _u8p, lib

pytestmark = pytest.mark.gpu

SENTINEL = 0xA5
# SHMR_SWEEP_SCALE=N multiplies the number of seeded cases (long sweeps on the
# GPU box: tools/sweep_long.sh); the default suite runs scale 1.
SCALE = max(1, int(os.environ.get("SHMR_SWEEP_SCALE", "1")))


def _shape(rng):
    k = int(rng.choice([1, 2, 3, 4, 5, 8, 10, 12, 17, 32, 64]))
    p = int(rng.integers(1, 9))
    L = int(rng.choice([1, 15, 16, 17, 255, 4095, 4096, 4097, 8192 + 48, 12288 - 16, int(rng.integers(1, 70000))]))
    B = int(rng.integers(1, 9))
    aligned = bool(rng.integers(0, 2))
    if aligned:
        spitch = (L + 15) // 16 * 16 + 16 * int(rng.integers(0, 4))
        off = 16 * int(rng.integers(0, 3))
    else:
        spitch = L + int(rng.integers(0, 40))
        off = int(rng.integers(0, 16))
    return k, p, L, B, spitch, off


def _stream():
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


@pytest.mark.parametrize("case", range(40 * SCALE))
def test_random_encode_batch_dev(gpu, case):
    import torch
    rng = np.random.default_rng([0x5EED, case])
    k, p, L, B, spitch, off = _shape(rng)
    bpitch = k * spitch + int(rng.integers(0, 2)) * 64
    pspitch = spitch
    pbpitch = p * pspitch
    data = rng.integers(0, 256, off + B * bpitch + 64, dtype=np.uint8)
    d_data = torch.from_numpy(data).to(gpu)
    d_par = torch.full((off + B * pbpitch + 64,), SENTINEL, dtype=torch.uint8, device=gpu)
    rs = shmr_amd.ReedSolomon(k, p)
    rc = lib().shmr_ec_encode_batch_dev(rs._h, ctypes.c_void_p(d_data.data_ptr() + off), spitch, bpitch,
                                        ctypes.c_void_p(d_par.data_ptr() + off), pspitch, pbpitch, B, L, 0, _stream())
    assert rc == 0, shmr_amd.Error(rc).name
    torch.cuda.synchronize()
    par = d_par.cpu().numpy()
    expect = np.full_like(par, SENTINEL)
    for b in range(B):
        ins = [data[off + b * bpitch + i * spitch: off + b * bpitch + i * spitch + L].copy() for i in range(k)]
        sh = ins + [np.zeros(L, np.uint8) for _ in range(p)]
        c_oracle.encode(k, p, sh)
        for r in range(p):
            o = off + b * pbpitch + r * pspitch
            expect[o:o + L] = sh[k + r]
    assert np.array_equal(par, expect), (k, p, L, B, spitch, off)


@pytest.mark.parametrize("case", range(40 * SCALE))
def test_random_reconstruct_batch_dev(gpu, case):
    import torch
    rng = np.random.default_rng([0xDEC0, case])
    k, p, L, B, spitch, off = _shape(rng)
    t = k + p
    bpitch = t * spitch + int(rng.integers(0, 2)) * 48
    data_only = bool(rng.integers(0, 2))
    buf = np.full(off + B * bpitch + 64, SENTINEL, dtype=np.uint8)
    present = np.ones((B, t), np.uint8)
    full = []
    for b in range(B):
        ins = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
        sh = ins + [np.zeros(L, np.uint8) for _ in range(p)]
        c_oracle.encode(k, p, sh)
        full.append(sh)
        for i in range(t):
            o = off + b * bpitch + i * spitch
            buf[o:o + L] = sh[i]
        if rng.integers(0, 4):   # 3 of 4 blocks lose something
            n = int(rng.integers(1, p + 1))
            present[b, rng.choice(t, size=n, replace=False)] = 0
    poisoned = buf.copy()
    for b in range(B):
        for i in range(t):
            if not present[b, i]:
                o = off + b * bpitch + i * spitch
                poisoned[o:o + L] = 0xEE
    d = torch.from_numpy(poisoned).to(gpu)
    rs = shmr_amd.ReedSolomon(k, p)
    pr = np.ascontiguousarray(present)
    rc = lib().shmr_ec_reconstruct_batch_dev(rs._h, ctypes.c_void_p(d.data_ptr() + off), spitch, bpitch,
                                             pr.ctypes.data_as(_u8p), B, L, int(data_only), 0, _stream())
    assert rc == 0, shmr_amd.Error(rc).name
    torch.cuda.synchronize()
    got = d.cpu().numpy()
    expect = buf.copy()
    if data_only:   # absent parity stays as it was (poisoned)
        for b in range(B):
            for i in range(k, t):
                if not present[b, i]:
                    o = off + b * bpitch + i * spitch
                    expect[o:o + L] = 0xEE
    assert np.array_equal(got, expect), (k, p, L, B, spitch, off, data_only)


@pytest.mark.parametrize("case", range(16 * SCALE))
def test_random_host_blocks(gpu, case):
    """Host-buffer batches: pageable and mapped buffers, random erasures."""
    rng = np.random.default_rng([0x4057, case])
    k, p, L, B, _, _ = _shape(rng)
    t = k + p
    mapped = bool(case % 2)
    keep = None
    if mapped:
        keep = shmr_amd.PinnedBuffer(B * t * L + 16)
        base = int(rng.integers(0, 16))
        arr = keep.array[base:base + B * t * L].reshape(B, t, L)
        blocks = [[arr[b, i] for i in range(t)] for b in range(B)]
    else:
        blocks = [[np.zeros(L, np.uint8) for _ in range(t)] for _ in range(B)]
    for blk in blocks:
        for i in range(k):
            blk[i][:] = rng.integers(0, 256, L, dtype=np.uint8)
    rs = shmr_amd.ReedSolomon(k, p)
    rs.encode_blocks_host(blocks)
    full = []
    for blk in blocks:
        sh = [x.copy() for x in blk[:k]] + [np.zeros(L, np.uint8) for _ in range(p)]
        c_oracle.encode(k, p, sh)
        for r in range(p):
            assert np.array_equal(blk[k + r], sh[k + r])
        full.append(sh)
    present = np.ones((B, t), np.uint8)
    for b in range(B):
        n = int(rng.integers(0, p + 1))
        if n:
            present[b, rng.choice(t, size=n, replace=False)] = 0
        for i in range(t):
            if not present[b, i]:
                blocks[b][i][:] = 0
    rs.reconstruct_blocks_host(blocks, present)
    for b in range(B):
        for i in range(t):
            assert np.array_equal(blocks[b][i], full[b][i]), (b, i)


def _scatter(rng, n, L, aligned):
    """Offsets of n regions of L bytes in shuffled order inside one buffer, with
    random gaps (16-byte aligned starts or any byte); returns (offsets, size)."""
    order = rng.permutation(n)
    offs = np.zeros(n, np.int64)
    pos = int(rng.integers(0, 16))
    for j in order:
        pos += int(rng.integers(0, 3)) * 16 + (0 if aligned else int(rng.integers(0, 16)))
        if aligned:
            pos = (pos + 15) // 16 * 16
        offs[j] = pos
        pos += L
    return offs, pos + 64


@pytest.mark.parametrize("case", range(24 * SCALE))
def test_random_ptrs(gpu, case):
    """Pointer tables (*_ptrs_dev, the crate's shard-per-Vec shape): every shard
    anywhere in a shared buffer, in shuffled memory order, aligned or not; encode,
    then rebuild random erasures into separate buffers (absent parity NULL under
    data_only).  Rows are permuted into plan order on the host (r04): a wrong
    permutation writes the wrong shard."""
    import torch
    rng = np.random.default_rng([0x9715, case])
    k, p, L, B, _, _ = _shape(rng)
    t = k + p
    aligned = bool(rng.integers(0, 2))
    offs, size = _scatter(rng, B * t, L, aligned)
    host = np.full(size, SENTINEL, np.uint8)
    full = []
    for b in range(B):
        sh = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)] + [np.zeros(L, np.uint8) for _ in range(p)]
        c_oracle.encode(k, p, sh)
        full.append(sh)
        for i in range(k):
            host[offs[b * t + i]:offs[b * t + i] + L] = sh[i]
    d = torch.from_numpy(host).to(gpu)
    base = d.data_ptr()
    tab = np.array([base + int(o) for o in offs], dtype=np.uint64)
    rs = shmr_amd.ReedSolomon(k, p)
    rc = lib().shmr_ec_encode_ptrs_dev(rs._h, tab.ctypes.data_as(ctypes.POINTER(_u8p)), B, L, 0, _stream())
    assert rc == 0, shmr_amd.Error(rc).name
    torch.cuda.synchronize()
    got = d.cpu().numpy()
    expect = host.copy()
    for b in range(B):
        for i in range(k, t):
            expect[offs[b * t + i]:offs[b * t + i] + L] = full[b][i]
    assert np.array_equal(got, expect), ("encode", k, p, L, B, aligned)
    # rebuild: absent shards point into a separate poisoned buffer
    data_only = bool(rng.integers(0, 2))
    present = np.ones((B, t), np.uint8)
    for b in range(B):
        if rng.integers(0, 4):
            present[b, rng.choice(t, size=int(rng.integers(1, p + 1)), replace=False)] = 0
    ooffs, osize = _scatter(rng, B * t, L, aligned)
    out = torch.full((osize,), 0xEE, dtype=torch.uint8, device=gpu)
    tab2 = tab.copy()
    for b in range(B):
        for i in range(t):
            if not present[b, i]:
                tab2[b * t + i] = 0 if (data_only and i >= k) else out.data_ptr() + int(ooffs[b * t + i])
    rc = lib().shmr_ec_reconstruct_ptrs_dev(rs._h, tab2.ctypes.data_as(ctypes.POINTER(_u8p)),
                                            present.ctypes.data_as(_u8p), B, L, int(data_only), 0, _stream())
    assert rc == 0, shmr_amd.Error(rc).name
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), expect), ("rebuild touched a present shard", k, p, L, B)
    got = out.cpu().numpy()
    want = np.full(osize, 0xEE, np.uint8)
    for b in range(B):
        for i in range(t):
            if not present[b, i] and not (data_only and i >= k):
                want[ooffs[b * t + i]:ooffs[b * t + i] + L] = full[b][i]
    assert np.array_equal(got, want), ("rebuild", k, p, L, B, aligned, data_only)


@pytest.mark.parametrize("case", range(24 * SCALE))
def test_random_reconstruct_out(gpu, case):
    """Compact rebuilds (shmr_ec_reconstruct_batch_dev_out, the crate's
    fresh-buffer-per-None semantics): absent slots poisoned and never read,
    rebuilt shards in ascending index into a separate output, nothing else
    written."""
    import torch
    rng = np.random.default_rng([0xC0DE, case])
    k, p, L, B, spitch, off = _shape(rng)
    t = k + p
    bpitch = t * spitch
    data_only = bool(rng.integers(0, 2))
    buf = np.full(off + B * bpitch + 64, SENTINEL, dtype=np.uint8)
    present = np.ones((B, t), np.uint8)
    full = []
    for b in range(B):
        sh = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)] + [np.zeros(L, np.uint8) for _ in range(p)]
        c_oracle.encode(k, p, sh)
        full.append(sh)
        for i in range(t):
            buf[off + b * bpitch + i * spitch: off + b * bpitch + i * spitch + L] = sh[i]
        if rng.integers(0, 4):
            present[b, rng.choice(t, size=int(rng.integers(1, p + 1)), replace=False)] = 0
    for b in range(B):
        for i in range(t):
            if not present[b, i]:
                buf[off + b * bpitch + i * spitch: off + b * bpitch + i * spitch + L] = 0xEE
    nout = max(1, int(max(((present[b] == 0) & ((np.arange(t) < k) | (not data_only))).sum() for b in range(B))))
    opitch = spitch + 16 * int(rng.integers(0, 2))
    obpitch = nout * opitch
    d = torch.from_numpy(buf).to(gpu)
    out = torch.full((off + B * obpitch + 64,), SENTINEL, dtype=torch.uint8, device=gpu)
    rs = shmr_amd.ReedSolomon(k, p)
    rc = lib().shmr_ec_reconstruct_batch_dev_out(rs._h, ctypes.c_void_p(d.data_ptr() + off), spitch, bpitch,
                                                 present.ctypes.data_as(_u8p), B, L, int(data_only),
                                                 ctypes.c_void_p(out.data_ptr() + off), opitch, obpitch, 0, _stream())
    assert rc == 0, shmr_amd.Error(rc).name
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), buf), "the compact rebuild wrote its input"
    want = np.full(off + B * obpitch + 64, SENTINEL, np.uint8)
    for b in range(B):
        j = 0
        for i in range(t):
            if not present[b, i] and (i < k or not data_only):
                o = off + b * obpitch + j * opitch
                want[o:o + L] = full[b][i]
                j += 1
    assert np.array_equal(out.cpu().numpy(), want), (k, p, L, B, spitch, off, data_only)


def _start(rs, fn, shards, present=None, data_only=False):
    """shmr_ec_encode_start / shmr_ec_reconstruct_start through ctypes: (rc, op)."""
    from shmr_amd.reed_solomon import _ptr
    n = len(shards)
    L = len(shards[0])
    ptrs = (_u8p * n)(*[_ptr(s) for s in shards])
    lens = (ctypes.c_size_t * n)(*[(L if present is None or present[i] else 0) for i in range(n)])
    op = ctypes.c_void_p()
    if fn == "encode":
        rc = rs._L.shmr_ec_encode_start(rs._h, ptrs, lens, n, ctypes.byref(op))
    else:
        pr = np.ascontiguousarray(present, dtype=np.uint8)
        rc = rs._L.shmr_ec_reconstruct_start(rs._h, ptrs, lens, _ptr(pr), n, int(data_only), ctypes.byref(op))
    return rc, op


@pytest.mark.parametrize("case", range(8 * SCALE))
def test_random_started_calls(gpu, case):
    """Started per-block calls (shmr_ec_*_start, the Block Cache's overlap of
    file I/O with the GPU work): up to six ops of random shapes in flight at
    once, mapped (zero-copy, pending until waited) or pageable, encodes and
    rebuilds with data_only, waited in random order -- every byte equal to the
    oracle's."""
    rng = np.random.default_rng([0x57A7, case])
    keep, pending = [], []
    for _ in range(int(rng.integers(1, 7))):
        k, p, L, _, _, _ = _shape(rng)
        t = k + p
        rs = shmr_amd.ReedSolomon(k, p)
        if rng.integers(0, 2):
            buf = shmr_amd.PinnedBuffer(t * L + 16)
            base = int(rng.integers(0, 16))
            arr = buf.array[base:base + t * L].reshape(t, L)
            sh = [arr[i] for i in range(t)]
            keep.append(buf)
        else:
            sh = [np.zeros(L, np.uint8) for _ in range(t)]
        for i in range(k):
            sh[i][:] = rng.integers(0, 256, L, dtype=np.uint8)
        full = [s.copy() for s in sh[:k]] + [np.zeros(L, np.uint8) for _ in range(p)]
        c_oracle.encode(k, p, full)
        if rng.integers(0, 2):
            for i in range(k, t):
                sh[i][:] = SENTINEL
            rc, op = _start(rs, "encode", sh)
            want = full
        else:
            for i in range(k, t):
                sh[i][:] = full[i]
            present = np.ones(t, np.uint8)
            present[rng.choice(t, size=int(rng.integers(1, p + 1)), replace=False)] = 0
            data_only = bool(rng.integers(0, 2))
            for i in np.flatnonzero(present == 0):
                sh[i][:] = 0xEE
            rc, op = _start(rs, "reconstruct", sh, present, data_only)
            want = [(np.full(L, 0xEE, np.uint8) if (not present[i] and data_only and i >= k) else full[i])
                    for i in range(t)]
        assert rc == 0 and op.value, shmr_amd.Error(rc).name if rc else "no op"
        pending.append((op, rs, sh, want, (k, p, L)))
    for j in rng.permutation(len(pending)):
        op, rs, sh, want, shape = pending[j]
        assert rs._L.shmr_ec_op_wait(op) == 0
        for i in range(len(sh)):
            assert np.array_equal(sh[i], want[i]), (shape, i)


@pytest.mark.parametrize("case", range(24 * SCALE))
def test_random_grid_tables(gpu, case):
    """Pointer tables that name a slot grid (knob ptrs_grid, r05): random grid
    geometry -- data and parity in one joint grid or two, pitches aligned or
    not, strides with gaps -- encoded, then rebuilt either in place (every
    shard on one grid) or into a second grid of fresh buffers (rebuilt shard j
    of block b), data_only random.  Every call must be recognised as a grid
    (counter ptr_table_grids), write exactly the oracle's bytes and nothing
    outside the shards."""
    import torch
    rng = np.random.default_rng([0x6D1D, case])
    k, p, L, B, spitch, off = _shape(rng)
    t = k + p
    aligned = spitch % 16 == 0 and off % 16 == 0
    joint = bool(rng.integers(0, 2))
    gap = int(rng.integers(0, 3)) * (16 if aligned else 7)
    if joint:                                          # [B][t] slots in one grid
        bp = t * spitch + gap
        addr = np.array([[off + b * bp + i * spitch for i in range(t)] for b in range(B)], np.int64)
        size = off + B * bp + 64
    else:                                              # data grid, then a parity grid after it
        bpd, bpp = k * spitch + gap, p * spitch + gap
        pbase = off + B * bpd + 32 * int(rng.integers(0, 3))
        addr = np.array([[off + b * bpd + i * spitch for i in range(k)] +
                         [pbase + b * bpp + r * spitch for r in range(p)] for b in range(B)], np.int64)
        size = pbase + B * bpp + 64
    host = np.full(size, SENTINEL, np.uint8)
    full = []
    for b in range(B):
        sh = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)] + [np.zeros(L, np.uint8) for _ in range(p)]
        c_oracle.encode(k, p, sh)
        full.append(sh)
        for i in range(k):
            host[addr[b, i]:addr[b, i] + L] = sh[i]
    d = torch.from_numpy(host).to(gpu)
    base = d.data_ptr()
    tab = np.ascontiguousarray((addr + base).astype(np.uint64).reshape(-1))
    rs = shmr_amd.ReedSolomon(k, p)
    g0 = shmr_amd.device_stats(0)["ptr_table_grids"]
    rc = lib().shmr_ec_encode_ptrs_dev(rs._h, tab.ctypes.data_as(ctypes.POINTER(_u8p)), B, L, 0, _stream())
    assert rc == 0, shmr_amd.Error(rc).name
    torch.cuda.synchronize()
    assert shmr_amd.device_stats(0)["ptr_table_grids"] == g0 + 1, ("encode not taken as a grid", joint, gap)
    expect = host.copy()
    for b in range(B):
        for i in range(k, t):
            expect[addr[b, i]:addr[b, i] + L] = full[b][i]
    assert np.array_equal(d.cpu().numpy(), expect), ("grid encode", k, p, L, B, joint, gap, aligned)
    # rebuild
    data_only = bool(rng.integers(0, 2))
    present = np.ones((B, t), np.uint8)
    for b in range(B):
        if rng.integers(0, 4):
            present[b, rng.choice(t, size=int(rng.integers(1, p + 1)), replace=False)] = 0
    written = (present == 0)
    if data_only:
        written[:, k:] = False
    fresh = bool(rng.integers(0, 2)) and written.any()
    work = expect.copy()
    for b in range(B):
        for i in range(t):
            if not present[b, i]:
                work[addr[b, i]:addr[b, i] + L] = 0x3C   # poison the absent shards' slots
    d = torch.from_numpy(work).to(gpu)
    tab2 = (addr + d.data_ptr()).astype(np.uint64)
    if fresh:                                          # rebuilt shard j of block b in an output grid
        nout = int(written.sum(axis=1).max())
        ospitch = spitch + (16 if aligned else 3) * int(rng.integers(0, 2))
        obp = nout * ospitch + gap
        out = torch.full((B * obp + 64,), 0xEE, dtype=torch.uint8, device=gpu)
        for b in range(B):
            j = 0
            for i in range(t):
                if written[b, i]:
                    tab2[b, i] = out.data_ptr() + b * obp + j * ospitch
                    j += 1
                elif not present[b, i]:
                    tab2[b, i] = 0                     # absent parity under data_only: NULL
    tab2 = np.ascontiguousarray(tab2.reshape(-1))
    g1 = shmr_amd.device_stats(0)["ptr_table_grids"]
    rc = lib().shmr_ec_reconstruct_ptrs_dev(rs._h, tab2.ctypes.data_as(ctypes.POINTER(_u8p)),
                                            present.ctypes.data_as(_u8p), B, L, int(data_only), 0, _stream())
    assert rc == 0, shmr_amd.Error(rc).name
    torch.cuda.synchronize()
    # (two grids: the present shards span both, so the table kernels may run --
    # bytes equal; nothing to rebuild -- every block whole, or only parity lost
    # under data_only -- launches nothing; rebuilt into fresh buffers from ONE
    # present shard per block, the input lattice's shard pitch is not
    # determined by the table -- the table kernels run)
    has_work = written.any(axis=1)
    one_present = fresh and bool((present[has_work].sum(axis=1) == 1).all())
    if joint and has_work.any() and not one_present:
        assert shmr_amd.device_stats(0)["ptr_table_grids"] == g1 + 1, ("rebuild not taken as a grid", fresh)
    got = d.cpu().numpy()
    want = work.copy()
    if not fresh:
        for b in range(B):
            for i in range(t):
                if written[b, i]:
                    want[addr[b, i]:addr[b, i] + L] = full[b][i]
        assert np.array_equal(got, want), ("grid rebuild in place", k, p, L, B, joint, data_only)
    else:
        assert np.array_equal(got, want), ("grid rebuild touched the shard buffer", k, p, L, B)
        o = out.cpu().numpy()
        ow = np.full(B * obp + 64, 0xEE, np.uint8)
        for b in range(B):
            j = 0
            for i in range(t):
                if written[b, i]:
                    ow[b * obp + j * ospitch:b * obp + j * ospitch + L] = full[b][i]
                    j += 1
        assert np.array_equal(o, ow), ("grid rebuild into fresh buffers", k, p, L, B, data_only)
