"""Every kernel of the product library, launched against the CPU oracle.

The product library's full-tile kernel list is not written by hand: gf_apply.hip
derives it at compile time from the launch policy (kern::policy_variant over
every valid kern::LaunchShape, include/shmr_ec.h shmr_ec_kernel_inventory), so
each compiled instantiation is reachable by some call.  This module makes those
calls -- one per launch shape, through the public entry points the reference's
two call sites would use (ReedSolomon::encode at src/vfs/block.rs:427 and
ReedSolomon::reconstruct at block.rs:560, batched and per-shard-buffer forms,
device-resident and host-resident) -- checks every output byte against the
oracle, and finally asserts from the library's per-kernel launch counters that
the sweep launched every instantiation in the inventory, the partial-tile
(mode 1), byte-granular (mode 2) and realigning (mode 3, knob uvec=0: what a
device without the unaligned access mode runs) kernels included.

Shape parameters (gf_apply.hpp LaunchShape) and how a call produces them:
  decode     encode (p = rows parity rows) / reconstruct (rows absent shards)
  small_k    k = 4 / k = 10
  host_mapped + ptrs
             device pitch batch (*_batch_dev) / device shard buffers (*_ptrs_dev)
             / mapped host slab (*_blocks_host over shmr_ec_host_alloc memory,
             zero-copy pointer tables) / pageable host slab (*_blocks_host,
             coded in place in the mapped pinned mirror)
  segs       reconstruct: two erasure patterns in two block runs / one pattern;
             encode (r06): pointer-table blocks on a slot lattice in two runs
             (slots 0-2 and 5-7: launch_slots' segment launch) / a pitch batch
  compact    reconstruct_batch_dev_out / in place
  sc1_ok     16-byte aligned outputs / an output (or, for pointer tables, a
             shard) off alignment
  fused      shard length with a partial last tile / a whole number of tiles
"""
import itertools

import numpy as np
import pytest

import shmr_amd
from oracle import c_oracle

pytestmark = pytest.mark.gpu

B = 6          # blocks per call
TILE = 4096    # 256 lanes x 16 B (U = 1); 4-row launches use U = 2


def _shapes():
    """Valid LaunchShapes (gf_apply.hpp shape_valid), as dicts."""
    for decode, small_k, hm, ptrs, segs, compact, sc1_ok, fused, rows in itertools.product(
            (False, True), (False, True), (False, True), (False, True), (False, True), (False, True),
            (False, True), (False, True), (1, 2, 3, 4)):
        if not decode and (compact or (segs and (ptrs or hm))):
            continue
        if compact and (ptrs or hm):
            continue
        if sc1_ok and hm:
            continue
        yield dict(decode=decode, small_k=small_k, hm=hm, ptrs=ptrs, segs=segs, compact=compact,
                   sc1_ok=sc1_ok, fused=fused, rows=rows)


def _shard_len(rows, fused):
    tile = TILE * (2 if rows >= 4 else 1)
    return 2 * tile + (48 if fused else 0)


def _codeword(k, p, L, rng):
    data = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    par = np.zeros((B, p, L), np.uint8)
    c_oracle.encode_batch(k, p, data, par, B, L, 8)
    return np.concatenate([data, par], axis=1)   # [B, t, L]


def _patterns(k, t, rows, segs):
    """present flags [B, t]: `rows` absent shards per block; with segs two
    patterns in two runs of blocks (a segment launch), else one pattern."""
    a = list(range(rows))
    b = [1, 2, 3, 5][:rows] if k == 4 else list(range(2, 2 + rows))
    pr = np.ones((B, t), np.uint8)
    for blk in range(B):
        for i in (b if segs and blk >= B // 2 else a):
            pr[blk, i] = 0
    return pr


def _dev_views(gpu, arr, misalign_one, idx=None):
    """Separate GPU buffers per shard (slices of one arena); one shard off
    16-byte alignment when misalign_one: shard `idx` (default the last) of block
    1 -- a shard the call touches (an encode's last parity row; a rebuild's
    input `rows`, the first present shard after the erased ones: removed shards
    are replaced by fresh, aligned buffers, and present shards past the first k
    are never read)."""
    import torch
    Bn, t, L = arr.shape
    slot = (L + 64 + 255) // 256 * 256
    arena = torch.zeros(Bn * t * slot + 256, dtype=torch.uint8, device=gpu)
    idx = t - 1 if idx is None else idx
    views = []
    for b in range(Bn):
        row = []
        for i in range(t):
            off = (b * t + i) * slot + (3 if misalign_one and b == 1 and i == idx else 0)
            v = arena[off:off + L]
            v.copy_(torch.from_numpy(np.ascontiguousarray(arr[b, i])).to(gpu))
            row.append(v)
        views.append(row)
    return arena, views


def _run_case(gpu, s, seed):
    import torch
    rng = np.random.default_rng(seed)
    rows, L = s["rows"], _shard_len(s["rows"], s["fused"])
    k = 4 if s["small_k"] else 10
    p = rows if not s["decode"] else 4
    t = k + p
    rs = shmr_amd.ReedSolomon(k, p)
    cw = _codeword(k, p, L, rng)
    if not s["decode"]:
        want = cw
        if s["hm"]:
            if s["ptrs"]:   # mapped Block-Cache slab: zero-copy pointer tables
                buf = shmr_amd.PinnedBuffer(B * t * L)
                arr = buf.array.reshape(B, t, L)
            else:           # pageable: coded in the mapped pinned mirror
                arr = np.zeros((B, t, L), np.uint8)
            arr[:, :k] = cw[:, :k]
            arr[:, k:] = 0x77
            rs.encode_blocks_host(arr)
            got = np.array(arr)
        elif s["ptrs"]:
            start = cw.copy()
            start[:, k:] = 0x77
            _, views = _dev_views(gpu, start, not s["sc1_ok"])
            rs.encode_ptrs_dev(views)
            torch.cuda.synchronize()
            got = np.stack([np.stack([v.cpu().numpy() for v in row]) for row in views])
        elif s["segs"]:   # block slots of one arena in two runs (a pool with a hole)
            pitch = (L + 255) // 256 * 256
            arena = torch.full(((B + 4) * t * pitch,), 0x77, dtype=torch.uint8, device=gpu)
            slots = list(range(B // 2)) + list(range(B // 2 + 2, B + 2))
            views = [[arena[(sl * t + i) * pitch:(sl * t + i) * pitch + L] for i in range(t)] for sl in slots]
            for b in range(B):
                for i in range(k):
                    views[b][i].copy_(torch.from_numpy(cw[b, i].copy()).to(gpu))
            shmr_amd.set_tuning(ptrs_grid=1)   # (the module runs with the table kernels)
            try:
                g0 = shmr_amd.device_stats(0)["ptr_table_grids"]
                rs.encode_ptrs_dev(views)
                assert shmr_amd.device_stats(0)["ptr_table_grids"] == g0 + 1
            finally:
                shmr_amd.set_tuning(ptrs_grid=0)
            torch.cuda.synchronize()
            got = np.stack([np.stack([v.cpu().numpy() for v in row]) for row in views])
        else:
            pitch = (L + 255) // 256 * 256
            data = torch.zeros((B, k, pitch), dtype=torch.uint8, device=gpu)
            data[:, :, :L] = torch.from_numpy(cw[:, :k]).to(gpu)
            off = 0 if s["sc1_ok"] else 1
            pflat = torch.full((B * p * (pitch + 16) + 64,), 0x77, dtype=torch.uint8, device=gpu)
            parity = pflat[off:off + B * p * (pitch + 16)].view(B, p, pitch + 16)
            rs.encode_batch_dev(data, parity, shard_len=L)
            torch.cuda.synchronize()
            got = np.concatenate([data[:, :, :L].cpu().numpy(), parity[:, :, :L].cpu().numpy()], axis=1)
        assert np.array_equal(got, want), s
        return
    pr = _patterns(k, t, rows, s["segs"])
    erased = cw.copy()
    erased[pr == 0] = 0xEE
    if s["hm"]:
        if s["ptrs"]:
            buf = shmr_amd.PinnedBuffer(B * t * L)
            arr = buf.array.reshape(B, t, L)
            arr[:] = erased
        else:
            arr = erased.copy()
        rs.reconstruct_blocks_host(arr, pr)
        assert np.array_equal(np.array(arr), cw), s
    elif s["ptrs"]:
        _, views = _dev_views(gpu, erased, not s["sc1_ok"], idx=rows)
        blocks = [[(v if pr[b, i] else None) for i, v in enumerate(row)] for b, row in enumerate(views)]
        rs.reconstruct_ptrs_dev(blocks)
        torch.cuda.synchronize()
        got = np.stack([np.stack([v.cpu().numpy() for v in row]) for row in blocks])
        assert np.array_equal(got, cw), s
    elif s["compact"]:
        pitch = (L + 255) // 256 * 256
        sh = torch.zeros((B, t, pitch), dtype=torch.uint8, device=gpu)
        sh[:, :, :L] = torch.from_numpy(erased).to(gpu)
        off = 0 if s["sc1_ok"] else 1
        oflat = torch.full((B * rows * pitch + 64,), 0x77, dtype=torch.uint8, device=gpu)
        out = oflat[off:off + B * rows * pitch].view(B, rows, pitch)
        rs.reconstruct_batch_dev_out(sh, pr, out, shard_len=L)
        torch.cuda.synchronize()
        o = out[:, :, :L].cpu().numpy()
        for b in range(B):
            absent = np.flatnonzero(pr[b] == 0)
            assert np.array_equal(o[b, :len(absent)], cw[b, absent]), (s, b)
        assert np.array_equal(sh[:, :, :L].cpu().numpy()[pr == 1], cw[pr == 1]), s   # inputs untouched
    else:
        pitch = (L + 255) // 256 * 256 + (0 if s["sc1_ok"] else 1)   # in place; odd pitch: misaligned shards
        flat = torch.zeros((B * t * pitch,), dtype=torch.uint8, device=gpu)
        sh = flat.view(B, t, pitch)
        sh[:, :, :L] = torch.from_numpy(erased).to(gpu)
        rs.reconstruct_batch_dev(sh, pr, shard_len=L)
        torch.cuda.synchronize()
        assert np.array_equal(sh[:, :, :L].cpu().numpy(), cw), s


@pytest.fixture(scope="module")
def before():
    # the sweep's device shard views sit on a slot grid: keep them on the
    # table kernels (knob ptrs_grid) so every pointer-table kernel is launched
    shmr_amd.set_tuning(ptrs_grid=0)
    try:
        yield shmr_amd.kernel_inventory()
    finally:
        shmr_amd.set_tuning(ptrs_grid=-2)


@pytest.mark.parametrize("decode", [False, True])
@pytest.mark.parametrize("small_k", [False, True])
def test_launch_shapes(gpu, before, decode, small_k):
    cases = [s for s in _shapes() if s["decode"] == decode and s["small_k"] == small_k]
    assert cases
    for n, s in enumerate(cases):
        _run_case(gpu, s, seed=1000 * int(decode) + 100 * int(small_k) + n)


@pytest.mark.parametrize("rows", [1, 2, 3, 4])
def test_tail_bytewise_realign_kernels(gpu, before, rows):
    """Mode 1 (shard shorter than one tile), mode 2 (mapped host shards off
    alignment: byte-granular) and mode 3 (knob uvec=0 on the reference's packed
    device buffer: the realigning kernel, plus mode 2 for the remainder)."""
    import torch
    rng = np.random.default_rng(77 + rows)
    k, p = 4, rows
    t = k + p
    rs = shmr_amd.ReedSolomon(k, p)
    # mode 1
    L = 1000
    cw = _codeword(k, p, L, rng)
    data = torch.from_numpy(cw[:, :k].copy()).to(gpu)
    parity = torch.zeros((B, p, L), dtype=torch.uint8, device=gpu)
    rs.encode_batch_dev(data, parity, shard_len=L)
    torch.cuda.synchronize()
    assert np.array_equal(parity.cpu().numpy(), cw[:, k:])
    # mode 2: mapped shards at odd offsets
    L = 3 * TILE + 5
    cw = _codeword(k, p, L, rng)
    buf = shmr_amd.PinnedBuffer(B * t * (L + 16) + 16)
    blocks = []
    for b in range(B):
        row = []
        for i in range(t):
            off = (b * t + i) * (L + 16) + 3
            v = buf.array[off:off + L]
            v[:] = cw[b, i] if i < k else 0
            row.append(v)
        blocks.append(row)
    rs.encode_blocks_host(blocks)
    assert all(np.array_equal(blocks[b][i], cw[b, i]) for b in range(B) for i in range(t))
    # mode 3: the packed block buffer (shard i at i * L, L odd) without the unaligned mode
    shmr_amd.set_tuning(uvec=0)
    try:
        flat = torch.zeros(B * t * L, dtype=torch.uint8, device=gpu)
        packed = flat.view(B, t, L)
        packed[:, :k] = torch.from_numpy(cw[:, :k].copy()).to(gpu)
        rs.encode_batch_dev(packed[:, :k], packed[:, k:], shard_len=L, data_shard_pitch=L, parity_shard_pitch=L)
        torch.cuda.synchronize()
        assert np.array_equal(packed.cpu().numpy(), cw)
    finally:
        shmr_amd.set_tuning(uvec=-2)


def test_every_kernel_launched(gpu, before):
    """Runs last in this module: the sweep above launched every kernel of the
    product library's inventory (launch counters since the module started)."""
    after = shmr_amd.kernel_inventory()
    assert [(e["rows"], e["chunks"], e["mode"], e["flags"]) for e in after] == \
        [(e["rows"], e["chunks"], e["mode"], e["flags"]) for e in before]
    missing = [e for e, b in zip(after, before) if e["launches"] == b["launches"]]
    assert not missing, f"{len(missing)} of {len(after)} kernels never launched: {missing[:8]}"
