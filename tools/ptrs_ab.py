#!/usr/bin/env python3
"""The crate's shard-per-buffer shape on device (*_ptrs_dev) against the
Block-Cache slot layout (*_batch_dev, bench.py's default), interleaved rounds
in one process (product library).  Splits the gap into the table kernels'
own cost and the buffers' placement, and measures the placements a Rust shim
can get:

  slots          bench.py's layout: data / parity (or compact rebuild output) in
                 page-padded slots (shard pitch roundup(S, 4 KiB), + 4 KiB when
                 that is a multiple of 64 KiB), torch tensors, *_batch_dev
  slab           shmr_ec_device_alloc_shards: all total shards of the batch in one
                 slab (+ a second slab for rebuilt shards, one per absent shard);
                 the table is a slot grid -> the strided kernels (knob ptrs_grid)
  slab_sep       encode: data and parity in slabs of their own (grid)
  slab_inplace   rebuild: absent shards rebuilt in their own slots of the slab (grid)
  slab_tab       the slab's table with ptrs_grid=0: the table kernels over the
                 same addresses -- any difference to `slab` is the table
  slab_sep_tab   encode: the separate slabs with ptrs_grid=0
  smajor         shard-major slab: shard i of block b at base + (i * B + b) * P (one
                 grid whose data and parity shards fill separate regions; rebuilt
                 shards in a second shard-major slab); _tab / _inplace as above
  hipmalloc      one shmr_ec_device_alloc (hipMalloc) per shard
  ptrs_torch     one torch allocation per shard (back to back in the caching allocator)
  ptrs_page      per-shard allocations spaced by S + 4 KiB, 16 B past a page, as
                 glibc's mmap-served Vec<u8> allocations of these sizes are
                 (reference src/vfs/block.rs:408-419)
  pool_dense     r06: shmr_ec_pool slots, every slot live, blocks in shuffled order
                 (the table sorts into one lattice run); rebuilds in place
  pool_holed     r06: a pool after churn: B + B/4 slots, a random quarter freed,
                 the B live blocks in shuffled order (lattice runs -> segment runs
                 or a block list); _tab: the same with ptrs_grid=0; _pl (rebuilds):
                 one launch set per erasure pattern (knob pattern_launches); _list:
                 knob lattice_list=1 (a block list where runs do not fit the kernel
                 arguments; default: the table kernels)
  pool_few       r06: B + 16 slots, 16 freed (at most 17 runs: segment launches)
  joint_padNk    r06, encode: one torch slab, block b's k + p shards at b * (t*P + N KiB)
                 + i * P (the pool's slot layout, with N KiB between slots)

    python tools/ptrs_ab.py --config encode83 --rounds 11
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import shmr_amd  # noqa: E402
from shmr_amd.reed_solomon import _ptr, _u8p  # noqa: E402

CFG = {"encode83": (8, 3, 4 << 20, 0, 512), "decode83": (8, 3, 4 << 20, 1, 512),
       "encode104": (10, 4, 16 << 20, 0, 64), "decode104": (10, 4, 16 << 20, 2, 64)}


def slot_pitch(S):
    pitch = (S + 4095) // 4096 * 4096
    return pitch + 4096 if pitch % 65536 == 0 else pitch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="encode83", choices=sorted(CFG))
    ap.add_argument("--rounds", type=int, default=11)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--legs", default="", help="comma-separated subset of the legs (default: all)")
    a = ap.parse_args()
    k, p, block, er, B = CFG[a.config]
    t = k + p
    S = shmr_amd.calculate_shard_size(block, k)
    P = slot_pitch(S)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    rs = shmr_amd.ReedSolomon(k, p)
    st = torch.cuda.current_stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    present = np.ones((B, t), np.uint8)
    rows = np.arange(B)
    if er == 1:
        present[rows, rows % k] = 0
    elif er:
        for j in range(er):
            present[rows, (rows + 3 * j) % min(t, 10)] = 0
    pr = _ptr(present)
    runs, keep, tables = {}, [], {}

    def table(addrs):   # [B * t] uint64 addresses -> ctypes table
        arr = np.ascontiguousarray(np.asarray(addrs, dtype=np.uint64).reshape(-1))
        keep.append(arr)
        return arr.ctypes.data_as(ctypes.POINTER(_u8p))

    def ptrs_run(tab, grid=True, use_list=False):
        def f():
            if not grid:
                shmr_amd.set_tuning(ptrs_grid=0)
            if use_list:
                shmr_amd.set_tuning(lattice_list=1)
            try:
                if er == 0:
                    return rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab, B, S, 0, sp)
                return rs._L.shmr_ec_reconstruct_ptrs_dev(rs._h, tab, pr, B, S, 0, 0, sp)
            finally:
                if not grid:
                    shmr_amd.set_tuning(ptrs_grid=-2)
                if use_list:
                    shmr_amd.set_tuning(lattice_list=-2)
        return f

    def rebuilt_into(addrs, out_addr):
        """addrs [B, t]: absent entries replaced by out_addr(b, j) (j-th absent shard)"""
        addrs = np.array(addrs, dtype=np.uint64).reshape(B, t)
        for b in range(B):
            for j, i in enumerate(np.flatnonzero(present[b] == 0)):
                addrs[b, i] = out_addr(b, j)
        return addrs

    # -- slots (bench layout) --------------------------------------------------
    if er == 0:
        data = torch.randint(0, 256, (B, k, P), dtype=torch.uint8, device=dev, generator=g)
        par = torch.empty((B, p, P), dtype=torch.uint8, device=dev)
        runs["slots"] = lambda: rs.encode_batch_dev(data, par, shard_len=S)
    else:
        sh = torch.zeros((B, t, P), dtype=torch.uint8, device=dev)
        sh[:, :k, :S] = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device=dev, generator=g)
        rs.encode_batch_dev(sh[:, :k], sh[:, k:], shard_len=S)
        out = torch.zeros((B, er, P), dtype=torch.uint8, device=dev)
        runs["slots"] = lambda: rs.reconstruct_batch_dev_out(sh, present, out, shard_len=S)

    # -- allocator slabs --------------------------------------------------------
    slab = shmr_amd.ShardSlab(B, t, S)
    sv = slab.tensor()
    sv[:, :k, :S] = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device=dev, generator=g)
    enc_tab = table(slab.ptrs)
    assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, enc_tab, B, S, 0, sp) == 0     # codewords for the rebuilds
    if er == 0:
        runs["slab"] = ptrs_run(enc_tab)
        runs["slab_tab"] = ptrs_run(enc_tab, grid=False)
        ds, ps = shmr_amd.ShardSlab(B, k, S), shmr_amd.ShardSlab(B, p, S)
        ds.tensor()[:, :, :S] = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device=dev, generator=g)
        sep = np.concatenate([ds.ptrs.reshape(B, k), ps.ptrs.reshape(B, p)], axis=1)
        sep_tab = table(sep)
        runs["slab_sep"] = ptrs_run(sep_tab)
        runs["slab_sep_tab"] = ptrs_run(sep_tab, grid=False)
        keep.extend([ds, ps])
    else:
        outs = shmr_amd.ShardSlab(B, er, S)
        dec_tab = table(rebuilt_into(slab.ptrs, lambda b, j: outs.ptrs[b * er + j]))
        runs["slab"] = ptrs_run(dec_tab)
        runs["slab_tab"] = ptrs_run(dec_tab, grid=False)
        runs["slab_inplace"] = ptrs_run(enc_tab)
        keep.append(outs)
    keep.append(slab)
    # shard-major slab: shard i of block b at base + (i * B + b) * P -- one grid
    # (spitch B * P, bpitch P) whose data and parity shards fill separate regions
    smaj = shmr_amd.DeviceBuffer(B * t * P, device=0, contiguous=False)
    m0 = int(smaj._p.value)
    mv = smaj.tensor((t, B, P))
    mv[:k, :, :S] = torch.randint(0, 256, (k, B, S), dtype=torch.uint8, device=dev, generator=g)
    sm = np.array([[m0 + (i * B + b) * P for i in range(t)] for b in range(B)], dtype=np.uint64)
    sm_tab = table(sm)
    assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, sm_tab, B, S, 0, sp) == 0
    keep.append(smaj)
    if er:
        souts = shmr_amd.DeviceBuffer(B * er * P, device=0, contiguous=False)
        keep.append(souts)
        o0 = int(souts._p.value)
        sm_dec = table(rebuilt_into(sm, lambda b, j: o0 + (j * B + b) * P))
        runs["smajor"] = ptrs_run(sm_dec)
        runs["smajor_tab"] = ptrs_run(sm_dec, grid=False)
        runs["smajor_inplace"] = ptrs_run(sm_tab)
    else:
        runs["smajor"] = ptrs_run(sm_tab)
        runs["smajor_tab"] = ptrs_run(sm_tab, grid=False)

    # -- r06: a slot pool (shmr_ec_pool_*), blocks taken in shuffled order ------------
    # pool_dense: B slots, all live (one lattice run once sorted); pool_holed: B + B/4
    # slots, a random quarter freed again (holes), the other B blocks in shuffled
    # order -- a Block Cache after churn.  Encodes write parity into the block's
    # own slot; rebuilds write the lost shard in place.  _tab: ptrs_grid=0.
    prng = np.random.default_rng(17)
    for name, extra in (("pool_dense", 0), ("pool_holed", B // 4), ("pool_few", 16)):
        pool = shmr_amd.ShardPool(t, S, B + extra)
        blocks = [pool.alloc() for _ in range(B + extra)]
        for j in sorted(prng.choice(B + extra, size=extra, replace=False).tolist(), reverse=True):
            pool.free(blocks.pop(j))
        order = prng.permutation(B)
        rows_ = np.stack([blocks[int(j)] for j in order])
        for r in rows_:
            for i in range(k):
                pool.shard(r, i).copy_(torch.randint(0, 256, (S,), dtype=torch.uint8, device=dev, generator=g))
        ptab = table(rows_)
        assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, ptab, B, S, 0, sp) == 0
        runs[name] = ptrs_run(ptab)
        runs[name + "_tab"] = ptrs_run(ptab, grid=False)
        runs[name + "_list"] = ptrs_run(ptab, use_list=True)
        if er:   # the rebuild's patterns as one launch set each (knob pattern_launches)
            def pl(f=ptrs_run(ptab)):
                shmr_amd.set_tuning(pattern_launches=1)
                try:
                    return f()
                finally:
                    shmr_amd.set_tuning(pattern_launches=-2)
            runs[name + "_pl"] = pl
        keep.append(pool)
    # -- r06: one joint slab per block slot (k + p shards at P), block pitch t*P + pad --
    if er == 0:
        for pad in (0, 4096, 8192, 65536, 69632, 1 << 20):
            BP = t * P + pad
            jt = torch.zeros((B * BP,), dtype=torch.uint8, device=dev)
            jv = jt.view(B, BP)
            for i in range(k):
                jv[:, i * P:i * P + S] = torch.randint(0, 256, (B, S), dtype=torch.uint8, device=dev, generator=g)
            keep.append(jt)

            def joint(jt=jt, BP=BP):
                b0 = jt.data_ptr()
                return rs._L.shmr_ec_encode_batch_dev(rs._h, ctypes.c_void_p(b0), P, BP, ctypes.c_void_p(b0 + k * P),
                                                      P, BP, B, S, 0, sp)
            runs[f"joint_pad{pad // 1024}k"] = joint

    # -- one hipMalloc per shard (shmr_ec_device_alloc) ------------------------------
    bufs = [[shmr_amd.DeviceBuffer(S, device=0, contiguous=False) for _ in range(t)] for _ in range(B)]
    for blk in bufs:
        for i in range(k):
            blk[i].tensor().copy_(torch.randint(0, 256, (S,), dtype=torch.uint8, device=dev, generator=g))
    keep.append(bufs)
    hm = np.array([[int(b_._p.value) for b_ in blk] for blk in bufs], dtype=np.uint64)
    hm_tab = table(hm)
    assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, hm_tab, B, S, 0, sp) == 0
    if er:
        obufs = [[shmr_amd.DeviceBuffer(S, device=0, contiguous=False) for _ in range(er)] for _ in range(B)]
        keep.append(obufs)
        hm_tab = table(rebuilt_into(hm, lambda b, j: int(obufs[b][j]._p.value)))
    runs["hipmalloc"] = ptrs_run(hm_tab)

    # -- one torch allocation per shard ----------------------------------------------
    tb = [[torch.randint(0, 256, (S,), dtype=torch.uint8, device=dev, generator=g) for _ in range(t)]
          for _ in range(B)]
    keep.append(tb)
    tt = np.array([[s.data_ptr() for s in blk] for blk in tb], dtype=np.uint64)
    t_tab = table(tt)
    assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, t_tab, B, S, 0, sp) == 0
    if er:
        tout = [[torch.zeros(S, dtype=torch.uint8, device=dev) for _ in range(er)] for _ in range(B)]
        keep.append(tout)
        t_tab = table(rebuilt_into(tt, lambda b, j: tout[b][j].data_ptr()))
    runs["ptrs_torch"] = ptrs_run(t_tab)

    # -- glibc-like placement ---------------------------------------------------------
    span = (S + 4096 + 4095) // 4096 * 4096
    arena = torch.randint(0, 256, ((B * t + (B * er if er else 0)) * span,), dtype=torch.uint8, device=dev,
                          generator=g)
    keep.append(arena)
    a0 = arena.data_ptr()
    pg = np.array([[a0 + (b * t + i) * span + 16 for i in range(t)] for b in range(B)], dtype=np.uint64)
    pg_tab = table(pg)
    assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, pg_tab, B, S, 0, sp) == 0
    if er:
        pg_tab = table(rebuilt_into(pg, lambda b, j: a0 + (B * t + b * er + j) * span + 16))
    runs["ptrs_page"] = ptrs_run(pg_tab)

    if a.legs:
        want = set(a.legs.split(","))
        runs = {n: f for n, f in runs.items() if n in want}
    algo = B * (k + (er or p)) * S
    for f in runs.values():
        assert f() in (None, 0)
    torch.cuda.synchronize()
    grids0 = shmr_amd.device_stats(0)["ptr_table_grids"]
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:   # clock ramp
        for f in runs.values():
            f()
        torch.cuda.synchronize()
    times = {n: [] for n in runs}
    for _ in range(a.rounds):
        for n, f in runs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.iters):
                rc = f()
                assert rc in (None, 0), rc
            e1.record(st)
            torch.cuda.synchronize()
            times[n].append(e0.elapsed_time(e1) / a.iters)
    grid_calls = shmr_amd.device_stats(0)["ptr_table_grids"] - grids0
    for n, ts in times.items():
        med = float(np.median(ts))
        print(json.dumps({"config": a.config, "layout": n, "median_ms": round(med, 4), "min_ms": round(min(ts), 4),
                          "frac": round(algo / (med / 1e3) / 8e12, 4),
                          "build_id": shmr_amd.reed_solomon.lib().shmr_ec_build_id().decode()}))
    print(json.dumps({"config": a.config, "grid_calls": grid_calls}))


if __name__ == "__main__":
    main()
