#!/usr/bin/env python3
"""Host-memory (PCIe-inclusive) rates of the erasure path -- BASELINE config 5.

The reference's path starts and ends in host memory (FUSE buffers / the Block
Cache, shard files on disk).  These numbers include H2D and D2H copies and are
reported in DESIGN.md; they are never bench.py's headline ``value``.

Measured (GiB/s of file data, RS(8,3), 4 MiB StorageBlocks):
  * host_batch_encode_{pageable,pinned_dma,mapped}  shmr_ec_encode_blocks_host
      over B blocks: pageable numpy (staged through a pinned mirror by copy
      threads), torch-pinned (DMA pipeline), mapped Block-Cache buffers from
      shmr_ec_host_alloc (zero-copy: the kernel reads/writes them over PCIe)
  * host_batch_reconstruct_{...}          1 missing data shard per block
  * per_block_encode_threads{,_mapped}    the literal drop-in call
      (shmr_ec_encode per block) from a thread pool, as rayon calls
      ReedSolomon::encode per block (src/vfs/mod.rs:93-96)
The batch entry points are timed through the C ABI with the shard-pointer
arrays marshalled once (the Python shim's per-call conversion of B*(k+p) numpy
views is not the library's cost).
  * virtual_file_roundtrip                 write -> sync_data (encode) -> erase a
      shard per block -> read (reconstruct) over a 256 MiB file, verified
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (share torch's HIP runtime)

import shmr_amd  # noqa: E402

K, P = 8, 3
BLOCK = 4 << 20
S = shmr_amd.calculate_shard_size(BLOCK, K)
GiB = float(1 << 30)


def timeit(fn, reps):
    fn()                                    # warm: plans, staging, clocks
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps


def make_blocks(B, kind, rng):
    blocks, keep = [], []
    for _ in range(B):
        if kind == "mapped":
            buf = shmr_amd.PinnedBuffer((K + P) * S)
            keep.append(buf)
            a = buf.array
        elif kind == "pinned_dma":
            t = torch.empty((K + P) * S, dtype=torch.uint8).pin_memory()
            keep.append(t)
            a = t.numpy()
        else:
            a = np.empty((K + P) * S, np.uint8)
        a[:K * S] = rng.integers(0, 256, K * S, dtype=np.uint8)
        a[K * S:] = 0
        blocks.append([a[i * S:(i + 1) * S] for i in range(K + P)])
    return blocks, keep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rs = shmr_amd.ReedSolomon(K, P)
    rng = np.random.default_rng(0)
    res = {"k": K, "p": P, "block_bytes": BLOCK, "shard_bytes": S, "blocks": a.blocks, "unit": "GiB/s of data"}
    data_bytes = a.blocks * K * S

    import ctypes
    from shmr_amd._native import _u8p, lib
    cdev = (ctypes.c_int * 1)(0)
    for tag in ("pageable", "pinned_dma", "mapped"):
        blocks, keep = make_blocks(a.blocks, tag, rng)
        _, _, cp = rs._host_ptrs(blocks)
        z0, s0 = shmr_amd.path_stats()
        dt = timeit(lambda: lib().shmr_ec_encode_blocks_host(rs._h, cp, a.blocks, S, cdev, 1), a.reps)
        z1, s1 = shmr_amd.path_stats()
        res[f"host_batch_encode_{tag}"] = round(data_bytes / dt / GiB, 2)
        res[f"host_batch_{tag}_path"] = "zero_copy" if z1 > z0 and s1 == s0 else "staged"
        want = [[x.copy() for x in blk[K:]] for blk in blocks[:4]]
        # one missing data shard per block (config 3 pattern), in place
        present = np.ones((a.blocks, K + P), np.uint8)
        present[np.arange(a.blocks), np.arange(a.blocks) % K] = 0
        ref = [blk[b % K].copy() for b, blk in enumerate(blocks)]
        for b, blk in enumerate(blocks):
            blk[b % K][:] = 0
        cpres = present.ctypes.data_as(_u8p)
        dt = timeit(lambda: lib().shmr_ec_reconstruct_blocks_host(rs._h, cp, cpres, a.blocks, S, 0, cdev, 1), a.reps)
        res[f"host_batch_reconstruct_{tag}"] = round(data_bytes / dt / GiB, 2)
        assert all(np.array_equal(blk[b % K], ref[b]) for b, blk in enumerate(blocks))
        assert all(np.array_equal(x, y) for blk, w in zip(blocks[:4], want) for x, y in zip(blk[K:], w))
        del blocks, keep

    # the literal drop-in: one shmr_ec_encode per block from a thread pool
    pool = ThreadPoolExecutor(a.threads)
    for tag in ("pageable", "mapped"):
        blocks, keep = make_blocks(64, tag, rng)
        sfx = "" if tag == "pageable" else "_mapped"
        dt = timeit(lambda: list(pool.map(lambda blk: rs.encode(blk), blocks)), a.reps)
        res[f"per_block_encode_threads{sfx}"] = round(64 * K * S / dt / GiB, 2)
        t1 = timeit(lambda: rs.encode(blocks[0]), a.reps * 4)
        res[f"per_block_encode_latency_ms{sfx}"] = round(t1 * 1e3, 3)
        del blocks, keep
    res["per_block_encode_threads_n"] = a.threads

    # VirtualFile round trip: 256 MiB file, write -> sync -> erase -> read
    nblk = 64
    file_bytes = nblk * BLOCK
    src = rng.integers(0, 256, file_bytes, dtype=np.uint8)
    cache = [shmr_amd.PinnedBuffer((K + P) * S) for _ in range(nblk)]      # Block Cache buffers
    t0 = time.perf_counter()
    for b in range(nblk):                                                  # VirtualFile::write
        cache[b].array[:BLOCK] = src[b * BLOCK:(b + 1) * BLOCK]
    t_write = time.perf_counter() - t0
    blocks = [[c.array[i * S:(i + 1) * S] for i in range(K + P)] for c in cache]
    t0 = time.perf_counter()
    rs.encode_blocks_host(blocks)                                          # VirtualFile::sync_data
    t_sync = time.perf_counter() - t0
    present = np.ones((nblk, K + P), np.uint8)
    for b in range(nblk):                                                  # lose one data shard per block
        present[b, b % K] = 0
        blocks[b][b % K][:] = 0
    t0 = time.perf_counter()
    rs.reconstruct_blocks_host(blocks, present)                            # load_block with erasure
    out = np.concatenate([c.array[:BLOCK] for c in cache])                 # VirtualFile::read
    t_read = time.perf_counter() - t0
    assert np.array_equal(out, src)
    res["virtual_file_roundtrip"] = {"file_MiB": file_bytes >> 20, "write_GiBps": round(file_bytes / t_write / GiB, 2),
                                     "sync_encode_GiBps": round(file_bytes / t_sync / GiB, 2),
                                     "read_reconstruct_GiBps": round(file_bytes / t_read / GiB, 2),
                                     "verified": True}
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
