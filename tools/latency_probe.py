#!/usr/bin/env python3
"""Per-call latency of the drop-in single-block calls (shmr_ec_encode /
shmr_ec_reconstruct, the reference's per-block shape, block.rs:427/560):
mapped (zero-copy) and pageable (staged) shards, tiny and 4 MiB blocks.
Median over many calls from one thread; prints one JSON line per case.

    python tools/latency_probe.py
"""
from __future__ import annotations

import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

import shmr_amd  # noqa: E402
from shmr_amd._native import _u8p, lib  # noqa: E402


def main():
    k, p = 8, 3
    out = []
    # mapped (pointer table read in place / uploaded); pageable staged; pageable bounced
    cases = [(True, None, -2), (True, None, 0), (False, 0, -2), (False, 65536, -2)]
    spin = int(os.environ.get("SPIN", "-2"))
    shmr_amd.set_tuning(sync_spin_us=spin)
    for S in (4096, 524288):
        for mapped, bounce, direct in cases:
            shmr_amd.set_tuning(ptrs_direct=direct)
            if bounce is not None:
                shmr_amd.set_tuning(bounce_kib=bounce)
            if mapped:
                keep = shmr_amd.PinnedBuffer((k + p) * S)
                arr = keep.array.reshape(k + p, S)
            else:
                keep = None
                arr = np.zeros((k + p, S), np.uint8)
            arr[:k] = np.random.default_rng(1).integers(0, 256, (k, S), dtype=np.uint8)
            rs = shmr_amd.ReedSolomon(k, p)
            ptrs = (_u8p * (k + p))(*[arr[i].ctypes.data_as(_u8p) for i in range(k + p)])
            lens = (ctypes.c_size_t * (k + p))(*([S] * (k + p)))
            pres = np.ones(k + p, np.uint8)
            pres[3] = 0
            cp = pres.ctypes.data_as(_u8p)
            for name, call in (("encode", lambda: lib().shmr_ec_encode(rs._h, ptrs, lens, k + p)),
                               ("reconstruct", lambda: lib().shmr_ec_reconstruct(rs._h, ptrs, lens, cp, k + p, 0))):
                for _ in range(20):
                    assert call() == 0
                ts = []
                for _ in range(200):
                    t0 = time.perf_counter()
                    call()
                    ts.append(time.perf_counter() - t0)
                rec = {"call": name, "shard_bytes": S,
                       "buffers": ("mapped" + ("" if direct else ", pointer table uploaded")) if mapped else
                                  ("pageable, bounced" if bounce else "pageable, staged DMA"),
                       "median_us": round(float(np.median(ts)) * 1e6, 1), "p10_us": round(float(np.percentile(ts, 10)) * 1e6, 1)}
                out.append(rec)
                print(json.dumps(rec), flush=True)
            del keep
    shmr_amd.set_tuning(bounce_kib=-2, ptrs_direct=-2)
    # the reference's shape: per-block encode calls from 8 threads, pageable 4 MiB blocks
    from concurrent.futures import ThreadPoolExecutor
    S = 524288
    rng = np.random.default_rng(2)
    blocks = [[rng.integers(0, 256, S, dtype=np.uint8) if i < k else np.zeros(S, np.uint8) for i in range(k + p)]
              for _ in range(64)]
    rs = shmr_amd.ReedSolomon(k, p)
    pool = ThreadPoolExecutor(8)
    for bounce in (0, 65536):
        shmr_amd.set_tuning(bounce_kib=bounce)
        list(pool.map(rs.encode, blocks))
        t0 = time.perf_counter()
        for _ in range(3):
            list(pool.map(rs.encode, blocks))
        dt = (time.perf_counter() - t0) / 3
        print(json.dumps({"call": "encode x64 blocks, 8 threads", "buffers": "pageable, bounced" if bounce else
                          "pageable, staged DMA", "data_GiBps": round(64 * k * S / dt / 2 ** 30, 2)}), flush=True)
    shmr_amd.set_tuning(bounce_kib=-2)


if __name__ == "__main__":
    main()
