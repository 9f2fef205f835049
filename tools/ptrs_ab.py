#!/usr/bin/env python3
"""Pointer tables against padded slots, interleaved rounds in one process
(product library).  Splits the gap between the crate's shard-per-buffer shape
(`*_ptrs_dev`) and the Block-Cache slot layout (`*_batch_dev`, bench.py's
default) into the kernel's own cost and the allocations' placement:

  slots        bench.py's layout: data / parity (or compact rebuild output) in
               page-padded slots (shard pitch roundup(S, 4 KiB), + 4 KiB when
               that is a multiple of 64 KiB)
  ptrs_slots   *_ptrs_dev over a pointer table naming exactly those slots: the
               same addresses and bytes -- any difference is the table
  ptrs_torch   *_ptrs_dev over one torch allocation per shard (bench.py
               --layout ptrs): the caching allocator packs them back to back
  ptrs_page    *_ptrs_dev over per-shard allocations spaced by S + 4 KiB, as
               glibc's mmap-served Vec<u8> allocations of these sizes are
               (reference src/vfs/block.rs:408-419)

    python tools/ptrs_ab.py --config encode83 --rounds 11
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

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
    runs, keep = {}, []

    def table(addr):   # addr(b, i) -> device address; a ctypes table [B * t]
        arr = np.array([addr(b, i) for b in range(B) for i in range(t)], dtype=np.uint64)
        keep.append(arr)
        return arr.ctypes.data_as(ctypes.POINTER(_u8p))

    def ptrs_run(tab):
        if er == 0:
            return lambda: rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab, B, S, 0, sp)
        return lambda: rs._L.shmr_ec_reconstruct_ptrs_dev(rs._h, tab, pr, B, S, 0, 0, sp)

    # slots: data [B, k, P], parity [B, p, P]; decode: all shards [B, t, P] + compact out [B, er, P]
    if er == 0:
        data = torch.randint(0, 256, (B, k, P), dtype=torch.uint8, device=dev, generator=g)
        par = torch.empty((B, p, P), dtype=torch.uint8, device=dev)
        runs["slots"] = lambda: rs.encode_batch_dev(data, par, shard_len=S)
        d0, p0 = data.data_ptr(), par.data_ptr()
        runs["ptrs_slots"] = ptrs_run(table(lambda b, i: d0 + (b * k + i) * P if i < k else p0 + (b * p + i - k) * P))
    else:
        sh = torch.zeros((B, t, P), dtype=torch.uint8, device=dev)
        sh[:, :k, :S] = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device=dev, generator=g)
        rs.encode_batch_dev(sh[:, :k], sh[:, k:], shard_len=S)
        out = torch.zeros((B, er, P), dtype=torch.uint8, device=dev)
        runs["slots"] = lambda: rs.reconstruct_batch_dev_out(sh, present, out, shard_len=S)
        s0, o0 = sh.data_ptr(), out.data_ptr()
        slot_of = {}
        for b in range(B):
            for j, i in enumerate(np.flatnonzero(present[b] == 0)):
                slot_of[(b, int(i))] = o0 + (b * er + j) * P
        runs["ptrs_slots"] = ptrs_run(table(lambda b, i: slot_of.get((b, i), s0 + (b * t + i) * P)))
    # one torch allocation per shard (back to back in the caching allocator)
    bufs = [[torch.randint(0, 256, (S,), dtype=torch.uint8, device=dev, generator=g) for _ in range(t)]
            for _ in range(B)]
    keep.append(bufs)
    runs["ptrs_torch"] = ptrs_run(table(lambda b, i: bufs[b][i].data_ptr()))
    # per-shard allocations spaced S + 4 KiB (glibc's mmap-served Vec<u8>: header page + data)
    span = (S + 4096 + 4095) // 4096 * 4096
    arena = torch.randint(0, 256, (B * t * span,), dtype=torch.uint8, device=dev, generator=g)
    a0 = arena.data_ptr()
    runs["ptrs_page"] = ptrs_run(table(lambda b, i: a0 + (b * t + i) * span + 16))
    # rebuild inputs of the pointer layouts must be codewords as well (a zero or random
    # parity input changes the rate): encode them first
    for name in ("ptrs_torch", "ptrs_page"):
        if er:
            tab = keep[-1] if name == "ptrs_page" else keep[-2]
            assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab.ctypes.data_as(ctypes.POINTER(_u8p)), B, S, 0, sp) == 0
    algo = B * (k + (er or p)) * S
    for f in runs.values():
        assert f() in (None, 0)
    torch.cuda.synchronize()
    import time
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
    for n, ts in times.items():
        med = float(np.median(ts))
        print(json.dumps({"config": a.config, "layout": n, "median_ms": round(med, 4), "min_ms": round(min(ts), 4),
                          "frac": round(algo / (med / 1e3) / 8e12, 4)}))


if __name__ == "__main__":
    main()
