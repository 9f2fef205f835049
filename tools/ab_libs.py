#!/usr/bin/env python3
"""A/B builds of libshmr_ec.so in ONE process (interleaved rounds): the
current in-tree library against other builds given by path, on the same
device buffers.  Both are loaded with RTLD_LOCAL, so each resolves its own
shmr_ec_* symbols and registers its own kernels.

    python tools/ab_libs.py tools/_ab/libshmr_ec_<rev>.so [more.so ...] [--config encode83]
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

from shmr_amd import _native  # noqa: E402

CFG = {"encode83": (8, 3, 4 << 20, 0, 512), "decode83": (8, 3, 4 << 20, 1, 512),
       "encode104": (10, 4, 16 << 20, 0, 64), "decode104": (10, 4, 16 << 20, 2, 64),
       "decode83e3": (8, 3, 4 << 20, 3, 512),
       "encode42": (4, 2, 1 << 20, 0, 1024)}


def load(path):
    L = ctypes.CDLL(path, mode=os.RTLD_LOCAL)
    for name, res, args in _native.SIGNATURES:
        if hasattr(L, name):
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("others", nargs="+")
    ap.add_argument("--config", default="encode83")
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--pitch-align", type=int, default=256, help="shard pitch alignment (bench.py uses 4096)")
    ap.add_argument("--compact", action="store_true",
                    help="decode: rebuild into a compact [B][erasures][pitch] output (shmr_ec_reconstruct_batch_dev_out)")
    ap.add_argument("--ptrs", action="store_true",
                    help="every shard its own torch allocation, through the *_ptrs_dev calls (bench.py --layout ptrs)")
    a = ap.parse_args()
    k, p, block, er, B = CFG[a.config]
    libs = {"current": load(_native.LIB_PATH)}
    for o in a.others:
        libs[os.path.basename(o)] = load(os.path.abspath(o))
    dev = torch.device("cuda", 0)
    S = int(libs["current"].shmr_ec_shard_size(block, k))
    pitch = (S + a.pitch_align - 1) // a.pitch_align * a.pitch_align
    st = torch.cuda.current_stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    runs = {}
    if a.ptrs:
        t = k + p
        blocks = [[torch.randint(0, 256, (S,), dtype=torch.uint8, device=dev, generator=g) for _ in range(k)]
                  + [torch.zeros(S, dtype=torch.uint8, device=dev) for _ in range(p)] for _ in range(B)]
        present = np.ones((B, t), np.uint8)
        rows = np.arange(B)
        if er == 1:
            present[rows, rows % k] = 0
        elif er:
            for j in range(er):   # {b, b+3, b+6, ...} mod min(total, 10), as tools/tune.py
                present[rows, (rows + 3 * j) % min(t, 10)] = 0
        outs = [[torch.zeros(S, dtype=torch.uint8, device=dev) for _ in range(t)] for _ in range(B)]
        table = [blocks[b][i] if present[b, i] else outs[b][i] for b in range(B) for i in range(t)]
        tab = (_native._u8p * (B * t))(*[ctypes.cast(x.data_ptr(), _native._u8p) for x in table])
        pr = present.ctypes.data_as(_native._u8p)
        algo = B * (k + (er or p)) * S
        for n, L in libs.items():
            h = ctypes.c_void_p()
            assert L.shmr_ec_new(k, p, ctypes.byref(h)) == 0

            def run(L=L, h=h):
                rc = (L.shmr_ec_encode_ptrs_dev(h, tab, B, S, 0, sp) if er == 0 else
                      L.shmr_ec_reconstruct_ptrs_dev(h, tab, pr, B, S, 0, 0, sp))
                assert rc == 0, rc
            runs[n] = run
    elif er == 0:
        data = torch.randint(0, 256, (B, k, pitch), dtype=torch.uint8, device=dev, generator=g)
        par = {n: torch.empty((B, p, pitch), dtype=torch.uint8, device=dev) for n in libs}
        algo = B * (k + p) * S
        for n, L in libs.items():
            h = ctypes.c_void_p()
            assert L.shmr_ec_new(k, p, ctypes.byref(h)) == 0

            def run(L=L, h=h, out=par[n]):
                rc = L.shmr_ec_encode_batch_dev(h, ctypes.c_void_p(data.data_ptr()), pitch, k * pitch,
                                                ctypes.c_void_p(out.data_ptr()), pitch, p * pitch, B, S, 0, sp)
                assert rc == 0, rc
            runs[n] = run
    else:
        shards = torch.zeros((B, k + p, pitch), dtype=torch.uint8, device=dev)
        shards[:, :k, :S] = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device=dev, generator=g)
        present = np.ones((B, k + p), np.uint8)
        rows = np.arange(B)
        if er == 1:
            present[rows, rows % k] = 0
        else:
            for j in range(er):
                present[rows, (rows + 3 * j) % min(k + p, 10)] = 0
        algo = B * (k + er) * S
        pr = present.ctypes.data_as(_native._u8p)
        if a.compact:   # real parity content (a zero parity input changes the rate)
            for n, L in libs.items():
                h = ctypes.c_void_p()
                assert L.shmr_ec_new(k, p, ctypes.byref(h)) == 0
                assert L.shmr_ec_encode_batch_dev(h, ctypes.c_void_p(shards.data_ptr()), pitch, (k + p) * pitch,
                                                  ctypes.c_void_p(shards.data_ptr() + k * pitch), pitch,
                                                  (k + p) * pitch, B, S, 0, sp) == 0
                break
        outs = {n: torch.zeros((B, er, pitch), dtype=torch.uint8, device=dev) for n in libs}
        for n, L in libs.items():
            h = ctypes.c_void_p()
            assert L.shmr_ec_new(k, p, ctypes.byref(h)) == 0

            def run(L=L, h=h, out=outs[n]):
                if a.compact:
                    rc = L.shmr_ec_reconstruct_batch_dev_out(h, ctypes.c_void_p(shards.data_ptr()), pitch,
                                                             (k + p) * pitch, pr, B, S, 0,
                                                             ctypes.c_void_p(out.data_ptr()), pitch, er * pitch, 0, sp)
                else:
                    rc = L.shmr_ec_reconstruct_batch_dev(h, ctypes.c_void_p(shards.data_ptr()), pitch,
                                                         (k + p) * pitch, pr, B, S, 0, 0, sp)
                assert rc == 0, rc
            runs[n] = run
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        for r in runs.values():
            r()
        torch.cuda.synchronize()
    times = {n: [] for n in runs}
    for _ in range(a.rounds):
        for n, r in runs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.iters):
                r()
            e1.record(st)
            torch.cuda.synchronize()
            times[n].append(e0.elapsed_time(e1) / a.iters)
    if er == 0 and not a.ptrs:
        for n in par:
            assert torch.equal(par["current"], par[n]), f"outputs differ: {n}"
    if er and a.compact and not a.ptrs:
        for n in outs:
            assert torch.equal(outs["current"], outs[n]), f"outputs differ: {n}"
    for n, ts in times.items():
        med = float(np.median(ts))
        print(json.dumps({"config": a.config, "lib": n, "median_ms": round(med, 4), "min_ms": round(min(ts), 4),
                          "frac": round(algo / (med / 1e3) / 8e12, 4)}))


if __name__ == "__main__":
    main()
