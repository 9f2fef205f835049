#!/usr/bin/env python3
"""Does the private-stream wait behind a mirrored readiness event (ec_core.hpp
record_mirrored) hold back another stream?  Stream A runs multi-pattern
rebuilds that take the upload-ring table launch (each call releases a ring slot
on A: one private-stream wait in a mirroring build); stream B runs short
encodes.  For each library build -- loaded side by side in one process,
interleaved rounds -- reports B's span alone and next to A's, and A's span.

    python tools/hol_probe.py tools/_hol/libshmr_ec_nomirror.so [--rounds 7]
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

from shmr_amd import _native  # noqa: E402


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
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    libs = {"current": load(_native.LIB_PATH)}
    for o in a.others:
        libs[os.path.basename(o)] = load(os.path.abspath(o))
    k, p = 8, 3
    t = k + p
    S = 1 << 19
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    BA, BB = 256, 8
    shards = torch.randint(0, 256, (BA, t, S), dtype=torch.uint8, device=dev, generator=g)
    present = np.ones((BA, t), np.uint8)
    present[np.arange(BA), np.arange(BA) % 2] = 0      # 256 one-block runs: the ring table launch
    pr = present.ctypes.data_as(_native._u8p)
    data = torch.randint(0, 256, (BB, k, S), dtype=torch.uint8, device=dev, generator=g)
    par = torch.empty((BB, p, S), dtype=torch.uint8, device=dev)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    pa, pb = ctypes.c_void_p(sa.cuda_stream), ctypes.c_void_p(sb.cuda_stream)
    hs = {}
    for n, L in libs.items():
        h = ctypes.c_void_p()
        assert L.shmr_ec_new(k, p, ctypes.byref(h)) == 0
        hs[n] = h

    def enc(L, h):
        assert L.shmr_ec_encode_batch_dev(h, ctypes.c_void_p(data.data_ptr()), S, k * S,
                                          ctypes.c_void_p(par.data_ptr()), S, p * S, BB, S, 0, pb) == 0

    def rec(L, h):
        assert L.shmr_ec_reconstruct_batch_dev(h, ctypes.c_void_p(shards.data_ptr()), S, t * S, pr, BA, S,
                                               0, 0, pa) == 0

    for n, L in libs.items():   # warm: plans, rings
        enc(L, hs[n])
        rec(L, hs[n])
    torch.cuda.synchronize()
    res = {n: {"b_alone": [], "b_mixed": [], "a_mixed": []} for n in libs}
    for _ in range(a.rounds):
        for n, L in libs.items():
            h = hs[n]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(sb)
            for _ in range(100):
                enc(L, h)
            e1.record(sb)
            torch.cuda.synchronize()
            res[n]["b_alone"].append(e0.elapsed_time(e1))
            ea0, ea1, eb0, eb1 = (torch.cuda.Event(enable_timing=True) for _ in range(4))
            ea0.record(sa)
            eb0.record(sb)
            for i in range(100):
                if i % 5 == 0:
                    rec(L, h)
                enc(L, h)
            ea1.record(sa)
            eb1.record(sb)
            torch.cuda.synchronize()
            res[n]["b_mixed"].append(eb0.elapsed_time(eb1))
            res[n]["a_mixed"].append(ea0.elapsed_time(ea1))
    for n, r in res.items():
        print(json.dumps({"lib": n, **{k_: round(float(np.median(v)), 3) for k_, v in r.items()}}), flush=True)


if __name__ == "__main__":
    main()
