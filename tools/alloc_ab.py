#!/usr/bin/env python3
"""Where a device Block Cache's memory comes from, and how its blocks are
named, at one layout: interleaved rounds in one process (tools build), RS(8,3)
4 MiB blocks, fraction of 8 TB/s from HIP events.

  sep_*     bench.py's layout: data [B][k][P] and parity [B][p][P], two buffers
  joint_*   one buffer [B][k+p][P] (a pool's block slots)
  *_torch   torch's caching allocator; *_hip hipMalloc (shmr_ec_device_alloc);
            *_contig physically contiguous VRAM (hipDeviceMallocContiguous)
  joint_torch_run / _list   the joint torch buffer named by a pointer table
            (encode_ptrs_dev): its slot lattice as one strided run, or forced
            through the uploaded block list (tools knob slots_list=1)
decode (one lost data shard per block, b mod 8):
  cmp_*     rebuilt into a compact output (reconstruct_batch_dev_out)
  inpl_*    rebuilt in place (reconstruct_batch_dev)
  one_pattern_list   every block the same lost shard, in place, block list

    python tools/alloc_ab.py --op encode --rounds 9
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
from shmr_amd import _native  # noqa: E402
from shmr_amd.reed_solomon import _ptr, _u8p  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", default="encode", choices=["encode", "decode"])
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--blocks", type=int, default=512)
    a = ap.parse_args()
    k, p, B = 8, 3, a.blocks
    t = k + p
    S = 512 * 1024
    P = S + 4096
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(9)
    with _native.tools():
        rs = shmr_amd.ReedSolomon(k, p)
        L = rs._L
        st = torch.cuda.current_stream()
        sp = ctypes.c_void_p(st.cuda_stream)
        keep = []

        def buf(kind, nbytes):
            if kind == "torch":
                x = torch.empty((nbytes,), dtype=torch.uint8, device=dev)
                keep.append(x)
                return x.data_ptr()
            d = shmr_amd.DeviceBuffer(nbytes, device=0, contiguous=(kind == "contig"))
            keep.append(d)
            return int(d._p.value)

        def fill(addr, nbytes):
            v = torch.as_tensor(shmr_amd.reed_solomon._RawView(None, addr, (nbytes,)), device=dev)
            v.copy_(torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=dev, generator=g))

        runs = {}
        present = np.ones((B, t), np.uint8)
        rows = np.arange(B)
        present[rows, rows % k] = 0
        one = np.ones((B, t), np.uint8)
        one[:, 3] = 0
        for kind in ("torch", "hip", "contig"):
            if a.op == "encode":
                d, q = buf(kind, B * k * P), buf(kind, B * p * P)
                fill(d, B * k * P)
                runs[f"sep_{kind}"] = (lambda d=d, q=q: L.shmr_ec_encode_batch_dev(
                    rs._h, ctypes.c_void_p(d), P, k * P, ctypes.c_void_p(q), P, p * P, B, S, 0, sp))
            j = buf(kind, B * t * P)
            fill(j, B * t * P)
            if a.op == "encode":
                runs[f"joint_{kind}"] = (lambda j=j: L.shmr_ec_encode_batch_dev(
                    rs._h, ctypes.c_void_p(j), P, t * P, ctypes.c_void_p(j + k * P), P, t * P, B, S, 0, sp))
                if kind == "torch":
                    tab = np.array([[j + b * t * P + i * P for i in range(t)] for b in range(B)], np.uint64).reshape(-1)
                    keep.append(tab)
                    tp = tab.ctypes.data_as(ctypes.POINTER(_u8p))

                    def run_tab(tp=tp, force=0):
                        shmr_amd.set_tuning(slots_list=force)
                        try:
                            return L.shmr_ec_encode_ptrs_dev(rs._h, tp, B, S, 0, sp)
                        finally:
                            shmr_amd.set_tuning(slots_list=0)
                    runs["joint_torch_run"] = (lambda f=run_tab: f(force=0))
                    runs["joint_torch_list"] = (lambda f=run_tab: f(force=1))
            else:
                assert L.shmr_ec_encode_batch_dev(rs._h, ctypes.c_void_p(j), P, t * P, ctypes.c_void_p(j + k * P), P,
                                                  t * P, B, S, 0, sp) == 0
                o = buf(kind, B * P)
                runs[f"cmp_{kind}"] = (lambda j=j, o=o: L.shmr_ec_reconstruct_batch_dev_out(
                    rs._h, ctypes.c_void_p(j), P, t * P, _ptr(present), B, S, 0, ctypes.c_void_p(o), P, P, 0, sp))
                runs[f"inpl_{kind}"] = (lambda j=j: L.shmr_ec_reconstruct_batch_dev(
                    rs._h, ctypes.c_void_p(j), P, t * P, _ptr(present), B, S, 0, 0, sp))
                if kind == "torch":
                    tab = np.array([[j + b * t * P + i * P for i in range(t)] for b in range(B)], np.uint64).reshape(-1)
                    keep.append(tab)
                    tp = tab.ctypes.data_as(ctypes.POINTER(_u8p))

                    def one_list(tp=tp, force=1):
                        shmr_amd.set_tuning(slots_list=force)
                        try:
                            return L.shmr_ec_reconstruct_ptrs_dev(rs._h, tp, _ptr(one), B, S, 0, 0, sp)
                        finally:
                            shmr_amd.set_tuning(slots_list=0)
                    runs["one_pattern_run"] = (lambda f=one_list: f(force=0))
                    runs["one_pattern_list"] = (lambda f=one_list: f(force=1))
        algo = B * ((k + p) if a.op == "encode" else (k + 1)) * S
        for f in runs.values():
            assert f() in (None, 0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.5:
            for f in runs.values():
                f()
            torch.cuda.synchronize()
        times = {n: [] for n in runs}
        for _ in range(a.rounds):
            for n, f in runs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(a.iters):
                    assert f() in (None, 0)
                e1.record(st)
                torch.cuda.synchronize()
                times[n].append(e0.elapsed_time(e1) / a.iters)
        for n, ts in times.items():
            med = float(np.median(ts))
            print(json.dumps({"op": a.op, "leg": n, "median_ms": round(med, 4), "min_ms": round(min(ts), 4),
                              "frac": round(algo / (med / 1e3) / 8e12, 4)}))
        sys.stdout.flush()


if __name__ == "__main__":
    main()
