#!/usr/bin/env python3
"""Table kernels with two neighbouring tiles per workgroup (tools knob `pair`)
against the policy's one tile per workgroup, interleaved rounds in one process
(tools build).  The table kernels' cost against the strided kernels is a
scalar-cache miss on each workgroup's block row of the pointer table
(DESIGN.md section 6): with a tile pair the second tile of a block finds the
row in the cache its first tile filled, and the grid has half the prologues.

Legs per config, over one torch allocation per shard (the table kernels):
  torch         the product policy (one tile per workgroup)
  torch_pair    knob pair=1
  slab          the same blocks in a library slab (the strided kernels: the
                ceiling the table kernels are measured against)
Each pair leg's outputs are compared byte for byte with the policy leg's.

    SHMR_EC_FLAVOUR=tools python tools/pair_ab.py --config encode83 --rounds 11
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="encode83", choices=sorted(CFG))
    ap.add_argument("--rounds", type=int, default=11)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    L = shmr_amd.reed_solomon.lib()
    assert L.shmr_ec_is_tools_build() == 1, "run with SHMR_EC_FLAVOUR=tools"
    k, p, block, er, B = CFG[a.config]
    t = k + p
    S = shmr_amd.calculate_shard_size(block, k)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(7)
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
    keep = []

    def table(addrs):
        arr = np.ascontiguousarray(np.asarray(addrs, dtype=np.uint64).reshape(-1))
        keep.append(arr)
        return arr.ctypes.data_as(ctypes.POINTER(_u8p))

    def call(tab, knobs=None):
        def f():
            if knobs:
                shmr_amd.set_tuning(**knobs)
            try:
                if er == 0:
                    return rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab, B, S, 0, sp)
                return rs._L.shmr_ec_reconstruct_ptrs_dev(rs._h, tab, pr, B, S, 0, 0, sp)
            finally:
                if knobs:
                    shmr_amd.set_tuning(**{kk: -2 for kk in knobs})
        return f

    # one torch allocation per shard; rebuilt shards into buffers of their own
    tb = [[torch.randint(0, 256, (S,), dtype=torch.uint8, device=dev, generator=g) for _ in range(t)]
          for _ in range(B)]
    tt = np.array([[s.data_ptr() for s in blk] for blk in tb], dtype=np.uint64)
    assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, table(tt), B, S, 0, sp) == 0
    outs = []
    if er:
        tout = [[torch.zeros(S, dtype=torch.uint8, device=dev) for _ in range(er)] for _ in range(B)]
        tt = tt.copy()
        for b in range(B):
            for j, i in enumerate(np.flatnonzero(present[b] == 0)):
                tt[b, i] = tout[b][j].data_ptr()
        outs = [s for blk in tout for s in blk]
        keep.append(tout)
    else:
        outs = [s for blk in tb for s in blk[k:]]
    t_tab = table(tt)
    runs = {"torch": call(t_tab), "torch_pair": call(t_tab, {"pair": 1})}

    # the same blocks in a slab (strided kernels)
    slab = shmr_amd.ShardSlab(B, t, S)
    sv = slab.tensor()
    sv[:, :k, :S] = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device=dev, generator=g)
    s_tab = table(slab.ptrs)
    assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, s_tab, B, S, 0, sp) == 0
    runs["slab"] = call(s_tab)
    keep.append(slab)

    # parity of the pair leg against the policy leg
    assert runs["torch"]() == 0
    torch.cuda.synchronize()
    want = [o.clone() for o in outs]
    for o in outs:
        o.fill_(0x5A)
    assert runs["torch_pair"]() == 0
    torch.cuda.synchronize()
    equal = all(torch.equal(x, y) for x, y in zip(want, outs))
    variants = {}
    for n, f in runs.items():
        s0 = shmr_amd.kernel_inventory()
        f()
        torch.cuda.synchronize()
        s1 = shmr_amd.kernel_inventory()
        before = {(e["rows"], e["chunks"], e["mode"], e["flags"]): e["launches"] for e in s0}
        variants[n] = sorted({f"<{e['rows']},{e['chunks']},{e['mode']},{e['flags']}>" for e in s1
                              if e["launches"] > before.get((e["rows"], e["chunks"], e["mode"], e["flags"]), 0)})

    algo = B * (k + (er or p)) * S
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
                assert f() == 0
            e1.record(st)
            torch.cuda.synchronize()
            times[n].append(e0.elapsed_time(e1) / a.iters)
    for n, ts in times.items():
        med = float(np.median(ts))
        print(json.dumps({"config": a.config, "layout": n, "median_ms": round(med, 4), "min_ms": round(min(ts), 4),
                          "frac": round(algo / (med / 1e3) / 8e12, 4), "kernels": variants[n],
                          "build_id": L.shmr_ec_build_id().decode()}))
    print(json.dumps({"config": a.config, "pair_equals_policy": equal}))
    if not equal:
        sys.exit(1)


if __name__ == "__main__":
    main()
