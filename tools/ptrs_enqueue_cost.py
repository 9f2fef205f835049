#!/usr/bin/env python3
"""Host time of one pointer-table call (`shmr_ec_encode_ptrs_dev`, the call the
submission queue makes per merged batch) against the number of blocks in it:
blocks of one slab (a slot lattice) in slot order (one arithmetic run), in
shuffled order (the queue's arrival order), with every 4th block missing
(holes), and the same shuffled table forced through the table kernels
(ptrs_grid=0).  RS(8,3), 512 KiB shards.  Enqueue time only (the GPU runs
behind); each point is the median of 30 calls after 5 warm calls.

    python tools/ptrs_enqueue_cost.py   (one JSON line per point)
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
import torch  # noqa: E402

import shmr_amd  # noqa: E402
from shmr_amd.reed_solomon import _u8p  # noqa: E402


def main():
    k, p, S = 8, 3, 512 * 1024
    t = k + p
    nmax = 1024
    rs = shmr_amd.ReedSolomon(k, p)
    slab = shmr_amd.ShardSlab(nmax, t, S)
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rng = np.random.default_rng(3)
    tabs = slab.ptrs.reshape(nmax, t)
    for n in (1, 4, 16, 64, 256, 1024):
        legs = {
            "run": tabs[:n],
            "shuffled": tabs[rng.permutation(n)],
            "holed": tabs[[b for b in range(min(nmax, n * 4 // 3 + 1)) if b % 4 != 3][:n]],
            "table": tabs[rng.permutation(n)],
        }
        for leg, tab in legs.items():
            tab = np.ascontiguousarray(tab, dtype=np.uint64)
            tp = tab.ctypes.data_as(ctypes.POINTER(_u8p))
            B = tab.shape[0]
            shmr_amd.set_tuning(ptrs_grid=0 if leg == "table" else -2)
            try:
                g0 = shmr_amd.device_stats(0)["ptr_table_grids"]
                ts = []
                for i in range(35):
                    a = time.perf_counter()
                    rc = rs._L.shmr_ec_encode_ptrs_dev(rs._h, tp, B, S, 0, sp)
                    b = time.perf_counter()
                    assert rc == 0
                    if i >= 5:
                        ts.append((b - a) * 1e6)
                    if i % 5 == 4:
                        torch.cuda.synchronize()
                grids = shmr_amd.device_stats(0)["ptr_table_grids"] - g0
            finally:
                shmr_amd.set_tuning(ptrs_grid=-2)
            torch.cuda.synchronize()
            med = float(np.median(ts))
            print(json.dumps({"blocks": B, "leg": leg, "enqueue_us_median": round(med, 1),
                              "us_per_block": round(med / B, 3), "min_us": round(min(ts), 1),
                              "lattice_calls": grids}), flush=True)


if __name__ == "__main__":
    main()
