#!/usr/bin/env python3
"""A caller stream held up by something outside the library (ADVICE r04 #3,
VERDICT r05 #5): does another thread's work on another stream wait for it?

Stream A is held by hipStreamWaitValue32 on a word in mapped host memory,
with library work queued behind the wait that takes a new erasure plan (its
first upload is on A) and upload-ring slots.  Meanwhile thread B, on stream B,
runs: a plain torch kernel (the runtime baseline: B's hardware queue may be
shared with A's), device-resident calls that need the same plan, pointer-table
calls that cycle every ring slot, the per-block queue call, and host-buffer
calls (mapped, and pageable through the staging pipe) larger than the ones made
before the hold, so their scratch buffers grow during it (r06 s40: a growth
that freed the old buffer -- hipFree waits for every stream of the device --
was held back by A).  The word is released after --hold seconds.  Each of B's steps reports
when it completed, relative to the hold; a step that completes only after the
release was held back by A.

    python tools/hol_held.py [--hold 1.0]   (prints one JSON line)
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import shmr_amd  # noqa: E402
from shmr_amd.reed_solomon import _ptr, _u8p  # noqa: E402

HIP = ctypes.CDLL("libamdhip64.so")
HIP.hipStreamWaitValue32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint, ctypes.c_uint32]
HIP.hipStreamWaitValue32.restype = ctypes.c_int
HIP_WAIT_GTE = 0   # hipStreamWaitValueGte


def run(hold: float = 1.0) -> dict:
    dev = torch.device("cuda", 0)
    k, p, S, B = 8, 3, 1 << 16, 64
    t = k + p
    rs = shmr_amd.ReedSolomon(k, p)
    shmr_amd.device_init(0)
    g = torch.Generator(device=dev).manual_seed(11)
    word_buf = shmr_amd.PinnedBuffer(4096)
    word = word_buf.array[:4].view(np.uint32)
    word[0] = 0
    waddr = word_buf.array.ctypes.data
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    pa, pb = ctypes.c_void_p(sa.cuda_stream), ctypes.c_void_p(sb.cuda_stream)
    slab = torch.randint(0, 256, (2, B, t, S), dtype=torch.uint8, device=dev, generator=g)
    torch.cuda.synchronize()
    # small host-buffer calls before the hold: the library's scratch for them
    # exists and must grow for the larger calls made during it
    small = shmr_amd.PinnedBuffer(t * 4096)
    rs.encode([small.array.reshape(t, 4096)[i] for i in range(t)])
    rs.encode([np.zeros(4096, np.uint8) for _ in range(t)])
    # pattern never used before: its plan's first upload goes on A
    present = np.ones((B, t), np.uint8)
    present[:, [1, 9]] = 0
    # A: held, then a pointer-table rebuild (one table row per block: shuffled
    # so the table path uploads it through the ring) with the new pattern
    order = np.random.default_rng(1).permutation(B)
    tabA = np.array([[slab[0, b, i].data_ptr() for i in range(t)] for b in order], np.uint64).reshape(-1)
    rcA = HIP.hipStreamWaitValue32(pa, ctypes.c_void_p(waddr), 1, HIP_WAIT_GTE, 0xFFFFFFFF)
    if rcA != 0:
        return {"error": f"hipStreamWaitValue32 -> {rcA}"}
    shmr_amd.set_tuning(ptrs_grid=0)   # the table path: ring slots on A
    try:
        assert rs._L.shmr_ec_reconstruct_ptrs_dev(rs._h, tabA.ctypes.data_as(ctypes.POINTER(_u8p)), _ptr(present), B,
                                                  S, 0, 0, pa) == 0
    finally:
        shmr_amd.set_tuning(ptrs_grid=-2)
    t0 = time.perf_counter()
    steps = {}

    def mark(name):
        steps[name] = round(time.perf_counter() - t0, 4)

    def side():
        try:
            x = torch.ones(1 << 20, device=dev)
            with torch.cuda.stream(sb):
                y = x * 2                                          # plain runtime work on B
            sb.synchronize()
            mark("torch_kernel_on_B")
            pr = _ptr(present)
            base = slab[1].data_ptr()
            assert rs._L.shmr_ec_reconstruct_batch_dev(rs._h, ctypes.c_void_p(base), S, t * S, pr, B, S, 0, 0, pb) == 0
            sb.synchronize()
            mark("batch_rebuild_same_plan_on_B")
            tabB = np.array([[slab[1, b, i].data_ptr() for i in range(t)] for b in order], np.uint64).reshape(-1)
            shmr_amd.set_tuning(ptrs_grid=0)
            try:
                for _ in range(40):                                 # > 32 ring slots
                    assert rs._L.shmr_ec_reconstruct_ptrs_dev(rs._h, tabB.ctypes.data_as(ctypes.POINTER(_u8p)),
                                                              pr, B, S, 0, 0, pb) == 0
            finally:
                shmr_amd.set_tuning(ptrs_grid=-2)
            mark("ptrs_calls_enqueued_on_B")
            sb.synchronize()
            mark("ptrs_calls_done_on_B")
            blk = [slab[1, 0, i] for i in range(t)]
            rs.encode_dev(blk)
            mark("queue_encode_dev")
            host = shmr_amd.PinnedBuffer(t * S)
            h = host.array.reshape(t, S)
            rs.encode([h[i] for i in range(t)])
            mark("host_mapped_encode")
            SP = 4 << 20
            rs.encode([np.full(SP, i, np.uint8) if i < k else np.zeros(SP, np.uint8) for i in range(t)])
            mark("host_pageable_encode")
            del y
        except Exception as e:  # noqa: BLE001
            steps["error"] = repr(e)

    th = threading.Thread(target=side)
    th.start()
    th.join(timeout=hold)
    word[0] = 1                                                    # release A
    released = round(time.perf_counter() - t0, 4)
    th.join(timeout=30)
    sa.synchronize()
    a_done = round(time.perf_counter() - t0, 4)
    held_back = sorted(n for n, v in steps.items() if isinstance(v, float) and v >= released)
    return {"hold_s": hold, "released_at_s": released, "a_done_s": a_done, "b_steps_s": steps,
            "b_steps_held_back": held_back, "b_finished": not th.is_alive()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hold", type=float, default=1.0)
    a = ap.parse_args()
    print(json.dumps(run(a.hold)), flush=True)


if __name__ == "__main__":
    main()
