#!/usr/bin/env python3
"""Host<->device transfer probe for the host-memory path (BASELINE config 5).

Measures, on one MI355X, the rates the host-buffer entry points are built
from: pinned H2D / D2H DMA alone and concurrently (two streams), and the GF
kernel reading its inputs / writing its outputs straight from / to pinned host
memory over PCIe (zero-copy: the kernel's own loads and stores cross the bus,
no staging copy).  Prints one JSON line per measurement.

    python tools/pcie_probe.py [--blocks 64]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

os.environ.setdefault("SHMR_EC_FLAVOUR", "tools")   # kernel knobs: the tools build
import shmr_amd  # noqa: E402


def timed(fn, iters=5, streams=None):
    dev = torch.device("cuda", 0)
    fn()
    torch.cuda.synchronize(dev)
    best = 1e9
    for _ in range(iters):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize(dev)
        best = min(best, time.perf_counter() - t0)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=64)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    k, p = 8, 3
    S = shmr_amd.calculate_shard_size(4 << 20, k)
    B = a.blocks
    GB = 1e9
    out = []

    def emit(name, nbytes, secs, **kw):
        rec = {"probe": name, "GB/s": round(nbytes / secs / GB, 2), "bytes": nbytes, "ms": round(secs * 1e3, 3)}
        rec.update(kw)
        out.append(rec)
        print(json.dumps(rec), flush=True)

    h_data = torch.randint(0, 256, (B, k, S), dtype=torch.uint8).pin_memory()
    h_par = torch.zeros((B, p, S), dtype=torch.uint8).pin_memory()
    d_data = torch.empty((B, k, S), dtype=torch.uint8, device=dev)
    d_par = torch.empty((B, p, S), dtype=torch.uint8, device=dev)
    h_big = torch.empty((B, k, S), dtype=torch.uint8).pin_memory()
    s1 = torch.cuda.Stream(dev)
    s2 = torch.cuda.Stream(dev)

    n_in = B * k * S
    n_out = B * p * S
    emit("h2d_pinned", n_in, timed(lambda: d_data.copy_(h_data, non_blocking=True), a.iters))
    emit("d2h_pinned", n_in, timed(lambda: h_big.copy_(d_data, non_blocking=True), a.iters))

    def both():
        with torch.cuda.stream(s1):
            d_data.copy_(h_data, non_blocking=True)
        with torch.cuda.stream(s2):
            h_big.copy_(d_data, non_blocking=True)
    emit("h2d+d2h_concurrent", 2 * n_in, timed(both, a.iters))

    rs = shmr_amd.ReedSolomon(k, p)
    # reference parity (device-resident)
    d_data.copy_(h_data)
    rs.encode_batch_dev(d_data, d_par)
    torch.cuda.synchronize(dev)
    ref = d_par.cpu()

    emit("kernel_dev_to_dev", n_in + n_out, timed(lambda: rs.encode_batch_dev(d_data, d_par), a.iters))
    sweep = [{}, {"depth": 3}, {"depth": 5}, {"depth": 9}, {"chunks": 2}, {"threads": 512},
             {"nt_load": 0}, {"nt_store": 0}, {"grid": 0}, {"depth": 5, "grid": 0}]
    for knobs in sweep:
        for kk, vv in knobs.items():
            shmr_amd.set_tuning(**{kk: vv})
        tag = ",".join(f"{kk}={vv}" for kk, vv in knobs.items()) or "auto"
        h_par.zero_()
        emit("zerocopy_host_to_host", n_in + n_out,
             timed(lambda: rs.encode_batch_dev(h_data, h_par), a.iters), tuning=tag,
             data_GiBps=None, bit_exact=bool(torch.equal(h_par, ref)))
        out[-1]["data_GiBps"] = round(n_in / (out[-1]["ms"] / 1e3) / 2 ** 30, 2)
        if not knobs:
            d_par.zero_()
            emit("zerocopy_host_in_dev_out", n_in + n_out,
                 timed(lambda: rs.encode_batch_dev(h_data, d_par), a.iters), tuning=tag,
                 bit_exact=bool(torch.equal(d_par.cpu(), ref)))
            h_par.zero_()
            emit("zerocopy_dev_in_host_out", n_in + n_out,
                 timed(lambda: rs.encode_batch_dev(d_data, h_par), a.iters), tuning=tag,
                 bit_exact=bool(torch.equal(h_par, ref)))
        for kk in knobs:
            shmr_amd.set_tuning(**{kk: -2 if kk in ("chunks", "nt_load", "nt_store", "depth") else
                                   {"threads": 256, "grid": -1}[kk]})

    # zero-copy reconstruct in place: 1 missing data shard per block (b mod 8)
    import numpy as np
    h_sh = torch.zeros((B, k + p, S), dtype=torch.uint8).pin_memory()
    h_sh[:, :k] = h_data
    h_sh[:, k:] = ref
    present = np.ones((B, k + p), np.uint8)
    present[np.arange(B), np.arange(B) % k] = 0
    for b in range(B):
        h_sh[b, b % k] = 0
    def rec():
        rs.reconstruct_batch_dev(h_sh, present, shard_len=S)
    n_rec = B * (k + 1) * S
    emit("zerocopy_reconstruct_host", n_rec, timed(rec, a.iters),
         data_GiBps=round(B * k * S / timed(rec, a.iters) / 2 ** 30, 2),
         bit_exact=bool(torch.equal(h_sh[:, :k], h_data)))

    # Host-buffer batch entry point on Block-Cache buffers: mapped memory from
    # shmr_ec_host_alloc (zero-copy) vs torch-pinned memory (staged DMA pipeline)
    import ctypes
    import numpy as np
    from shmr_amd._native import _u8p, lib
    cdev = (ctypes.c_int * 1)(0)
    hb = shmr_amd.PinnedBuffer(B * (k + p) * S)
    arr_zc = hb.array.reshape(B, k + p, S)
    t_pin = torch.zeros((B, k + p, S), dtype=torch.uint8).pin_memory()
    arr_st = t_pin.numpy()
    for arr, tag in ((arr_zc, "zero_copy"), (arr_st, "staged_dma")):
        arr[:, :k] = h_data.numpy()
        arr[:, k:] = 0
        blocks = [[arr[b, i] for i in range(k + p)] for b in range(B)]
        _, _, cp = rs._host_ptrs(blocks)     # marshalled once: time the library, not the shim
        z0, s0 = shmr_amd.path_stats()
        secs = timed(lambda: lib().shmr_ec_encode_blocks_host(rs._h, cp, B, S, cdev, 1), a.iters)
        z1, s1_ = shmr_amd.path_stats()
        emit("encode_blocks_host", n_in + n_out, secs, path=tag, data_GiBps=round(n_in / secs / 2 ** 30, 2),
             zero_copy_blocks=z1 - z0, staged_blocks=s1_ - s0,
             bit_exact=bool((arr[:, k:] == ref.numpy()).all()))
        present = np.ones((B, k + p), np.uint8)
        present[np.arange(B), np.arange(B) % k] = 0
        cpres = present.ctypes.data_as(_u8p)
        secs = timed(lambda: lib().shmr_ec_reconstruct_blocks_host(rs._h, cp, cpres, B, S, 0, cdev, 1), a.iters)
        emit("reconstruct_blocks_host", B * (k + 1) * S, secs, path=tag,
             data_GiBps=round(n_in / secs / 2 ** 30, 2),
             bit_exact=bool((arr[:, :k] == h_data.numpy()).all()))
    # Shard-pointer (Block Cache) launches vs the same buffers as a strided
    # device batch, per kernel variant
    tz = torch.from_numpy(arr_zc)
    arr_zc[:, :k] = h_data.numpy()
    blocks = [[arr_zc[b, i] for i in range(k + p)] for b in range(B)]
    # pointer arrays built once (the Python shim's per-call marshalling of
    # B*(k+p) numpy views is not the library's cost)
    _, _, c_ptrs = rs._host_ptrs(blocks)
    c_devs = (ctypes.c_int * 1)(0)

    def encode_ptrs():
        assert lib().shmr_ec_encode_blocks_host(rs._h, c_ptrs, B, S, c_devs, 1) == 0
    for knobs in ({}, {"chunks": 2}, {"grid": 0}, {"chunks": 2, "grid": 0}, {"nt_load": 1}):
        for kk, vv in knobs.items():
            shmr_amd.set_tuning(**{kk: vv})
        tag = ",".join(f"{kk}={vv}" for kk, vv in knobs.items()) or "auto"
        secs_raw = timed(lambda: rs.encode_batch_dev(tz[:, :k], tz[:, k:]), a.iters)
        secs_ptr = timed(encode_ptrs, a.iters)
        emit("zc_strided_vs_ptr", n_in + n_out, secs_ptr, tuning=tag, strided_ms=round(secs_raw * 1e3, 3),
             strided_GBps=round((n_in + n_out) / secs_raw / GB, 2), data_GiBps=round(n_in / secs_ptr / 2 ** 30, 2),
             bit_exact=bool((arr_zc[:, k:] == ref.numpy()).all()))
        for kk in knobs:
            shmr_amd.set_tuning(**{kk: -2 if kk in ("chunks", "nt_load", "nt_store", "depth") else
                                   {"threads": 256, "grid": -1}[kk]})

    # per-block drop-in calls (one block per call, as VirtualBlock::sync_data)
    blocks = [[arr_zc[b, i] for i in range(k + p)] for b in range(B)]
    def per_block():
        for blk in blocks:
            rs.encode(blk)
    secs = timed(per_block, 2)
    emit("encode_per_block_calls", n_in + n_out, secs, path="zero_copy", data_GiBps=round(n_in / secs / 2 ** 30, 2),
         ms_per_block=round(secs / B * 1e3, 3))
    with open(os.path.join(ROOT, "gpurun_out", "pcie_probe.jsonl"), "w") as f:
        for r in out:
            f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
