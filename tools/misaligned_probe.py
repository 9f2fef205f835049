#!/usr/bin/env python3
"""Misaligned-shard probe: RS(10,4) 16 MiB blocks (S = 1,677,722, so shard i of
the reference's contiguous block buffer starts at i*S, not 16-byte aligned)
encoded (a) device-resident with shard pitch S vs a 4 KiB-aligned pitch and
(b) from mapped host Block-Cache buffers (zero-copy) laid out contiguously vs
with 4 KiB-aligned shard slots.  Prints GiB/s of data per layout and checks the
parity of every layout against the aligned device result.

    python tools/misaligned_probe.py --blocks 32
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import shmr_amd  # noqa: E402

K, P = 10, 4
BLOCK = 16 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=32)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    B = a.blocks
    S = shmr_amd.calculate_shard_size(BLOCK, K)
    A = (S + 4095) // 4096 * 4096
    dev = torch.device("cuda", 0)
    rs = shmr_amd.ReedSolomon(K, P)
    rng = np.random.default_rng(7)
    host = rng.integers(0, 256, (B, K, S), dtype=np.uint8)
    out = []

    def rate(sec):
        return B * K * S / sec / 2 ** 30

    # (a) device-resident, pitch S (the reference's contiguous buffer) vs aligned slots
    ref_par = None
    for name, pitch in (("device_aligned_4KiB", A), ("device_contiguous_pitchS", S)):
        d = torch.zeros((B, K * pitch), dtype=torch.uint8, device=dev)
        dv = d.view(B, K * pitch)
        for i in range(K):
            dv[:, i * pitch:i * pitch + S] = torch.from_numpy(host[:, i]).to(dev)
        par = torch.zeros((B, P * pitch), dtype=torch.uint8, device=dev)
        data3 = d.as_strided((B, K, S), (K * pitch, pitch, 1))
        par3 = par.as_strided((B, P, S), (P * pitch, pitch, 1))

        def run():
            rs.encode_batch_dev(data3, par3, shard_len=S, data_shard_pitch=pitch, parity_shard_pitch=pitch)
        run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            run()
        torch.cuda.synchronize()
        sec = (time.perf_counter() - t0) / a.reps
        got = np.stack([par3[:, r, :].cpu().numpy() for r in range(P)], axis=1)
        if ref_par is None:
            ref_par = got
        out.append({"layout": name, "pitch": pitch, "GiBps": round(rate(sec), 2), "ms": round(sec * 1e3, 3),
                    "frac_of_8TBps": round(B * (K + P) * S / sec / 8e12, 4),
                    "parity_equal": bool(np.array_equal(got, ref_par))})
        del d, par
    # (b) mapped host Block-Cache buffers (zero-copy), contiguous vs aligned slots
    for name, pitch in (("mapped_aligned_4KiB", A), ("mapped_contiguous_pitchS", S)):
        bufs, blocks = [], []
        for b in range(B):
            buf = shmr_amd.PinnedBuffer((K + P) * pitch)
            bufs.append(buf)
            arr = buf.array
            for i in range(K):
                arr[i * pitch:i * pitch + S] = host[b, i]
            blocks.append([arr[i * pitch:i * pitch + S] for i in range(K + P)])
        rs.encode_blocks_host(blocks)
        t0 = time.perf_counter()
        for _ in range(a.reps):
            rs.encode_blocks_host(blocks)
        sec = (time.perf_counter() - t0) / a.reps
        got = np.stack([np.stack([blocks[b][K + r] for r in range(P)]) for b in range(B)])
        out.append({"layout": name, "pitch": pitch, "GiBps": round(rate(sec), 2), "ms": round(sec * 1e3, 3),
                    "parity_equal": bool(np.array_equal(got, ref_par))})
        del blocks, bufs
    for o in out:
        print(json.dumps(o), flush=True)


if __name__ == "__main__":
    main()
