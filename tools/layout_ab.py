#!/usr/bin/env python3
"""Encode-layout A/B on one GPU, interleaved rounds in one process: the same
RS(k,p) batch encoded (a) with data and parity in separate allocations
([B,k,S] + [B,p,S], bench.py's layout) and (b) in the reference's in-place
block buffer layout ([B, k+p, S]: parity shards right after the block's data
shards, block.rs:408-423), plus (c) a padded shard pitch.

    python tools/layout_ab.py [--k 8 --p 3 --block-mib 4 --blocks 512]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

os.environ.setdefault("SHMR_EC_FLAVOUR", "tools")   # kernel knobs: the tools build
import shmr_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--p", type=int, default=3)
    ap.add_argument("--block-mib", type=int, default=4)
    ap.add_argument("--blocks", type=int, default=512)
    ap.add_argument("--rounds", type=int, default=11)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--decode", type=int, default=0, help="erasures per block: time reconstruct instead")
    a = ap.parse_args()
    k, p, B = a.k, a.p, a.blocks
    S = shmr_amd.calculate_shard_size(a.block_mib << 20, k)
    P = (S + 255) // 256 * 256
    dev = torch.device("cuda", 0)
    rs = shmr_amd.ReedSolomon(k, p)
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    sep_d = torch.randint(0, 256, (B, k, P), dtype=torch.uint8, device=dev, generator=g)
    sep_p = torch.empty((B, p, P), dtype=torch.uint8, device=dev)
    blk = torch.empty((B, k + p, P), dtype=torch.uint8, device=dev)
    blk[:, :k] = sep_d
    Q = P + 4096 + 256   # padded pitch: breaks the power-of-two shard stride
    pad = torch.empty((B, k + p, Q), dtype=torch.uint8, device=dev)
    pad[:, :k, :P] = sep_d
    if a.decode:
        present = np.ones((B, k + p), np.uint8)
        b = np.arange(B)
        for e in range(a.decode):
            present[b, (b + 3 * e) % k] = 0
        rs.encode_batch_dev(blk[:, :k], blk[:, k:], shard_len=S)
        rs.encode_batch_dev(pad[:, :k], pad[:, k:], shard_len=S)
        runs = {f"decode_pitch_{P}": lambda: rs.reconstruct_batch_dev(blk, present, shard_len=S),
                f"decode_pitch_{Q}": lambda: rs.reconstruct_batch_dev(pad, present, shard_len=S)}
        for d in (4096, 8192 + 256, 65536 + 256):
            t = torch.empty((B, k + p, P + d), dtype=torch.uint8, device=dev)
            t[:, :, :P] = blk
            runs[f"decode_pitch_{P + d}"] = (lambda t=t: rs.reconstruct_batch_dev(t, present, shard_len=S))
    else:
        runs = {}
    runs.update({} if a.decode else {
        "separate": lambda: rs.encode_batch_dev(sep_d, sep_p, shard_len=S),
        "block_buffer": lambda: rs.encode_batch_dev(blk[:, :k], blk[:, k:], shard_len=S),
        "block_buffer_padded": lambda: rs.encode_batch_dev(pad[:, :k], pad[:, k:], shard_len=S),
    })
    st = torch.cuda.current_stream()
    for r in runs.values():
        for _ in range(50):
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
    if not a.decode:
        assert torch.equal(blk[:, k:, :S], sep_p[:, :, :S]) and torch.equal(pad[:, k:, :S], sep_p[:, :, :S])
    algo = B * ((k + a.decode) if a.decode else (k + p)) * S
    for n, ts in times.items():
        med = float(np.median(ts))
        print(json.dumps({"layout": n, "k": k, "p": p, "S": S, "median_ms": round(med, 4),
                          "frac": round(algo / (med / 1e3) / 8e12, 4)}))


if __name__ == "__main__":
    main()
