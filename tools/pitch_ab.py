#!/usr/bin/env python3
"""Shard-pitch A/B of the device-batch encode, interleaved rounds in one
process: the same RS(k,p) batch (bench.py's separate data / parity layout)
with the shard pitch rounded to 256 B (bench.py), to 4 KiB and 8 KiB, and
with a tile-multiple shard length (no partial tail tile), to separate the
cost of the unaligned RS(10,4) shard length S = 1,677,722 from the layout.

    python tools/pitch_ab.py [--k 10 --p 4 --block-mib 16 --blocks 64]
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
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--p", type=int, default=4)
    ap.add_argument("--block-mib", type=int, default=16)
    ap.add_argument("--blocks", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=11)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    k, p, B = a.k, a.p, a.blocks
    S = shmr_amd.calculate_shard_size(a.block_mib << 20, k)
    dev = torch.device("cuda", 0)
    rs = shmr_amd.ReedSolomon(k, p)
    g = torch.Generator(device=dev)
    g.manual_seed(7)

    def rup(x, m):
        return (x + m - 1) // m * m

    cases = {}
    for name, pitch, slen in (("pitch256", rup(S, 256), S),
                              ("pitch4k", rup(S, 4096), S),
                              ("pitch8k", rup(S, 8192), S),
                              ("pitch64k+256", rup(S, 65536) + 256, S),
                              ("tilemult_S", rup(S, 8192), rup(S, 8192)),
                              ("tilemult_S_down", rup(S, 8192), S // 8192 * 8192)):
        d = torch.randint(0, 256, (B, k, pitch), dtype=torch.uint8, device=dev, generator=g)
        par = torch.empty((B, p, pitch), dtype=torch.uint8, device=dev)
        cases[name] = (d, par, slen)
    runs = {n: (lambda c=c: rs.encode_batch_dev(c[0], c[1], shard_len=c[2])) for n, c in cases.items()}
    st = torch.cuda.current_stream()
    for r in runs.values():
        for _ in range(100):
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
    for n, ts in times.items():
        slen = cases[n][2]
        med = float(np.median(ts))
        algo = B * (k + p) * slen
        print(json.dumps({"case": n, "k": k, "p": p, "blocks": B, "pitch": cases[n][0].shape[2],
                          "shard_len": slen, "median_ms": round(med, 4),
                          "frac": round(algo / (med / 1e3) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
