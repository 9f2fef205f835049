#!/usr/bin/env python3
"""Where the packed-layout loss sits: the RS(k,p) device encode with the data
shards and the parity shards each either in the reference's packed block
buffer (shard i of block b at (b*(k+p) + i) * S, off 16-byte alignment when
S % 16 != 0; block.rs:408-419) or in 4 KiB-aligned slots, interleaved rounds
in one process, the product policy against the DPP-realigned loads (tools
knobs uvec=1, realign=1) and the realigned aligned stores (st_align=1, with
and without the early prologue).

    python tools/misalign_split.py [--k 10 --p 4 --block-mib 16 --blocks 64]
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

_AUTO = dict(uvec=-2, realign=-2, wave_run=-2, early=-2, serial=-2, st_align=-2)
VARIANTS = {"policy": _AUTO, "realign": dict(_AUTO, uvec=1, realign=1), "st_align": dict(_AUTO, st_align=1),
            "st_align_plain": dict(_AUTO, st_align=1, early=0, serial=0)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--p", type=int, default=4)
    ap.add_argument("--block-mib", type=int, default=16)
    ap.add_argument("--blocks", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    k, p, B = a.k, a.p, a.blocks
    t = k + p
    S = shmr_amd.calculate_shard_size(a.block_mib << 20, k)
    P = (S + 4095) // 4096 * 4096
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    flat = torch.randint(0, 256, (B * t * S,), dtype=torch.uint8, device=dev, generator=g)
    packed_data = flat.as_strided((B, k, S), (t * S, S, 1))
    packed_par = flat[k * S:].as_strided((B, p, S), (t * S, S, 1))
    slot_data = torch.randint(0, 256, (B, k, P), dtype=torch.uint8, device=dev, generator=g)
    slot_par = torch.empty((B, p, P), dtype=torch.uint8, device=dev)
    layouts = {"aligned": (slot_data, slot_par), "in_packed": (packed_data, slot_par),
               "out_packed": (slot_data, packed_par), "packed": (packed_data, packed_par)}
    rs = shmr_amd.ReedSolomon(k, p)
    algo = B * t * S

    def run(name):
        d, q = layouts[name]
        rs.encode_batch_dev(d, q, shard_len=S, data_shard_pitch=d.stride(1), parity_shard_pitch=q.stride(1))

    # parity check of every (layout, variant) against the aligned policy result
    ref = None
    for name in layouts:
        for vn, kn in VARIANTS.items():
            shmr_amd.set_tuning(**kn)
            d, q = layouts[name]
            if name in ("in_packed", "packed"):
                d.copy_(slot_data[:, :, :S])
            run(name)
            torch.cuda.synchronize()
            got = q[:, :, :S].cpu().numpy()
            if ref is None:
                ref = got
            assert np.array_equal(ref, got), (name, vn)
    st = torch.cuda.current_stream()
    times = {(ln, vn): [] for ln in layouts for vn in VARIANTS}
    for _ in range(3):
        for key in times:
            shmr_amd.set_tuning(**VARIANTS[key[1]])
            run(key[0])
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for key in times:
            shmr_amd.set_tuning(**VARIANTS[key[1]])
            run(key[0])
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.iters):
                run(key[0])
            e1.record(st)
            torch.cuda.synchronize()
            times[key].append(e0.elapsed_time(e1) / a.iters)
    shmr_amd.set_tuning(**VARIANTS["policy"])
    print(f"k={k} p={p} S={S} B={B} algo_bytes={algo}")
    for key, ts in sorted(times.items(), key=lambda kv: np.median(kv[1])):
        med = float(np.median(ts))
        print(json.dumps({"layout": key[0], "variant": key[1], "median_ms": round(med, 4),
                          "frac": round(algo / (med / 1e3) / 8e12, 4)}))


if __name__ == "__main__":
    main()
