#!/usr/bin/env python3
"""A/B kernel variants of the encode/decode path in ONE process, interleaved
rounds (cdna_hip_programming.md rule 24).  Prints a table of median/min kernel
times and the HBM roofline fraction of each variant.

    python tools/tune.py --config encode83 --rounds 5
"""
from __future__ import annotations

import argparse
import json
import time
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

os.environ.setdefault("SHMR_EC_FLAVOUR", "tools")   # kernel knobs: the tools build
import shmr_amd  # noqa: E402

CFG = {
    "encode83": (8, 3, 4 << 20, 0, 512),
    "decode83": (8, 3, 4 << 20, 1, 512),
    "encode104": (10, 4, 16 << 20, 0, 64),
    "decode104": (10, 4, 16 << 20, 2, 64),
    "decode104e4": (10, 4, 16 << 20, 4, 64),   # worst-case rebuild: 4 erasures per block
    "decode104e3": (10, 4, 16 << 20, 3, 64),
    "decode83e3": (8, 3, 4 << 20, 3, 512),
    "encode42": (4, 2, 1 << 20, 0, 1024),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="encode83")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--variants", default="chunks=1;nt_load=1;nt_store=1;nt_load=1,nt_store=1;"
                    "occ8=1,nt_load=1,nt_store=1;chunks=2;"
                    "chunks=2,nt_load=1,nt_store=1;chunks=4,nt_load=1,nt_store=1;grid=0;nt_load=1,nt_store=1,grid=0",
                    help="';'-separated knob sets applied on top of the defaults (prefix-free keys)")
    ap.add_argument("--json", default="")
    ap.add_argument("--pad", type=int, default=0, help="extra bytes per shard pitch (de-alias 2^n strides)")
    ap.add_argument("--align", type=int, default=256, help="shard pitch = S rounded up to this (bench.py: 4096)")
    ap.add_argument("--bpad", type=int, default=0, help="encode: extra bytes per block pitch")
    ap.add_argument("--ppad", type=int, default=None,
                    help="encode: parity shard pitch = S rounded to 256 B plus this (default: --pad, as the data)")
    ap.add_argument("--diag", action="store_true", help="also time the XOR-only ceiling kernel")
    ap.add_argument("--ref", action="store_true", help="also time torch copy / xor references")
    ap.add_argument("--same-pattern", action="store_true", help="decode: every block loses the same shards")
    ap.add_argument("--packed", action="store_true",
                    help="the reference's block buffer: shard i of block b at (b*(k+p) + i) * S, no padding "
                         "(block.rs:408-419; off 16-byte alignment when S % 16 != 0)")
    ap.add_argument("--compact", action="store_true",
                    help="decode: rebuild into a compact [B][erasures][pitch] output (reconstruct_batch_dev_out)")
    ap.add_argument("--ptrs", action="store_true",
                    help="every shard its own torch allocation, named by a pointer table (shmr_ec_*_ptrs_dev; "
                         "bench.py --layout ptrs); decodes rebuild into separate buffers")
    a = ap.parse_args()
    if a.config in CFG:
        k, p, block, er, B = CFG[a.config]
    else:  # "k,p,block_MiB,blocks[,erasures]" (erasures {b, b+3, ...} mod 10, or b mod k for one)
        parts = a.config.split(",")
        kk, pp, mb, bb = parts[:4]
        k, p, block, er, B = int(kk), int(pp), int(mb) << 20, int(parts[4]) if len(parts) > 4 else 0, int(bb)
    S = shmr_amd.calculate_shard_size(block, k)
    dev = torch.device("cuda", 0)
    rs = shmr_amd.ReedSolomon(k, p)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    if a.ptrs:
        import ctypes
        t = k + p
        blocks = [[torch.randint(0, 256, (S,), dtype=torch.uint8, device=dev, generator=g) for _ in range(k)]
                  + [torch.zeros(S, dtype=torch.uint8, device=dev) for _ in range(p)] for _ in range(B)]
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        if er == 0:
            keep, _, _, tab = rs._dev_table(blocks, lambda b, i: True)
            algo = B * (k + p) * S

            def run():
                assert rs._L.shmr_ec_encode_ptrs_dev(rs._h, tab, B, S, 0, stream) == 0
        else:
            rs.encode_ptrs_dev(blocks)
            present = np.ones((B, t), np.uint8)
            rows = np.arange(B)
            if er == 1:
                present[rows, rows % k] = 0
            else:
                for j in range(er):
                    present[rows, (rows + 3 * j) % min(t, 10)] = 0
            table = [[blk[i] if present[b, i] else torch.zeros(S, dtype=torch.uint8, device=dev) for i in range(t)]
                     for b, blk in enumerate(blocks)]
            keep, _, _, tab = rs._dev_table(table, lambda b, i: True)
            algo = B * (k + er) * S
            pp = present.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))

            def run():
                assert rs._L.shmr_ec_reconstruct_ptrs_dev(rs._h, tab, pp, B, S, 0, 0, stream) == 0
    elif er == 0 and a.packed:
        t = k + p
        flat = torch.randint(0, 256, (B * t * S,), dtype=torch.uint8, device=dev, generator=g)
        data = flat.as_strided((B, k, S), (t * S, S, 1))
        parity = flat[k * S:].as_strided((B, p, S), (t * S, S, 1))
        algo = B * (k + p) * S

        def run():
            rs.encode_batch_dev(data, parity, shard_len=S, data_shard_pitch=S, parity_shard_pitch=S)
    elif er == 0:
        P = (S + a.align - 1) // a.align * a.align + a.pad
        if a.bpad:   # extra bytes per block pitch (block stride != k * shard pitch)
            flat = torch.randint(0, 256, (B * (k * P + a.bpad),), dtype=torch.uint8, device=dev, generator=g)
            data = flat.as_strided((B, k, P), (k * P + a.bpad, P, 1))
            parity = torch.empty((B * (p * P + a.bpad),), dtype=torch.uint8, device=dev).as_strided(
                (B, p, P), (p * P + a.bpad, P, 1))
        else:
            data = torch.randint(0, 256, (B, k, P), dtype=torch.uint8, device=dev, generator=g)
            PP = P if a.ppad is None else (S + a.align - 1) // a.align * a.align + a.ppad
            parity = torch.empty((B, p, PP), dtype=torch.uint8, device=dev)
        algo = B * (k + p) * S

        def run():
            rs.encode_batch_dev(data, parity, shard_len=S)
    else:
        pitch = S if a.packed else (S + a.align - 1) // a.align * a.align + a.pad
        shards = torch.zeros((B, k + p, pitch), dtype=torch.uint8, device=dev)
        shards[:, :k, :S] = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device=dev, generator=g)
        # real parity (the bench's content): a zero parity shard among the
        # inputs measurably changes the decode rate
        rs.encode_batch_dev(shards[:, :k], shards[:, k:], shard_len=S, data_shard_pitch=pitch, parity_shard_pitch=pitch)
        present = np.ones((B, k + p), np.uint8)
        rows = np.arange(B)
        b = rows * (0 if a.same_pattern else 1)
        if er == 1:
            present[rows, b % k] = 0
        else:
            n = min(k + p, 10)
            for j in range(er):   # {b, b+3, b+6, b+9} mod n (n = 10, or k+p if smaller): distinct for n >= 3*er - 2
                present[rows, (b + 3 * j) % n] = 0
        algo = B * (k + er) * S
        out = torch.zeros((B, er, pitch), dtype=torch.uint8, device=dev)
        mode = {"compact": a.compact}

        def run():
            # pseudo-knob compact=0/1 in a variant picks the output form per variant
            if mode["compact"]:
                rs.reconstruct_batch_dev_out(shards, present, out, shard_len=S)
            else:
                rs.reconstruct_batch_dev(shards, present, shard_len=S)
    base = {"chunks": 1, "nt_load": 0, "nt_store": 0, "occ8": 0, "grid": -1, "diag": 0, "depth": 3, "wgs_per_cu": 0, "occ": 0, "early": 0, "spre": 0,
            "threads": 256, "fuse_tail": 0, "glds": 0, "serial": 0, "uvec": -2, "sc1_store": 0, "realign": 0, "peel": 0, "wave_run": 0, "st_align": 0, "xcd": 0, "ptrs_segs": 1}
    variants = []
    for spec in a.variants.split(";"):
        kn = dict(base)
        for kv in filter(None, spec.split(",")):
            kk, vv = kv.split("=")
            kn[kk] = int(vv)
        variants.append(tuple(sorted(kn.items())))
    if a.diag:
        variants.append(tuple(sorted(dict(base, diag=1).items())))
        variants.append(tuple(sorted(dict(base, diag=1, nt_load=1, nt_store=1).items())))
    times = {v: [] for v in variants}
    st = torch.cuda.current_stream()
    t_ramp = time.perf_counter()          # untimed clock ramp (see bench.py)
    while time.perf_counter() - t_ramp < 0.5:
        for _ in range(8):
            run()
        torch.cuda.synchronize()
    for rnd in range(a.rounds):
        for v in variants:
            kn = dict(v)
            if "compact" in kn:
                mode["compact"] = bool(kn.pop("compact"))
            shmr_amd.set_tuning(**kn)
            run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.iters):
                run()
            e1.record(st)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / a.iters)
    rows = []
    if a.ref:
        n = 2 << 30
        src = torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev)
        dst = torch.empty_like(src)
        x2 = src.view(torch.int64)
        o2 = dst.view(torch.int64)[: x2.numel() // 2]
        refs = {"copy_2GiB": (lambda: dst.copy_(src), 2 * n),
                "xor_2in_1out_1GiB": (lambda: torch.bitwise_xor(x2[: x2.numel() // 2], x2[x2.numel() // 2:], out=o2), 1.5 * n)}
        for name, (fn, nbytes) in refs.items():
            fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(a.rounds):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(a.iters):
                    fn()
                e1.record(st)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / a.iters)
            med = float(np.median(ts))
            print(json.dumps({"ref": name, "median_ms": round(med, 4), "TBps": round(nbytes / med / 1e9, 3),
                              "frac": round(nbytes / (med / 1e3) / 8e12, 4)}))
        del src, dst
    for v in variants:
        med, mn = float(np.median(times[v])), float(np.min(times[v]))
        rows.append({"knobs": {kk: vv for kk, vv in v if vv != base.get(kk)}, "median_ms": round(med, 4),
                     "min_ms": round(mn, 4), "TBps": round(algo / med / 1e9, 3),
                     "frac": round(algo / (med / 1e3) / 8e12, 4)})
    rows.sort(key=lambda r: r["median_ms"])
    print(f"config={a.config} k={k} p={p} S={S} B={B} algo_bytes={algo}")
    for r in rows:
        print(json.dumps(r))
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"config": a.config, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
