#!/usr/bin/env python3
"""CU-mask probe: does the encode run faster on fewer CUs?

The HBM-bound kernels keep ~1,000-1,500 short workgroups in flight; the
occupancy caps of DESIGN.md §6 lowered that count per CU (and lost on the
encodes).  This probe lowers it per chip instead: the same product kernel is
enqueued on streams created with hipExtStreamCreateWithCUMask over all 256
CUs, over whole XCDs only, over fewer CUs on every XCD, and (for contrast) over
CUs picked evenly from the mask's bit order, interleaved in one process
(rounds x iters launches per stream).

    python tools/cumask_ab.py --config encode83 --rounds 9
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

CFG = {"encode83": (8, 3, 4 << 20, 512, 4096), "encode104": (10, 4, 16 << 20, 64, 0),
       "encode42": (4, 2, 1 << 20, 1024, 4096)}


def mask_bits(ncu: int, spec: str):
    """CU indices (mask bit numbers) kept by `spec`.  Measured on MI355X: mask
    bit i belongs to XCD i % 8 (a mask that halves one XCD's CUs halves the
    whole launch's rate: its round-robin share of workgroups straggles).
      default  torch's current stream, no CU mask (control)
      all      every CU
      xN       XCDs 0 .. N-1 whole (N * 32 CUs)
      cN       N CUs on every XCD (bits i with i // 8 < N within each group of 32 per XCD)
      evenN    N CUs spread evenly over the bit order (not XCD-aware)"""
    if spec in ("all", "default"):
        return list(range(ncu))
    if spec.startswith("x"):
        n = int(spec[1:])
        return [i for i in range(ncu) if i % 8 < n]
    if spec.startswith("c"):
        n = int(spec[1:])
        return [i for i in range(ncu) if i // 8 < n]
    if spec.startswith("even"):
        n = int(spec[4:])
        return sorted({(i * ncu) // n for i in range(n)})
    raise ValueError(spec)


def masked_stream(hip, ncu_total: int, keep):
    words = (ncu_total + 31) // 32
    mask = [0] * words
    for cu in keep:
        mask[cu // 32] |= 1 << (cu % 32)
    arr = (ctypes.c_uint32 * words)(*mask)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), arr)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask: {rc}")
    return torch.cuda.ExternalStream(s.value)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="encode83", choices=sorted(CFG))
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--keep", default="default,all,x7,x6,x4,c28,c24,c16,even240")
    a = ap.parse_args()
    k, p, block, B, pad = CFG[a.config]
    S = shmr_amd.calculate_shard_size(block, k)
    P = (S + 4095) // 4096 * 4096
    P += pad if P % 65536 == 0 else 0        # the bench's shard slot (bench.py --pitch-pad auto)
    dev = torch.device("cuda", 0)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    hip = ctypes.CDLL("libamdhip64.so")
    rs = shmr_amd.ReedSolomon(k, p)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    data = torch.randint(0, 256, (B, k, P), dtype=torch.uint8, device=dev, generator=g)
    parity = torch.empty((B, p, P), dtype=torch.uint8, device=dev)
    ref = torch.empty_like(parity)
    rs.encode_batch_dev(data, ref, shard_len=S)
    torch.cuda.synchronize()
    keeps = a.keep.split(",")
    bits = {kp: mask_bits(ncu, kp) for kp in keeps}
    streams = {kp: (torch.cuda.current_stream(dev) if kp == "default" else masked_stream(hip, ncu, bits[kp]))
               for kp in keeps}
    algo = B * (k + p) * S
    t_ramp = time.perf_counter()
    while time.perf_counter() - t_ramp < 0.5:
        for _ in range(8):
            rs.encode_batch_dev(data, parity, shard_len=S)
        torch.cuda.synchronize()
    times = {kp: [] for kp in keeps}
    for _ in range(a.rounds):
        for kp, st in streams.items():
            with torch.cuda.stream(st):
                rs.encode_batch_dev(data, parity, shard_len=S)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(a.iters):
                    rs.encode_batch_dev(data, parity, shard_len=S)
                e1.record(st)
            torch.cuda.synchronize()
            times[kp].append(e0.elapsed_time(e1) / a.iters)
    ok = bool(torch.equal(parity[:, :, :S], ref[:, :, :S]))
    print(f"config={a.config} k={k} p={p} S={S} pitch={P} B={B} cus={ncu} algo_bytes={algo} parity_ok={ok}")
    for kp in keeps:
        med = float(np.median(times[kp]))
        print(json.dumps({"mask": kp, "cus": len(bits[kp]), "median_ms": round(med, 4), "min_ms": round(min(times[kp]), 4),
                          "TBps": round(algo / med / 1e9, 3), "frac": round(algo / (med / 1e3) / 8e12, 4)}))


if __name__ == "__main__":
    main()
