#!/usr/bin/env python3
"""Inter-launch gaps of the headline step (RS(8,3) encode, 512 blocks on the
bench's slots), interleaved in one process: K back-to-back steps timed with an
event after every step (bench.py's timed region) against only a start and an
end event, and against the same K launches captured in one HIP graph.  The
difference between ms per step and the kernel's own duration is the gap the
bench's value pays between dispatches.

    python tools/gap_probe.py --rounds 11 --steps 20
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

import shmr_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=11)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    k, p, B = 8, 3, 512
    S = shmr_amd.calculate_shard_size(4 << 20, k)
    P = S + 4096
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    data = torch.randint(0, 256, (B, k, P), dtype=torch.uint8, device=dev, generator=g)
    par = torch.empty((B, p, P), dtype=torch.uint8, device=dev)
    rs = shmr_amd.ReedSolomon(k, p)
    st = torch.cuda.Stream()
    shmr_amd.device_init(0)

    def step():
        rs.encode_batch_dev(data, par, shard_len=S)

    with torch.cuda.stream(st):
        for _ in range(200):
            step()
    st.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=st):
        for _ in range(a.steps):
            step()
    res = {"per_step_events": [], "two_events": [], "graph": []}
    for _ in range(a.rounds):
        with torch.cuda.stream(st):
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
            evs[0].record(st)
            for i in range(a.steps):
                step()
                evs[i + 1].record(st)
            st.synchronize()
            res["per_step_events"].append(evs[0].elapsed_time(evs[-1]) / a.steps)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for i in range(a.steps):
                step()
            e1.record(st)
            st.synchronize()
            res["two_events"].append(e0.elapsed_time(e1) / a.steps)
            e0.record(st)
            graph.replay()
            e1.record(st)
            st.synchronize()
            res["graph"].append(e0.elapsed_time(e1) / a.steps)
    algo = B * (k + p) * S
    for n, v in res.items():
        med = float(np.median(v))
        print(json.dumps({"timing": n, "ms_per_step_median": round(med, 4), "min": round(min(v), 4),
                          "frac_of_8TBps": round(algo / (med / 1e3) / 8e12, 4)}))


if __name__ == "__main__":
    main()
