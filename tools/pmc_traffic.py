#!/usr/bin/env python3
"""Summarise a tools/profile.sh run: per-kernel average duration (kernel trace)
and HBM bytes per launch from the FETCH_SIZE / WRITE_SIZE PMC passes.

gfx950 corrections (MI355X_MICROARCH.md, HBM section): both counters are in
KiB; FETCH_SIZE reports exactly half the bytes of a wide coalesced streaming
read (16 B/lane global_load), so read bytes = 2 * FETCH_SIZE * 1024;
WRITE_SIZE is exact for 16 B/lane streaming stores: write bytes =
WRITE_SIZE * 1024.

    python tools/pmc_traffic.py gpurun_out/prof_r01 --config encode83 --blocks 512 \
        --algo-bytes 2952790016 --merge profiles/pmc_traffic.json
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import statistics


def rows(path_glob):
    out = []
    for p in glob.glob(path_glob, recursive=True):
        with open(p) as f:
            out.extend(csv.DictReader(f))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--config", required=True)
    ap.add_argument("--blocks", type=int, required=True)
    ap.add_argument("--algo-bytes", type=int, required=True, help="algorithmic bytes per main launch")
    ap.add_argument("--kernel", default="gf_apply_kernel")
    ap.add_argument("--merge", default="")
    ap.add_argument("--sum-kernels", action="store_true",
                    help="steps of several launches (codec104: encode + reconstruct): per-step figures = "
                         "sum over every matching kernel of its average duration / median counter")
    a = ap.parse_args()

    stats = rows(os.path.join(a.dir, "kt", "**", "*kernel_stats.csv"))
    dur = {}
    for r in stats:
        if a.kernel in r["Name"]:
            dur[r["Name"]] = (int(r["Calls"]), float(r["AverageNs"]))
    # dominant = most total time
    main_name = max(dur, key=lambda n: dur[n][0] * dur[n][1]) if dur else None
    names = sorted(dur) if a.sum_kernels else [main_name]

    def counter(name):
        recs = rows(os.path.join(a.dir, name, "**", "*counter_collection.csv"))
        total = 0.0
        for kn in names:
            vals = [float(r["Counter_Value"]) for r in recs
                    if r["Kernel_Name"] == kn and r["Counter_Name"] == name]
            if not vals:
                return None
            total += statistics.median(vals)
        return total

    fetch, write = counter("FETCH_SIZE"), counter("WRITE_SIZE")
    # The bench line of the kernel-trace run names the library build and the
    # kernel variant that ran; bench.py reports this record's traffic only
    # while both still match (traffic_source).
    build_id = variant = None
    logs = [os.path.join(a.dir, "kt.log")] + [os.path.join(a.dir, c + ".log") for c in ("FETCH_SIZE", "WRITE_SIZE")]
    seen = set()
    for log in logs:
        try:
            with open(log) as f:
                for line in f:
                    if line.startswith("{"):
                        b = json.loads(line)
                        seen.add((b["library"]["build_id"], b["config"]["tuning"], b["config"]["blocks_per_gpu"]))
        except (OSError, ValueError, KeyError):
            pass
    if len(seen) == 1:
        build_id, variant, blocks = seen.pop()
        assert blocks == a.blocks, (blocks, a.blocks)
    elif seen:
        raise SystemExit(f"passes ran different builds/variants: {seen}")
    rec = {
        "build_id": build_id,
        "variant": variant,
        "blocks": a.blocks,
        "kernel": main_name if not a.sum_kernels else names,
        "calls": dur[main_name][0] if main_name else None,
        "avg_duration_ns": (sum(dur[n][1] for n in names) if main_name else None),
        "FETCH_SIZE_KiB": fetch,
        "WRITE_SIZE_KiB": write,
        "read_bytes_per_launch": 2 * fetch * 1024 if fetch is not None else None,
        "write_bytes_per_launch": write * 1024 if write is not None else None,
        "algorithmic_bytes_per_launch": a.algo_bytes,
    }
    if a.sum_kernels:
        rec["per"] = "step (sum over the step's launches; *_per_launch keys hold per-step figures)"
    if fetch is not None and write is not None:
        hbm = 2 * fetch * 1024 + write * 1024
        rec["hbm_bytes_per_launch"] = int(hbm)
        rec["traffic_over_algorithmic"] = round(hbm / a.algo_bytes, 4)
    if rec["avg_duration_ns"]:
        rec["achieved_GBps_rocprof"] = round(a.algo_bytes / rec["avg_duration_ns"], 2)
    print(json.dumps(rec, indent=1))
    if a.merge:
        db = {}
        if os.path.exists(a.merge):
            with open(a.merge) as f:
                db = json.load(f)
        db[a.config] = rec
        with open(a.merge, "w") as f:
            json.dump(db, f, indent=1)


if __name__ == "__main__":
    main()
