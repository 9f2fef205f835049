#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --pmc passes (any counters): for every
kernel whose name contains --kernel, the dispatch count and the median and
mean of each counter per dispatch, plus the kernel-trace average duration when
the pass wrote one.  Writes one small JSON (the raw per-dispatch CSVs are
large; GPU scripts delete them after summarising).

    python tools/pmc_summary.py /tmp/pmcraw/encode83_p1 --out gpurun_out/r05b/encode83_p1.json
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", required=True)
    ap.add_argument("--kernel", default="gf_apply_kernel")
    a = ap.parse_args()
    vals = defaultdict(lambda: defaultdict(list))
    for p in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                if a.kernel in r["Kernel_Name"]:
                    vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    durs = defaultdict(list)
    for p in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                if a.kernel in r["Kernel_Name"]:
                    durs[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = {}
    for kn in sorted(set(vals) | set(durs)):
        rec = {"dispatches": max([len(v) for v in vals[kn].values()] + [len(durs[kn])]),
               "duration_ns_median": statistics.median(durs[kn]) if durs[kn] else None,
               "counters": {c: {"median": statistics.median(v), "mean": statistics.fmean(v), "n": len(v)}
                            for c, v in sorted(vals[kn].items())}}
        out[kn] = rec
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(f"{a.out}: {len(out)} kernels")


if __name__ == "__main__":
    main()
