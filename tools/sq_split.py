#!/usr/bin/env python3
"""Summarise one rocprofv3 SQ-counter pass (tools/sq_passes.sh) of a bench
run: per dominant kernel, the median of each counter over its launches and the
derived wave-cycle split (SQ_* wave counters count quad-cycles; only ratios of
SQ counters are quoted because they cover a subset of the waves).

    python tools/sq_split.py gpurun_out/sq_<tag> --tag encode104_u2 --dwords-per-wave 80
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--tag", required=True)
    ap.add_argument("--kernel", default="gf_apply_kernel")
    ap.add_argument("--dwords-per-wave", type=float, default=0.0,
                    help="input dwords one wave loads per lane (k shards x U x 4), for VALU per dword")
    ap.add_argument("--merge", default="")
    a = ap.parse_args()
    rows = []
    for p in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            rows.extend(r for r in csv.DictReader(f) if a.kernel in r["Kernel_Name"])
    per = {}
    for r in rows:
        per.setdefault(r["Kernel_Name"], {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    if not per:
        raise SystemExit("no counter rows for " + a.kernel)
    name = max(per, key=lambda n: len(next(iter(per[n].values()))))
    med = {c: statistics.median(v) for c, v in per[name].items()}
    wc = med.get("SQ_WAVE_CYCLES", 0.0)
    out = {"tag": a.tag, "kernel": name, "launches": len(next(iter(per[name].values()))), "median_counters": med}
    if wc:
        out["wave_cycle_split"] = {
            "waiting_waitcnt_or_barrier": round(med.get("SQ_WAIT_ANY", 0) / wc, 4),
            "issue_stalled": round(med.get("SQ_WAIT_INST_ANY", 0) / wc, 4),
            "issuing": round(med.get("SQ_ACTIVE_INST_ANY", 0) / wc, 4),
        }
    if med.get("SQ_WAVES"):
        vpw = med.get("SQ_INSTS_VALU", 0) / med["SQ_WAVES"]
        out["valu_insts_per_wave"] = round(vpw, 1)
        if a.dwords_per_wave:
            out["valu_insts_per_loaded_dword"] = round(vpw / a.dwords_per_wave, 2)
        out["wave_quadcycles_per_wave"] = round(wc / med["SQ_WAVES"], 1)
    if med.get("SQ_BUSY_CYCLES") and med.get("SQ_ACTIVE_INST_VALU"):
        out["valu_active_per_busy_cycle"] = round(med["SQ_ACTIVE_INST_VALU"] / med["SQ_BUSY_CYCLES"], 3)
    print(json.dumps(out, indent=1))
    if a.merge:
        db = {}
        if os.path.exists(a.merge):
            with open(a.merge) as f:
                db = json.load(f)
        db[a.tag] = out
        with open(a.merge, "w") as f:
            json.dump(db, f, indent=1)


if __name__ == "__main__":
    main()
