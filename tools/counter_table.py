#!/usr/bin/env python3
"""Per-byte memory-pipeline counters from tools/counter_passes.sh.

For each subject (GF encode kernel on page-aligned slots, on the reference's
packed buffer, and the 10 -> 4 XOR replica at U = 1 / 2) takes the median over
dispatches of every counter of the dominant kernel, and normalises by the
kernel's algorithmic bytes (B * (k + R) * S) -- "per KiB" columns -- so kernels
of slightly different shard sizes compare directly.

    python tools/counter_table.py gpurun_out/ctr --json profiles/r03/counters_encode104.json
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import statistics

SUBJECTS = {
    # name: (directory prefix, kernel-name filter, algorithmic bytes per dispatch)
    "gf_encode104_slots": ("gf", "gf_apply_kernel<4, 2, 0", 64 * 14 * 1677722),
    "gf_encode104_packed": ("gfpack", "gf_apply_kernel<4, 2, 0", 64 * 14 * 1677722),
    # r04: the same encode with the peeled ring, and the realigning kernel (MODE 3, knob uvec=0)
    # on the packed buffer -- it covers the 409 full 4 KiB tiles of each shard (the rest is MODE 2)
    "gf_encode104_peel": ("gfpeel", "gf_apply_kernel<4, 2, 0", 64 * 14 * 1677722),
    "gf_encode104_packed_mode3": ("gfpack3", "gf_apply_kernel<4, 1, 3", 64 * 14 * 409 * 4096),
    "xor_10to4_U1": ("xor", "kin_rout<10, 4, 1", 64 * 14 * 1671168),
    "xor_10to4_U2": ("xor", "kin_rout<10, 4, 2", 64 * 14 * 1671168),
}


def load(path_glob, kfilter):
    vals, dur = {}, []
    for p in glob.glob(path_glob, recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                if kfilter not in r.get("Kernel_Name", ""):
                    continue
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in vals.items()}


def durations(path_glob, kfilter):
    ds = []
    for p in glob.glob(path_glob, recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                if kfilter in r.get("Kernel_Name", ""):
                    ds.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return statistics.median(ds) if ds else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    table = {}
    for name, (prefix, kf, algo) in SUBJECTS.items():
        ctr, dur = {}, []
        for d in sorted(glob.glob(os.path.join(a.dir, prefix + "_p*"))):
            for k, v in load(os.path.join(d, "**", "*counter_collection.csv"), kf).items():
                ctr.setdefault(k, v)
            x = durations(os.path.join(d, "**", "*kernel_trace.csv"), kf)
            if x:
                dur.append(x)
        if not ctr:
            continue
        kib = algo / 1024
        row = {"algorithmic_bytes": algo, "kernel_ns_median": statistics.median(dur) if dur else None}
        if row["kernel_ns_median"]:
            row["frac_of_8TBps"] = round(algo / row["kernel_ns_median"] / 8000, 4)
        for k, v in sorted(ctr.items()):
            row[k] = v
            row[k + "_per_KiB"] = round(v / kib, 4)
        table[name] = row
    keys = ["frac_of_8TBps", "TCC_EA0_RDREQ_sum_per_KiB", "TCC_EA0_RDREQ_128B_sum_per_KiB", "TCC_EA0_WRREQ_sum_per_KiB",
            "TCC_EA0_WRREQ_64B_sum_per_KiB", "TCC_REQ_sum_per_KiB", "TCC_HIT_sum_per_KiB", "TCC_MISS_sum_per_KiB",
            "TCC_STREAMING_REQ_sum_per_KiB", "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum_per_KiB",
            "TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum_per_KiB", "TCC_EA0_RDREQ_LEVEL_sum_per_KiB",
            "TCC_EA0_WRREQ_LEVEL_sum_per_KiB", "TA_FLAT_READ_WAVEFRONTS_sum_per_KiB",
            "TA_FLAT_WRITE_WAVEFRONTS_sum_per_KiB", "TA_ADDR_STALLED_BY_TC_CYCLES_sum_per_KiB",
            "TA_DATA_STALLED_BY_TC_CYCLES_sum_per_KiB", "TD_TD_BUSY_sum_per_KiB", "TD_TC_STALL_sum_per_KiB",
            "TCP_TCC_READ_REQ_sum_per_KiB", "TCP_TCC_WRITE_REQ_sum_per_KiB", "TCP_TOTAL_CACHE_ACCESSES_sum_per_KiB",
            "TCP_PENDING_STALL_CYCLES_sum_per_KiB", "TCP_TCR_TCP_STALL_CYCLES_sum_per_KiB",
            "TCP_UTCL1_REQUEST_sum_per_KiB", "TCP_UTCL1_TRANSLATION_MISS_sum_per_KiB",
            "SQ_INSTS_VMEM_RD_per_KiB", "SQ_INSTS_VMEM_WR_per_KiB", "SQ_INST_LEVEL_VMEM_per_KiB",
            "SQ_WAIT_ANY_per_KiB", "SQ_WAVE_CYCLES_per_KiB", "GRBM_GUI_ACTIVE_per_KiB"]
    names = list(table)
    print("| counter (per KiB of algorithmic bytes) | " + " | ".join(names) + " |")
    print("|---|" + "---|" * len(names))
    for k in keys:
        print(f"| {k.replace('_per_KiB', '')} | " + " | ".join(str(table[n].get(k, "")) for n in names) + " |")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(table, f, indent=1)


if __name__ == "__main__":
    main()
