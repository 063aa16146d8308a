#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output for the CRC kernel (measurement tooling).

    python tools/pmc_summary.py <kernel_trace_dir> <fetch_dir> <write_dir> <sq_dir> <out.json>

Applies the gfx950 corrections of /opt/skills/guides/MI355X_MICROARCH.md
(HBM section): FETCH_SIZE is in KiB and reports exactly half of the bytes of a
wide coalesced 16-B/lane streaming read, so HBM read bytes = 2 * 1024 *
FETCH_SIZE; WRITE_SIZE (KiB) is exact for 16-B stores and dword stores here
are negligible.  Effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel time.
"""
import csv
import glob
import json
import os
import statistics
import sys

import re

KERNEL = "crc32_batch_kernel"
# the read-ceiling form (kAblate = 1, any depth): never the product's
ABLATED = re.compile(r"crc32_batch_kernel<false, \d+u, 1,")


def product(name: str) -> bool:
    return KERNEL in name and not ABLATED.search(name)


def per_dispatch(d, counter):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if product(r["Kernel_Name"]) and r["Counter_Name"] == counter:
                vals.setdefault(r["Dispatch_Id"], 0.0)
                vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return list(vals.values())


def main():
    kt, fetch, write, sq, out = sys.argv[1:6]
    durs = []
    for f in glob.glob(os.path.join(kt, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if product(r["Kernel_Name"]):
                durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    stats = {}
    for f in glob.glob(os.path.join(kt, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            stats[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"]),
                                "pct": float(r["Percentage"])}
    fs = per_dispatch(fetch, "FETCH_SIZE")
    ws = per_dispatch(write, "WRITE_SIZE")
    res = {
        "kernel": KERNEL,
        "kernel_trace": {"dispatches": len(durs), "avg_ms": 1e3 * statistics.mean(durs) if durs else None,
                         "median_ms": 1e3 * statistics.median(durs) if durs else None},
        "kernel_stats": stats,
        "fetch_size_kib_per_launch_raw": statistics.median(fs) if fs else None,
        "hbm_read_bytes_per_launch": 2 * 1024 * statistics.median(fs) if fs else None,
        "hbm_write_bytes_per_launch": 1024 * statistics.median(ws) if ws else None,
        "correction": "read bytes = 2 x 1024 x FETCH_SIZE (gfx950 reports half of 16-B/lane streamed bytes)",
    }
    sqd = {}
    for c in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VALU",
              "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "GRBM_GUI_ACTIVE"):
        v = per_dispatch(sq, c)
        if v:
            sqd[c] = statistics.median(v)
    res["sq"] = sqd
    if "GRBM_GUI_ACTIVE" in sqd and durs:
        res["effective_clock_ghz"] = sqd["GRBM_GUI_ACTIVE"] / 8 / statistics.median(durs) / 1e9
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
