#!/usr/bin/env python3
"""Per-kernel breakdown of block-parallel inflate calls from a rocprofv3
kernel-trace CSV (measurement tooling): one line per zcrc_inflate_device call
(find, spec, chain, tails, body, serial fall-back) with the call's span.

    python tools/kt_split.py <run_kernel_trace.csv>
"""
import csv
import sys


def short(name):
    for key, s in (("find", "find"), ("spec", "spec"), ("chain", "chain"), ("tails", "tails"), ("body", "body"),
                   ("inflate_kernel", "serial")):
        if key in name:
            return s
    return None


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    seq = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    seq = [x for x in seq if x[0]]
    i = 0
    while i < len(seq):
        if seq[i][0] != "find":
            i += 1
            continue
        grp = seq[i:i + 6]
        i += 6
        span = (grp[-1][2] - grp[0][1]) / 1e3
        print(" ".join(f"{s}={(e - b) / 1e3:.1f}" for s, b, e in grp), f"| span={span:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
