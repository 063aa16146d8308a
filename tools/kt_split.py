#!/usr/bin/env python3
"""Per-kernel breakdown of block-parallel inflate calls from a rocprofv3
kernel-trace CSV (measurement tooling): one line per zcrc_inflate_device call
(find, spec, chain, window build / jumps / store, body, serial fall-back;
times summed per kernel kind) with the call's span.

    python tools/kt_split.py <run_kernel_trace.csv>
"""
import csv
import sys


def short(name):
    for key, s in (("find", "find"), ("probe", "probe"), ("spec", "spec"), ("chain", "chain"), ("tails", "tails"),
                   ("win_build", "wbuild"), ("win_jump", "wjump"), ("win_store", "wstore"), ("body", "body"),
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
        j = i
        while j < len(seq) and seq[j][0] != "serial":
            j += 1
        grp = seq[i:j + 1]
        i = j + 1
        span = (grp[-1][2] - grp[0][1]) / 1e3
        tot = {}
        for s, b, e in grp:
            tot[s] = tot.get(s, 0.0) + (e - b) / 1e3
        njump = sum(1 for s, _, _ in grp if s == "wjump")
        print(" ".join(f"{s}={v:.1f}" for s, v in tot.items()), f"(jumps {njump}) | span={span:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
