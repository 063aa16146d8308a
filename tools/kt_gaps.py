#!/usr/bin/env python3
"""Inter-launch gaps of one kernel in a rocprofv3 kernel trace (measurement
tooling): duration, start-to-start and end-to-next-start per dispatch of the
kernels whose name contains PATTERN, over the longest back-to-back run.
    python3 tools/kt_gaps.py TRACE.csv PATTERN [--skip N]"""
import csv
import statistics
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 0
    rows = [r for r in csv.DictReader(open(path)) if pat in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[skip:]
    st = [int(r["Start_Timestamp"]) for r in rows]
    en = [int(r["End_Timestamp"]) for r in rows]
    dur = [(e - s) / 1e3 for s, e in zip(st, en)]
    s2s = [(st[i + 1] - st[i]) / 1e3 for i in range(len(st) - 1)]
    e2s = [(st[i + 1] - en[i]) / 1e3 for i in range(len(st) - 1)]
    # back-to-back: a gap under 100 us (the bench's timed loop)
    b2b = [i for i in range(len(e2s)) if e2s[i] < 100]
    q = lambda v: "p10 %.2f p50 %.2f p90 %.2f mean %.2f" % (
        sorted(v)[len(v) // 10], statistics.median(v), sorted(v)[9 * len(v) // 10], statistics.mean(v))
    print(f"{len(rows)} dispatches of *{pat}*; {len(b2b)} back-to-back pairs")
    print("duration us        ", q(dur))
    print("start-to-start us  ", q([s2s[i] for i in b2b]))
    print("end-to-next-start us", q([e2s[i] for i in b2b]))


if __name__ == "__main__":
    main()
