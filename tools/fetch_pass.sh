#!/bin/bash
# One rocprofv3 FETCH_SIZE pass and one kernel-trace pass of a bench.py
# command (measurement tooling; run on the GPU box from the repo root):
#     tools/fetch_pass.sh <work_dir> <bench args...>
# prints the median HBM read bytes per crc32_batch_kernel launch (2 x 1024 x
# FETCH_SIZE, the gfx950 correction) and the average kernel duration.
set -e -o pipefail
W=$1; shift
export TMPDIR=/tmp
mkdir -p "$W"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$W/kt" -o bench -- python3 bench.py "$@" > "$W/kt.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$W/fetch" -o bench -- python3 bench.py "$@" > "$W/fetch.log" 2>&1
python3 - "$W" <<'PY'
import csv, glob, os, statistics, sys
w = sys.argv[1]
fs, durs = {}, []
for f in glob.glob(os.path.join(w, "fetch", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "crc32_batch_kernel" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE":
            fs[r["Dispatch_Id"]] = fs.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
for f in glob.glob(os.path.join(w, "kt", "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "crc32_batch_kernel" in r["Kernel_Name"]:
            durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
print({"read_bytes_per_launch": 2 * 1024 * statistics.median(fs.values()), "launches": len(fs),
       "avg_kernel_ms": statistics.mean(durs), "median_kernel_ms": statistics.median(durs)})
PY
