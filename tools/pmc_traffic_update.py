#!/usr/bin/env python3
"""Fold a pmc_summary_config<C>.json (tools/collect_profiles.sh) into
profiles/pmc_traffic.json, the per-config PMC traffic bench.py reports as
roofline.traffic (measurement tooling).

    python tools/pmc_traffic_update.py <config> <pmc_summary.json>
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from zipsfs_amd.crc32 import kernel_source_hash  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BYTES = {2: 4096 * 65536, 3: 65536 << 20, 4: 13123505587, 5: 131072 << 20}


def main():
    cfg, path = int(sys.argv[1]), sys.argv[2]
    s = json.load(open(path))
    kern = [k for k in s["kernel_stats"] if "crc32_batch_kernel" in k]
    rel = os.path.relpath(os.path.abspath(path), ROOT)
    out_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    cur = json.load(open(out_path)) if os.path.exists(out_path) else {}
    cur[str(cfg)] = {
        "bytes_per_gpu_per_step": BYTES[cfg],
        "traffic_bytes_per_launch": s["hbm_read_bytes_per_launch"] + s["hbm_write_bytes_per_launch"],
        "read_bytes": s["hbm_read_bytes_per_launch"],
        "write_bytes": s["hbm_write_bytes_per_launch"],
        "kernel": kern[0].replace("void ", "").split("(")[0] if kern else "crc32_batch_kernel",
        "rocprof_avg_kernel_ms": s["kernel_trace"]["avg_ms"],
        "kernel_source_hash": kernel_source_hash(),
        "source": f"{rel}: tools/collect_profiles.sh (rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate "
                  f"passes of python3 bench.py --config {cfg} --steps 5 --warmup 1 --no-cpu-baseline); "
                  f"{s['correction']}",
    }
    json.dump(cur, open(out_path, "w"), indent=1)
    print(json.dumps(cur[str(cfg)]))


if __name__ == "__main__":
    main()
