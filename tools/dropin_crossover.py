#!/usr/bin/env python3
"""Single-entry latency of the drop-in's two paths on this host + GPU.

For each entry size: median wall time of zcrc32_checked (the GPU path:
pinned staging, H2D, kernel, result back) and of zcrc32 with the threshold
raised above every size (libzcrc's host CRC), over host buffers that were
just written (as an entry is, right after its last zip_fread).  The two
answers must agree.  Picks the smallest size from which the GPU is faster
at every larger size: the drop-in's default ZCRC_GPU_MIN_BYTES.  Prints one
JSON object.  Measurement tooling, not the bench contract.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from zipsfs_amd import _lib
    lib = _lib.lib()
    sizes = [1 << k for k in range(12, 29)]  # 4 KiB .. 256 MiB
    rng = np.random.default_rng(7)
    buf = rng.integers(0, 256, size=sizes[-1], dtype=np.uint8)
    out = ctypes.c_uint32()
    lib.zcrc32_checked(buf.ctypes.data, 4096, 0, ctypes.byref(out))  # device init + staging
    rows = []
    for n in sizes:
        reps = 15 if n <= (16 << 20) else 5
        g, h = [], []
        for _ in range(reps):
            buf[:n:4096] += 1  # touch: the entry was just written
            t = time.perf_counter()
            rc = lib.zcrc32_checked(buf.ctypes.data, n, 0, ctypes.byref(out))
            g.append(time.perf_counter() - t)
            assert rc == 0
            gv = out.value
            old = lib.zcrc32_set_gpu_min_bytes(ctypes.c_size_t(-1).value)
            t = time.perf_counter()
            hv = lib.zcrc32(buf.ctypes.data, n, 0)
            h.append(time.perf_counter() - t)
            lib.zcrc32_set_gpu_min_bytes(old)
            assert gv == hv, (n, gv, hv)
        rows.append({"bytes": n, "gpu_us": round(1e6 * float(np.median(g)), 1),
                     "host_us": round(1e6 * float(np.median(h)), 1)})
    cross = None
    for i in range(len(rows)):
        if all(r["gpu_us"] < r["host_us"] for r in rows[i:]):
            cross = rows[i]["bytes"]
            break
    print(json.dumps({"rows": rows, "gpu_faster_from_bytes": cross}))


if __name__ == "__main__":
    main()
