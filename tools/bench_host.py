#!/usr/bin/env python3
"""Host-resident CRC throughput (pinned staging + H2D + kernel + D2H).

The ZIPsFS path starts and ends in host RAM (the preloaded entry buffer), so
this measures what the drop-in cg_crc32()/zcrc32_batch() deliver including
PCIe.  Prints one JSON object.  Measurement tooling, not the bench contract.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import zipsfs_amd as z
    rng = np.random.default_rng(1)
    res = {}
    # many 1 MiB buffers (config-3-like, host-resident)
    bufs = [rng.integers(0, 256, size=1 << 20, dtype=np.uint8) for _ in range(1024)]
    z.crc32_batch(bufs[:8])
    t = time.perf_counter()
    reps = 3
    for _ in range(reps):
        z.crc32_batch(bufs)
    el = time.perf_counter() - t
    res["batch_1024x1MiB_GiBs"] = round(reps * 1024 / 1024 / el, 2)
    # one large entry through the drop-in signature (zcrc32)
    big = rng.integers(0, 256, size=512 << 20, dtype=np.uint8)
    z.cg_crc32(big[:4096])
    t = time.perf_counter()
    z.cg_crc32(big)
    el = time.perf_counter() - t
    res["dropin_single_512MiB_GiBs"] = round(0.5 / el, 2)
    # latency of the drop-in for small entries (median ZIP entry ~4 KiB)
    for n in (64, 4096, 16384, 32768, 65536, 1 << 20, 16 << 20):
        d = big[:n]
        lat = []
        for _ in range(20):
            t = time.perf_counter()
            z.cg_crc32(d)
            lat.append(time.perf_counter() - t)
        res[f"dropin_latency_us_{n}"] = round(1e6 * float(np.median(lat)), 1)
    # zipf (config-4-like) sample, host-resident
    sys.path.insert(0, ROOT)
    from bench import zipf_lens
    lens = zipf_lens(20000)
    zb = [rng.integers(0, 256, size=int(L), dtype=np.uint8) for L in lens]
    tot = float(lens.sum())
    z.crc32_batch(zb[:10])
    t = time.perf_counter()
    z.crc32_batch(zb)
    el = time.perf_counter() - t
    res["batch_zipf20k_GiBs"] = round(tot / el / (1 << 30), 2)
    res["batch_zipf20k_bytes"] = int(tot)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
