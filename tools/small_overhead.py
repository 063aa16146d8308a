"""tools/small_overhead.py -- where a small-buffer API call's time goes
(measurement only).

For uniform 1 GiB batches of `L`-byte buffers (two batches rotated), through
the strided and the device (pointer/length arrays) entry points, prints per
call: the host time to queue it (no synchronize inside the loop), the GPU
time between two events around `reps` x 2 back-to-back calls, and the kernel
time of the same calls from per-launch dispatch timestamps (z.profile()).
The gap between the last two is queue time between launches; a host time
above the GPU time means the GPU waited for the host.

  python tools/small_overhead.py [reps] [len ...]
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import zipsfs_amd as z  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    lengths = [int(x) for x in sys.argv[2:]] or [1024, 4096]
    dev = "cuda:0"
    for L in lengths:
        n = (1 << 30) // L
        bat = []
        for b in range(2):
            mem = torch.empty(n * L + 64, dtype=torch.uint8, device=dev)
            ptrs = mem.data_ptr() + torch.arange(n, dtype=torch.int64, device=dev) * L
            lens = torch.full((n,), L, dtype=torch.int64, device=dev)
            z.fill_synthetic(ptrs, lens, index0=7 * b, seed=0xC0FFEE)
            bat.append((mem, ptrs, lens, torch.empty(n, dtype=torch.int32, device=dev)))
        for api in ("device", "strided", "device", "strided"):  # twice: order effects
            def call(b):
                mem, ptrs, lens, out = bat[b]
                if api == "device":
                    z.crc32_batch_device(ptrs, lens, out=out)
                else:
                    z.crc32_batch_strided(mem, L, L, n, out=out)
            for b in range(2):  # warm
                call(b)
            torch.cuda.synchronize()
            for _ in range(50):  # >= 15 ms of work before the timed calls
                for b in range(2):
                    call(b)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            t0 = time.perf_counter()
            for _ in range(reps):
                for b in range(2):
                    call(b)
            t1 = time.perf_counter()
            e1.record()
            e1.synchronize()
            calls = 2 * reps
            gpu_ms = e0.elapsed_time(e1) / calls
            with z.profile() as prof:
                for _ in range(reps):
                    for b in range(2):
                        call(b)
                torch.cuda.synchronize()
            print(json.dumps({"len": L, "n": n, "api": api, "host_us_per_call": round((t1 - t0) / calls * 1e6, 1),
                              "gpu_us_per_call": round(gpu_ms * 1e3, 1),
                              "kernel_us_per_call": round((prof.total_ms + prof.small_ms) / calls * 1e3, 1),
                              "launches_per_call": (prof.launches + prof.small_launches) / calls}), flush=True)
        del bat


if __name__ == "__main__":
    main()
