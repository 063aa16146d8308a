"""tools/small_timing_ab.py -- why do bench.py's small-buffer secondary and
tools/small_batches.py disagree on the same box?  (measurement only)

Same batches (1 GiB of L-byte buffers, two rotated), same APIs; two ways of
timing k calls between one HIP event pair:
  idle    torch.cuda.synchronize() after the warm calls, then the timed calls
          (bench.py's small_batches until round 6 session 15): the GPU starts
          the timed block idle, so the host's per-call time shows whenever it
          exceeds the kernel's
  queued  the timed calls queued behind the warm ones, no synchronize
          (tools/small_batches.py): the host's time hides behind the backlog
and the host's own time per call (perf_counter around the k calls); the
*_newout variants let the API allocate each call's result tensor, as
tools/small_batches.py does.

  python tools/small_timing_ab.py [len ...]
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import zipsfs_amd as z  # noqa: E402


def main():
    lengths = [int(a) for a in sys.argv[1:]] or [1024, 4096]
    dev = "cuda:0"
    for L in lengths:
        n = (1 << 30) // L
        bat = []
        for b in range(2):
            mem = torch.empty(n * L + 64, dtype=torch.uint8, device=dev)
            ptrs = mem.data_ptr() + torch.arange(n, dtype=torch.int64, device=dev) * L
            lens = torch.full((n,), L, dtype=torch.int64, device=dev)
            z.fill_synthetic(ptrs, lens, index0=b * n, seed=0xC0FFEE)
            bat.append((mem, ptrs, lens, torch.empty(n, dtype=torch.int32, device=dev)))
        apis = {
            "device": lambda b: z.crc32_batch_device(bat[b][1], bat[b][2], out=bat[b][3]),
            "device_maxlen": lambda b: z.crc32_batch_device(bat[b][1], bat[b][2], out=bat[b][3], max_len=L),
            "strided": lambda b: z.crc32_batch_strided(bat[b][0], L, L, n, out=bat[b][3]),
            # a fresh result tensor per call, as tools/small_batches.py calls it
            "device_newout": lambda b: z.crc32_batch_device(bat[b][1], bat[b][2]),
            "device_maxlen_newout": lambda b: z.crc32_batch_device(bat[b][1], bat[b][2], max_len=L),
        }
        for mode in ("idle", "queued", "idle", "queued"):
            for name, fn in apis.items():
                for s in range(100):
                    fn(s % 2)
                if mode == "idle":
                    torch.cuda.synchronize()
                k = 40
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                h0 = time.perf_counter()
                for s in range(k):
                    fn(s % 2)
                h1 = time.perf_counter()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / k
                print(json.dumps({"len": L, "api": name, "mode": mode, "gpu_us_per_call": round(ms * 1e3, 1),
                                  "host_us_per_call": round((h1 - h0) / k * 1e6, 1),
                                  "tbs": round(n * L / (ms * 1e-3) / 1e12, 3)}), flush=True)
        del bat
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
