"""tools/small_batches.py -- uniform batches of small buffers through the
product entry points (measurement only).

For each length, two distinct 1 GiB batches (rotated, so the MALL cannot serve
repeats) are checksummed through zcrc32_batch_device (general form: device
pointer and length arrays; above 8192 buffers the split plan routes buffers
of <= 8 KiB to the small-buffer kernel), zcrc32_batch_device_maxlen (the
caller's bound: one small-kernel launch, no plan) and
zcrc32_batch_device_strided, with
ZCRC_SMALL=1 (default) and 0 (batch kernel only).  Reported per call: the
GPU time between two events on the stream around `reps` x 2 back-to-back
calls (plans and launch gaps included; no per-launch events, which leave a
~10 us bubble before each launch: profiles/r03/s2).  Results of all four
routes are compared.

  python tools/small_batches.py [reps] [len,len,... | len len ...] > out.jsonl
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import zipsfs_amd as z  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    lengths = ([int(x) for a in sys.argv[2:] for x in a.split(",")] if len(sys.argv) > 2
               else [1024, 2048, 3000, 4096, 8192, 16384])
    dev = "cuda:0"
    for L in lengths:
        n = (1 << 30) // L
        bat = []
        for b in range(2):
            mem = torch.empty(n * L + 64, dtype=torch.uint8, device=dev)
            ptrs = mem.data_ptr() + torch.arange(n, dtype=torch.int64, device=dev) * L
            lens = torch.full((n,), L, dtype=torch.int64, device=dev)
            z.fill_synthetic(ptrs, lens, index0=7 * b, seed=0xC0FFEE)
            bat.append((mem, ptrs, lens))
        ref = None
        for small in ("1", "0"):
            os.environ["ZCRC_SMALL"] = small
            for api in ("device", "device_maxlen", "strided"):
                if api == "device_maxlen" and small == "0":
                    continue  # (the hint is the small kernel's route)

                def call(b):
                    mem, ptrs, lens = bat[b]
                    if api == "device":
                        return z.crc32_batch_device(ptrs, lens)
                    if api == "device_maxlen":  # zcrc32_batch_device_maxlen: the caller's bound, no plan
                        return z.crc32_batch_device(ptrs, lens, max_len=L)
                    return z.crc32_batch_strided(mem, L, L, n)
                outs = [call(b) for b in range(2)]  # warm (scratch, first use)
                torch.cuda.synchronize()
                for _ in range(50):  # >= 15 ms of work before the timed calls (clocks; the first
                    for b in range(2):  # calls after the fill read up to 30 us slower)
                        call(b)
                if ref is None:
                    ref = [o.clone() for o in outs]
                same = all(torch.equal(o, r) for o, r in zip(outs, ref))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for r in range(reps):
                    for b in range(2):
                        call(b)
                e1.record()
                e1.synchronize()
                calls = 2 * reps
                w_ms = e0.elapsed_time(e1) / calls
                print(json.dumps({"len": L, "n": n, "api": api, "small": small == "1", "wall_ms": round(w_ms, 4),
                                  "wall_GBps": round(n * L / (w_ms * 1e-3) / 1e9, 1),
                                  "same_results": same}), flush=True)
        del bat


if __name__ == "__main__":
    main()
