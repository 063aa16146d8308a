"""Per-call host cost of zcrc32_batch_device (what bounds small batches).

Times K back-to-back calls on a tiny batch (GPU work ~ nothing), with and
without z.profile(), and the same for a config-2-sized batch, so the
difference between the per-step time and the kernel time can be attributed.
"""
import sys
import time

import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import zipsfs_amd as z


def run(ptrs, lens, out, k, prof):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if prof:
        with z.profile() as p:
            for _ in range(k):
                z.crc32_batch_device(ptrs, lens, out=out)
            ti = time.perf_counter()
            torch.cuda.synchronize()
    else:
        p = None
        for _ in range(k):
            z.crc32_batch_device(ptrs, lens, out=out)
        ti = time.perf_counter()
        torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / k
    return dt * 1e6, (p.total_ms / p.launches * 1e3 if p else None), (ti - t0) / k * 1e6


def main():
    dev = torch.device("cuda:0")
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    for n, L in ((1, 64), (4096, 64), (4096, 65536)):
        mem = torch.zeros(n * L + 64, dtype=torch.uint8, device=dev)
        ptrs = mem.data_ptr() + torch.arange(n, dtype=torch.int64, device=dev) * L
        lens = torch.full((n,), L, dtype=torch.int64, device=dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        run(ptrs, lens, out, 50, False)
        us, _, iss = run(ptrs, lens, out, k, False)
        _, _, iss50 = run(ptrs, lens, out, 50, False)
        print(f"  first 50 calls: host issue {iss50:5.1f} us/call")
        usp, kus, issp = run(ptrs, lens, out, k, True)
        print(f"n={n:5d} len={L:6d}: {us:7.1f} us/call plain (host issue {iss:5.1f}), {usp:7.1f} us/call "
              f"profiled (host issue {issp:5.1f}), kernel {kus:6.1f} us")


if __name__ == "__main__":
    main()


def burst(fn, k=50):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    ti = time.perf_counter()
    torch.cuda.synchronize()
    return (ti - t0) / k * 1e6, (time.perf_counter() - t0) / k * 1e6


def apis():
    """Which entry point blocks the host?  Config-2 shape, 50-call bursts."""
    dev = torch.device("cuda:0")
    n, L = 4096, 65536
    mem = torch.zeros(n * L + 64, dtype=torch.uint8, device=dev)
    ptrs = mem.data_ptr() + torch.arange(n, dtype=torch.int64, device=dev) * L
    lens = torch.full((n,), L, dtype=torch.int64, device=dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    scratch = torch.empty(z.scratch_bytes(n), dtype=torch.uint8, device=dev)
    for name, fn in (("batch_device", lambda: z.crc32_batch_device(ptrs, lens, out=out)),
                     ("batch_device_ws", lambda: z.crc32_batch_device_ws(ptrs, lens, scratch, out=out)),
                     ("strided", lambda: z.crc32_batch_strided(mem, L, L, n, out=out))):
        burst(fn, 10)
        iss, tot = burst(fn)
        print(f"{name:16s} host issue {iss:6.1f} us/call, total {tot:6.1f} us/call")


if __name__ == "__main__" and os.environ.get("HOST_OVH_APIS"):
    apis()
