"""tools/order_ab.py -- the batch kernel's window order (BatchView::wp) against
the range order (ZCRC_AB_FLAGS=8), interleaved in ONE process over the same
allocation (measurement only; round 6).

tools/region_probe showed that a config-3 read's rate depends on where its
64 GiB landed (one box: 9.81 against 10.49 ms for the product, three
allocations) -- a comparison across processes mixes that in.  Here both
orders run on the same buffers, alternating blocks of k calls, each block
between one HIP event pair on the launch stream; medians.  Workloads:
config 3 through zcrc32_batch_device (pointer and length arrays: the split
plan finds the lengths equal) and through zcrc32_batch_device_strided, and
(--shard) config 5's per-GPU shard, 131,072 x 1 MiB.  Every block's results
are compared with the reference-generated golden samples.

  python tools/order_ab.py [rounds] [--shard | --c4 | --n=N] [--dyn | --chunk]
  (--dyn: also the window order with an eighth, half or none of the bytes
  dynamic; --chunk: the chunked window order, ab_flags bit 6; --c4: config
  4's 100k Zipf-sized buffers instead of config 3)
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import zipsfs_amd as z  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 5
    shard = "--shard" in sys.argv
    dev = "cuda:0"
    g = np.load(os.path.join(ROOT, "tests", "golden", "configs.npz"))
    c4 = "--c4" in sys.argv
    n = 131072 if shard else (100000 if c4 else 65536)
    for a in sys.argv:  # --n=N: N x 1 MiB instead (config 3's goldens below N)
        if a.startswith("--n="):
            n = int(a[4:])
    L = 1 << 20
    if c4:  # config 4: bench.py's Zipf lengths, 16-B aligned, one allocation
        sys.path.insert(0, ROOT)
        from bench import zipf_lens
        ln = zipf_lens(n)
        offs = np.zeros(n, dtype=np.int64)
        offs[1:] = np.cumsum((ln + 15) // 16 * 16)[:-1]
        mem = torch.empty(int(offs[-1] + ln[-1] + 16), dtype=torch.uint8, device=dev)
        ptrs = mem.data_ptr() + torch.tensor(offs, device=dev)
        lens = torch.tensor(ln, device=dev)
        for k in range(0, n, 4096):
            z.fill_synthetic(ptrs[k:k + 4096], lens[k:k + 4096], index0=k, seed=0xC0FFEE)
        total = int(ln.sum())
    else:
        mem = torch.empty(n * L, dtype=torch.uint8, device=dev)
        ptrs = mem.data_ptr() + torch.arange(n, dtype=torch.int64, device=dev) * L
        lens = torch.full((n,), L, dtype=torch.int64, device=dev)
        z.fill_synthetic(ptrs, lens, index0=0, seed=0xC0FFEE)
        total = n * L
    out = torch.empty(n, dtype=torch.int32, device=dev)
    if c4:
        idx, exp = g["cfg4_idx"].astype(np.int64), g["cfg4"]
    elif shard:
        idx, exp = g["cfg5_idx"].astype(np.int64), g["cfg5"]
        keep = idx < n
        idx, exp = idx[keep], exp[keep]
    else:
        idx, exp = g["cfg3_idx"].astype(np.int64), g["cfg3"]
        keep = idx < n
        idx, exp = idx[keep], exp[keep]
    apis = {"device": lambda: z.crc32_batch_device(ptrs, lens, out=out)}
    if not c4:
        apis["strided"] = lambda: z.crc32_batch_strided(mem, L, L, n, out=out)
    k = 5
    res = {}
    # orders x dynamic shares (ZCRC_AB_FLAGS bits 3 and 4-5, read per call)
    variants = (("window", "0"), ("range", "8"), ("window-dyn1/8", "16"), ("window-dyn1/2", "32"),
                ("window-nodyn", "48")) if "--dyn" in sys.argv else (("window", "0"), ("range", "8"))
    if "--chunk" in sys.argv:  # the chunked window order (ab_flags bit 6)
        variants = (("window", "0"), ("range", "8"), ("chunked-1M", "64"), ("chunked-512K", "192"),
                    ("chunked-256K", "320"), ("chunked-128K", "448"))
    for api, fn in apis.items():
        for order, flags in variants:
            os.environ["ZCRC_AB_FLAGS"] = flags
            for _ in range(3):
                fn()
        torch.cuda.synchronize()
        for r in range(rounds):
            for order, flags in variants:
                os.environ["ZCRC_AB_FLAGS"] = flags
                out.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(k):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                got = out.cpu().numpy().view(np.uint32)
                ok = int((got[idx] == exp).sum())
                res.setdefault((api, order), []).append((e0.elapsed_time(e1) / k, ok))
    os.environ.pop("ZCRC_AB_FLAGS", None)
    for (api, order), v in res.items():
        ms = [a for a, _ in v]
        print(json.dumps({"workload": "config4" if c4 else "config5-shard" if shard else f"{n}x1MiB", "api": api,
                          "order": order,
                          "ms_median": round(float(np.median(ms)), 4), "ms": [round(a, 4) for a in ms],
                          "gbs_median": round(total / (float(np.median(ms)) * 1e-3) / 1e9, 1),
                          "parity": f"{min(o for _, o in v)}/{len(idx)}"}), flush=True)


if __name__ == "__main__":
    main()
