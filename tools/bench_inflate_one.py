#!/usr/bin/env python3
"""ONE deflated entry, inflated on the GPU: block-parallel (zcrc_inflate_device)
against the batched kernel with a batch of one (one wave) and against the
system zlib on one host core (what libzip's zip_fread() does for ZIPsFS's
preloadram_now, src/ZIPsFS_preloadfileram.c:286-306) -- measurement tooling.

Payloads: tests/inflate_streams.py (text-like and mass-spectrum-like),
deflated by the image's zlib 1.2.11 at level 6.  GPU times are HIP events
around the call with the compressed stream already in HBM; the rate counts
uncompressed bytes.  Prints one JSON line per (kind, size).

    python tools/bench_inflate_one.py [--sizes 1,16,64] [--reps 5]
"""
import argparse
import json
import os
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,16,64", help="MiB, comma separated")
    ap.add_argument("--kinds", default="text,spectrum")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--no-serial", action="store_true", help="skip the one-wave batch kernel (slow on large entries)")
    args = ap.parse_args()
    import torch
    import inflate_streams as S
    import zipsfs_amd as z

    dev = "cuda:0"
    for kind in args.kinds.split(","):
        for mib in [int(x) for x in args.sizes.split(",")]:
            size = mib << 20
            data = S.PAYLOADS[kind](size, 77)
            comp = S.deflate(data, 6)
            src = torch.frombuffer(bytearray(comp), dtype=torch.uint8).to(dev)
            dst = torch.empty(size, dtype=torch.uint8, device=dev)
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

            def split_once():
                return z.inflate_device(src, dst, chunk_bytes=args.chunk)

            ol, st = split_once()
            torch.cuda.synchronize()
            ok = int(st.item()) == 0 and int(ol.item()) == size
            ok = ok and zlib.crc32(bytes(dst.cpu().numpy())) == zlib.crc32(data)
            ts = []
            for _ in range(args.reps):
                ev0.record()
                split_once()
                ev1.record()
                torch.cuda.synchronize()
                ts.append(ev0.elapsed_time(ev1))
            t_split = sorted(ts)[len(ts) // 2]

            t_serial = None
            if not args.no_serial:
                sp = torch.tensor([src.data_ptr()], dtype=torch.int64, device=dev)
                sl = torch.tensor([len(comp)], dtype=torch.int64, device=dev)
                dp = torch.tensor([dst.data_ptr()], dtype=torch.int64, device=dev)
                cp = torch.tensor([size], dtype=torch.int64, device=dev)
                z.inflate_batch_device(sp, sl, dp, cp)
                torch.cuda.synchronize()
                ev0.record()
                z.inflate_batch_device(sp, sl, dp, cp)
                ev1.record()
                torch.cuda.synchronize()
                t_serial = ev0.elapsed_time(ev1)

            reps_cpu = max(1, min(args.reps, int(2e8 // size)))
            t0 = time.perf_counter()
            for _ in range(reps_cpu):
                zlib.decompress(comp, -15)
            t_cpu = (time.perf_counter() - t0) / reps_cpu * 1e3
            line = {"kind": kind, "size_mib": mib, "compressed": len(comp), "ok": bool(ok),
                    "split_ms": round(t_split, 3), "split_gbs": round(size / t_split / 1e6, 2),
                    "one_wave_ms": None if t_serial is None else round(t_serial, 3),
                    "zlib_1core_ms": round(t_cpu, 3), "zlib_1core_gbs": round(size / t_cpu / 1e6, 3),
                    "speedup_vs_1core": round(t_cpu / t_split, 2), "chunk": args.chunk or "auto"}
            print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
