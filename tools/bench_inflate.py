#!/usr/bin/env python3
"""Batched GPU inflate throughput -- measurement tooling.

Workload ("many ZIP entries"): U distinct payloads (half text-like, half
mass-spectrum-like binary, tests/inflate_streams.py), deflated by the image's
zlib 1.2.11 at level 6, replicated into N device-resident entries.  Timed with
HIP events around the inflate launch (and around inflate + batched CRC, the
ZIP-verification shape).  GB/s counts *uncompressed* output bytes, the unit
zip_fread() delivers to ZIPsFS.  CPU baseline: system zlib raw inflate (what
libzip calls) over a bounded sample with a pthread pool.

    python tools/bench_inflate.py [--entries 4096] [--size 1048576] [--reps 5]

Prints one JSON line.  Not the bench.py contract (that is the CRC metric).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--entries", type=int, default=4096)
    ap.add_argument("--size", type=int, default=1 << 20)
    ap.add_argument("--unique", type=int, default=32)
    ap.add_argument("--level", type=int, default=6)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-budget-s", type=float, default=10.0)
    ap.add_argument("--kind", default="mixed", choices=["mixed", "text", "spectrum"])
    ap.add_argument("--lib", default=None, help="alternate libzcrc build (measurement variants)")
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    if args.lib:
        import zipsfs_amd._lib as L
        L.LIB_PATH = os.path.abspath(args.lib)

    import torch
    import zlib
    import inflate_streams as S
    import zipsfs_amd as z
    from oracle import oracle as o

    dev = "cuda:0"
    raw, comp = [], []
    for u in range(args.unique):
        if args.kind == "mixed":
            gen = S.text_payload if u % 2 == 0 else S.spectrum_payload
        else:
            gen = S.text_payload if args.kind == "text" else S.spectrum_payload
        data = gen(args.size, 7000 + u)
        raw.append(data)
        comp.append(S.deflate(data, args.level))
    pick = [k % args.unique for k in range(args.entries)]
    # compressed entries packed back to back (unaligned), outputs in one arena
    src_off = np.zeros(args.entries, dtype=np.int64)
    sizes = np.array([len(comp[p]) for p in pick], dtype=np.int64)
    src_off[1:] = np.cumsum(sizes)[:-1]
    host = np.empty(int(sizes.sum()), dtype=np.uint8)
    for k, p in enumerate(pick):
        host[src_off[k]:src_off[k] + sizes[k]] = np.frombuffer(comp[p], dtype=np.uint8)
    src = torch.from_numpy(host).to(dev)
    caps = np.array([len(raw[p]) for p in pick], dtype=np.int64)
    dst_off = np.zeros(args.entries, dtype=np.int64)
    dst_off[1:] = np.cumsum(caps)[:-1]
    arena = torch.empty(int(caps.sum()), dtype=torch.uint8, device=dev)
    sp = src.data_ptr() + torch.from_numpy(src_off).to(dev)
    sl = torch.from_numpy(sizes).to(dev)
    dp = arena.data_ptr() + torch.from_numpy(dst_off).to(dev)
    cp = torch.from_numpy(caps).to(dev)
    ol = torch.empty(args.entries, dtype=torch.int64, device=dev)
    st = torch.empty(args.entries, dtype=torch.int32, device=dev)
    out_bytes = int(caps.sum())
    in_bytes = int(sizes.sum())

    def run(fused):
        z.inflate_batch_device(sp, sl, dp, cp, out_lens=ol, status=st)
        if fused:
            return z.crc32_batch_device(dp, ol)
        return None

    run(True)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0, "inflate failed"
    check = args.lib is None  # ablation builds produce wrong bytes by design
    crcs = run(True).cpu().numpy().view(np.uint32)
    want = [zlib.crc32(raw[p]) for p in pick[: args.unique]]
    assert not check or list(crcs[: args.unique]) == want, "parity"
    host_out = arena[: min(out_bytes, 64 << 20)].cpu().numpy()
    for k in range(min(args.unique, 8)):
        a = int(dst_off[k])
        if check and a + caps[k] <= host_out.size:
            assert host_out[a:a + caps[k]].tobytes() == raw[pick[k]]

    res = {}
    for fused in (False, True):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(args.reps):
            run(fused)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.reps
        key = "inflate_crc" if fused else "inflate"
        res[key] = {"ms": round(ms, 3), "out_GBs": round(out_bytes / ms / 1e6, 2),
                    "in_GBs": round(in_bytes / ms / 1e6, 2)}

    if args.no_cpu:
        print(json.dumps({"kind": args.kind, "lib": args.lib, "gpu": res}), flush=True)
        return
    # CPU baseline: system zlib (libzip's inflate), bounded sample
    nsamp = max(args.cpu_threads, min(args.entries, 64))
    streams = [comp[pick[k]] for k in range(nsamp)]
    scaps = [len(raw[pick[k]]) for k in range(nsamp)]
    o.zlib_inflate_batch(streams[: args.cpu_threads], scaps[: args.cpu_threads], nthreads=args.cpu_threads)
    t0 = time.perf_counter()
    reps = 0
    while True:
        zs, zl, _ = o.zlib_inflate_batch(streams, scaps, nthreads=args.cpu_threads)
        reps += 1
        el = time.perf_counter() - t0
        if el > args.cpu_budget_s or reps >= 50:
            break
    assert (zs == 0).all()
    cpu_gbs = reps * sum(scaps) / el / 1e9
    t0 = time.perf_counter()
    o.zlib_inflate_batch(streams[:4], scaps[:4], nthreads=1)
    one = sum(scaps[:4]) / (time.perf_counter() - t0) / 1e9

    line = {
        "metric": "batched raw-DEFLATE inflate, GB/s of uncompressed output (device-resident)",
        "value": res["inflate"]["out_GBs"],
        "unit": "GB/s",
        "workload": f"{args.entries} entries x {args.size} B ({args.unique} distinct text/spectrum payloads, "
                    f"zlib level {args.level}), compressed {in_bytes} B -> {out_bytes} B",
        "gpu": res,
        "cpu_baseline": {"value": round(cpu_gbs, 2), "unit": "GB/s", "cores": args.cpu_threads,
                         "kind": "reference",
                         "sample": f"{nsamp} of the same entries, system zlib {zlib.ZLIB_RUNTIME_VERSION} raw "
                                   f"inflate (libzip's inflate), pthread pool",
                         "single_core_GBs": round(one, 3)},
        "device": torch.cuda.get_device_name(0),
    }
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
