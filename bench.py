#!/usr/bin/env python3
"""bench.py -- device-resident batched CRC-32 throughput on MI355X.

Metric (BASELINE.json): "CRC32 GiB/s device-resident (batched chunks) and %
of HBM3E read peak".  A *step* is one pass of the hot path over one batch of
synthetic buffers already resident in HBM: the plan (prefix scan) + the
persistent CRC kernel of zcrc32_batch_device, and for N>1 the RCCL
all-gather of the 32-bit results.  Default workload = SURVEY 8(d) config 3,
65536 x 1 MiB buffers per GPU (config 5's per-GPU shard shape at N>1: global
buffer i lives on rank i mod N, weak scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5]

Prints ONE JSON line on rank 0.  `roofline.achieved` is algorithmic bytes per
launch (sum of buffer lengths) / average kernel time, the kernel timed with
HIP events recorded by libzcrc on the stream it launches on.
`cpu_baseline` times the reference's own src/cg_crc32.c (oracle/_ref, built
from the reference sources) on the host cores over a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GiB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
PAYLOAD_SEED = 0xC0FFEE
METRIC = "CRC32 GiB/s device-resident (batched chunks) and % of HBM3E read peak"


def mix64_np(z: np.ndarray) -> np.ndarray:
    z = z + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def zipf_lens(n: int) -> np.ndarray:
    """Config-4 bounded power law on [1 KiB, 16 MiB]."""
    with np.errstate(over="ignore"):
        i = np.arange(n, dtype=np.uint64)
        h = mix64_np(np.uint64(0x5A1F5EED) ^ ((i + np.uint64(1)) * np.uint64(0xD1B54A32D192ED03)))
    u = (h >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    t = 1.0 - u * 127.0 / 128.0
    return np.clip(np.floor(1024.0 / (t * t)), 1024, 1 << 24).astype(np.int64)


class Workload:
    """Device buffers + descriptor tensors for this rank's shard."""

    def __init__(self, cfg: int, rank: int, world: int, dev):
        import torch
        import zipsfs_amd as z
        self.cfg, self.rank, self.world = cfg, rank, world
        self.batches = []  # list of (ptrs, lens) device tensors
        self.mem = []
        if cfg in (3, 5):
            n = 65536 if cfg == 3 else 131072
            L = 1 << 20
            self.desc = f"config{cfg}: {n} x 1 MiB buffers per GPU (global buffer i on rank i mod N)"
            self._strided(n, L, pools=1, dev=dev)
        elif cfg == 2:
            n, L, pools = 4096, 65536, 16
            self.desc = (f"config2: {n} x 64 KiB buffers per GPU per step, rotating over {pools} distinct "
                         "resident batches (4 GiB) so the 256 MB MALL cannot serve repeats")
            self._strided(n, L, pools=pools, dev=dev)
        elif cfg == 4:
            lens_all = zipf_lens(100000)
            mine = np.arange(rank, 100000, world)
            L = lens_all[mine]
            offs = np.zeros(len(L), dtype=np.int64)
            offs[1:] = np.cumsum((L + 15) // 16 * 16)[:-1]
            mem = torch.empty(int(offs[-1] + L[-1] + 16), dtype=torch.uint8, device=dev)
            ptrs = mem.data_ptr() + torch.tensor(offs, device=dev)
            lens = torch.tensor(L, device=dev)
            for k in range(0, len(mine), 4096):  # payload index = global buffer index
                sl = slice(k, min(k + 4096, len(mine)))
                idx0 = int(mine[sl][0])
                z.fill_synthetic(ptrs[sl], lens[sl], index0=idx0, index_step=world, seed=PAYLOAD_SEED)
            self.mem.append(mem)
            self.batches.append((ptrs, lens))
            self.n_local = len(L)
            self.n_total = 100000
            self.bytes_local = int(L.sum())
            self.desc = ("config4: 100k ZIP-entry-like buffers, bounded power law 1 KiB-16 MiB "
                         "(sum 13,123,505,587 B), 16-B aligned, round-robin over ranks")
        else:
            raise ValueError(f"unknown config {cfg}")
        torch.cuda.synchronize()

    def _strided(self, n, L, pools, dev):
        import torch
        import zipsfs_amd as z
        for p in range(pools):
            mem = torch.empty(n * L, dtype=torch.uint8, device=dev)
            ptrs = mem.data_ptr() + torch.arange(n, dtype=torch.int64, device=dev) * L
            lens = torch.full((n,), L, dtype=torch.int64, device=dev)
            # global buffer id g = p*n*world + rank + world*k ; payload index = g
            z.fill_synthetic(ptrs, lens, index0=p * n * self.world + self.rank, index_step=self.world,
                             seed=PAYLOAD_SEED)
            self.mem.append(mem)
            self.batches.append((ptrs, lens))
        self.n_local = n
        self.n_total = n * self.world
        self.bytes_local = n * L


def golden_check(cfg: int, glob: np.ndarray) -> str:
    """Compare CRCs (global buffer order) with the reference-generated fixtures."""
    path = os.path.join(ROOT, "tests", "golden", "configs.npz")
    if not os.path.exists(path):
        return "skipped (no fixtures)"
    g = np.load(path)
    if cfg == 3:
        idx, exp = g["cfg3_idx"].astype(np.int64), g["cfg3"]
    elif cfg == 2:
        k = min(4096, len(glob))
        idx, exp = np.arange(k), g["cfg2"][:k]
    elif cfg == 4:
        idx, exp = g["cfg4_idx"].astype(np.int64), g["cfg4"]
    else:
        return "no fixture for config 5 (see tests/test_gpu_parity.py)"
    ok = int((glob[idx] == exp).sum())
    if ok != len(idx):
        raise SystemExit(f"PARITY FAILURE: {len(idx) - ok} of {len(idx)} sampled CRCs differ from the reference")
    return f"{ok}/{len(idx)} sampled CRCs equal the reference golden vectors"


def cpu_baseline(cfg: int, budget_s: float) -> dict:
    """Reference src/cg_crc32.c (oracle/_ref, -O2) on host cores, bounded sample."""
    from oracle import oracle as o  # the only oracle use in bench.py
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    threads = max(1, min(threads, 64))
    if cfg in (3, 5):
        nb, L = 512, 1 << 20
        sample = f"512 x 1 MiB buffers of the same synthetic payload (512 MiB host-resident), {threads} threads"
    elif cfg == 2:
        nb, L = 4096, 65536
        sample = f"4096 x 64 KiB buffers (256 MiB host-resident), {threads} threads"
    else:
        nb, L = 2000, None
        sample = f"first 2000 config-4 buffers (host-resident), {threads} threads"
    lens = zipf_lens(nb) if L is None else np.full(nb, L, dtype=np.int64)
    bufs = [o.payload(int(lens[i]), i) for i in range(nb)]
    ptrs = np.array([b.ctypes.data for b in bufs], dtype=np.uint64)
    ln = lens.astype(np.uint64)
    total = float(ln.sum())
    use_ref = o.ref_available()
    kind = "reference" if use_ref else "port"
    fn = (lambda nt: o.ref_crc32_batch(ptrs, ln, None, nt)) if use_ref else (lambda nt: o.crc32_batch(ptrs, ln, None, nt))
    fn(threads)  # warm
    reps, t0 = 0, time.perf_counter()
    while True:
        fn(threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= budget_s * 0.7 or reps >= 200:
            break
    rate = reps * total / el / GiB
    # single core, for context
    t1 = time.perf_counter()
    fn(1)
    single = total / (time.perf_counter() - t1) / GiB
    o0 = None
    if use_ref and o.ref_available(o0=True):
        sub = max(1, nb // 8)
        t2 = time.perf_counter()
        o.ref_crc32_batch(ptrs[:sub], ln[:sub], None, 1, o0=True)
        o0 = float(ln[:sub].sum()) / (time.perf_counter() - t2) / GiB
    return {"value": round(rate, 3), "unit": "GiB/s", "cores": threads, "kind": kind,
            "sample": sample + (" -- src/cg_crc32.c compiled -O2 by oracle/Makefile" if use_ref else
                                " -- CPU restatement oracle/crc32_port.c -O2"),
            "single_core_gibs": round(single, 3),
            "single_core_O0_as_shipped_gibs": None if o0 is None else round(o0, 3),
            "host": host_cpu()}


def host_cpu() -> dict:
    """CPU model and counts of the box the baseline ran on."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        allowed = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = None
    return {"model": model, "logical_cpus": os.cpu_count(), "cpus_allowed": allowed}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=3, choices=[2, 3, 4, 5])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (default); gloo only to rehearse ranks sharing one GPU")
    ap.add_argument("--cpu-budget-s", type=float, default=12.0)
    ap.add_argument("--pmc-traffic-bytes", type=float, default=None,
                    help="HBM bytes per launch from a separate rocprofv3 --pmc pass (corrected)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import zipsfs_amd as z
    from zipsfs_amd import shard

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    gpu = local % max(ndev, 1)
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    def barrier():
        if world > 1:
            if args.dist_backend == "nccl":
                dist.barrier(device_ids=[gpu])
            else:
                dist.barrier()

    wl = Workload(args.config, rank, world, dev)
    out = torch.empty(wl.n_local, dtype=torch.int32, device=dev)
    result = {"global": out}

    def step(s: int) -> None:
        ptrs, lens = wl.batches[s % len(wl.batches)]
        z.crc32_batch_device(ptrs, lens, out=out)
        if world > 1:  # the one exchange: all-gather of the 32-bit CRCs
            result["global"] = shard.gather_crcs(out, wl.n_total)

    for s in range(args.warmup):
        step(s)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    with z.profile() as prof:
        t0 = time.perf_counter()
        for s in range(args.steps):
            step(args.warmup + s)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    if world > 1:
        rdev = dev if args.dist_backend == "nccl" else torch.device("cpu")
        et = torch.tensor([elapsed], dtype=torch.float64, device=rdev)
        dist.all_reduce(et, op=dist.ReduceOp.MAX)
        elapsed = float(et.item())
        bt = torch.tensor([wl.bytes_local], dtype=torch.int64, device=rdev)
        dist.all_reduce(bt, op=dist.ReduceOp.SUM)
        bytes_all = int(bt.item())
    else:
        bytes_all = wl.bytes_local

    # parity spot-check: run batch 0 once more (collective at N>1) and compare
    # sampled CRCs with the reference-generated golden vectors (data only)
    step(0)
    torch.cuda.synchronize()
    glob = result["global"].cpu().numpy().view(np.uint32)
    parity = golden_check(args.config, glob) if rank == 0 else None

    ms_per_step = elapsed / args.steps * 1e3
    value = bytes_all * args.steps / elapsed / GiB
    avg_kernel_ms = prof.total_ms / max(prof.launches, 1)
    achieved = wl.bytes_local / (avg_kernel_ms * 1e-3) / 1e9
    traffic = args.pmc_traffic_bytes
    traffic_src = "--pmc-traffic-bytes" if traffic is not None else None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if traffic is None and os.path.exists(pmc_path):
        # PMC traffic per config, collected by tools/collect_profiles.sh for
        # the kernel this build launches (same workload bytes)
        pm = json.load(open(pmc_path)).get(str(args.config))
        if pm and pm.get("bytes_per_gpu_per_step") == wl.bytes_local:
            traffic = pm["traffic_bytes_per_launch"]
            traffic_src = pm["source"]
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.config, args.cpu_budget_s)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world if args.dist_backend == "nccl" else min(world, ndev),
            "ranks": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic: counter-based splitmix64 payload generated in HBM (SURVEY 8d), seed 0xC0FFEE",
            "config": {
                "workload": wl.desc,
                "buffers_per_gpu": wl.n_local,
                "bytes_per_gpu_per_step": wl.bytes_local,
                "api": "zcrc32_batch_device (plan scan + persistent CRC kernel)" +
                       (f" + {'RCCL' if args.dist_backend == 'nccl' else 'gloo'} all_gather of uint32 CRCs"
                        if world > 1 else ""),
                "parallelism": f"round-robin buffer sharding over {world} GPU(s)",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": None if traffic is None else int(traffic),
                "traffic_unit": "bytes per launch (HBM read+write, PMC)",
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": wl.bytes_local,
                "kernel": "zcrc::crc32_batch_kernel<false, 4u, 0, true, false, 1, 2>",
                "avg_kernel_ms": round(avg_kernel_ms, 4),
                "launches_timed": prof.launches,
            },
            "cpu_baseline": cpu,
            "parity": parity,
            "device": torch.cuda.get_device_name(dev),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
