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
launch (sum of buffer lengths) / average kernel time: one HIP event pair on
the stream the launches go to, around the timed steps, divided by the
launches (back-to-back launches leave no gap on the stream; per-launch events
did, ~10 us each: ZCRC_BENCH_KERNEL_EVENTS=1).
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

    def __init__(self, cfg: int, rank: int, world: int, dev, n_override=None):
        import torch
        import zipsfs_amd as z
        self.cfg, self.rank, self.world = cfg, rank, world
        self.batches = []  # list of (ptrs, lens) device tensors
        self.regions = []  # per batch: (device address, bytes) of the contiguous region holding its buffers
        self.mem = []
        if cfg in (3, 5):
            n = n_override or (65536 if cfg == 3 else 131072)
            L = 1 << 20
            self.desc = (f"config{cfg}: {n} x 1 MiB buffers per GPU, {n * world} in all "
                         f"(global buffer i on rank i mod {world})")
            self._strided(n, L, pools=1, dev=dev)
        elif cfg == 2:
            n, L, pools = 4096, 65536, 16
            self.desc = (f"config2: {n} x 64 KiB buffers per GPU per step, rotating over {pools} distinct "
                         "resident batches (4 GiB) so the 256 MB MALL cannot serve repeats")
            self._strided(n, L, pools=pools, dev=dev)
        elif cfg == 4:
            lens_all = zipf_lens(100000)
            rnd = int(os.environ.get("ZCRC_BENCH_LEN_ROUND", "0"))  # traffic experiments only:
            if rnd:                                                  # lengths rounded up (parity then fails)
                lens_all = (lens_all + rnd - 1) // rnd * rnd
            mine = np.arange(rank, 100000, world)
            L = lens_all[mine]
            # buffer start alignment (16 B; ZCRC_BENCH_ALIGN: a measurement knob for
            # the HBM-traffic experiments of DESIGN.md section 7b)
            al = int(os.environ.get("ZCRC_BENCH_ALIGN", "16"))
            offs = np.zeros(len(L), dtype=np.int64)
            offs[1:] = np.cumsum((L + al - 1) // al * al)[:-1]
            mem = torch.empty(int(offs[-1] + L[-1] + 16), dtype=torch.uint8, device=dev)
            ptrs = mem.data_ptr() + torch.tensor(offs, device=dev)
            lens = torch.tensor(L, device=dev)
            for k in range(0, len(mine), 4096):  # payload index = global buffer index
                sl = slice(k, min(k + 4096, len(mine)))
                idx0 = int(mine[sl][0])
                z.fill_synthetic(ptrs[sl], lens[sl], index0=idx0, index_step=world, seed=PAYLOAD_SEED)
            self.mem.append(mem)
            self.batches.append((ptrs, lens))
            self.regions.append((mem.data_ptr(), int(offs[-1] + L[-1]) // 16 * 16))
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
            self.regions.append((mem.data_ptr(), n * L))
        self.n_local = n
        self.n_total = n * self.world
        self.bytes_local = n * L


class _NoProfile:
    total_ms, launches, small_ms, small_launches = float("nan"), 0, 0.0, 0

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


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
    else:  # config 5: samples spread over [0, 2^20); check those this run holds
        idx, exp = g["cfg5_idx"].astype(np.int64), g["cfg5"]
        keep = idx < len(glob)
        idx, exp = idx[keep], exp[keep]
        if len(idx) < 256:
            raise SystemExit(f"PARITY: only {len(idx)} config-5 samples fall inside {len(glob)} buffers")
    ok = int((glob[idx] == exp).sum())
    if ok != len(idx) and cfg == 4 and os.environ.get("ZCRC_BENCH_LEN_ROUND"):
        return "not checked: ZCRC_BENCH_LEN_ROUND changed the workload (traffic experiment)"
    if ok != len(idx):
        raise SystemExit(f"PARITY FAILURE: {len(idx) - ok} of {len(idx)} sampled CRCs differ from the reference")
    return f"{ok}/{len(idx)} sampled CRCs equal the reference golden vectors"


def baseline_sample(cfg: int, sample_bytes: int) -> tuple:
    """(lens, payload indices, description) of the CPU baseline's host sample:
    the same synthetic buffers as the GPU workload, at least `sample_bytes`
    in all, so that the sample is several times the host's L3."""
    if cfg in (3, 5):
        L = 1 << 20
        nb = max(1, -(-sample_bytes // L))
        return np.full(nb, L, dtype=np.int64), np.arange(nb), f"{nb} x 1 MiB buffers"
    if cfg == 2:
        L = 65536
        nb = max(1, -(-sample_bytes // L))
        return np.full(nb, L, dtype=np.int64), np.arange(nb), f"{nb} x 64 KiB buffers"
    lens = zipf_lens(100000)
    nb = int(np.searchsorted(np.cumsum(lens), sample_bytes)) + 1
    nb = min(nb, 100000)
    return lens[:nb], np.arange(nb), f"the first {nb} config-4 buffers"


def cpu_baseline(cfg: int, budget_s: float, sample_gib: float) -> dict:
    """The reference's src/cg_crc32.c (oracle/_ref) on this host's cores.

    SURVEY 8(d): a pthread pool with round-robin buffer ownership, wall clock
    per pass over a host-resident sample of >= sample_gib GiB of the same
    payload, at -O2 and at -O0 (as shipped, src/ZIPsFS.compile.sh:319).  Each
    thread count runs on a sample that its own workers filled (first touch:
    pages on the NUMA node of the core that checksums them).  The thread
    counts from 1 to all allowed CPUs are swept; `value` and `cores` are the
    fastest one (256 threads on one-thread-filled memory ran
    slower than 16)."""
    from oracle import oracle as o  # the only oracle use in bench.py
    host = host_cpu()
    allowed = host["cpus_allowed"] or os.cpu_count() or 1
    quota = host["cgroup_quota_cpus"]  # the GPU box's cgroup grants 16 CPUs of its 256
    cap = min(allowed, 2 * quota) if quota else allowed
    forced = int(os.environ.get("ZCRC_BASELINE_THREADS", "0") or 0)
    counts = [forced] if forced else sorted({t for t in (1, 4, 8, 12, 16, 24, 32, 64, 128, 256, cap) if t <= cap})
    lens, idx, what = baseline_sample(cfg, int(sample_gib * GiB))
    offs = np.zeros(len(lens), dtype=np.int64)
    offs[1:] = np.cumsum((lens + 4095) // 4096 * 4096)[:-1]  # page-aligned: no page shared by two owners
    total = float(lens.sum())
    use_ref = o.ref_available()
    kind = "reference" if use_ref else "port"
    ln = lens.astype(np.uint64)
    gidx = idx.astype(np.uint64)

    def sample(nt: int):
        arena = np.empty(int(offs[-1] + lens[-1] + 16), dtype=np.uint8)  # untouched pages
        ptrs = (arena.ctypes.data + offs).astype(np.uint64)
        o.port().oracle_fill_payload_batch(ptrs.ctypes.data, ln.ctypes.data, gidx.ctypes.data, PAYLOAD_SEED,
                                           len(lens), nt)
        return arena, ptrs

    def run(nt: int, o0: bool, p, l=ln):
        return o.ref_crc32_batch(p, l, None, nt, o0=o0) if use_ref else o.crc32_batch(p, l, None, nt)

    def rate(nt: int, o0: bool, budget: float, p) -> float:
        run(nt, o0, p)  # warm: spawn, caches
        reps, t0 = 0, time.perf_counter()
        while True:
            run(nt, o0, p)
            reps += 1
            el = time.perf_counter() - t0
            if el >= budget or reps >= 50:
                return reps * total / el / GiB

    sweep = {}
    for nt in counts[1:] if len(counts) > 1 else counts:  # one thread: below, on a 1 GiB prefix
        arena, ptrs = sample(nt)
        sweep[nt] = rate(nt, False, budget_s * 0.5 / max(1, len(counts) - 1), ptrs)
        del arena
    best = max(sweep, key=sweep.get)
    arena, ptrs = sample(best)
    best_o0 = rate(best, True, budget_s * 0.15, ptrs) if use_ref and o.ref_available(o0=True) else None
    # one thread: a >= 1 GiB prefix of the sample (still > L3), one pass
    k = max(1, int(np.searchsorted(np.cumsum(lens), min(total, GiB))) + 1)
    sub_p, sub_l = ptrs[:k], ln[:k]
    sub_total = float(sub_l.sum())

    def one(o0: bool) -> float:
        t0 = time.perf_counter()
        run(1, o0, sub_p, sub_l)
        return sub_total / (time.perf_counter() - t0) / GiB

    one_o2 = one(False)
    one_o0 = one(True) if use_ref and o.ref_available(o0=True) else None
    del arena
    r3 = lambda v: None if v is None else round(v, 3)
    cores = min(best, quota) if quota else best
    return {"value": r3(sweep[best]), "unit": "GiB/s", "cores": cores, "kind": kind,
            "sample": (f"{what} ({total / GiB:.2f} GiB host-resident, same synthetic payload, filled by the "
                       f"owning threads), {best} threads (fastest of {sorted(sweep)})" +
                       (f" under a cgroup quota of {quota} CPUs" if quota else "") +
                       ", round-robin buffer ownership, wall clock per pass -- " +
                       ("src/cg_crc32.c compiled -O2 by oracle/Makefile" if use_ref else
                        "CPU restatement oracle/crc32_port.c -O2")),
            "threads_sweep_gibs": {str(t): r3(v) for t, v in sorted(sweep.items())},
            "best_threads_O0_as_shipped_gibs": r3(best_o0),
            "single_core_gibs": r3(one_o2),
            "single_core_O0_as_shipped_gibs": r3(one_o0),
            "single_core_sample_gib": round(sub_total / GiB, 3),
            "host": host}


def host_cpu() -> dict:
    """CPU model, counts, cgroup CPU quota and NUMA layout of the box the
    baseline ran on."""
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
    quota, quota_cpus = None, None
    try:  # cgroup v2: "<quota> <period>" or "max <period>"
        quota = open("/sys/fs/cgroup/cpu.max").read().strip()
        q, per = quota.split()[:2]
        if q != "max":
            quota_cpus = max(1, int(q) // int(per))
    except (OSError, ValueError):
        try:  # cgroup v1
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            quota = f"{q} {per}"
            if q > 0:
                quota_cpus = max(1, q // per)
        except (OSError, ValueError):
            pass
    nodes = {}
    try:
        base = "/sys/devices/system/node"
        for d in sorted(os.listdir(base)):
            if d.startswith("node") and d[4:].isdigit():
                nodes[d] = open(os.path.join(base, d, "cpulist")).read().strip()
    except OSError:
        pass
    return {"model": model, "logical_cpus": os.cpu_count(), "cpus_allowed": allowed,
            "cgroup_cpu_max": quota, "cgroup_quota_cpus": quota_cpus, "numa_nodes": nodes or None}


def resolve_world(gpus, world_env) -> tuple:
    """(world size, whether bench.py must start the ranks itself).

    Under torchrun WORLD_SIZE is set and must equal --gpus when both are
    given; without it, --gpus N > 1 means this process spawns N ranks."""
    if world_env is not None:
        world = int(world_env)
        if gpus is not None and gpus != world:
            raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}; they must agree")
        return world, False
    n = 1 if gpus is None else int(gpus)
    if n < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    return n, n > 1


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def rank_env(base: dict, rank: int, world: int, port: int) -> dict:
    env = dict(base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                "MASTER_PORT": str(port)})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def spawn_ranks(world: int, argv: list) -> int:
    """Start `world` fresh bench.py processes (one per GPU) and wait for them.

    Rank 0 prints the JSON line; the exit code is the first non-zero child
    code.  A failed rank stops the others (by their exact PIDs)."""
    import subprocess
    port = free_port()
    cmd = [sys.executable, os.path.abspath(__file__)] + list(argv)
    procs = [subprocess.Popen(cmd, env=rank_env(os.environ, r, world, port)) for r in range(world)]
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 1
                    for q in pending:
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without WORLD_SIZE in the env, bench.py starts them itself")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=None, choices=[2, 3, 4, 5],
                    help="SURVEY 8(d) config; default 3 at one rank, 5 (its per-GPU shard) at N>1")
    ap.add_argument("--buffers-per-gpu", type=int, default=None,
                    help="configs 3/5: override the per-GPU buffer count (rehearsals with ranks sharing a GPU)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="N=1 config 3: skip the configs 2 and 4 timed after the headline")
    ap.add_argument("--collective", action="store_true",
                    help="init the process group and gather the CRCs even at one rank (exercises the "
                         "RCCL path on a one-GPU box: init_process_group, all_gather on the device)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (default); gloo only to rehearse ranks sharing one GPU")
    ap.add_argument("--cpu-budget-s", type=float, default=None,
                    help="CPU-baseline wall-clock budget (default 12 s at one rank, 24 s at N > 1)")
    ap.add_argument("--cpu-sample-gib", type=float, default=None,
                    help="host-resident CPU-baseline sample, >= 2x the host L3 (default 4 GiB at one rank; "
                         "16 GiB of config 5 at N > 1, SURVEY 8(d))")
    ap.add_argument("--no-read-ceiling", action="store_true",
                    help="skip the same-process read ceiling (profiling runs: only the product kernel launches)")
    ap.add_argument("--host-resident-gib", type=float, default=4.0,
                    help="configs 3/5: host-resident zcrc32_batch over this many GiB of the workload's buffers "
                         "(0: skip); at N > 1 rank 0 runs it over every visible GPU")
    ap.add_argument("--pmc-traffic-bytes", type=float, default=None,
                    help="HBM bytes per launch from a separate rocprofv3 --pmc pass (corrected)")
    args = ap.parse_args()
    world, spawn_needed = resolve_world(args.gpus, os.environ.get("WORLD_SIZE"))
    if spawn_needed:
        # no launcher: start the ranks here, before this process touches torch
        # or the GPU (children are fresh interpreters, never an exec of this one)
        sys.exit(spawn_ranks(world, sys.argv[1:]))
    if args.config is None:
        args.config = 3 if world == 1 else 5

    import torch
    import torch.distributed as dist
    import zipsfs_amd as z
    from zipsfs_amd import shard

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()  # does not initialise the GPU on this image
    if world > 1 and args.dist_backend == "nccl" and world > ndev:
        raise SystemExit(f"bench.py: {world} ranks over RCCL need {world} GPUs, {ndev} visible "
                         "(--dist-backend gloo rehearses ranks sharing a GPU)")
    gpu = local % max(ndev, 1)
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    use_dist = world > 1 or args.collective
    if use_dist:
        if world == 1:  # --collective without a launcher: a one-rank group on 127.0.0.1
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(free_port()))
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    def barrier():
        if use_dist:
            if args.dist_backend == "nccl":
                dist.barrier(device_ids=[gpu])
            else:
                dist.barrier()

    def measure(cfg: int, steps: int, warmup: int, n_override=None, extra=None) -> dict:
        """Warmup, then exactly `steps` timed steps between barriers and
        synchronizes (max over ranks), then a parity spot-check, then (outside
        the timed region) the same-shape read ceiling and `extra(wl, crcs)`."""
        wl = Workload(cfg, rank, world, dev, n_override)
        out = torch.empty(wl.n_local, dtype=torch.int32, device=dev)
        result = {"global": out}

        def step(s: int) -> None:
            ptrs, lens = wl.batches[s % len(wl.batches)]
            z.crc32_batch_device(ptrs, lens, out=out)
            if use_dist:  # the one exchange: all-gather of the 32-bit CRCs
                result["global"] = shard.gather_crcs(out, wl.n_total)

        for s in range(warmup):
            step(s)
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        # Kernel time: one HIP event pair on the stream the launches go to
        # (torch's current stream), bracketing the timed steps -- GPU time per
        # step / CRC launches per step.  Back-to-back launches leave no gap on
        # the stream (rocprofv3 kernel trace: end-to-next-start 0 us), so this
        # is the average launch duration; when a plan kernel precedes the CRC
        # launch (n > 8192) its few us are counted in too (conservative).
        # Events on every launch (hipExtLaunchKernel; ZCRC_BENCH_KERNEL_EVENTS=1
        # restores them) left a ~10 us bubble before each launch: config 2
        # stepped at 54.9 us instead of 51.2 (profiles/r03/s2).
        per_launch = os.environ.get("ZCRC_BENCH_KERNEL_EVENTS") == "1"
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        with (z.profile() if per_launch else _NoProfile()) as prof:
            t0 = time.perf_counter()
            ev0.record()
            for s in range(steps):
                step(warmup + s)
            ev1.record()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
        barrier()
        elapsed = t1 - t0
        if per_launch:
            avg_kernel_ms, launches, timing = prof.total_ms / max(prof.launches, 1), prof.launches, \
                "HIP events on every CRC launch (hipExtLaunchKernel)"
        else:
            avg_kernel_ms, launches, timing = ev0.elapsed_time(ev1) / steps, steps, \
                "one HIP event pair on the launch stream around the timed steps / launches"
        if use_dist:
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
        gathered_on = str(result["global"].device)
        glob = result["global"].cpu().numpy().view(np.uint32)
        parity = golden_check(cfg, glob) if rank == 0 else None
        try:  # measurement beside the line's numbers: never fails the run
            ceiling = (read_ceiling(wl, out, steps) if not args.no_read_ceiling else
                       {"skipped": "--no-read-ceiling", "read_ceiling_gbs": None})
        except Exception as e:
            ceiling = {"error": f"{type(e).__name__}: {e}", "read_ceiling_gbs": None}
        extra_res = extra(wl, out.cpu().numpy().view(np.uint32)) if extra else None
        per_rank = rank_spread(avg_kernel_ms, ceiling) if use_dist else None
        # the device path runs in one batch-kernel launch per step (the split
        # plan's small list, when it splits, runs inside it: zcrc_kernels.hip)
        res = {"wl_desc": wl.desc, "n_local": wl.n_local, "kernel": z.kernel_name_for(wl.n_local),
               "bytes_local": wl.bytes_local, "elapsed": elapsed, "bytes_all": bytes_all,
               "avg_kernel_ms": avg_kernel_ms, "kernel_timing": timing, "launches": launches, "parity": parity,
               "gathered_on": gathered_on, "bytes_main": wl.bytes_local, "small": None, "ceiling": ceiling,
               "extra": extra_res, "per_rank": per_rank}
        del wl, out, result
        torch.cuda.empty_cache()
        return res

    def rank_spread(avg_kernel_ms: float, ceiling: dict) -> dict:
        """Min/max over ranks of each rank's own kernel time and read ceilings
        (VERDICT r5 next #1): a straggling GPU shows in the one line rank 0
        prints.  One all_gather of 3 float64 per rank."""
        rdev = dev if args.dist_backend == "nccl" else torch.device("cpu")
        nan = float("nan")
        mine = torch.tensor([avg_kernel_ms, ceiling.get("read_ceiling_gbs") or nan,
                             ceiling.get("stream_read_gbs") or nan], dtype=torch.float64, device=rdev)
        allr = torch.empty(world * 3, dtype=torch.float64, device=rdev)
        dist.all_gather_into_tensor(allr, mine)
        a = allr.cpu().numpy().reshape(world, 3)
        out = {}
        for j, key in enumerate(("avg_kernel_ms", "read_ceiling_gbs", "stream_read_gbs")):
            col = a[:, j]
            if np.isnan(col).all():
                out[key] = None
                continue
            out[key] = {"min": round(float(np.nanmin(col)), 4), "max": round(float(np.nanmax(col)), 4),
                        "argmin_rank": int(np.nanargmin(col)), "argmax_rank": int(np.nanargmax(col))}
        return out

    def read_ceiling(wl, out, steps: int) -> dict:
        """Two ceilings over the same bytes, interleaved with the CRC in one
        process: 3 rounds of k CRC launches,
        k launches of the same-shape ceiling (zcrc32_batch_device_read_ceiling:
        the same plan, workgroups, loads and fold, one VALU op per dword
        instead of the table lookups) and k plain stream reads of the batch's
        contiguous region (zcrc_read_sweep_device: one grid-stride sweep, no
        per-buffer structure -- the chip's stream-read peak on these bytes),
        each block timed by one HIP event pair on the launch stream, medians.
        same-shape / stream-read is the access pattern's own loss; CRC /
        same-shape what the CRC costs over its loads.  Ratios measured minutes
        apart in one process make an A/B independent of the box's HBM rate."""
        k = max(5, steps // 2)
        sink = torch.empty(max(out.numel(), 1024), dtype=torch.int32, device=out.device)

        def block(fn) -> float:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for s in range(k):
                b = s % len(wl.batches)
                fn(b)
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / k

        crc = lambda b: z.crc32_batch_device(*wl.batches[b], out=sink[:wl.n_local])
        ceil = lambda b: z.batch_device_read_ceiling(*wl.batches[b], out=sink[:wl.n_local])
        sweep = lambda b: z.read_sweep_device(wl.regions[b][0], wl.regions[b][1], sink)
        block(ceil)  # warm both measurement kernels' code objects
        block(sweep)
        rounds = [(block(crc), block(ceil), block(sweep)) for _ in range(3)]
        crc_ms = float(np.median([a for a, _, _ in rounds]))
        ceil_ms = float(np.median([b for _, b, _ in rounds]))
        sweep_ms = float(np.median([c for _, _, c in rounds]))
        region = float(np.mean([r[1] for r in wl.regions]))
        gbs = wl.bytes_local / (ceil_ms * 1e-3) / 1e9
        sgbs = region / (sweep_ms * 1e-3) / 1e9
        return {"read_ceiling_gbs": round(gbs, 1), "ceiling_ms": round(ceil_ms, 4),
                "stream_read_gbs": round(sgbs, 1), "stream_read_ms": round(sweep_ms, 4),
                "stream_read_bytes": int(region),
                "ceiling_frac_of_stream_read": round(gbs / sgbs, 4),
                "crc_ms_interleaved": round(crc_ms, 4), "frac_of_ceiling_interleaved": round(ceil_ms / crc_ms, 4),
                "frac_of_stream_read_interleaved": round((wl.bytes_local / (crc_ms * 1e-3) / 1e9) / sgbs, 4),
                "rounds_ms": [[round(a, 4), round(b, 4), round(c, 4)] for a, b, c in rounds],
                "launches_per_block": k,
                "method": "3 interleaved rounds of k CRC launches, k same-shape read-ceiling launches "
                          "(zcrc32_batch_device_read_ceiling: same plan, loads and fold, table lookups "
                          "replaced by one VALU op) and k stream reads of the batch's contiguous region "
                          "(zcrc_read_sweep_device: grid-stride sweep, 1024-thread workgroup per CU, nt 16-B "
                          "loads), HIP events per block, medians"}

    def host_resident(wl, crcs, n_host: int, reps: int) -> dict:
        """SURVEY 8(d)/north_star: the path starts and ends in host memory.
        zcrc32_batch over n_host x 1 MiB config-3 buffers in pageable host
        memory (copied out of the workload), i.e. the library's pinned staging
        and PCIe transfer included, over the device set (ZCRC_DEVICES, default
        every visible GPU); results checked against the device path's CRCs of
        the same buffers (themselves checked against the golden vectors)."""
        import ctypes
        try:
            L = 1 << 20
            n_host = min(n_host, wl.n_local)
            host = wl.mem[0][: n_host * L].cpu()  # pageable, like ZIPsFS's preload buffers
            ptrs = np.arange(n_host, dtype=np.uint64) * np.uint64(L) + np.uint64(host.data_ptr())
            lens = np.full(n_host, L, dtype=np.uint64)
            res = np.zeros(n_host, dtype=np.uint32)
            lib = z.lib()

            def run() -> None:
                rc = lib.zcrc32_batch(ptrs.ctypes.data, lens.ctypes.data, None, res.ctypes.data, n_host, 0)
                if rc:
                    raise RuntimeError(f"zcrc32_batch failed ({rc}): {lib.zcrc_last_error().decode()}")

            run()  # warm: staging slots, device set
            t = []
            for _ in range(reps):
                res[:] = 0
                t0 = time.perf_counter()
                run()
                t.append(time.perf_counter() - t0)
            bad = int((res != crcs[:n_host]).sum())
            devs = z.device_set()
            st = z.staging_info()
            out = {"value": round(n_host * L / float(np.median(t)) / GiB, 2), "unit": "GiB/s",
                   "bytes_per_call": n_host * L, "reps": reps, "seconds": [round(x, 4) for x in t],
                   "devices": devs, "bytes_per_device": n_host * L // max(1, len(devs)),
                   "parity": (f"{n_host - bad}/{n_host} equal the device path's CRCs of the same buffers"),
                   "staging": st,
                   "api": "zcrc32_batch (host pointers; pinned staging + PCIe inside, zero-copy kernel reads)"}
            if bad:
                out["error"] = f"{bad} CRCs differ from the device path"
            del host
            return out
        except Exception as e:  # reported in the line, never failing the run
            return {"error": f"{type(e).__name__}: {e}"}

    def pmc_traffic(cfg: int, bytes_local: int):
        """PMC traffic per launch recorded for this workload AND these kernel
        sources (tools/collect_profiles.sh -> profiles/pmc_traffic.json)."""
        path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if not os.path.exists(path):
            return None, None
        pm = json.load(open(path)).get(str(cfg))
        if (pm and pm.get("bytes_per_gpu_per_step") == bytes_local
                and pm.get("kernel_source_hash") == z.kernel_source_hash()):
            return pm["traffic_bytes_per_launch"], pm["source"]
        return None, None

    def small_batches() -> dict:
        """Uniform batches of small buffers -- the ZIP-entry regime (config 4's
        median entry is 3,971 B): 1 GiB of L-byte
        buffers (buffer i = payload(L, i)), two batches rotated, through
        zcrc32_batch_device (no bound: the split plan's two scans and the CRC
        launch), zcrc32_batch_device_maxlen (the caller's bound L: one launch)
        and zcrc32_batch_device_strided; k calls per API between one HIP event
        pair queued behind >= 15 ms of warm calls, the stream read of the same region
        beside them; every API's results checked against reference-generated
        samples (tests/golden/small.npz) and against each other."""
        g = np.load(os.path.join(ROOT, "tests", "golden", "small.npz"))
        res = {}
        for L in (1024, 4096):
            n = (1 << 30) // L
            bat = []
            for b in range(2):
                mem = torch.empty(n * L + 64, dtype=torch.uint8, device=dev)
                ptrs = mem.data_ptr() + torch.arange(n, dtype=torch.int64, device=dev) * L
                lens = torch.full((n,), L, dtype=torch.int64, device=dev)
                z.fill_synthetic(ptrs, lens, index0=b * n, seed=PAYLOAD_SEED)
                bat.append((mem, ptrs, lens, torch.empty(n, dtype=torch.int32, device=dev)))
            sink = torch.empty(1024, dtype=torch.int32, device=dev)
            apis = {
                "device": lambda b: z.crc32_batch_device(bat[b][1], bat[b][2], out=bat[b][3]),
                "device_maxlen": lambda b: z.crc32_batch_device(bat[b][1], bat[b][2], out=bat[b][3], max_len=L),
                "strided": lambda b: z.crc32_batch_strided(bat[b][0], L, L, n, out=bat[b][3]),
                "stream_read": lambda b: z.read_sweep_device(bat[b][0].data_ptr(), n * L, sink),
            }
            idx = g[f"len{L}_idx"].astype(np.int64)
            first = None
            row = {"buffers": n, "bytes_per_call": n * L}
            # timed back to back, the parity checks after all of them: an idle
            # GPU between blocks (a host-side check) left the next block's
            # calls up to 15% slower after 40 warm calls (session 15:
            # tools/small_timing_ab.py agrees with tools/small_batches.py once
            # the blocks follow each other)
            for name, fn in apis.items():
                for s in range(100):  # >= 15 ms of work in front of the timed calls
                    fn(s % 2)
                k = 40
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for s in range(k):
                    fn(s % 2)
                e1.record()
                e1.synchronize()
                ms = e0.elapsed_time(e1) / k
                row[f"{name}_us_per_call"] = round(ms * 1e3, 1)
                row[f"{name}_tbs"] = round(n * L / (ms * 1e-3) / 1e12, 3)
            for name, fn in apis.items():
                if name == "stream_read":
                    continue
                fn(0)
                torch.cuda.synchronize()
                got = bat[0][3].cpu().numpy().view(np.uint32)
                ok = int((got[idx] == g[f"len{L}"]).sum())
                if ok != len(idx) or (first is not None and not np.array_equal(got, first)):
                    raise SystemExit(f"PARITY FAILURE: small buffers {L} B through {name}: "
                                     f"{len(idx) - ok} of {len(idx)} samples differ, or differs from another API")
                first = got.copy() if first is None else first
            for name in ("device", "device_maxlen", "strided"):
                row[f"{name}_frac_of_stream_read"] = round(row[f"{name}_tbs"] / row["stream_read_tbs"], 4)
            row["parity"] = (f"{len(idx)}/{len(idx)} reference samples equal on every API; the three APIs' "
                             f"{n} results equal")
            res[f"len{L}"] = row
            del bat, sink
            torch.cuda.empty_cache()
        res["method"] = ("uniform L-byte buffers, 2 x 1 GiB batches rotated, k = 40 calls per API between one "
                         "HIP event pair on the launch stream, queued behind 100 warm calls; device = zcrc32_batch_device "
                         "(split plan: 2 scan kernels + the CRC launch), device_maxlen = "
                         "zcrc32_batch_device_maxlen(max_len = L) (one small-kernel launch), strided = "
                         "zcrc32_batch_device_strided; stream_read = zcrc_read_sweep_device over the batch")
        return res

    host_extra = None
    if args.config in (3, 5) and args.host_resident_gib > 0:
        n_host = int(args.host_resident_gib * 1024)
        if world == 1:
            host_extra = lambda wl, crcs: host_resident(wl, crcs, n_host, 3)
        else:
            # N > 1: after the timed steps, rank 0 alone runs a host batch over
            # every visible GPU (the in-process device set, ZIPsFS's one
            # process) while the other ranks wait
            def host_extra(wl, crcs):
                r = host_resident(wl, crcs, n_host, 3) if rank == 0 else None
                barrier()
                return r
    m = measure(args.config, args.steps, args.warmup, args.buffers_per_gpu, extra=host_extra)
    elapsed, bytes_all = m["elapsed"], m["bytes_all"]

    class _WL:  # the headline workload's figures, for the line below
        desc, n_local, bytes_local = m["wl_desc"], m["n_local"], m["bytes_local"]
    wl = _WL()
    parity = m["parity"]

    # Secondary configs (N = 1 only): SURVEY 8(d) configs 2 and 4, timed the
    # same way in the same run, so that they too carry the driver's clock, and
    # uniform batches of 1 KiB / 4 KiB buffers through the three device APIs.
    secondary = None
    if world == 1 and args.config == 3 and not args.no_secondary:
        secondary = {}
        for c in (2, 4):
            # config 2's 50 us steps: 200 of them, so that the first launch's
            # latency (~30 us) does not weigh on the per-step figure, behind
            # >= 20 ms of untimed warmup (3 warmup steps left the timed steps
            # 2-3 us slower than the same launches a few ms later, in the read
            # ceiling's pairs: profiles/r05/s4, s7)
            ks = max(args.steps, 200 if c == 2 else 20)
            r = measure(c, ks, max(args.warmup, 400 if c == 2 else 10))
            ach = r["bytes_main"] / (r["avg_kernel_ms"] * 1e-3) / 1e9
            tr, _ = pmc_traffic(c, r["bytes_local"])
            ce = r["ceiling"]
            secondary[f"config{c}"] = {
                "workload": r["wl_desc"], "value": round(r["bytes_all"] * ks / r["elapsed"] / GiB, 2),
                "read_ceiling_gbs": ce["read_ceiling_gbs"],
                "frac_of_ceiling": round(ach / ce["read_ceiling_gbs"], 4) if ce["read_ceiling_gbs"] else None,
                "stream_read_gbs": ce.get("stream_read_gbs"),
                "frac_of_stream_read": round(ach / ce["stream_read_gbs"], 4) if ce.get("stream_read_gbs") else None,
                "read_ceiling": ce,
                "unit": "GiB/s", "steps": ks, "ms_per_step": round(r["elapsed"] / ks * 1e3, 4),
                "avg_kernel_ms": round(r["avg_kernel_ms"], 4), "achieved": round(ach, 1),
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None if tr is None else int(tr),
                "algorithmic_bytes_per_launch": r["bytes_main"], "kernel": r["kernel"], "small_kernel": r["small"],
                "parity": r["parity"]}

        try:
            secondary["small_buffers"] = small_batches()
        except SystemExit:
            raise
        except Exception as e:  # measurement beside the line: reported, never failing the run
            secondary["small_buffers"] = {"error": f"{type(e).__name__}: {e}"}

    if m["extra"] is not None:  # host-resident rate (N = 1) / host batch over the device set (N > 1)
        secondary = secondary or {}
        secondary["host_resident" if world == 1 else "host_multi_device"] = m["extra"]

    ms_per_step = elapsed / args.steps * 1e3
    value = bytes_all * args.steps / elapsed / GiB
    avg_kernel_ms = m["avg_kernel_ms"]
    achieved = m["bytes_main"] / (avg_kernel_ms * 1e-3) / 1e9
    traffic = args.pmc_traffic_bytes
    traffic_src = "--pmc-traffic-bytes" if traffic is not None else None
    if traffic is None:
        traffic, traffic_src = pmc_traffic(args.config, wl.bytes_local)
    if use_dist:
        # every rank's GPU work is done: leave the group, so that rank 0's CPU
        # baseline below runs with the other ranks gone (no rank polling a
        # barrier on the host cores it measures)
        barrier()
        dist.destroy_process_group()
        use_dist_done = True
    else:
        use_dist_done = False
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        # N > 1 too: the reference timed on this box's
        # host cores in the same run, over a fixed config-5 subset (SURVEY 8(d):
        # 16 GiB by default at N > 1 -- global buffers 0 .. 16383)
        sample_gib = args.cpu_sample_gib if args.cpu_sample_gib is not None else (4.0 if world == 1 else 16.0)
        budget = args.cpu_budget_s if args.cpu_budget_s is not None else (12.0 if world == 1 else 24.0)
        cpu = cpu_baseline(args.config, budget, sample_gib)

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
                "api": ("zcrc32_batch_device (one persistent CRC launch, lengths scanned in-kernel)"
                        if m["kernel"] != z.kernel_name() else
                        "zcrc32_batch_device (plan scan + persistent CRC kernel)") +
                       (f" + {'RCCL' if args.dist_backend == 'nccl' else 'gloo'} all_gather of uint32 CRCs"
                        if use_dist else ""),
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
                "algorithmic_bytes_per_launch": m["bytes_main"],
                "kernel": m["kernel"],
                "kernel_source_hash": z.kernel_source_hash(),
                "avg_kernel_ms": round(avg_kernel_ms, 4),
                "launches_timed": m["launches"],
                "kernel_timing": m["kernel_timing"],
                "small_kernel": m["small"],
                "read_ceiling_gbs": m["ceiling"]["read_ceiling_gbs"],
                "frac_of_ceiling": (round(achieved / m["ceiling"]["read_ceiling_gbs"], 4)
                                    if m["ceiling"]["read_ceiling_gbs"] else None),
                "stream_read_gbs": m["ceiling"].get("stream_read_gbs"),
                "frac_of_stream_read": (round(achieved / m["ceiling"]["stream_read_gbs"], 4)
                                        if m["ceiling"].get("stream_read_gbs") else None),
                "read_ceiling": m["ceiling"],
                "per_rank": m["per_rank"],
            },
            "cpu_baseline": cpu,
            "parity": parity,
            "collective": None if not use_dist else {
                "backend": "RCCL" if args.dist_backend == "nccl" else "gloo", "ranks": world,
                "op": "all_gather_into_tensor of the int32 CRCs (zipsfs_amd/shard.py)",
                "results_on": m["gathered_on"]},
            "secondary": secondary,
            "device": torch.cuda.get_device_name(dev),
        }
        print(json.dumps(line), flush=True)
    if use_dist and not use_dist_done:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
