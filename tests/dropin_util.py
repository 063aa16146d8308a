"""Builds and feeds tests/dropin/dropin_main.c, ZIPsFS's cg_crc32 call site
compiled against the drop-in (zipsfs_amd/cg_crc32.c + libzcrc).

Records carry the reference-generated golden CRCs (tests/golden/) as the
expected central-directory value; their bytes are the fixtures' inputs
(KAT strings, the counter-based payload), regenerated here by the test-side
oracle."""
from __future__ import annotations

import json
import os
import struct
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
BIG = 40 << 20  # above the drop-in's default GPU threshold
DEFAULT_GPU_MIN = 4 << 20  # zcrc_runtime.hip kDefaultGpuMinBytes


def build_harness(tmp_path) -> str:
    exe = os.path.join(str(tmp_path), "dropin_main")
    cmd = ["gcc", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "zipsfs_amd"), "-I",
           os.path.join(ROOT, "include"), os.path.join(HERE, "dropin", "dropin_main.c"), "-o", exe,
           "-L", os.path.join(ROOT, "zipsfs_amd"), "-lzcrc", "-Wl,-rpath," + os.path.join(ROOT, "zipsfs_amd"),
           "-pthread"]
    subprocess.run(cmd, check=True)
    return exe


def golden_records(big: bool = True) -> list:
    """[(bytes, expected crc, seed)] from the golden fixtures."""
    from oracle import oracle as o  # test-side input generator only
    meta = json.load(open(os.path.join(HERE, "golden", "golden.json")))
    recs = []
    for k in meta["kats"]:
        if "hex" in k:
            data = bytes.fromhex(k["hex"])
        else:
            a, b = k["text_seq"]
            data = "".join(f"{i}\n" for i in range(a, b + 1)).encode()
        recs.append((data, k["crc"], 0))
    lo = np.load(os.path.join(HERE, "golden", "lengths_offsets.npz"))
    base = o.payload(int(lo["payload_len"]), int(lo["payload_index"])).tobytes()
    lengths = lo["lengths"]
    for a in range(0, len(lengths), 37):
        for off in (0, 3, 8, 13):
            L = int(lengths[a])
            recs.append((base[off:off + L], int(lo["crc"][a, off]), 0))
    for c in meta["chains"][:40]:  # cg_crc32(data, n, seed): the chaining form
        recs.append((o.payload(c["len"], c["index"]).tobytes(), c["crc"], c["seed"]))
    c1 = meta["config1"]
    recs.append((o.payload(c1["len"], c1["index"]).tobytes(), c1["crc"], 0))
    if big:
        recs.append((o.payload(BIG, 3).tobytes(), o.payload_crc(BIG, 3), 0))
    return recs


def write_records(path, recs) -> None:
    with open(path, "wb") as f:
        for data, crc, seed in recs:
            f.write(struct.pack("<QII", len(data), crc & 0xFFFFFFFF, seed & 0xFFFFFFFF))
            f.write(data)


def run_harness(exe, records_path, env_extra=None) -> tuple:
    """-> (returncode, [(index, crc, ok)], stats dict, stderr)."""
    env = dict(os.environ)
    env.update(env_extra or {})
    p = subprocess.run([exe, str(records_path)], capture_output=True, text=True, env=env, timeout=300)
    rows, stats = [], {}
    for line in p.stdout.splitlines():
        if line.startswith("stats "):
            stats = {k: int(v) for k, v in (kv.split("=") for kv in line.split()[1:])}
        else:
            i, crc, st = line.split()
            rows.append((int(i), int(crc, 16), st == "ok"))
    return p.returncode, rows, stats, p.stderr


def build_preload_harness(tmp_path) -> str:
    """tests/dropin/preload_main.c: preloadram_now's read loop + the CRC check."""
    exe = os.path.join(str(tmp_path), "preload_main")
    cmd = ["gcc", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "zipsfs_amd"), "-I",
           os.path.join(ROOT, "include"), os.path.join(HERE, "dropin", "preload_main.c"), "-o", exe,
           "-L", os.path.join(ROOT, "zipsfs_amd"), "-lzcrc", "-Wl,-rpath," + os.path.join(ROOT, "zipsfs_amd"),
           "-pthread", "-ldl", "-lz"]
    subprocess.run(cmd, check=True)
    return exe


REF_O0 = os.path.join(ROOT, "oracle", "_ref", "libref_cg_crc32_O0.so")


def run_preload(exe, entry_path, expected, reps, modes, env_extra=None) -> tuple:
    """-> (returncode, {mode: row}, stats, stderr)."""
    env = dict(os.environ)
    env["ZCRC_REF_LIB"] = REF_O0
    env.update(env_extra or {})
    p = subprocess.run([exe, str(entry_path), f"{expected & 0xFFFFFFFF:08x}", str(reps)] + list(modes),
                       capture_output=True, text=True, env=env, timeout=600)
    rows, stats = {}, {}
    for line in p.stdout.splitlines():
        d = json.loads(line)
        if "stats" in d:
            stats = d["stats"]
        else:
            rows[d["mode"]] = d
    return p.returncode, rows, stats, p.stderr
