"""C-ABI boundary checks that need no GPU: libzcrc loads, exports every
function include/zcrc.h declares, the host-only GF(2) combine is right, the
drop-in cg_crc32.c compiles as C and C++ against the header, and the product
package contains no CPU CRC path."""
import os
import random
import subprocess
import zlib

import pytest

import zipsfs_amd
from zipsfs_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_header_symbols():
    names = _lib.exported_symbols_from_header()
    assert "zcrc32" in names and "zcrc32_batch_device" in names
    lib = _lib.lib()
    for n in names:
        assert hasattr(lib, n), n
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines()}
    assert set(names) <= exported


def test_hip_symbols_resolve_against_torch_runtime():
    """libzcrc is loaded next to PyTorch's bundled libamdhip64 (ROCm 7.0):
    every versioned HIP symbol it imports must exist there (a hip_7.1-only
    call made the library fail to load on the GPU box)."""
    import re
    torch = pytest.importorskip("torch")
    hip = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
    if not os.path.exists(hip):
        pytest.skip("no bundled libamdhip64")
    need = subprocess.run(["objdump", "-T", _lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    have = subprocess.run(["objdump", "-T", hip], capture_output=True, text=True, check=True).stdout
    have_syms = {(m.group(1), m.group(2)) for m in re.finditer(r"\(?(hip_[0-9.]+)\)?\s+(\w+)$", have, re.M)}
    und = list(re.finditer(r"\*UND\*\s+\S+\s+\(?(hip_[0-9.]+)\)?\s+(\w+)$", need, re.M))
    assert len(und) > 10, "objdump format not understood"
    for m in und:
        assert (m.group(1), m.group(2)) in have_syms, f"{m.group(2)}@{m.group(1)} missing from torch's HIP runtime"


def test_combine_matches_zlib():
    rnd = random.Random(1)
    for _ in range(200):
        a = bytes(rnd.getrandbits(8) for _ in range(rnd.randint(0, 300)))
        b = bytes(rnd.getrandbits(8) for _ in range(rnd.randint(0, 300)))
        assert zipsfs_amd.crc32_combine(zlib.crc32(a), zlib.crc32(b), len(b)) == zlib.crc32(a + b)
    # large length: combine with 2^40 zero bytes is consistent with repeated squaring
    z = zipsfs_amd.crc32_combine(0x12345678, 0, 1 << 40)
    assert isinstance(z, int)


def test_version_and_gfx950_only():
    assert "gfx950" in zipsfs_amd.version()


@pytest.mark.parametrize("compiler,lang", [("gcc", "c"), ("g++", "c++")])
def test_dropin_compiles(tmp_path, compiler, lang):
    src = tmp_path / ("main.c" if lang == "c" else "main.cpp")
    src.write_text(
        '#include "cg_crc32.c"\n'
        "#include <stdio.h>\n"
        "int main(void){ pthread_mutex_t m = PTHREAD_MUTEX_INITIALIZER;\n"
        '  printf("%08x\\n", cg_crc32("123456789", 9, 0, &m)); return 0; }\n')
    exe = tmp_path / "a.out"
    cmd = [compiler, "-Wall", "-Werror", "-I", os.path.join(ROOT, "zipsfs_amd"), "-I", os.path.join(ROOT, "include"),
           str(src), "-o", str(exe), "-L", os.path.join(ROOT, "zipsfs_amd"), "-lzcrc",
           "-Wl,-rpath," + os.path.join(ROOT, "zipsfs_amd"), "-pthread"]
    subprocess.run(cmd, check=True)
    assert exe.exists()


def test_product_has_no_cpu_crc_path():
    """The shipped package must not import the oracle or compute CRCs on the CPU.

    Source files may not reference the oracle or the reference build; Python
    modules may import zlib only for inflate and never call a zlib/binascii
    checksum (AST check).  The C library's one host CRC (zcrc_host.cpp) is
    reachable only from the drop-in zcrc32(): no other source
    calls host_crc32."""
    import ast
    pkg = os.path.join(ROOT, "zipsfs_amd")
    banned_attrs = {"crc32", "adler32", "crc_hqx", "crc32_combine"}
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            path = os.path.join(dirpath, f)
            if not f.endswith((".py", ".hip", ".h", ".c", ".cpp")):
                continue
            text = open(path).read()
            for bad in ("from oracle", "import oracle", "liboracle", "libref_cg_crc32", "crc32_port", "binascii"):
                assert bad not in text, (f, bad)
            if f.endswith(".py"):
                tree = ast.parse(text)
                aliases = set()
                for node in ast.walk(tree):
                    if isinstance(node, ast.Import):
                        for a in node.names:
                            if a.name in ("zlib", "binascii"):
                                aliases.add(a.asname or a.name)
                    if isinstance(node, ast.ImportFrom) and node.module in ("zlib", "binascii"):
                        for a in node.names:
                            assert a.name not in banned_attrs, (f, a.name)
                for node in ast.walk(tree):
                    if isinstance(node, ast.Attribute) and isinstance(node.value, ast.Name):
                        if node.value.id in aliases:
                            assert node.attr not in banned_attrs, (f, node.attr)
    callers = {}
    csrc = os.path.join(pkg, "csrc")
    for f in os.listdir(csrc):
        if f.endswith((".hip", ".h", ".cpp")):
            text = "\n".join(l.split("//")[0] for l in open(os.path.join(csrc, f)).read().splitlines())
            if "host_crc32(" in text:
                callers[f] = text
    assert set(callers) == {"zcrc_host.cpp", "zcrc_internal.h", "zcrc_runtime.hip"}, sorted(callers)
    rt = callers["zcrc_runtime.hip"]
    body = rt[rt.index("uint32_t zcrc32(const void *data"):]
    body = body[:body.index("\n}\n")]
    # below threshold or no device; every staging slot busy; GPU failure
    assert rt.count("host_crc32(") == body.count("host_crc32(") == 3


def test_missing_gpu_fails_loudly():
    """Without a device the API raises; it never answers from the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(zipsfs_amd.ZcrcError):
        zipsfs_amd.cg_crc32(b"123456789")


REF_SRC = "/root/reference/src"


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_SRC, "cg_crc32.c")), reason="reference tree absent")
def test_dropin_shadows_reference(tmp_path):
    """INTEGRATION.md recipe: -include the drop-in ahead of a TU that does
    `#include "cg_crc32.c"` from the reference's own src/; the reference body
    must vanish behind the shared include guard and the call go to zcrc32."""
    tu = tmp_path / "tu.c"
    tu.write_text('#include "cg_crc32.c"\n'
                  "uint32_t check(const void *p, size_t n) { return cg_crc32(p, n, 0, NULL); }\n")
    obj = tmp_path / "tu.o"
    subprocess.run(["gcc", "-c", "-O0", "-I", REF_SRC, "-I", os.path.join(ROOT, "include"),
                    "-include", os.path.join(ROOT, "zipsfs_amd", "cg_crc32.c"), str(tu), "-o", str(obj)], check=True)
    syms = subprocess.run(["nm", str(obj)], capture_output=True, text=True, check=True).stdout
    assert " U zcrc32" in syms
    assert "crc32_for_byte" not in syms and "cg_crc32_init_tables" not in syms


def test_argument_errors_are_reported_not_computed():
    """Invalid arguments return ZCRC_ERR_ARG (-2) before any device work."""
    import ctypes
    lib = _lib.lib()
    assert lib.zcrc32_batch_device(None, None, None, None, 5, None) == -2
    assert lib.zcrc32_batch(None, None, None, None, 3, 0) == -2
    assert lib.zcrc32_batch_device(None, None, None, None, 0, None) == 0  # empty batch: nothing to do
    # the caller-bound form: its one-launch route and the unhinted one check alike
    assert lib.zcrc32_batch_device_maxlen(None, None, None, None, 9000, 1024, None) == -2
    assert lib.zcrc32_batch_device_maxlen(None, None, None, None, 5, 1024, None) == -2
    assert lib.zcrc32_batch_device_maxlen(None, None, None, None, 9000, 0, None) == -2
    # the stream-read measurement: null, misaligned (checked before any device work), empty
    assert lib.zcrc_read_sweep_device(None, 4096, None, None) == -2
    assert lib.zcrc_read_sweep_device(ctypes.c_void_p(0x1008), 4096, ctypes.c_void_p(0x2000), None) == -2
    assert b"aligned" in lib.zcrc_last_error()
    assert lib.zcrc_read_sweep_device(None, 0, None, None) == 0
    out = ctypes.c_uint32()
    assert lib.zcrc32_checked(None, 10, 0, ctypes.byref(out)) == -2
    assert b"null" in lib.zcrc_last_error()
    assert lib.zcrc32_batch_device_scratch_bytes(8192) == 256 + 8 * 8193 + 8  # counter line | prefix | one plan tile
    # above kFusedMaxN the split plan's layout: counters | prefix | 7 tile words x T tiles | tile prefixes
    # 7 x (T + 1) | ptrs | seeds, oidx | small-list descriptors (16 B, 16-B aligned)
    # (T = the split plan's tiles: tests/kernel_model.py split_tile mirrors split_per_thread)
    import kernel_model as km
    for n in (8193, 100_000, 262_144, 262_145, 600_000, 1_048_577, 4_200_000):
        T = -(-n // km.split_tile(n))
        head = 256 + 8 * (n + 1) + 8 * 7 * T + 8 * 7 * (T + 1) + 8 * n + 8 * n
        assert lib.zcrc32_batch_device_scratch_bytes(n) == (head + 15) // 16 * 16 + 16 * n, n


def test_no_kernel_waits_on_another_workgroup():
    """No product kernel spins on a flag that another workgroup writes (the
    fused plan did, and aborted a concurrent-streams GPU test; DESIGN.md
    section 4, "Plan").  Such a wait needs a poll loop, so none of its
    markers may appear in the kernel sources: a sleep, an atomic load, or a
    trap as the loop's bound."""
    csrc = os.path.join(ROOT, "zipsfs_amd", "csrc")
    for f in sorted(os.listdir(csrc)):
        if not f.endswith((".hip", ".h")):
            continue
        text = open(os.path.join(csrc, f)).read()
        code = "\n".join(line.split("//")[0] for line in text.splitlines())
        for marker in ("s_sleep", "__hip_atomic_load", "__builtin_trap", "__atomic_load"):
            assert marker not in code, (f, marker)


# ------------------------------------------------- drop-in contract (8(b))

def _dropin_lib():
    import ctypes
    lib = _lib.lib()
    return lib, ctypes


def test_host_crc_pinned_by_golden_vectors():
    """The drop-in's host CRC (zcrc_host.cpp) against the reference-generated
    fixtures: every length 0..4096 at 16 offsets, seeds/chains, KATs, 1 MiB."""
    import json
    import numpy as np
    from oracle import oracle as o
    lib, ctypes = _dropin_lib()
    old = lib.zcrc32_set_gpu_min_bytes(ctypes.c_size_t(-1).value)  # everything on the host
    try:
        g = os.path.join(ROOT, "tests", "golden")
        lo = np.load(os.path.join(g, "lengths_offsets.npz"))
        base = o.payload(int(lo["payload_len"]), int(lo["payload_index"]))
        addr = base.ctypes.data
        for a, L in enumerate(lo["lengths"]):
            for off in range(16):
                assert lib.zcrc32(addr + off, int(L), 0) == lo["crc"][a, off], (int(L), off)
        meta = json.load(open(os.path.join(g, "golden.json")))
        for c in meta["chains"]:
            d = o.payload(c["len"], c["index"])
            assert lib.zcrc32(d.ctypes.data, c["len"], c["seed"]) == c["crc"]
            cut = c["cut"]
            mid = lib.zcrc32(d.ctypes.data, cut, c["seed"])
            assert lib.zcrc32(d.ctypes.data + cut, c["len"] - cut, mid) == c["crc"]
        d = o.payload(meta["config1"]["len"], meta["config1"]["index"])
        assert lib.zcrc32(d.ctypes.data, d.size, 0) == meta["config1"]["crc"]
        assert lib.zcrc32(b"123456789", 9, 0) == 0xCBF43926
        assert lib.zcrc32(None, 0, 0x1234) == 0x1234
        gpu, host, fb = (ctypes.c_uint64() for _ in range(3))
        lib.zcrc32_dropin_stats(ctypes.byref(gpu), ctypes.byref(host), ctypes.byref(fb))
        assert host.value > 24000
    finally:
        lib.zcrc32_set_gpu_min_bytes(old)


def test_dropin_never_aborts_without_gpu(tmp_path):
    """ZIPsFS's call site (fhandle_check_crc32 shape) built against the
    drop-in, run with no visible GPU: every golden CRC comes back -- the
    entry above the GPU threshold through the counted fallback -- and a
    wrong expected CRC is reported as a mismatch, not a crash."""
    import dropin_util as du
    exe = du.build_harness(tmp_path)
    recs = du.golden_records(big=True)
    path = tmp_path / "recs.bin"
    du.write_records(path, recs)
    rc, rows, stats, err = du.run_harness(exe, path, {"HIP_VISIBLE_DEVICES": "", "ROCR_VISIBLE_DEVICES": ""})
    assert rc == 0, err
    assert len(rows) == len(recs) and all(ok for _, _, ok in rows)
    assert [crc for _, crc, _ in rows] == [c & 0xFFFFFFFF for _, c, _ in recs]
    assert stats["gpu"] == 0 and stats["fallback"] == 1 and stats["host"] == len(recs) - 1
    assert "answering from the host CRC" in err
    bad = [(b"123456789", 0xCBF43927, 0)]
    du.write_records(tmp_path / "bad.bin", bad)
    rc, rows, _, err = du.run_harness(exe, tmp_path / "bad.bin", {"HIP_VISIBLE_DEVICES": ""})
    assert rc == 1 and rows == [(0, 0xCBF43926, False)] and "crc32-mismatch" in err


def test_preload_harness_without_gpu(tmp_path):
    """The preloadram_now harness (tests/dropin/preload_main.c) built against
    the drop-in runs without a GPU: the drop-in answers from libzcrc's host
    CRC, never aborts, and equals the reference's own cg_crc32 (-O0)."""
    import dropin_util as du
    from oracle import oracle as o
    exe = du.build_preload_harness(tmp_path)
    path = tmp_path / "entry.bin"
    o.payload(300_001, 9).tofile(path)
    exp = o.payload_crc(300_001, 9)
    modes = ["dropin"] + (["ref"] if os.path.exists(du.REF_O0) else [])
    rc, rows, stats, err = du.run_preload(exe, path, exp, 2, modes, {"HIP_VISIBLE_DEVICES": ""})
    assert rc == 0, err
    assert all(r["ok"] for r in rows.values()), rows
    assert stats["fallback"] == 0 and stats["gpu"] == 0
