"""GPU: the host staging pool under ZIPsFS's thread model.

ZIPsFS preloads with one thread per root, up to ROOTS=32
(src/ZIPsFS_configuration.h:110, src/ZIPsFS_async.c:468), and each calls
cg_crc32 under mutex_fhandle.  libzcrc stages host data through a
process-wide pool of 16 MiB pinned + 16 MiB HBM slots under a fixed budget
(include/zcrc.h, zcrc32_batch).  32 threads at once: drop-in calls (which
never wait for staging), GPU-path calls, batches, and a stream
open/update/final/close per entry -- every CRC bit-exact, the pool within
its budget, every slot returned."""
import zlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import zipsfs_amd as z
from zipsfs_amd import _lib
from oracle import oracle as o

pytestmark = pytest.mark.gpu

SLOT = 16 << 20


def test_staging_pool_32_threads():
    lib = _lib.lib()
    sizes = [5 << 20, 40 << 10, 20 << 20, 1 << 20, 33 << 20 | 7, 3, 0]
    bufs = [o.payload(L, 900 + i) for i, L in enumerate(sizes)]
    exp = [zlib.crc32(b.tobytes()) for b in bufs]

    def work(t):
        got = []
        for b in bufs[t % 3:] + bufs[: t % 3]:
            r = [lib.zcrc32(b.ctypes.data, b.size, 0), z.cg_crc32(b)]
            s = z.Crc32Stream()
            for off in range(0, b.size, SLOT):
                s.update(b[off: off + SLOT])
            r.append(s.final())
            s.close()
            got.append((b.size, r))
        got.append(("batch", list(z.crc32_batch(bufs))))
        return got

    with ThreadPoolExecutor(32) as ex:
        res = list(ex.map(work, range(32)))
    by_size = {b.size: e for b, e in zip(bufs, exp)}
    for t, got in enumerate(res):
        for key, r in got:
            if key == "batch":
                assert r == exp, t
            else:
                assert r == [by_size[key]] * 3, (t, key, r)
    info = z.staging_info()
    assert info["slots_in_use"] == 0, info
    assert 1 <= info["slots_peak"] <= info["slots_budget"], info
    assert info["pinned_bytes"] <= info["slots_budget"] * (SLOT + (1 << 20)), info
    print("staging after 32 threads:", info)


def test_stream_objects_are_reused():
    """Opening and closing a stream per ZIP entry allocates nothing after the
    first: the pool hands the same object back, and an idle stream holds no
    staging slot."""
    a = z.Crc32Stream(seed=7)
    a.update(np.arange(1000, dtype=np.uint8))
    assert a.final() == zlib.crc32(bytes(range(256)) * 3 + bytes(range(232)), 7)
    assert z.staging_info()["slots_in_use"] == 0  # final() returned the slots
    a.close()
    for k in range(50):
        with z.Crc32Stream(seed=k) as s:
            s.update(np.full(100, k, dtype=np.uint8))
            assert s.final() == zlib.crc32(bytes([k]) * 100, k)
    assert z.staging_info()["slots_in_use"] == 0


_ONE_SLOT = r"""
import ctypes, sys, threading, zlib
import numpy as np
sys.path.insert(0, ".")
import zipsfs_amd as z
from zipsfs_amd import _lib
from oracle import oracle as o
lib = _lib.lib()
big = [o.payload(L, 50 + i) for i, L in enumerate([40 << 20, (16 << 20) + 5, 33 << 20])]
exp = [zlib.crc32(b.tobytes()) for b in big]
# one slot: every launch of a > 16 MiB buffer chains through the same slot
assert list(z.crc32_batch(big)) == exp, "batch through one slot"
assert [z.cg_crc32(b) for b in big] == exp, "checked path through one slot"
# a stream holds the only slot: the drop-in does not wait, answers on the host
s = z.Crc32Stream()
s.update(big[0][: 1 << 20])
before = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
lib.zcrc32_dropin_stats(*[ctypes.byref(x) for x in before])
got = lib.zcrc32(big[1].ctypes.data, big[1].size, 0)
after = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
lib.zcrc32_dropin_stats(*[ctypes.byref(x) for x in after])
assert got == exp[1]
assert after[1].value == before[1].value + 1 and after[0].value == before[0].value, "busy pool -> host answer"
# a second stream finds no slot either: its pieces are copied from pageable
# memory by the HIP runtime (it never waits for a slot and never returns a
# partial CRC: ADVICE r2)
t = z.Crc32Stream(seed=9)
for off in range(0, big[2].size, 16 << 20):
    t.update(big[2][off: off + (16 << 20)])
assert t.final() == zlib.crc32(big[2].tobytes(), 9), "pageable stream pieces"
st = t.stats()
assert st["pageable"] == -(-big[2].size // (4 << 20)) and st["staged"] == 0 and st["registered"] == 0, st
t.close()
# a registered segment needs no slot at all: the kernels read its pieces in place
seg = big[0].copy()
r = z.Crc32Stream(segment=seg)
for off in range(0, seg.size, 16 << 20):
    r.update(seg[off: off + (16 << 20)])
assert r.final() == exp[0], "registered stream with the pool exhausted"
assert r.stats() == {"registered": 10, "staged": 0, "pageable": 0}, r.stats()
r.close()
assert s.final() == zlib.crc32(big[0][: 1 << 20].tobytes())
assert s.stats()["staged"] == 1, s.stats()
s.close()
info = z.staging_info()
assert info["slots_budget"] == 1 and info["slots_peak"] == 1 and info["slots_in_use"] == 0, info
print("one-slot pool ok", info)
"""


def test_staging_pool_with_one_slot(tmp_path):
    """ZCRC_STAGING_MIB=16 (one slot): buffers larger than a slot chain their
    launches through it, the waiting GPU path works, and while a stream holds
    the only slot a drop-in call is answered by the host CRC instead of
    waiting (it runs under mutex_fhandle), a second stream copies its pieces
    from pageable memory, and a registered stream reads its segment in place."""
    import os
    import subprocess
    import sys
    script = tmp_path / "one_slot.py"
    script.write_text(_ONE_SLOT)
    env = dict(os.environ, ZCRC_STAGING_MIB="16", ZCRC_GPU_MIN_BYTES="0")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, str(script)], cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    print(p.stdout.strip())
