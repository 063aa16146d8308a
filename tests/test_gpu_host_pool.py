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
