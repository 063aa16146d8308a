"""GPU: the streaming CRC of preloadram_now with the
caller's preload segment registered (zero-copy: the kernels read it over
PCIe) and the stream's error contract.

ZIPsFS reads an entry into one mmap'd segment in <= 16 MiB zip_fread() chunks
(src/ZIPsFS_preloadfileram.c:284-306, src/cg_textbuffer.c:103-106) and then
checks the CRC under mutex_fhandle (:309-321).  A stream opened on the
registered segment (zcrc32_stream_open_registered) checksums each chunk
where it lies; chunks outside it go through pinned staging; a failed update
makes the stream fail until it is closed (never a partial CRC)."""
import mmap
import zlib

import numpy as np
import pytest

import zipsfs_amd as z
from zipsfs_amd import _lib
from oracle import oracle as o

pytestmark = pytest.mark.gpu

CHUNK = 16 << 20  # PRELOADRAM_READ_BYTES_NUM (src/ZIPsFS_configuration.h:112)


@pytest.mark.parametrize("size,seed", [(64 << 20, 0), ((40 << 20) + 12345, 0xC0DE), (5 << 20, 3), (4096, 0)])
def test_registered_segment_is_read_in_place(size, seed):
    seg = o.payload(size, 77)
    exp = zlib.crc32(seg.tobytes(), seed)
    with z.Crc32Stream(seed=seed, segment=seg) as s:
        for off in range(0, size, CHUNK):
            s.update(seg[off: off + CHUNK])
        assert s.final() == exp
        st = s.stats()
    assert st == {"registered": -(-size // (4 << 20)), "staged": 0, "pageable": 0}, st


def test_registered_mmap_segment_ragged_chunks_and_outside_data():
    """An anonymous mmap'd segment as ZIPsFS allocates it (filled in place
    after registration), ragged chunk sizes, and one update from outside the
    segment (staged) in the middle: the CRC of the concatenation."""
    size = (24 << 20) + 999
    mm = mmap.mmap(-1, size)
    seg = np.frombuffer(mm, dtype=np.uint8)
    other = o.payload(3 << 20, 5)
    with z.Crc32Stream(segment=seg) as s:
        seg[:] = o.payload(size, 78)  # written after the stream registered the segment
        cuts = [0, 1, 4097, 7 << 20, (7 << 20) + 3, 20 << 20, size]
        for a, b in zip(cuts, cuts[1:]):
            s.update(seg[a:b])
            if a == 4097:
                s.update(other)
        crc = s.final()
        st = s.stats()
    exp = zlib.crc32(seg[:7 << 20].tobytes())
    exp = zlib.crc32(other.tobytes(), exp)
    exp = zlib.crc32(seg[7 << 20:].tobytes(), exp)
    assert crc == exp
    assert st["staged"] == 1 and st["pageable"] == 0 and st["registered"] >= 6, st
    del seg
    mm.close()


def test_failed_update_is_sticky():
    """A failed update poisons the stream: later updates and final() report
    the error instead of a CRC of part of the entry; a reopened stream (the
    same pooled object) starts clean."""
    lib = _lib.lib()
    s = z.Crc32Stream(seed=1)
    s.update(np.arange(100, dtype=np.uint8))
    assert lib.zcrc32_stream_update(s._s, None, 10) != 0  # null data: the bytes are missing
    with pytest.raises(z.ZcrcError):
        s.update(np.arange(100, dtype=np.uint8))
    with pytest.raises(z.ZcrcError):
        s.final()
    s.close()
    t = z.Crc32Stream(seed=1)
    t.update(np.arange(100, dtype=np.uint8))
    assert t.final() == zlib.crc32(bytes(range(100)), 1)
    t.close()


def test_prewarm_creates_staging_for_the_dropin():
    """zcrc32_prewarm creates slots outside any lock; the drop-in then finds
    one free and checksums on the GPU."""
    z.prewarm(2)
    info = z.staging_info()
    assert info["pinned_bytes"] >= 2 * (16 << 20), info
    lib = _lib.lib()
    old = lib.zcrc32_set_gpu_min_bytes(0)
    try:
        with z.profile() as p:
            data = o.payload(6 << 20, 3)
            assert lib.zcrc32(data.ctypes.data, data.size, 0) == zlib.crc32(data.tobytes())
        assert p.launches >= 1
    finally:
        lib.zcrc32_set_gpu_min_bytes(old)
