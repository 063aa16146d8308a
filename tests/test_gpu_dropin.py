"""GPU: ZIPsFS's cg_crc32 call site (fhandle_check_crc32 shape) built
against the drop-in and run on the MI355X, plus the drop-in's routing.

SURVEY 8(b): the replacement keeps cg_crc32's static signature
(src/cg_crc32.c:26), never fails, answers small entries on the host and
checksums entries at or above the threshold on the GPU."""
import ctypes
import os

import numpy as np
import pytest

import dropin_util as du
import zipsfs_amd as z
from zipsfs_amd import _lib

pytestmark = pytest.mark.gpu


def test_dropin_executable_all_on_gpu(tmp_path):
    exe = du.build_harness(tmp_path)
    recs = du.golden_records(big=True)
    path = tmp_path / "recs.bin"
    du.write_records(path, recs)
    rc, rows, stats, err = du.run_harness(exe, path, {"ZCRC_GPU_MIN_BYTES": "0"})
    assert rc == 0, err
    assert [crc for _, crc, _ in rows] == [c & 0xFFFFFFFF for _, c, _ in recs]
    assert stats == {"gpu": len(recs), "host": 0, "fallback": 0}, stats
    print(f"drop-in on GPU: {len(recs)} golden entries bit-exact, stats {stats}")


def test_dropin_executable_default_threshold(tmp_path):
    exe = du.build_harness(tmp_path)
    recs = du.golden_records(big=True)
    path = tmp_path / "recs.bin"
    du.write_records(path, recs)
    rc, rows, stats, err = du.run_harness(exe, path, {})
    assert rc == 0, err
    assert [crc for _, crc, _ in rows] == [c & 0xFFFFFFFF for _, c, _ in recs]
    n_big = sum(1 for d, _, _ in recs if len(d) >= du.DEFAULT_GPU_MIN)
    assert stats == {"gpu": n_big, "host": len(recs) - n_big, "fallback": 0}, stats


def test_dropin_gpu_path_launches_kernel():
    """Above the threshold zcrc32 runs the CRC kernel (launch count), below
    it no kernel runs; both answers are the reference's."""
    from oracle import oracle as o
    lib = _lib.lib()
    z.prewarm(1)  # the drop-in never creates a staging slot itself (it runs under mutex_fhandle)
    data = o.payload(3 << 20, 11)
    exp = o.payload_crc(3 << 20, 11)
    old = lib.zcrc32_set_gpu_min_bytes(1 << 20)
    try:
        with z.profile() as p_gpu:
            got = lib.zcrc32(data.ctypes.data, data.size, 0)
        assert got == exp and p_gpu.launches >= 1
        small = data[: 100_000]
        with z.profile() as p_host:
            got = lib.zcrc32(small.ctypes.data, small.size, 0)
        assert got == o.payload_crc(100_000, 11) and p_host.launches == 0
    finally:
        lib.zcrc32_set_gpu_min_bytes(old)
