"""CPU test of the block-parallel inflate's block-start test (the host build
of zipsfs_amd/csrc/zcrc_inflate_find.h via tools/find_check.hip): over every
bit position of zlib streams, the quick filter and the full check pass every
true dynamic block start (a miss would silently cost parallelism, never
correctness), the full check agrees with the model's exact header decode
(tests/inflate_split_model.py header_ok) on every position the quick filter
lets through, and the quick filter keeps ~0.1% of the positions."""
import ctypes
import os
import subprocess
import zlib

import numpy as np
import pytest

import inflate_split_model as M
import inflate_streams as S
from test_inflate_split_model import _block_starts

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("find") / "find_check.so")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17", "-fPIC", "-shared", "-o",
                    out, os.path.join(ROOT, "tools", "find_check.hip")], check=True)
    L = ctypes.CDLL(out)
    L.find_flags.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    return L


def _flags(lib, comp: bytes) -> np.ndarray:
    arr = np.frombuffer(comp, dtype=np.uint8).copy()
    fl = np.zeros(8 * len(comp), dtype=np.uint8)
    lib.find_flags(arr.ctypes.data, len(comp), fl.ctypes.data)
    return fl


@pytest.mark.parametrize("kind,level,strategy", [("text", 6, "default"), ("spectrum", 6, "default"),
                                                 ("text", 9, "filtered"), ("spectrum", 1, "default"),
                                                 ("runs", 6, "rle")])
def test_find_passes_true_starts_and_agrees_with_model(lib, kind, level, strategy):
    data = S.PAYLOADS[kind](400 << 10, 17)
    comp = S.deflate(data, level, strategy)
    fl = _flags(lib, comp)
    dyn = [p for p, t in _block_starts(comp) if t == 2]
    assert dyn, "no dynamic block in the stream"
    for p in dyn:
        assert fl[p] == 3, p
    quick = np.nonzero(fl & 1)[0]
    for q in quick:
        assert bool(fl[q] & 2) == M.header_ok(comp, int(q)), int(q)
    # the quick filter's pass rate on compressed data (the finder's survivors)
    assert len(quick) / len(fl) < 0.004


def test_find_flush_blocks(lib):
    data = S.text_payload(150 << 10, 2)
    comp = S.deflate_chunked(data, 20000)
    fl = _flags(lib, comp)
    for p, t in _block_starts(comp):
        if t == 2:
            assert fl[p] == 3
    assert zlib.decompress(comp, -15) == data
