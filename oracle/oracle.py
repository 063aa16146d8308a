"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes front-end for the CPU restatements (oracle/crc32_port.c, the CRC;
oracle/inflate_port.c, raw DEFLATE as zlib 1.2.11 accepts it), the system-zlib
inflate baseline (oracle/zlib_baseline.c) and, when it has been built, the
reference's own src/cg_crc32.c (oracle/_ref/).  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module; the product package zipsfs_amd never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_PORT = os.path.join(HERE, "liboracle.so")
_PORT_O0 = os.path.join(HERE, "liboracle_O0.so")
_REF = os.path.join(HERE, "_ref", "libref_cg_crc32.so")
_REF_O0 = os.path.join(HERE, "_ref", "libref_cg_crc32_O0.so")

_u8p = ctypes.POINTER(ctypes.c_uint8)


def build() -> None:
    """Compile the restatement (and oracle/_ref when /root/reference exists)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _load(path: str) -> ctypes.CDLL:
    if not os.path.exists(path):
        build()
    lib = ctypes.CDLL(path)
    return lib


def _setup_port(lib: ctypes.CDLL) -> ctypes.CDLL:
    lib.oracle_cg_crc32.restype = ctypes.c_uint32
    lib.oracle_cg_crc32.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32]
    lib.oracle_crc32_bitwise.restype = ctypes.c_uint32
    lib.oracle_crc32_bitwise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32]
    lib.oracle_comp_table_literal.restype = ctypes.c_uint32
    lib.oracle_comp_table_literal.argtypes = [ctypes.c_uint32]
    lib.oracle_comp_table_entry.restype = ctypes.c_uint32
    lib.oracle_comp_table_entry.argtypes = [ctypes.c_uint32]
    lib.oracle_mix64.restype = ctypes.c_uint64
    lib.oracle_mix64.argtypes = [ctypes.c_uint64]
    lib.oracle_fill_payload.restype = None
    lib.oracle_fill_payload.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
    lib.oracle_fill_payload_batch.restype = ctypes.c_int
    lib.oracle_fill_payload_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                              ctypes.c_uint64, ctypes.c_int]
    lib.oracle_zipf_len.restype = ctypes.c_uint64
    lib.oracle_zipf_len.argtypes = [ctypes.c_uint64]
    lib.oracle_crc_payload.restype = ctypes.c_uint32
    lib.oracle_crc_payload.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]
    lib.oracle_crc32_batch.restype = ctypes.c_int
    lib.oracle_crc32_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int]
    lib.oracle_inflate.restype = ctypes.c_int
    lib.oracle_inflate.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                   ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]
    for fn in (lib.oracle_inflate_batch, lib.oracle_zlib_inflate_batch):
        fn.restype = ctypes.c_int
        fn.argtypes = [ctypes.c_void_p] * 6 + [ctypes.c_size_t, ctypes.c_int]
    lib.oracle_crc32_batch_fn.restype = ctypes.c_int
    lib.oracle_crc32_batch_fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int]
    return lib


_port = None
_port_o0 = None


def port(o0: bool = False) -> ctypes.CDLL:
    global _port, _port_o0
    if o0:
        if _port_o0 is None:
            _port_o0 = _setup_port(_load(_PORT_O0))
        return _port_o0
    if _port is None:
        _port = _setup_port(_load(_PORT))
    return _port


def ref_available(o0: bool = False) -> bool:
    return os.path.exists(_REF_O0 if o0 else _REF)


_ref_libs: dict = {}


def ref(o0: bool = False) -> ctypes.CDLL:
    """The reference's own cg_crc32 (compiled from /root/reference/src)."""
    path = _REF_O0 if o0 else _REF
    if path not in _ref_libs:
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} not built (needs /root/reference at build time)")
        lib = ctypes.CDLL(path)
        lib.ref_cg_crc32.restype = ctypes.c_uint32
        lib.ref_cg_crc32.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32]
        _ref_libs[path] = lib
    return _ref_libs[path]


def _buf(data) -> tuple:
    arr = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    arr = np.ascontiguousarray(arr, dtype=np.uint8)
    return arr, arr.ctypes.data


def cg_crc32(data, crc: int = 0) -> int:
    """Restatement of src/cg_crc32.c:26 (zlib crc32(crc, data, n) semantics)."""
    arr, ptr = _buf(data)
    return int(port().oracle_cg_crc32(ptr, arr.size, crc & 0xFFFFFFFF))


def crc32_bitwise(data, crc: int = 0) -> int:
    arr, ptr = _buf(data)
    return int(port().oracle_crc32_bitwise(ptr, arr.size, crc & 0xFFFFFFFF))


def ref_cg_crc32(data, crc: int = 0, o0: bool = False) -> int:
    arr, ptr = _buf(data)
    return int(ref(o0).ref_cg_crc32(ptr, arr.size, crc & 0xFFFFFFFF))


PAYLOAD_SEED = 0xC0FFEE


def mix64(z: int) -> int:
    return int(port().oracle_mix64(z & 0xFFFFFFFFFFFFFFFF))


def payload(length: int, index: int, seed: int = PAYLOAD_SEED) -> np.ndarray:
    out = np.empty(max(length, 1), dtype=np.uint8)
    port().oracle_fill_payload(out.ctypes.data, length, index, seed)
    return out[:length]


def payload_crc(length: int, index: int, seed: int = PAYLOAD_SEED, crc: int = 0) -> int:
    return int(port().oracle_crc_payload(length, index, seed, crc & 0xFFFFFFFF))


def zipf_lens(n: int) -> np.ndarray:
    """Config-4 bounded power-law lengths."""
    lib = port()
    return np.array([lib.oracle_zipf_len(i) for i in range(n)], dtype=np.uint64)


def crc32_batch(ptrs: np.ndarray, lens: np.ndarray, seeds=None, nthreads: int = 1) -> np.ndarray:
    """Restatement over many host buffers (pthread pool, round-robin)."""
    ptrs = np.ascontiguousarray(ptrs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    out = np.zeros(len(lens), dtype=np.uint32)
    sp = None
    if seeds is not None:
        seeds = np.ascontiguousarray(seeds, dtype=np.uint32)
        sp = seeds.ctypes.data
    rc = port().oracle_crc32_batch(ptrs.ctypes.data, lens.ctypes.data, sp, out.ctypes.data,
                                   len(lens), nthreads)
    if rc != 0:
        raise RuntimeError("oracle batch failed")
    return out


def ref_crc32_batch(ptrs: np.ndarray, lens: np.ndarray, seeds=None, nthreads: int = 1,
                    o0: bool = False) -> np.ndarray:
    """The reference's cg_crc32 over many host buffers, same thread pool."""
    fn = ctypes.cast(ref(o0).ref_cg_crc32, ctypes.c_void_p).value
    ptrs = np.ascontiguousarray(ptrs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    out = np.zeros(len(lens), dtype=np.uint32)
    sp = None
    if seeds is not None:
        seeds = np.ascontiguousarray(seeds, dtype=np.uint32)
        sp = seeds.ctypes.data
    rc = port().oracle_crc32_batch_fn(fn, ptrs.ctypes.data, lens.ctypes.data, sp, out.ctypes.data,
                                      len(lens), nthreads)
    if rc != 0:
        raise RuntimeError("reference batch failed")
    return out


# ------------------------------------------------------------- inflate

INFLATE_STATUS = {0: "ok", 1: "block type", 2: "stored length", 3: "code lengths", 4: "symbol",
                  5: "distance too far", 6: "output overflow", 7: "input exhausted"}


def inflate(src, cap: int) -> tuple:
    """Raw DEFLATE -> (status, bytes, consumed).  status 0 = ok."""
    arr, ptr = _buf(src)
    dst = np.zeros(max(cap, 1), dtype=np.uint8)
    ol, used = ctypes.c_size_t(0), ctypes.c_size_t(0)
    rc = port().oracle_inflate(ptr, arr.size, dst.ctypes.data, cap, ctypes.byref(ol), ctypes.byref(used))
    return rc, dst[:ol.value].tobytes() if rc == 0 else b"", used.value


def _inflate_batch(fn, srcs, caps, nthreads):
    n = len(srcs)
    keep = [np.frombuffer(bytes(s), dtype=np.uint8) if not isinstance(s, np.ndarray) else s for s in srcs]
    sp = np.array([k.ctypes.data for k in keep], dtype=np.uint64)
    sl = np.array([k.size for k in keep], dtype=np.uint64)
    caps = np.asarray(caps, dtype=np.uint64)
    outs = [np.empty(max(int(c), 1), dtype=np.uint8) for c in caps]
    dp = np.array([o.ctypes.data for o in outs], dtype=np.uint64)
    ol = np.zeros(n, dtype=np.uint64)
    st = np.zeros(n, dtype=np.int32)
    if fn(sp.ctypes.data, sl.ctypes.data, dp.ctypes.data, caps.ctypes.data, ol.ctypes.data, st.ctypes.data,
          n, nthreads) != 0:
        raise RuntimeError("inflate batch failed to start")
    return st, ol, outs


def inflate_batch(srcs, caps, nthreads: int = 1):
    """Restatement over many streams (pthread pool) -> (status[], out_len[], outs[])."""
    return _inflate_batch(port().oracle_inflate_batch, srcs, caps, nthreads)


def zlib_inflate_batch(srcs, caps, nthreads: int = 1):
    """System zlib 1.2.11 raw inflate over many streams: the CPU baseline."""
    return _inflate_batch(port().oracle_zlib_inflate_batch, srcs, caps, nthreads)
