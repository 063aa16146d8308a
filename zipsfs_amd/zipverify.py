"""Batched verification of ZIP archives on the GPU.

ZIPsFS reads each entry's expected CRC from the central directory through
libzip (``zip_stat`` -> ``st.crc``, src/ZIPsFS.c:998; shown to users as
``<entry>@ARCHIVECRC32.TXT``, src/ZIPsFS_special_file.c:155-163) and checks
it after a full preload (src/ZIPsFS_preloadfileram.c:237-250).  This module
checks a whole archive at once: libzcrc parses the central directory
(ZIP64 aware), checksums every stored entry in one batched GPU launch, and
inflates every deflated entry on the GPU (zcrc_inflate.hip, SURVEY 8(f) rank
4) into HBM, where the same batched CRC kernel checks the outputs.  Nothing is
decompressed or checksummed on the host.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from ._lib import ZcrcError, check, lib

ZIP_OK, ZIP_MISMATCH, ZIP_UNVERIFIED, ZIP_BAD, ZIP_INFLATE_ERROR = 1, 0, -1, -2, -3


class _Entry(ctypes.Structure):
    _fields_ = [("data_offset", ctypes.c_uint64), ("comp_size", ctypes.c_uint64),
                ("uncomp_size", ctypes.c_uint64), ("name_offset", ctypes.c_uint64),
                ("name_len", ctypes.c_uint32), ("crc_expected", ctypes.c_uint32),
                ("crc_computed", ctypes.c_uint32), ("method", ctypes.c_uint16),
                ("flags", ctypes.c_uint16), ("status", ctypes.c_int32), ("inflate_status", ctypes.c_int32)]


_SIGS = False


def _setup():
    global _SIGS
    if _SIGS:
        return lib()
    l = lib()
    l.zcrc_zip_scan.restype = ctypes.c_int
    l.zcrc_zip_scan.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                ctypes.POINTER(ctypes.c_size_t)]
    l.zcrc_zip_verify_host.restype = ctypes.c_int
    l.zcrc_zip_verify_host.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
    l.zcrc_zip_verify_device.restype = ctypes.c_int
    l.zcrc_zip_verify_device.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                         ctypes.c_void_p]
    for f in (l.zcrc_zip_extract_stored_host, l.zcrc_zip_extract_stored_device):
        f.restype = ctypes.c_int
    l.zcrc_zip_extract_stored_host.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_size_t]
    l.zcrc_zip_extract_stored_device.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    _SIGS = True
    return l


@dataclass
class ZipEntryCheck:
    name: str
    method: int
    comp_size: int
    uncomp_size: int
    data_offset: int
    crc_expected: int
    crc_computed: Optional[int]
    status: int
    inflate_status: int = 0

    @property
    def ok(self) -> bool:
        return self.status == ZIP_OK


def _as_array(archive) -> np.ndarray:
    import os
    if isinstance(archive, (str, os.PathLike)):
        return np.fromfile(archive, dtype=np.uint8)
    if isinstance(archive, np.ndarray):
        return np.ascontiguousarray(archive, dtype=np.uint8)
    return np.frombuffer(bytes(archive) if not isinstance(archive, (bytes, bytearray, memoryview)) else archive,
                         dtype=np.uint8)


def scan(archive) -> List[ZipEntryCheck]:
    """Central-directory listing (no CRCs computed)."""
    a = _as_array(archive)
    return [_to_check(a, e) for e in _scan_raw(a)]


def _scan_raw(a: np.ndarray):
    l = _setup()
    n = ctypes.c_size_t(0)
    check(l.zcrc_zip_scan(a.ctypes.data, a.size, None, 0, ctypes.byref(n)), "zcrc_zip_scan")
    arr = (_Entry * max(n.value, 1))()
    check(l.zcrc_zip_scan(a.ctypes.data, a.size, arr, n.value, ctypes.byref(n)), "zcrc_zip_scan")
    return arr[: n.value]


def _to_check(a: np.ndarray, e) -> ZipEntryCheck:
    name = a[e.name_offset: e.name_offset + e.name_len].tobytes().decode("utf-8", "replace")
    computed = e.crc_computed if e.status in (ZIP_OK, ZIP_MISMATCH) else None
    return ZipEntryCheck(name, e.method, e.comp_size, e.uncomp_size, e.data_offset, e.crc_expected, computed,
                         e.status, e.inflate_status)


def verify(archive, device: bool = True) -> List[ZipEntryCheck]:
    """Verify every entry's CRC-32 (and size) against the central directory.

    device=True stages the archive image into HBM through torch and calls
    zcrc_zip_verify_device; device=False hands the host image to
    zcrc_zip_verify_host, which stages it itself.  Either way stored entries
    are checksummed in one batch, deflated entries are inflated on the GPU
    and their outputs checksummed in one more; encrypted entries and other
    methods come back ZIP_UNVERIFIED, broken deflate streams
    ZIP_INFLATE_ERROR (inflate_status says why).
    """
    a = _as_array(archive)
    l = _setup()
    entries = _scan_raw(a)
    arr = (_Entry * max(len(entries), 1))(*entries)
    if device:
        import torch
        from .crc32 import _stream_ptr
        d = torch.from_numpy(a if a.flags.writeable else a.copy()).to("cuda")
        check(l.zcrc_zip_verify_device(d.data_ptr(), a.size, arr, len(entries), _stream_ptr(None)),
              "zcrc_zip_verify_device")
    else:
        check(l.zcrc_zip_verify_host(a.ctypes.data, a.size, arr, len(entries)), "zcrc_zip_verify_host")
    return [_to_check(a, e) for e in arr[: len(entries)]]


def extract_stored(archive, device: bool = True):
    """Stored-entry extraction: the bytes zip_fread()
    would deliver for every stored entry (src/ZIPsFS_preloadfileram.c:286-288)
    plus fhandle_check_crc32's verdict on them (:237-250), in one call.

    Returns a list of (ZipEntryCheck, data) in central-directory order; data
    is a uint8 torch tensor in HBM (device=True: zcrc_zip_extract_stored_device,
    one copy launch + one CRC launch) or a numpy array (device=False:
    zcrc_zip_extract_stored_host, host memcpy + one zcrc32_batch), or None for
    entries that are not extracted (not stored, encrypted, out of range:
    status ZIP_UNVERIFIED or ZIP_BAD)."""
    a = _as_array(archive)
    l = _setup()
    entries = _scan_raw(a)
    n = len(entries)
    arr = (_Entry * max(n, 1))(*entries)
    want = [e.status != ZIP_BAD and e.method == 0 and not (e.flags & 1) and e.comp_size == e.uncomp_size
            and e.data_offset + e.comp_size <= a.size for e in entries]
    cap = np.array([e.comp_size if w else 0 for e, w in zip(entries, want)], dtype=np.uint64)
    bufs = [None] * n
    if device:
        import torch
        from .crc32 import _stream_ptr
        d = torch.from_numpy(a if a.flags.writeable else a.copy()).to("cuda")
        for i in range(n):
            if want[i]:
                bufs[i] = torch.empty(int(cap[i]), dtype=torch.uint8, device="cuda")
        ptrs = np.array([b.data_ptr() if b is not None else 0 for b in bufs], dtype=np.uint64)
        check(l.zcrc_zip_extract_stored_device(d.data_ptr(), a.size, arr, ptrs.ctypes.data, cap.ctypes.data, n,
                                               _stream_ptr(None)), "zcrc_zip_extract_stored_device")
    else:
        for i in range(n):
            if want[i]:
                bufs[i] = np.empty(int(cap[i]), dtype=np.uint8)
        ptrs = np.array([b.ctypes.data if b is not None else 0 for b in bufs], dtype=np.uint64)
        check(l.zcrc_zip_extract_stored_host(a.ctypes.data, a.size, arr, ptrs.ctypes.data, cap.ctypes.data, n),
              "zcrc_zip_extract_stored_host")
    out = []
    for i, e in enumerate(arr[:n]):
        c = _to_check(a, e)
        out.append((c, bufs[i] if c.status in (ZIP_OK, ZIP_MISMATCH) else None))
    return out
