"""ctypes binding of the in-tree libzcrc.so (include/zcrc.h).

The library is the product: every CRC this package returns is computed by
its HIP kernels.  If the .so is missing or a GPU call fails, the functions
here raise -- there is no CPU fallback anywhere in this package (only the C
drop-in zcrc32() answers from libzcrc's host CRC).
"""
from __future__ import annotations

import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libzcrc.so")

# The C header is the single source of truth for the exported surface.
HEADER_PATH = os.path.join(os.path.dirname(HERE), "include", "zcrc.h")

_lock = threading.Lock()
_lib = None

_c_u32 = ctypes.c_uint32
_c_u64 = ctypes.c_uint64
_c_sz = ctypes.c_size_t
_c_p = ctypes.c_void_p
_c_int = ctypes.c_int

_SIGNATURES = {
    "zcrc32": (_c_u32, [_c_p, _c_sz, _c_u32]),
    "zcrc32_checked": (_c_int, [_c_p, _c_sz, _c_u32, ctypes.POINTER(_c_u32)]),
    "zcrc32_set_gpu_min_bytes": (_c_sz, [_c_sz]),
    "zcrc32_dropin_stats": (None, [ctypes.POINTER(_c_u64)] * 3),
    "zcrc_staging_info": (ctypes.c_int, [ctypes.POINTER(_c_u64)] * 4),
    "zcrc32_batch": (_c_int, [_c_p, _c_p, _c_p, _c_p, _c_sz, ctypes.c_uint]),
    "zcrc32_batch_device": (_c_int, [_c_p, _c_p, _c_p, _c_p, _c_sz, _c_p]),
    "zcrc32_batch_device_maxlen": (_c_int, [_c_p, _c_p, _c_p, _c_p, _c_sz, _c_u64, _c_p]),
    "zcrc32_batch_device_scratch_bytes": (_c_sz, [_c_sz]),
    "zcrc32_batch_device_ws": (_c_int, [_c_p, _c_p, _c_p, _c_p, _c_sz, _c_p, _c_sz, _c_p]),
    "zcrc32_batch_device_strided": (_c_int, [_c_p, _c_u64, _c_u64, _c_sz, _c_p, _c_p, _c_p]),
    "zcrc32_batch_device_faults": (_c_int, [_c_p, _c_p, ctypes.POINTER(_c_u32)]),
    "zcrc32_batch_device_read_ceiling": (_c_int, [_c_p, _c_p, _c_p, _c_sz, _c_p]),
    "zcrc_read_sweep_device": (_c_int, [_c_p, _c_u64, _c_p, _c_p]),
    "zcrc_release_cached": (_c_int, [ctypes.POINTER(_c_u64)]),
    "zcrc_cache_info": (_c_int, [_c_int] + [ctypes.POINTER(_c_u64)] * 3),
    "zcrc32_combine": (_c_u32, [_c_u32, _c_u32, _c_u64]),
    "zcrc_inflate_batch_device": (_c_int, [_c_p] * 6 + [_c_sz, _c_p]),
    "zcrc_inflate_batch": (_c_int, [_c_p] * 7 + [_c_sz, ctypes.c_uint]),
    "zcrc_inflate_device": (_c_int, [_c_p, ctypes.c_uint64, _c_p, ctypes.c_uint64, _c_p, _c_p, ctypes.c_uint64, _c_p]),
    "zcrc32_stream_open": (_c_p, [_c_u32]),
    "zcrc32_stream_update": (_c_int, [_c_p, _c_p, _c_sz]),
    "zcrc32_stream_final": (_c_int, [_c_p, ctypes.POINTER(_c_u32)]),
    "zcrc32_stream_close": (None, [_c_p]),
    "zcrc32_stream_open_registered": (_c_p, [_c_u32, _c_p, _c_sz]),
    "zcrc32_stream_stats": (_c_int, [_c_p] + [ctypes.POINTER(_c_u64)] * 3),
    "zcrc32_prewarm": (_c_int, [_c_sz]),
    "zcrc_fill_synthetic": (_c_int, [_c_p, _c_p, _c_sz, _c_u64, _c_u64, _c_u64, _c_p]),
    "zcrc_last_error": (ctypes.c_char_p, []),
    "zcrc_version": (ctypes.c_char_p, []),
    "zcrc_kernel_name": (ctypes.c_char_p, []),
    "zcrc_kernel_name_for": (ctypes.c_char_p, [ctypes.c_size_t]),
    "zcrc_small_kernel_name": (ctypes.c_char_p, []),
    "zcrc_device_info": (_c_int, [ctypes.POINTER(_c_int)] * 3),
    "zcrc_device_set": (_c_int, [_c_p, _c_sz, ctypes.POINTER(_c_sz)]),
    "zcrc_shard_plan": (_c_int, [_c_p, _c_sz, _c_sz, _c_p, _c_p, _c_p]),
    "zcrc_profile_enable": (None, [_c_int]),
    "zcrc_profile_read": (_c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_c_int)]),
    "zcrc_profile_read_kind": (_c_int, [_c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_c_int)]),
    "zcrc_profile_reset": (None, []),
}


class ZcrcError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    """Load libzcrc.so (once).  Raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ZcrcError(
                f"{LIB_PATH} is missing: build it with `make -C zipsfs_amd/csrc` or "
                "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        # torch ships its own libamdhip64.so (SONAME libamdhip64.so.7).  Importing
        # torch first makes libzcrc bind to that same runtime instead of loading
        # /opt/rocm's copy beside it, so device pointers and streams are shared.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        l = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(l, name)
            fn.restype = res
            fn.argtypes = args
        _lib = l
        return l


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().zcrc_last_error()
        raise ZcrcError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def exported_symbols_from_header() -> list:
    """Function names declared in include/zcrc.h (for ABI tests)."""
    import re
    text = open(HEADER_PATH).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"\b(zcrc\w*)\s*\(", text)
    return sorted(set(names))
