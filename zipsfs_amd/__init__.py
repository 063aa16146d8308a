"""zipsfs_amd -- MI355X-native drop-in for ZIPsFS's CRC-32 hot path.

ZIPsFS (christophgil/ZIPsFS) verifies every ZIP entry it preloads into RAM
with src/cg_crc32.c.  This package replaces that path with libzcrc, a
hand-written HIP (gfx950) batched CRC-32 engine behind the same C signature
(include/zcrc.h, zipsfs_amd/cg_crc32.c) plus this Python mirror of the
interface.  GPU only: a missing library or device raises ZcrcError.
"""
from ._lib import ZcrcError, lib  # noqa: F401
from .crc32 import (  # noqa: F401
    Crc32Stream, cg_crc32, crc32_batch, crc32_batch_device, crc32_batch_device_ws, crc32_batch_strided,
    crc32_combine, crc32_tensors, device_info, fhandle_check_crc32, fill_synthetic, profile,
    scratch_bytes, staging_info, prewarm, batch_device_faults, verify_entries, version, kernel_name, kernel_name_for, small_kernel_name, kernel_source_hash, inflate_batch_device, inflate_to_device, inflate_batch, inflate_device, INFLATE_STATUS,
    device_set, shard_plan, batch_device_read_ceiling, read_sweep_device, release_cached, cache_info,
)

__version__ = "0.1.0"
