#!/usr/bin/env python3
"""Debug tooling: inflate a few tiny streams on the GPU and print status and
bytes next to zlib's.  With --trace the printf build of the kernel
(make -C zipsfs_amd/csrc trace -> tools/libzcrc_trace.so) is loaded instead."""
import os
import sys
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import zipsfs_amd._lib as L  # noqa: E402

if "--trace" in sys.argv:
    L.LIB_PATH = os.path.join(ROOT, "tools", "libzcrc_trace.so")

import zipsfs_amd as z  # noqa: E402


def deflate(d, lvl=6):
    c = zlib.compressobj(lvl, zlib.DEFLATED, -15)
    return c.compress(d) + c.flush()


cases = [b"T", b"\xc8", b"hello hello hello", b"", bytes(range(256)) * 4]
streams = [deflate(d, 1) for d in cases]
arena, dp, ol, st = z.inflate_to_device(streams, [len(d) + 8 for d in cases], device="cuda:0")
import torch  # noqa: E402
torch.cuda.synchronize()
st = st.cpu().numpy()
ol = ol.cpu().numpy()
host = arena.cpu().numpy()
offs = (dp.cpu().numpy() - arena.data_ptr())
for k, d in enumerate(cases):
    got = host[offs[k]:offs[k] + ol[k]].tobytes()
    print(k, "stream", streams[k][:16].hex(), "status", st[k], "len", ol[k], "ok", got == d, got[:16].hex(), flush=True)
