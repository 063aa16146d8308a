"""Child process of tests/test_gpu_multidevice.py (TEST INFRASTRUCTURE): runs
libzcrc's host-memory entry points over the device set the environment
names (ZCRC_DEVICES is read once per process, hence a process of its own)
and prints one JSON line of check results.  Every CRC is compared with the
reference-generated golden vectors (tests/golden/) or, for the inflate and
ZIP checks, with zlib / the central directory."""
from __future__ import annotations

import io
import json
import os
import sys
import threading
import time
import zipfile
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

import inflate_streams as S  # noqa: E402
import zipsfs_amd as z  # noqa: E402
from oracle import oracle as o  # noqa: E402
from zipsfs_amd import _lib, zipverify as zv  # noqa: E402


def main() -> int:
    g = os.path.join(HERE, "golden")
    meta = json.load(open(os.path.join(g, "golden.json")))
    cfg = np.load(os.path.join(g, "configs.npz"))
    res = {"device_set": z.device_set()}
    z.prewarm(2)

    # config 2 in full, host-resident: 4096 x 64 KiB (256 MiB, byte-balanced shards)
    bufs = [o.payload(65536, i) for i in range(4096)]
    got = z.crc32_batch(bufs)
    res["config2"] = [int((got == cfg["cfg2"]).sum()), 4096]
    del bufs

    # config 4's golden sample: 1,023 Zipf-sized buffers (1 KiB .. 16 MiB)
    idx, L = cfg["cfg4_idx"].astype(np.int64), cfg["cfg4_len"].astype(np.int64)
    bufs = [o.payload(int(n), int(i)) for n, i in zip(L, idx)]
    got = z.crc32_batch(bufs)
    res["config4"] = [int((got == cfg["cfg4"]).sum()), len(bufs)]
    del bufs

    # seeds and chains: first pieces take the seed, later pieces start from 0
    chains = meta["chains"]
    datas = [o.payload(c["len"], c["index"]) for c in chains]
    got = z.crc32_batch(datas, seeds=[c["seed"] for c in chains])
    res["chains"] = [int(sum(int(a) == c["crc"] for a, c in zip(got, chains))), len(chains)]

    # one large entry through zcrc32_checked (cut across the devices) and the drop-in zcrc32
    big = o.payload(40 << 20, 3)
    exp = o.payload_crc(40 << 20, 3)
    lib = _lib.lib()
    old = lib.zcrc32_set_gpu_min_bytes(0)
    try:
        dropin = [lib.zcrc32(big.ctypes.data, big.size, 0) for _ in range(3)]
    finally:
        lib.zcrc32_set_gpu_min_bytes(old)
    res["checked"] = z.cg_crc32(big) == exp
    res["dropin"] = all(v == exp for v in dropin)
    res["dropin_stats"] = _dropin_stats(lib)

    # streams opened from several threads (each bound to the least loaded device)
    want = o.payload_crc(24 << 20, 5)
    data = o.payload(24 << 20, 5)
    outs = [None] * 6

    segs = [data.copy() if k % 2 else data for k in range(6)]  # one registration per segment

    def one(k):
        seg = segs[k]
        with z.Crc32Stream(0, segment=seg if k % 2 else None) as s:
            for off in range(0, seg.size, 5 << 20):
                s.update(seg[off:off + (5 << 20)])
            outs[k] = s.final()

    th = [threading.Thread(target=one, args=(k,)) for k in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    res["streams"] = all(v == want for v in outs)

    # concurrent sharded callers: 8 host threads, each batch cut
    # across the logical devices; every result checked, every caller finishes
    bufs = [o.payload(4 << 20, 1000 + i) for i in range(8)]
    want_c = np.array([o.payload_crc(4 << 20, 1000 + i) for i in range(8)], dtype=np.uint32)
    conc = [None] * 8

    def caller(k):
        t0 = time.perf_counter()
        ok = 0
        for _ in range(3):
            ok += int((z.crc32_batch(bufs) == want_c).all())
        conc[k] = (ok, time.perf_counter() - t0)

    th = [threading.Thread(target=caller, args=(k,)) for k in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    res["concurrent"] = [sum(c[0] for c in conc if c), 24]
    res["concurrent_s"] = [round(c[1], 4) for c in conc if c]
    del bufs

    # ZIP verification from host memory (runs of entries per device) and host inflate batches
    buf = io.BytesIO()
    with zipfile.ZipFile(buf, "w") as zf:
        for i in range(24):
            payload = (S.text_payload if i % 2 else S.spectrum_payload)(200_000 + 9_973 * i, 100 + i)
            zf.writestr(f"e{i}.bin", payload, compress_type=zipfile.ZIP_STORED if i % 3 == 0 else zipfile.ZIP_DEFLATED)
    arch = buf.getvalue()
    checks = zv.verify(arch, device=False)
    res["zip"] = [sum(c.ok for c in checks), len(checks)]
    datas = [(S.text_payload if i % 2 else S.spectrum_payload)(300_000 + 1_000 * i, 200 + i) for i in range(12)]
    comps = [S.deflate(d, 6) for d in datas]
    out = z.inflate_batch(comps, [len(d) for d in datas])
    res["inflate"] = [sum(st == 0 and b == d and c == zlib.crc32(d) for (st, b, c), d in zip(out, datas)), len(datas)]
    print(json.dumps(res))
    return 0


def _dropin_stats(lib):
    import ctypes
    v = [ctypes.c_uint64() for _ in range(3)]
    lib.zcrc32_dropin_stats(*[ctypes.byref(x) for x in v])
    return {"gpu": v[0].value, "host": v[1].value, "fallback": v[2].value}


if __name__ == "__main__":
    sys.exit(main())
