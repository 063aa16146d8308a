#!/usr/bin/env python3
"""Debug tooling: GPU inflate of corpus items, first mismatch per stream."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import inflate_streams as S  # noqa: E402
import zipsfs_amd as z  # noqa: E402

items = []
for n in [8191, 8192, 8193, 16384, 20000, 32767, 32768, 32769, 40000, 65536, 100000]:
    for lvl in (1, 6):
        d = S.text_payload(n, 5)[:n]
        items.append((f"text-{n}-L{lvl}", S.deflate(d, lvl), d))
arena, dp, ol, st = z.inflate_to_device([s for _, s, _ in items], [len(d) for _, _, d in items], device="cuda:0")
st = st.cpu().numpy(); ol = ol.cpu().numpy(); host = arena.cpu().numpy()
offs = dp.cpu().numpy() - arena.data_ptr()
for k, (name, s, d) in enumerate(items):
    got = host[offs[k]:offs[k] + ol[k]]
    exp = np.frombuffer(d, dtype=np.uint8)
    if st[k] or len(got) != len(exp):
        print(name, "status", st[k], "len", ol[k], len(exp)); continue
    bad = np.nonzero(got != exp)[0]
    print(name, "dst%16", offs[k] % 16, "ok" if bad.size == 0 else f"{bad.size} bad, first {bad[:8]} last {bad[-4:]}", flush=True)
