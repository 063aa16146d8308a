"""GPU: preloadram_now's read loop with the CRC check (SURVEY 8(a) a6/a5 and
8(f) rank 1), as a C program against the drop-in and the stream API.

tests/dropin/preload_main.c reads an entry file in 16 MiB read() calls into
one mmap'd segment (src/ZIPsFS_preloadfileram.c:284-306) and checks the CRC
under mutex_fhandle (:309-321): with the drop-in cg_crc32 after the loop,
with zcrc32_stream_update per chunk and zcrc32_stream_final after it, and
with the reference's own cg_crc32 built -O0 as shipped (oracle/_ref, test
infrastructure).  Every mode must produce the expected CRC; the lock hold
times are printed (and written to $ZCRC_PRELOAD_TABLE as JSON lines when
set, for DESIGN.md section 10b)."""
import json
import os

import pytest

import dropin_util as du
from oracle import oracle as o

pytestmark = pytest.mark.gpu

SIZES = [4 << 10, 1 << 20, 16 << 20, 64 << 20, 256 << 20]


@pytest.mark.parametrize("size", SIZES)
def test_preload_loop_modes(tmp_path, size):
    exe = du.build_preload_harness(tmp_path)
    path = tmp_path / "entry.bin"
    o.payload(size, 41).tofile(path)
    exp = o.payload_crc(size, 41)
    reps = 7 if size <= (16 << 20) else 5
    modes = ["none", "dropin", "stream", "stream_reg"] + (["ref"] if os.path.exists(du.REF_O0) else [])
    rc, rows, stats, err = du.run_preload(exe, path, exp, reps, modes)
    assert rc == 0, err
    rc2, rows_gpu, stats2, err2 = du.run_preload(exe, path, exp, reps, ["dropin"], {"ZCRC_GPU_MIN_BYTES": "0"})
    assert rc2 == 0, err2
    rows["dropin_all_gpu"] = dict(rows_gpu["dropin"], mode="dropin_all_gpu")
    for m, r in rows.items():
        if "skipped" not in r:
            assert r["ok"] and int(r["crc"], 16) == exp, (m, r)
    assert set(rows) >= {"none", "dropin", "stream", "stream_reg", "dropin_all_gpu"}, rows.keys()
    assert stats2 == {"gpu": reps, "host": 0, "fallback": 0}, stats2
    line = {"size": size, "rows": rows}
    print(json.dumps(line))
    out = os.environ.get("ZCRC_PRELOAD_TABLE")
    if out:
        with open(out, "a") as f:
            f.write(json.dumps(line) + "\n")


@pytest.mark.parametrize("kind,size", [("text", 1 << 20), ("spectrum", 1 << 20), ("text", 16 << 20),
                                       ("spectrum", 16 << 20)])
def test_preload_deflated_entry_modes(tmp_path, kind, size):
    """A deflated entry through the same loop: zlib raw
    inflate in 16 MiB pieces + the reference cg_crc32 (-O0) -- what ZIPsFS
    does through zip_fread -- against the drop-in after the same loop and one
    zcrc_inflate_batch call (inflate + CRC on the GPU).  Every mode must give
    the entry's CRC; timings go to $ZCRC_PRELOAD_TABLE."""
    import zlib
    import inflate_streams as S
    exe = du.build_preload_harness(tmp_path)
    data = S.PAYLOADS[kind](size, 17)
    path = tmp_path / "entry.deflate"
    path.write_bytes(S.deflate(data, 6))
    exp = zlib.crc32(data)
    modes = ["zlib_dropin", "gpu_inflate"] + (["zlib_ref"] if os.path.exists(du.REF_O0) else [])
    rc, rows, stats, err = du.run_preload(exe, path, exp, 3, modes, {"ZCRC_PRELOAD_DEFLATED": str(len(data))})
    assert rc == 0, err
    for m, r in rows.items():
        if "skipped" not in r:
            assert r["ok"] and int(r["crc"], 16) == exp, (m, r)
    assert {"zlib_dropin", "gpu_inflate"} <= set(rows)
    line = {"size": size, "kind": kind, "deflated": True, "rows": rows}
    print(json.dumps(line))
    out = os.environ.get("ZCRC_PRELOAD_TABLE")
    if out:
        with open(out, "a") as f:
            f.write(json.dumps(line) + "\n")
