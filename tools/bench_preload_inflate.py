"""The preloadram_now loop on deflated entries (measurement tool; VERDICT r3
next #5): tests/dropin/preload_main.c in its deflated modes -- zlib raw
inflate in 16 MiB pieces + the reference cg_crc32 -O0 (ZIPsFS through
zip_fread), the same loop + the drop-in, and one zcrc_inflate_batch call
(GPU inflate + CRC) -- for text- and spectrum-like entries, every column
from the same run on the same box.  One JSON line per (kind, size).

    python3 tools/bench_preload_inflate.py [--sizes 1,16,64,256] [--reps 3]
"""
import argparse
import json
import os
import sys
import tempfile
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import dropin_util as du  # noqa: E402
import inflate_streams as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,16,64,256", help="MiB")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--kinds", default="text,spectrum")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as td:
        exe = du.build_preload_harness(td)
        for kind in a.kinds.split(","):
            for mib in [int(x) for x in a.sizes.split(",")]:
                data = S.PAYLOADS[kind](mib << 20, 17)
                comp = S.deflate(data, 6)
                path = os.path.join(td, "entry.deflate")
                with open(path, "wb") as f:
                    f.write(comp)
                modes = ["zlib_ref", "zlib_dropin", "gpu_inflate"]
                rc, rows, stats, err = du.run_preload(exe, path, zlib.crc32(data), a.reps, modes,
                                                      {"ZCRC_PRELOAD_DEFLATED": str(len(data))})
                print(json.dumps({"kind": kind, "mib": mib, "compressed": len(comp), "rc": rc, "rows": rows,
                                  "err": err[-400:] if rc else ""}), flush=True)
                del data, comp


if __name__ == "__main__":
    main()
