"""Generate the golden vectors in tests/golden/ from the REFERENCE itself.

Run in the build container (needs /root/reference): it compiles
/root/reference/src/cg_crc32.c via oracle/Makefile into oracle/_ref/ and
calls that build (ref_cg_crc32 = the reference's static cg_crc32).  Every
value is cross-checked against Python's zlib.crc32 before it is written.
Inputs are the counter-based payload of SURVEY.md 8(d) (oracle.payload), so
the fixtures hold parameters + expected CRCs, never copied source.

    python tests/golden/gen_golden.py [--small-only]
"""
from __future__ import annotations

import json
import os
import random
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as o  # noqa: E402

SEED = o.PAYLOAD_SEED


def ref(data: bytes, crc: int = 0) -> int:
    r = o.ref_cg_crc32(data, crc)
    r0 = o.ref_cg_crc32(data, crc, o0=True)
    z = zlib.crc32(data, crc)
    assert r == r0 == z, (len(data), crc, r, r0, z)
    return r


SMALL_LENS = (1024, 4096)


def gen_small() -> None:
    """small.npz: uniform batches of small buffers, the ZIP-entry regime
    (config 4's median entry is 3,971 B): 1 GiB of L-byte buffers, buffer i
    = payload(L, i), for L in SMALL_LENS -- 256 sampled indices each, for the
    bench line's small-buffer secondary (bench.py) and its tests."""
    rnd = random.Random(20261018)
    out = {}
    for L in SMALL_LENS:
        n = (1 << 30) // L
        idx = np.array(sorted(rnd.sample(range(n), 255) + [n - 1]), dtype=np.uint64)
        out[f"len{L}_idx"] = idx
        out[f"len{L}"] = np.array([ref(o.payload(L, int(i)).tobytes()) for i in idx], dtype=np.uint32)
    np.savez_compressed(os.path.join(HERE, "small.npz"), **out)


def main() -> None:
    if "--small-only" in sys.argv:  # (the other fixtures stay as they are)
        o.build()
        gen_small()
        print("wrote tests/golden/small.npz")
        return
    o.build()
    assert o.ref_available(), "oracle/_ref not built: /root/reference missing?"
    rnd = random.Random(20261015)

    # 1. known-answer tests
    seq1000 = "".join(f"{i}\n" for i in range(1, 1001)).encode()
    kats = [
        {"name": "check-123456789", "hex": b"123456789".hex(), "crc": ref(b"123456789")},
        {"name": "empty", "hex": "", "crc": ref(b"")},
        {"name": "seq1000 (testing/testfiles/ZIPsFS_testfiles_preload.sh:30,32,53)",
         "text_seq": [1, 1000], "len": len(seq1000), "crc": ref(seq1000)},
        {"name": "zero-byte", "hex": "00", "crc": ref(b"\0")},
        {"name": "ff x 32", "hex": "ff" * 32, "crc": ref(b"\xff" * 32)},
    ]
    assert kats[0]["crc"] == 0xCBF43926 and kats[2]["crc"] == 0x8DC4565D

    # 2. lengths x offsets over payload buffer 7: data = payload(5000, 7)[off:off+L]
    base = o.payload(5000, 7).tobytes()
    lengths = list(range(0, 1101)) + list(range(1101, 4097, 7)) + [4096]
    lo = np.zeros((len(lengths), 16), dtype=np.uint32)
    for a, L in enumerate(lengths):
        for off in range(16):
            lo[a, off] = ref(base[off:off + L])
    np.savez_compressed(os.path.join(HERE, "lengths_offsets.npz"), lengths=np.array(lengths, dtype=np.uint32),
                        crc=lo, payload_len=5000, payload_index=7)

    # 3. seeds and chain splits (zlib chaining semantics)
    chains = []
    for _ in range(600):
        L = rnd.choice([rnd.randint(0, 64), rnd.randint(0, 5000), rnd.randint(0, 70000)])
        idx = rnd.randint(0, 1 << 20)
        data = o.payload(L, idx).tobytes()
        seed = rnd.getrandbits(32)
        full = ref(data, seed)
        cut = rnd.randint(0, L)
        part = ref(data[cut:], ref(data[:cut], seed))
        assert part == full
        chains.append({"index": idx, "len": L, "seed": seed, "cut": cut, "crc": full})

    # 4. synthetic configs; payload seed 0xC0FFEE
    cfg1 = {"len": 1 << 20, "index": 0, "crc": ref(o.payload(1 << 20, 0).tobytes())}
    cfg2 = np.array([ref(o.payload(65536, i).tobytes()) for i in range(4096)], dtype=np.uint32)
    cfg3_idx = np.array(sorted(rnd.sample(range(65536), 256)), dtype=np.uint64)
    cfg3 = np.array([ref(o.payload(1 << 20, int(i)).tobytes()) for i in cfg3_idx], dtype=np.uint32)
    zl = o.zipf_lens(100000)
    big = [i for i in range(100000) if zl[i] >= (1 << 20)]
    cfg4_idx = np.array(sorted(set(rnd.sample(range(100000), 1000)) | set(big[:24])), dtype=np.uint64)
    cfg4 = np.array([ref(o.payload(int(zl[i]), int(i)).tobytes()) for i in cfg4_idx], dtype=np.uint32)
    # config 5: 1M x 1 MiB over 8 GPUs (buffer i on rank i mod N).  256
    # samples in each of [0,2^15), [2^15,2^16), ..., [2^19,2^20), so that runs
    # with fewer ranks or fewer buffers per rank still hold >= 256 of them.
    r5 = random.Random(5)
    cfg5_idx = []
    for lo, hi in [(0, 1 << 15)] + [(1 << k, 1 << (k + 1)) for k in range(15, 20)]:
        cfg5_idx += r5.sample(range(lo, hi), 256)
    cfg5_idx = np.array(sorted(cfg5_idx), dtype=np.uint64)
    cfg5 = np.array([ref(o.payload(1 << 20, int(i)).tobytes()) for i in cfg5_idx], dtype=np.uint32)
    np.savez_compressed(os.path.join(HERE, "configs.npz"), cfg2=cfg2, cfg3_idx=cfg3_idx, cfg3=cfg3,
                        cfg4_idx=cfg4_idx, cfg4_len=zl[cfg4_idx], cfg4=cfg4, cfg5_idx=cfg5_idx, cfg5=cfg5)

    meta = {
        "generator": "tests/golden/gen_golden.py",
        "reference": "/root/reference/src/cg_crc32.c compiled by oracle/Makefile (-O2 and -O0), "
                     "cross-checked with zlib.crc32",
        "payload": "word j of buffer I = splitmix64(0xC0FFEE ^ (I<<32 | j)), little-endian (SURVEY.md 8d)",
        "config4_sum_len": int(zl.sum()),
        "config4_first_lens": [int(x) for x in zl[:4]],
        "kats": kats,
        "config1": cfg1,
        "chains": chains,
    }
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1)
    gen_small()
    print("wrote golden fixtures:", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    main()
