"""The CPU oracle (oracle/crc32_port.c) pinned against the reference's own
golden vectors (tests/golden/, generated from /root/reference/src/cg_crc32.c
by gen_golden.py), the reference test-suite KAT and zlib."""
import random
import zlib

import numpy as np
import pytest

from oracle import oracle as o


def test_kats(golden):
    for k in golden["meta"]["kats"]:
        if "text_seq" in k:
            a, b = k["text_seq"]
            data = "".join(f"{i}\n" for i in range(a, b + 1)).encode()
            assert len(data) == k["len"]
        else:
            data = bytes.fromhex(k["hex"])
        assert o.cg_crc32(data) == k["crc"], k["name"]
        assert zlib.crc32(data) == k["crc"]
    assert o.cg_crc32(b"123456789") == 0xCBF43926
    seq = "".join(f"{i}\n" for i in range(1, 1001)).encode()
    assert o.cg_crc32(seq) == 0x8DC4565D  # testing/testfiles/ZIPsFS_testfiles_preload.sh:30


def test_complemented_table_identity():
    lib = o.port()
    for i in range(256):
        assert lib.oracle_comp_table_literal(i) == lib.oracle_comp_table_entry(i)


def test_lengths_offsets(golden):
    lo = golden["lo"]
    base = o.payload(int(lo["payload_len"]), int(lo["payload_index"])).tobytes()
    lengths = lo["lengths"]
    crc = lo["crc"]
    for a in range(0, len(lengths), 3):
        L = int(lengths[a])
        for off in range(16):
            assert o.cg_crc32(base[off:off + L]) == crc[a, off], (L, off)


def test_chains(golden):
    for c in golden["meta"]["chains"]:
        data = o.payload(c["len"], c["index"]).tobytes()
        assert o.cg_crc32(data, c["seed"]) == c["crc"]
        cut = c["cut"]
        assert o.cg_crc32(data[cut:], o.cg_crc32(data[:cut], c["seed"])) == c["crc"]


def test_configs(golden):
    cfg = golden["cfg"]
    meta = golden["meta"]
    assert o.payload_crc(meta["config1"]["len"], meta["config1"]["index"]) == meta["config1"]["crc"]
    for i in range(0, 4096, 97):
        assert o.payload_crc(65536, i) == cfg["cfg2"][i]
    for i, c in zip(cfg["cfg3_idx"][:16], cfg["cfg3"][:16]):
        assert o.payload_crc(1 << 20, int(i)) == c
    for i, L, c in zip(cfg["cfg4_idx"][:64], cfg["cfg4_len"][:64], cfg["cfg4"][:64]):
        assert o.payload_crc(int(L), int(i)) == c
    # config 5: 1536 samples, 256 per octave of [0, 2^20)
    idx5 = cfg["cfg5_idx"].astype(np.int64)
    assert len(idx5) == 1536 and len(set(idx5.tolist())) == 1536 and idx5.max() < (1 << 20)
    assert int((idx5 < (1 << 15)).sum()) == 256 and int((idx5 >= (1 << 19)).sum()) == 256
    for i, c in zip(cfg["cfg5_idx"][::96], cfg["cfg5"][::96]):
        assert o.payload_crc(1 << 20, int(i)) == c


def test_small_buffer_fixtures():
    """tests/golden/small.npz (uniform 1 KiB / 4 KiB batches, bench.py's
    small-buffer secondary): every sample against the oracle."""
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "small.npz"))
    for L in (1024, 4096):
        idx, crc = g[f"len{L}_idx"], g[f"len{L}"]
        assert len(idx) == 256 and int(idx.max()) == (1 << 30) // L - 1
        for i, c in zip(idx, crc):
            assert o.payload_crc(L, int(i)) == c


def test_zipf_pinned_totals(golden):
    L = o.zipf_lens(100000)
    assert int(L.sum()) == 13_123_505_587 == golden["meta"]["config4_sum_len"]
    assert [int(x) for x in L[:4]] == [3411, 5161, 1161, 4239]
    assert int(np.median(L)) == 3971
    assert int((L >= (1 << 20)).sum()) == 2339 and int((L < 65536).sum()) == 88481


def test_payload_generator_matches_streaming_crc():
    for L in (0, 1, 7, 8, 9, 65535, 65536, 65537, 200001):
        assert o.payload_crc(L, 3) == zlib.crc32(o.payload(L, 3).tobytes())


def test_random_vs_zlib_and_bitwise():
    rnd = random.Random(5)
    for _ in range(300):
        L = rnd.randint(0, 3000)
        data = bytes(rnd.getrandbits(8) for _ in range(L))
        s = rnd.getrandbits(32)
        assert o.cg_crc32(data, s) == zlib.crc32(data, s) == o.crc32_bitwise(data, s)


def test_batch_pool():
    bufs = [o.payload(L, i) for i, L in enumerate([0, 1, 100, 5000, 70000, 3])]
    ptrs = np.array([b.ctypes.data for b in bufs], dtype=np.uint64)
    lens = np.array([b.size for b in bufs], dtype=np.uint64)
    seeds = np.arange(len(bufs), dtype=np.uint32) * 77
    exp = [zlib.crc32(b.tobytes(), int(s)) for b, s in zip(bufs, seeds)]
    assert list(o.crc32_batch(ptrs, lens, seeds, nthreads=3)) == exp


@pytest.mark.skipif(not o.ref_available(), reason="oracle/_ref not built")
def test_reference_build_agrees():
    rnd = random.Random(9)
    for _ in range(200):
        L = rnd.randint(0, 2000)
        data = bytes(rnd.getrandbits(8) for _ in range(L))
        s = rnd.getrandbits(32)
        assert o.ref_cg_crc32(data, s) == o.cg_crc32(data, s)
