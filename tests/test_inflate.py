"""CPU parity of the inflate oracle (oracle/inflate_port.c) with zlib 1.2.11,
and with the reference's own archive when the reference tree is present.
The GPU inflate is checked against the same corpus in test_gpu_inflate.py."""
import os
import struct
import zlib

import numpy as np
import pytest

import inflate_streams as S
from oracle import oracle as o

REF_ZIP = "/root/reference/for_the_author_only.zip"


def test_oracle_matches_zlib_on_corpus():
    for name, stream, data in S.corpus():
        st, out, used = o.inflate(stream, len(data))
        assert st == 0, (name, o.INFLATE_STATUS[st])
        assert out == data, name
        ok, ref = S.zlib_inflate(stream)
        assert ok and ref == data


def test_oracle_error_iff_zlib_error_on_corruptions():
    n_err = n_ok = 0
    for i, (name, stream, data) in enumerate(S.corpus()):
        if i % 3:
            continue
        for bad in S.corrupt_variants(stream, seed=i):
            ok, ref = S.zlib_inflate(bad)
            st, out, _ = o.inflate(bad, 300 * len(bad) + 1024)
            assert (st == 0) == ok, (name, o.INFLATE_STATUS[st], ok)
            if ok:
                assert out == ref, name
                n_ok += 1
            else:
                n_err += 1
    assert n_err > 50 and n_ok > 5


def test_oracle_output_capacity_and_status_codes():
    data = S.text_payload(5000, 1)
    stream = S.deflate(data)
    assert o.inflate(stream, len(data) - 1)[0] == 6  # output overflow
    assert o.inflate(stream[:-3], len(data))[0] == 7  # input exhausted
    assert o.inflate(bytes([0x07]), 10)[0] == 1  # block type 3
    assert o.inflate(bytes([0x01, 0x05, 0x00, 0x00, 0x00]), 10)[0] == 2  # LEN != ~NLEN
    # distance 1 before any output: fixed block, length code 257 (7 bits 0000001), dist code 0
    bits = [1, 1, 0] + [0, 0, 0, 0, 0, 0, 1] + [0, 0, 0, 0, 0]
    v = sum(b << k for k, b in enumerate(bits))
    assert o.inflate(v.to_bytes(3, "little"), 100)[0] == 5


def test_oracle_batch_and_zlib_baseline_agree():
    items = S.corpus()[:120]
    srcs = [s for _, s, _ in items]
    caps = [len(d) for _, _, d in items]
    st, ol, outs = o.inflate_batch(srcs, caps, nthreads=4)
    zs, zl, zouts = o.zlib_inflate_batch(srcs, caps, nthreads=4)
    for k, (name, _, data) in enumerate(items):
        assert st[k] == 0 and zs[k] == 0, name
        assert ol[k] == zl[k] == len(data)
        assert outs[k][:ol[k]].tobytes() == data == zouts[k][:zl[k]].tobytes()


@pytest.mark.skipif(not os.path.exists(REF_ZIP), reason="reference tree absent")
def test_oracle_on_reference_archive_entries():
    """Every deflated entry of the reference's own for_the_author_only.zip:
    inflated size and CRC-32 equal the central directory's (read live, not
    copied into this repository)."""
    import zipfile
    raw = open(REF_ZIP, "rb").read()
    zf = zipfile.ZipFile(REF_ZIP)
    n = 0
    for info in zf.infolist():
        if info.compress_type != zipfile.ZIP_DEFLATED:
            continue
        h = info.header_offset
        fnlen, exlen = struct.unpack("<HH", raw[h + 26:h + 30])
        start = h + 30 + fnlen + exlen
        st, out, used = o.inflate(raw[start:start + info.compress_size], info.file_size)
        assert st == 0, info.filename
        assert len(out) == info.file_size and zlib.crc32(out) == info.CRC, info.filename
        assert used <= info.compress_size
        n += 1
    assert n >= 20
