"""ZIP central-directory scan (CPU) against Python's zipfile, incl. ZIP64."""
import io
import os
import random
import zipfile

import numpy as np
import pytest

from zipsfs_amd import zipverify as zv


def make_archive(n_small=20, zip64=False, comment=b"", seed=0):
    rnd = random.Random(seed)
    buf = io.BytesIO()
    names = []
    with zipfile.ZipFile(buf, "w", allowZip64=True) as zf:
        for i in range(n_small):
            data = bytes(rnd.getrandbits(8) for _ in range(rnd.choice([0, 1, 7, 100, 5000, 70000])))
            method = rnd.choice([zipfile.ZIP_STORED, zipfile.ZIP_DEFLATED])
            name = f"d{i % 3}/f{i}.bin"
            if zip64 and i % 4 == 0:
                with zf.open(zipfile.ZipInfo(name), "w", force_zip64=True) as f:
                    f.write(data)
            else:
                zf.writestr(name, data, compress_type=method)
            names.append(name)
        zf.writestr("dir/", b"")
        zf.comment = comment
    return buf.getvalue()


@pytest.mark.parametrize("zip64,comment", [(False, b""), (True, b"x" * 300), (False, b"c")])
def test_scan_matches_zipfile(zip64, comment):
    data = make_archive(zip64=zip64, comment=comment, seed=int(zip64))
    ents = zv.scan(data)
    infos = zipfile.ZipFile(io.BytesIO(data)).infolist()
    assert len(ents) == len(infos)
    arr = np.frombuffer(data, dtype=np.uint8)
    for e, z in zip(ents, infos):
        assert e.name == z.filename
        assert e.crc_expected == z.CRC
        assert e.comp_size == z.compress_size and e.uncomp_size == z.file_size
        assert e.method == z.compress_type
        if z.compress_type == zipfile.ZIP_STORED:
            with zipfile.ZipFile(io.BytesIO(data)) as zf:
                assert arr[e.data_offset: e.data_offset + e.comp_size].tobytes() == zf.read(z.filename)


def test_many_entries_zip64_eocd():
    """> 65535 entries forces the ZIP64 end-of-central-directory record."""
    buf = io.BytesIO()
    with zipfile.ZipFile(buf, "w", allowZip64=True) as zf:
        for i in range(66000):
            zf.writestr(f"{i}", b"")
    ents = zv.scan(buf.getvalue())
    assert len(ents) == 66000 and ents[-1].name == "65999"


def test_malformed_archives():
    from zipsfs_amd import ZcrcError
    with pytest.raises(ZcrcError):
        zv.scan(b"not a zip at all, definitely not")
    data = bytearray(make_archive(n_small=3))
    with pytest.raises(ZcrcError):
        zv.scan(bytes(data[: len(data) // 2]))  # truncated: no EOCD / CD outside
    # corrupt the first local header signature -> that entry is BAD, others fine
    assert data[0:4] == b"PK\x03\x04"
    data[0] = 0
    ents = zv.scan(bytes(data))
    assert ents[0].status == zv.ZIP_BAD
    assert all(e.status != zv.ZIP_BAD for e in ents[1:])


# ------------------------------------------- crafted archives
import struct  # noqa: E402
import zlib  # noqa: E402

SAT = 0xFFFFFFFF


def crafted_zip(data: bytes, method: int, *, usize64=None, lho64=None, z64_locator_off=None) -> bytes:
    """One-entry archive written by hand.  usize64 / lho64 put that value in
    a ZIP64 extra field (header field saturated); z64_locator_off adds a ZIP64
    EOCD locator pointing there."""
    payload = zlib.compress(data)[2:-4] if method == 8 else data
    crc = zlib.crc32(data)
    name = b"e.bin"
    local = struct.pack("<IHHHHHIIIHH", 0x04034B50, 20, 0, method, 0, 0, crc, len(payload), len(data), len(name), 0)
    body = local + name + payload
    extra = b""
    fields = []
    usize = len(data)
    lho = 0
    if usize64 is not None:
        usize = SAT
        fields.append(usize64)
    if lho64 is not None:
        lho = SAT
        fields.append(lho64)
    if fields:
        extra = struct.pack("<HH", 1, 8 * len(fields)) + b"".join(struct.pack("<Q", v) for v in fields)
    central = struct.pack("<IHHHHHHIIIHHHHHII", 0x02014B50, 45, 45, 0, method, 0, 0, crc, len(payload), usize,
                          len(name), len(extra), 0, 0, 0, 0, lho) + name + extra
    cd_off = len(body)
    tail = b""
    if z64_locator_off is not None:
        tail = struct.pack("<IIQI", 0x07064B50, 0, z64_locator_off, 1)
    eocd = struct.pack("<IHHHHIIH", 0x06054B50, 0, 0, 1, 1, len(central), cd_off, 0)
    return body + central + tail + eocd


def test_crafted_zip64_fields_never_wrap():
    from zipsfs_amd import ZcrcError
    data = bytes(range(256)) * 40
    ok = zv.scan(crafted_zip(data, 8))
    assert ok[0].uncomp_size == len(data) and ok[0].status == zv.ZIP_UNVERIFIED
    huge = zv.scan(crafted_zip(data, 8, usize64=0xFFFFFFFFFFFFFFF0))
    assert huge[0].uncomp_size == 0xFFFFFFFFFFFFFFF0 and huge[0].status == zv.ZIP_UNVERIFIED
    # a local-header offset near 2^64 must not wrap the bounds check
    for lho in (0xFFFFFFFFFFFFFFF0, 0xFFFFFFFFFFFFFFE2, 1 << 63):
        bad = zv.scan(crafted_zip(data, 0, lho64=lho))
        assert bad[0].status == zv.ZIP_BAD, hex(lho)
    # a ZIP64 EOCD offset near 2^64 must be rejected, not read before the image
    for z in (0xFFFFFFFFFFFFFFF0, 0xFFFFFFFFFFFFFFC8):
        with pytest.raises(ZcrcError):
            zv.scan(crafted_zip(data, 0, z64_locator_off=z))
