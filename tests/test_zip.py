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
