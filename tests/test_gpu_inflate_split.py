"""GPU parity of the block-parallel single-stream inflate (zcrc_inflate_device,
zipsfs_amd/csrc/zcrc_inflate_split.hip) with zlib 1.2.11 and the inflate
oracle (oracle/inflate_port.c): every output equals zlib.decompress; streams
that the chain cannot stitch (corrupt, truncated, output cap, a region
overflow) come back with the serial decoder's bytes and status, i.e. the
oracle's.  Chunk sizes down to 512 bytes put many chunks (and many
candidate-less ones) on small streams."""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import inflate_streams as S  # noqa: E402
import zipsfs_amd as z  # noqa: E402
from oracle import oracle as o  # noqa: E402

DEV = "cuda:0"


def _dev(b: bytes, pad: int = 0):
    t = torch.zeros(len(b) + pad + 1, dtype=torch.uint8)
    if b:
        t[:len(b)] = torch.frombuffer(bytearray(b), dtype=torch.uint8)
    return t.to(DEV)


def _run(comp: bytes, cap: int, chunk: int = 0, src_shift: int = 0):
    src = _dev(b"\0" * src_shift + comp)[src_shift:]
    dst = torch.zeros(max(cap, 1), dtype=torch.uint8, device=DEV)
    out_len, status = z.inflate_device(src, dst, src_len=len(comp), cap=cap, chunk_bytes=chunk)
    torch.cuda.synchronize()
    n, st = int(out_len.item()), int(status.item())
    return st, bytes(dst[:n].cpu().numpy()) if st == 0 else b""


CORPUS = [("text", 6, "default", 1 << 20), ("spectrum", 6, "default", 1 << 20), ("text", 1, "default", 600000),
          ("spectrum", 9, "filtered", 700000), ("random", 6, "default", 300000), ("far", 9, "default", 500000),
          ("runs", 6, "rle", 400000), ("text", 6, "huffman", 300000), ("text", 6, "fixed", 300000)]


@pytest.mark.parametrize("kind,level,strategy,size", CORPUS)
@pytest.mark.parametrize("chunk", [0, 4096, 512])
def test_split_inflate_equals_zlib(kind, level, strategy, size, chunk):
    data = S.PAYLOADS[kind](size, 21)
    comp = S.deflate(data, level, strategy)
    st, out = _run(comp, len(data), chunk)
    assert st == 0
    assert out == data


def test_split_inflate_flushes_and_unaligned_source():
    data = S.text_payload(700000, 5) + S.spectrum_payload(500000, 6)
    comp = S.deflate_chunked(data, 70000)
    for shift in (0, 1, 3, 7):
        st, out = _run(comp, len(data), 2048, src_shift=shift)
        assert st == 0 and out == data


def test_split_inflate_mixed_ratio_regions():
    """Stretches of very different ratio: a chunk's output may exceed its
    region (then the serial decoder runs) -- either way the bytes are zlib's."""
    data = b"\0" * (3 << 20) + S.spectrum_payload(1 << 20, 8) + S.text_payload(1 << 20, 9) + b"A" * (2 << 20)
    comp = S.deflate(data, 6)
    for chunk in (0, 1024):
        st, out = _run(comp, len(data), chunk)
        assert st == 0 and out == data


def test_split_inflate_large_streams():
    for kind, size in (("text", 24 << 20), ("spectrum", 16 << 20)):
        data = S.PAYLOADS[kind](size, 33)
        comp = S.deflate(data, 6)
        st, out = _run(comp, len(data))
        assert st == 0
        assert zlib.crc32(out) == zlib.crc32(data) and out == data


def test_split_inflate_small_and_empty():
    for data in (b"", b"a", b"hello world" * 10, S.text_payload(70000, 1)):
        comp = S.deflate(data, 6)
        st, out = _run(comp, max(len(data), 1))
        assert st == 0 and out == data
    st, _ = _run(b"", 16)
    assert st == 7  # empty input: input exhausted (ZCRC_INFLATE_ERR_INPUT), as the batch kernel says


def test_split_inflate_errors_match_oracle():
    """Corrupted and truncated streams: the status is the oracle's (the serial
    fall-back decodes them), and a stream the flip leaves valid is zlib's."""
    rng = np.random.default_rng(4)
    data = S.text_payload(400000, 12) + S.spectrum_payload(300000, 13)
    comp = S.deflate(data, 6)
    cases = []
    for _ in range(12):
        b = bytearray(comp)
        for p in rng.integers(0, len(b), 1 + int(rng.integers(0, 3))):
            b[int(p)] ^= 1 << int(rng.integers(0, 8))
        cases.append((bytes(b), len(data)))
    for cut in (1, 7, len(comp) // 3, len(comp) // 2):
        cases.append((comp[:-cut], len(data)))
    cases.append((comp, len(data) - 1))  # output cap
    for src, cap in cases:
        want_st, want_out, _ = o.inflate(src, cap)
        st, out = _run(src, cap, 2048)
        assert st == want_st
        if st == 0:
            assert out == bytes(want_out)


def test_split_inflate_random_bytes_like_oracle():
    rng = np.random.default_rng(9)
    for i in range(8):
        src = rng.integers(0, 256, int(rng.integers(70000, 200000)), dtype=np.uint8).tobytes()
        want_st, want_out, _ = o.inflate(src, 1 << 20)
        st, out = _run(src, 1 << 20, 1024)
        assert st == want_st, i
        if st == 0:
            assert out == bytes(want_out)


def test_split_inflate_repeated_calls_reuse_scratch():
    """Alternating sizes on one stream (the per-stream scratch grows and is
    reused in stream order)."""
    streams = []
    for i, size in enumerate((200000, 3 << 20, 90000, 1 << 20)):
        data = S.PAYLOADS["text" if i % 2 else "spectrum"](size, 40 + i)
        streams.append((S.deflate(data, 6), data))
    for rep in range(2):
        for comp, data in streams:
            st, out = _run(comp, len(data), 4096 if rep else 0)
            assert st == 0 and out == data


def test_host_batch_routes_large_entries_through_split():
    """zcrc_inflate_batch (host memory, the preload of deflated entries):
    one large entry (split path), a few large ones next to many small ones
    (the cost model splits the large and batches the rest) -- bytes, status
    and CRC-32 equal zlib's either way."""
    one = S.text_payload(3 << 20, 50)
    res = z.inflate_batch([S.deflate(one, 6)], [len(one)])
    assert res[0][0] == 0 and res[0][1] == one and res[0][2] == zlib.crc32(one)
    datas = [S.spectrum_payload(2 << 20, 60), S.text_payload(5 << 20, 61)]
    datas += [S.PAYLOADS["text" if i % 2 else "spectrum"](20000 + 977 * i, 70 + i) for i in range(40)]
    comps = [S.deflate(d, 6) for d in datas]
    res = z.inflate_batch(comps, [len(d) for d in datas])
    for (st, out, crc), d in zip(res, datas):
        assert st == 0 and out == d and crc == zlib.crc32(d)


@pytest.mark.parametrize("parts,probe", [(1, 0), (8, 0), (8, 2), (3, 5)])
def test_split_inflate_parts_and_unsynchronised_probes(monkeypatch, parts, probe):
    """Parts per chunk forced (ZCRC_SPLIT_PARTS) and probes of a few tokens
    (ZCRC_SPLIT_PROBE): part starts that are not token boundaries are
    stepped over by the part before -- the bytes stay zlib's."""
    monkeypatch.setenv("ZCRC_SPLIT_PARTS", str(parts))
    if probe:
        monkeypatch.setenv("ZCRC_SPLIT_PROBE", str(probe))
    for kind, size in (("text", 900000), ("spectrum", 700000), ("runs", 500000)):
        data = S.PAYLOADS[kind](size, 90 + parts + probe)
        comp = S.deflate(data, 6)
        for chunk in (0, 4096):
            st, out = _run(comp, len(data), chunk)
            assert st == 0 and out == data, (kind, chunk)


@pytest.mark.parametrize("parts", [1, 8])
def test_sp16_matches_just_past_the_ring(monkeypatch, parts):
    """with the 16 Ki ring forced, back-references at
    distances in (16 Ki, 16 Ki + len) that reach before a chunk's start
    (copy_spec) must not read ring slots an earlier 64-lane step of the same
    copy overwrote.  Block starts at several offsets put such copies at every
    position relative to the chunk start (tests/test_inflate_split_model.py
    checks the stream holds them)."""
    monkeypatch.setenv("ZCRC_SPLIT_RING", "16")
    monkeypatch.setenv("ZCRC_SPLIT_PARTS", str(parts))
    data = S.near_ring_payload(1 << 20, 3)
    for every in (24000, 33000, 40000):
        comp = S.deflate_sync(data, every)
        for chunk in (0, 4096, 512):
            st, out = _run(comp, len(data), chunk)
            assert st == 0 and out == data, (every, chunk)


@pytest.mark.parametrize("parts,probe,borrow", [(1, 0, "0"), (1, 0, "1"), (4, 0, "1"), (16, 3, "1"), (2, 0, "1")])
def test_split_inflate_borrowed_items(monkeypatch, capfd, parts, probe, borrow):
    """A chunk with a block start takes over the items of the candidate-less
    chunks after it (its block spans them): with 1-2 KiB chunks a text block
    spans 15-30 chunks, so up to kMaxParts = 64 parts of one block land on
    each other (a mask of 64 usable lanes) -- and with unsynchronised probes
    the parts step over each other's starts."""
    monkeypatch.setenv("ZCRC_SPLIT_PARTS", str(parts))
    monkeypatch.setenv("ZCRC_SPLIT_BORROW", borrow)
    monkeypatch.setenv("ZCRC_SPLIT_TRACE", "1")
    if probe:
        monkeypatch.setenv("ZCRC_SPLIT_PROBE", str(probe))
    for kind, size in (("text", 1 << 20), ("spectrum", 600000), ("far", 400000)):
        data = S.PAYLOADS[kind](size, 7 + parts)
        comp = S.deflate(data, 6)
        for chunk in (1024, 2048):
            st, out = _run(comp, len(data), chunk)
            assert st == 0 and out == data, (kind, chunk)
            line = [l for l in capfd.readouterr().err.splitlines() if l.startswith("[split] src")][-1]
            assert " serial 0" in line, (kind, chunk, line)  # the chain formed: no serial fall-back


def test_finder_finds_every_block_start(monkeypatch, capfd):
    """Every dynamic block start of a zlib stream is found (a missed one only
    costs parallelism, so the parity tests would not notice): with one part
    per chunk and chunks smaller than a block, the chain has one item per
    block (ZCRC_SPLIT_TRACE prints it; ZCRC_SPLIT_BORROW=0: no chunk takes
    over the items of the candidate-less chunks after it)."""
    import inflate_split_model as M
    from test_inflate_split_model import _block_starts
    monkeypatch.setenv("ZCRC_SPLIT_PARTS", "1")
    monkeypatch.setenv("ZCRC_SPLIT_BORROW", "0")
    monkeypatch.setenv("ZCRC_SPLIT_TRACE", "1")
    for kind in ("text", "spectrum"):
        data = S.PAYLOADS[kind](1 << 20, 5)
        comp = S.deflate(data, 6)
        blocks = _block_starts(comp)
        assert all(t == 2 for _, t in blocks)
        st, out = _run(comp, len(data), 4096)
        assert st == 0 and out == data
        err = capfd.readouterr().err
        line = [l for l in err.splitlines() if l.startswith("[split] src")][-1]
        chain = int(line.split("chain ")[1].split()[0])
        # one item per 4 KiB chunk that holds a block start (its first one)
        want = len({p // (8 * 4096) for p, _ in blocks})
        assert chain == want, (kind, chain, want, len(blocks))
