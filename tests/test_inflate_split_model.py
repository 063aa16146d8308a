"""CPU tests of the block-parallel inflate model (tests/inflate_split_model.py),
the specification of zcrc_inflate_split.hip: the model's bytes equal
zlib.decompress (zlib 1.2.11, the library libzip inflates ZIPsFS entries with)
on streams cut into many small chunks, and its fall-backs trigger where the
GPU path falls back to the serial decoder.  Sizes are kept small: the model
decodes in pure Python."""
import zlib

import pytest

import inflate_split_model as M
import inflate_streams as S


def _zlib(comp: bytes) -> bytes:
    return zlib.decompress(comp, -15)


@pytest.mark.parametrize("kind,level,strategy", [
    ("text", 6, "default"), ("spectrum", 6, "default"), ("text", 1, "default"), ("spectrum", 9, "filtered"),
    ("random", 6, "default"), ("far", 6, "default"), ("runs", 6, "rle"), ("text", 6, "huffman"),
    ("text", 6, "fixed"),
])
def test_model_equals_zlib(kind, level, strategy):
    data = S.PAYLOADS[kind](96 << 10, 11)
    comp = S.deflate(data, level, strategy)
    st, out, stats = M.inflate_split(comp, len(data), 1024)
    assert stats["fallback"] is None, stats
    assert st == M.OK and out == _zlib(comp)


def test_model_flush_blocks_and_many_chunks():
    """Sync/full flushes put empty stored blocks and byte-aligned block starts
    between dynamic blocks; 512-byte chunks make most chunks candidate-less."""
    data = S.text_payload(80 << 10, 3) + S.spectrum_payload(40 << 10, 4)
    comp = S.deflate_chunked(data, 9000)
    st, out, stats = M.inflate_split(comp, len(data), 512)
    assert st == M.OK and out == data, stats
    assert stats["chain"] >= 3


def test_model_history_markers_cross_chunks():
    """Matches reaching 32 KiB back across every chunk boundary (markers
    resolved through the chain of tails)."""
    data = S.far_repeat_payload(200 << 10, 5)
    comp = S.deflate(data, 9)
    st, out, stats = M.inflate_split(comp, len(data), 700)
    assert st == M.OK and out == data, stats


def test_model_header_check_passes_every_true_block_start():
    data = S.text_payload(200 << 10, 9) + S.spectrum_payload(100 << 10, 9)
    comp = S.deflate(data, 6)
    starts = _block_starts(comp)
    dyn = [p for p, t in starts if t == 2]
    assert len(dyn) >= 3
    assert all(M.header_ok(comp, p) for p in dyn)


def _block_starts(comp: bytes):
    """(bit position, BTYPE) of every block, by an exact decode."""
    out, res = [], []
    br = M.Bits(comp, 0)
    while True:
        res.append((br.pos, (br.peek(3) >> 1) & 3))
        last = br.get(1)
        typ = br.get(2)
        if typ == 0:
            br.pos = (br.pos + 7) & ~7
            ln = br.get(16)
            br.get(16)
            br.pos += 8 * ln
        else:
            if typ == 1:
                ll, dd = M.fixed_codes()
            else:
                _, ll, dd = M.read_dynamic(br)
            assert M.codes(br, ll, dd, out, M.ChunkResult(0), False) == M.OK
        if last:
            return res


def test_model_corrupt_stream_falls_back():
    data = S.text_payload(60 << 10, 2)
    comp = bytearray(S.deflate(data, 6))
    comp[len(comp) // 2] ^= 0x5A
    st, out, stats = M.inflate_split(bytes(comp), len(data), 2048)
    if st is None:
        assert stats["fallback"]
    else:  # the flip may leave a valid stream: then it must be zlib's
        try:
            want = _zlib(bytes(comp))
        except zlib.error:
            want = None
        assert out == want


def test_model_output_cap_falls_back():
    data = S.spectrum_payload(64 << 10, 1)
    comp = S.deflate(data, 6)
    st, _, stats = M.inflate_split(comp, len(data) - 1, 1024)
    assert st is None and stats["fallback"] == "output"


def test_model_truncated_stream_falls_back():
    data = S.spectrum_payload(64 << 10, 1)
    comp = S.deflate(data, 6)[:-3]
    st, _, stats = M.inflate_split(comp, len(data), 1024)
    assert st is None and stats["fallback"]


@pytest.mark.parametrize("kind,level,strategy", [("text", 6, "default"), ("spectrum", 6, "default"),
                                                 ("runs", 6, "rle"), ("text", 6, "fixed"), ("far", 9, "default")])
def test_model_parts_equal_zlib(kind, level, strategy):
    """Second level: each chunk's first block cut into 8 parts that start at
    probed token boundaries; parts land on each other per token."""
    data = S.PAYLOADS[kind](160 << 10, 13)
    comp = S.deflate(data, level, strategy)
    st, out, stats = M.inflate_split_parts(comp, len(data), 4096, parts=8, probe_tokens=64)
    assert stats["fallback"] is None, stats
    assert st == M.OK and out == _zlib(comp)


def test_model_parts_survive_unsynchronised_probes():
    """With 2-token probes most part starts are not token boundaries: the
    earlier part steps over them and decodes on -- slower, never wrong."""
    data = S.text_payload(120 << 10, 21)
    comp = S.deflate(data, 6)
    st, out, stats = M.inflate_split_parts(comp, len(data), 4096, parts=8, probe_tokens=2)
    assert st == M.OK and out == data, stats
    assert stats["chain"] < stats["items"]


def test_near_ring_stream_holds_aliasing_copies(monkeypatch):
    """The stream of tests/test_gpu_inflate_split.py::test_sp16_matches_just_past_the_ring
    really holds speculative copies that reach before the chunk start at
    16 Ki < dist < 16 Ki + len, where a 64-lane step would read a ring slot an
    earlier step of the same copy wrote."""
    hits = []

    def hook(p, length, dist, spec):
        if not spec or dist <= p or not 16384 < dist < 16384 + length:
            return
        for i in range(max(dist - p, 0), length):  # source p - dist + i >= 0: a ring element
            w = i - (dist - 16384)                   # the element whose slot it shares
            if 0 <= w and w // 64 < i // 64:
                hits.append((p, length, dist))
                return

    monkeypatch.setattr(M, "MATCH_HOOK", hook)
    data = S.near_ring_payload(320 << 10, 3)
    for every in (24000, 40000):
        comp = S.deflate_sync(data, every)
        assert _zlib(comp) == data
        cand = M.find_candidates(comp, 4096)
        for k, c in enumerate(cand):
            if c is not None:
                M.spec_decode(comp, c, cand, k, True)
    assert hits


@pytest.mark.parametrize("parts,max_parts,probe", [(1, 64, 64), (2, 64, 64), (4, 16, 3)])
def test_model_borrowed_items_equal_zlib(parts, max_parts, probe):
    """A chunk with a block start borrows the items of the candidate-less
    chunks after it: with 1 KiB chunks a text block spans many chunks and is
    cut into up to max_parts parts."""
    data = S.text_payload(160 << 10, 31)
    comp = S.deflate(data, 6)
    st, out, stats = M.inflate_split_parts(comp, len(data), 1024, parts=parts, probe_tokens=probe,
                                           max_parts=max_parts)
    assert stats["fallback"] is None, stats
    assert st == M.OK and out == data
    assert stats["items"] > len([c for c in M.find_candidates(comp, 1024) if c is not None]) * parts
