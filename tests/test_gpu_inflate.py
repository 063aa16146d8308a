"""GPU parity of libzcrc's batched inflate (zcrc_inflate.hip) with zlib
1.2.11 and the inflate oracle (oracle/inflate_port.c): same corpus as
tests/test_inflate.py, streams packed unaligned into one device buffer, one
launch per batch.  Valid streams: bytes identical.  Corrupted streams: the
GPU reports an error exactly when zlib does, and identical bytes otherwise."""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import inflate_streams as S  # noqa: E402
import zipsfs_amd as z  # noqa: E402
from oracle import oracle as o  # noqa: E402

DEV = "cuda:0"


def _run(streams, caps):
    arena, dp, out_lens, status = z.inflate_to_device(streams, caps, device=DEV)
    st = status.cpu().numpy()
    ol = out_lens.cpu().numpy()
    host = arena.cpu().numpy()
    base = arena.data_ptr()
    offs = (dp.cpu().numpy() - base).astype(np.int64)
    outs = [host[offs[k]:offs[k] + ol[k]].tobytes() for k in range(len(streams))]
    return st, ol, outs, arena, dp, out_lens


def test_inflate_corpus_bitexact():
    items = S.corpus()
    streams = [s for _, s, _ in items]
    st, ol, outs, *_ = _run(streams, [len(d) for _, _, d in items])
    for k, (name, _, data) in enumerate(items):
        assert st[k] == 0, (name, z.INFLATE_STATUS[int(st[k])])
        assert ol[k] == len(data) and outs[k] == data, name


def test_inflate_large_streams():
    items = []
    for k, (pname, gen) in enumerate(S.PAYLOADS.items()):
        data = gen(3_000_000 + 12345 * k, 500 + k)
        items.append((pname, S.deflate(data, 6), data))
    items.append(("text-64MiB", S.deflate(S.text_payload(64 << 20, 3), 1), None))
    caps = [len(d) if d is not None else 64 << 20 for _, _, d in items]
    st, ol, outs, *_ = _run([s for _, s, _ in items], caps)
    for k, (name, _, data) in enumerate(items):
        assert st[k] == 0, name
        exp = data if data is not None else S.text_payload(64 << 20, 3)
        assert outs[k] == exp, name


def test_inflate_errors_iff_zlib_errors():
    items = S.corpus()
    streams, caps, exp = [], [], []
    for i, (name, stream, data) in enumerate(items):
        if i % 2:
            continue
        for bad in S.corrupt_variants(stream, seed=i):
            ok, ref = S.zlib_inflate(bad)
            streams.append(bad)
            caps.append(300 * len(bad) + 1024)
            exp.append((name, ok, ref))
    st, ol, outs, *_ = _run(streams, caps)
    want = [o.inflate(b, c)[0] for b, c in zip(streams, caps)]
    n_err = 0
    for k, (name, ok, ref) in enumerate(exp):
        assert (st[k] == 0) == ok, (name, z.INFLATE_STATUS[int(st[k])], ok)
        # not just "an error": the oracle's status code (input exhaustion
        # wins over what zero bits past the end would have decoded to)
        assert st[k] == want[k], (name, z.INFLATE_STATUS[int(st[k])], z.INFLATE_STATUS[want[k]])
        if ok:
            assert outs[k] == ref, name
        else:
            n_err += 1
    assert n_err > 50


def test_inflate_status_codes_match_oracle():
    data = S.text_payload(5000, 1)
    stream = S.deflate(data)
    bits = [1, 1, 0] + [0, 0, 0, 0, 0, 0, 1] + [0, 0, 0, 0, 0]
    far = sum(b << k for k, b in enumerate(bits)).to_bytes(3, "little")
    cases = [(stream, len(data) - 1), (stream[:-3], len(data)), (bytes([0x07]), 10),
             (bytes([0x01, 0x05, 0x00, 0x00, 0x00]), 10), (far, 100), (b"", 10)]
    st, ol, outs, *_ = _run([c[0] for c in cases], [c[1] for c in cases])
    want = [o.inflate(s, c)[0] if s else 7 for s, c in cases]
    assert list(st) == want == [6, 7, 1, 2, 5, 7]


def test_inflate_then_crc_on_device():
    """The ZIP verification shape: inflate a batch in HBM, then CRC the
    outputs with the batched CRC kernel -- no host round trip."""
    items = [it for it in S.corpus() if len(it[2]) > 0][:200]
    st, ol, outs, arena, dp, out_lens = _run([s for _, s, _ in items], [len(d) for _, _, d in items])
    assert (st == 0).all()
    crcs = z.crc32_batch_device(dp, out_lens).cpu().numpy().view(np.uint32)
    assert list(crcs) == [zlib.crc32(d) for _, _, d in items]


def test_inflate_host_batch_with_crc():
    """zcrc_inflate_batch: host streams in, host bytes + CRC-32 out (the
    deflated-entry preload shape), including an error entry and grouping."""
    items = [it for it in S.corpus() if it[0].startswith(("text", "spectrum"))][:150]
    streams = [s for _, s, _ in items] + [b"\x07", b""]
    caps = [len(d) for _, _, d in items] + [10, 0]
    res = z.inflate_batch(streams, caps)
    for (name, _, data), (st, out, crc) in zip(items, res):
        assert st == 0 and out == data and crc == zlib.crc32(data), name
    assert res[-2][0] == 1 and res[-1][0] == 7


def test_inflate_random_bytes_terminate_like_oracle():
    """Arbitrary bytes as deflate streams (the adversarial shape: random
    headers, over-subscribed codes, distances before the start, streams that
    end anywhere).  Every launch must terminate, and every status (and every
    output, where one is produced) must equal the oracle's."""
    import random
    rnd = random.Random(11)
    streams, caps = [], []
    for k in range(3000):
        n = rnd.choice([1, 2, 3, 5, 8, 16, 40, 100, 600, 4000])
        b = bytearray(rnd.randrange(256) for _ in range(n))
        if k % 3 == 0 and n > 2:  # force a fixed or dynamic block header on some
            b[0] = (b[0] & ~6) | (2 if k % 2 else 4)
        streams.append(bytes(b))
        caps.append(rnd.choice([0, 1, 64, 5000, 1 << 16]))
    st, ol, outs, *_ = _run(streams, caps)
    want = [o.inflate(s_, c) for s_, c in zip(streams, caps)]
    for k, (ws, wout, _) in enumerate(want):
        assert st[k] == ws, (k, z.INFLATE_STATUS[int(st[k])], z.INFLATE_STATUS[ws])
        if ws == 0:
            assert outs[k] == wout, k
    assert sum(1 for w in want if w[0] == 0) >= 5  # a few decode cleanly


def test_inflate_corpus_both_window_kernels():
    """launch_inflate picks the 32 KiB-window kernel when every stream of the
    batch is resident at once (<= 4 per CU), the 16 KiB-ring kernel (far
    matches read back from dst) up to 8 per CU, and above that the 8 KiB-ring
    kernel (16 per CU) with the streams dispatched longest-first through a
    device-sorted order: run the corpus on all three."""
    items = S.corpus()
    cus = z.device_info()["num_cus"]
    assert len(items) <= 4 * cus
    for reps in (1, (4 * cus) // len(items) + 2, (8 * cus) // len(items) + 2):
        batch = items * reps
        st, ol, outs, *_ = _run([s for _, s, _ in batch], [len(d) for _, _, d in batch])
        for k, (name, _, data) in enumerate(batch):
            assert st[k] == 0 and outs[k] == data, (reps, name)


def test_inflate_host_batch_large_mixed_sizes_longest_first():
    """The host entry point with more streams than the GPU holds at once
    (> 8 per CU: 8 KiB-ring kernel, longest-first order built on the device
    from per-stream scratch), sizes spread over four octaves so the order
    really permutes, plus error entries scattered through the batch: every
    result lands at its own index with zlib's bytes and CRC."""
    import random
    rnd = random.Random(11)
    cus = z.device_info()["num_cus"]
    n = 8 * cus + 300
    base = [it for it in S.corpus() if it[0].startswith(("text", "spectrum"))]
    streams, caps, want = [], [], []
    for k in range(n):
        if k % 97 == 13:  # invalid block type / empty input
            streams.append(b"\x07" if k % 2 else b"")
            caps.append(10)
            want.append(None)
            continue
        name, s, data = base[rnd.randrange(len(base))]
        cut = rnd.choice([len(data), len(data) // 3, len(data) // 9, 4000])
        d = data[:cut]
        streams.append(zlib.compress(d, 6)[2:-4])
        caps.append(len(d))
        want.append(d)
    res = z.inflate_batch(streams, caps)
    assert len(res) == n
    for k, ((st, out, crc), w) in enumerate(zip(res, want)):
        if w is None:
            assert st != 0, k
        else:
            assert st == 0 and out == w and crc == zlib.crc32(w), k
