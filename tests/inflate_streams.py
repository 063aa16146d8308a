"""Deterministic raw-DEFLATE test streams (TEST INFRASTRUCTURE).

Streams are produced here, at test time, by the image's zlib 1.2.11 (the
library ZIPsFS's libzip inflates with); payloads are generated, never taken
from the reference tree.  Shared by the CPU oracle tests and the GPU parity
tests, so both see the same bytes."""
from __future__ import annotations

import random
import struct
import zlib

import numpy as np

WORDS = ("the of and to in is was for on that with as by at from spectrum peak mass charge ion scan "
         "retention time intensity sample file zip entry preload cache root fuse mount read").split()


def text_payload(n: int, seed: int) -> bytes:
    rnd = random.Random(seed)
    out, size = [], 0
    while size < n:
        w = rnd.choice(WORDS) + (" " if rnd.random() < 0.85 else "\n")
        out.append(w)
        size += len(w)
    return "".join(out).encode()[:n]


def spectrum_payload(n: int, seed: int) -> bytes:
    """Mass-spec-like binary: sorted float64 m/z with float32 intensities."""
    rng = np.random.default_rng(seed)
    k = max(1, n // 12 + 1)
    mz = np.sort(rng.uniform(100.0, 2000.0, k)).astype(np.float64)
    it = (rng.gamma(2.0, 500.0, k)).astype(np.float32)
    rec = np.empty(k, dtype=[("mz", "<f8"), ("i", "<f4")])
    rec["mz"], rec["i"] = mz, it
    return rec.tobytes()[:n]


def random_payload(n: int, seed: int) -> bytes:
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


def far_repeat_payload(n: int, seed: int) -> bytes:
    """Matches at distances near the 32 KiB window edge."""
    blk = random_payload(32768 - 7, seed)
    return (blk * (n // len(blk) + 2))[:n]


def near_ring_payload(n: int, seed: int, period: int = 16484, fresh: int = 8000) -> bytes:
    """Periods of `fresh` random bytes followed by a copy of the bytes one
    period back: the copies deflate to length-258 matches at distance
    `period`, just past a 16 Ki ring (the sp16 decoder's copy_spec
    aliased ring slots for kWin < dist < kWin + len)."""
    rng = np.random.default_rng(seed)
    out = bytearray(rng.integers(0, 256, period, dtype=np.uint8).tobytes())
    while len(out) < n:
        base = len(out)
        out += rng.integers(0, 256, fresh, dtype=np.uint8).tobytes()
        out += out[base + fresh - period: base]  # the bytes one period back
    return bytes(out[:n])


def runs_payload(n: int, seed: int) -> bytes:
    rnd = random.Random(seed)
    out = bytearray()
    while len(out) < n:
        out += bytes([rnd.randrange(256)]) * rnd.randint(1, 700)
    return bytes(out[:n])


PAYLOADS = {"text": text_payload, "spectrum": spectrum_payload, "random": random_payload,
            "far": far_repeat_payload, "runs": runs_payload}
STRATEGIES = {"default": zlib.Z_DEFAULT_STRATEGY, "filtered": zlib.Z_FILTERED, "huffman": zlib.Z_HUFFMAN_ONLY,
              "rle": zlib.Z_RLE, "fixed": zlib.Z_FIXED}


def deflate(data: bytes, level: int = 6, strategy: str = "default", mem_level: int = 8) -> bytes:
    c = zlib.compressobj(level, zlib.DEFLATED, -15, mem_level, STRATEGIES[strategy])
    return c.compress(data) + c.flush()


def deflate_chunked(data: bytes, chunk: int, level: int = 6) -> bytes:
    """Many blocks: Z_FULL_FLUSH / Z_SYNC_FLUSH between chunks (empty stored
    blocks and byte-aligned block starts)."""
    c = zlib.compressobj(level, zlib.DEFLATED, -15)
    out = []
    for k in range(0, len(data), chunk):
        out.append(c.compress(data[k:k + chunk]))
        out.append(c.flush(zlib.Z_FULL_FLUSH if (k // chunk) % 2 else zlib.Z_SYNC_FLUSH))
    out.append(c.flush())
    return b"".join(out)


def deflate_sync(data: bytes, every: int, level: int = 6) -> bytes:
    """A Z_SYNC_FLUSH every `every` input bytes: block starts at chosen output
    positions, the history kept across them."""
    c = zlib.compressobj(level, zlib.DEFLATED, -15)
    out = []
    for k in range(0, len(data), every):
        out.append(c.compress(data[k:k + every]))
        out.append(c.flush(zlib.Z_SYNC_FLUSH))
    out.append(c.flush())
    return b"".join(out)


def corpus(scale: int = 1):
    """(name, deflate stream, expected output) -- the parity corpus."""
    items = []
    sizes = [0, 1, 2, 3, 17, 258, 259, 1000, 4096, 32768, 32769, 70_000 * scale, 300_000 * scale]
    k = 0
    for pname, gen in PAYLOADS.items():
        for n in sizes:
            data = gen(n, 1000 + k)
            k += 1
            for level in (0, 1, 6, 9):
                items.append((f"{pname}-{n}-L{level}", deflate(data, level), data))
            for strat in ("filtered", "huffman", "rle", "fixed"):
                items.append((f"{pname}-{n}-{strat}", deflate(data, 6, strat), data))
        data = gen(200_000 * scale, 7)
        items.append((f"{pname}-chunked", deflate_chunked(data, 9_999), data))
        items.append((f"{pname}-memlevel1", deflate(data, 9, "default", 1), data))
    # hand-made edge streams
    items.append(("empty-fixed", bytes([0x03, 0x00]), b""))
    items.append(("empty-stored", bytes([0x01, 0x00, 0x00, 0xFF, 0xFF]), b""))
    stored = b"stored block payload " * 3
    items.append(("stored-manual", bytes([0x01]) + struct.pack("<HH", len(stored), len(stored) ^ 0xFFFF) + stored,
                  stored))
    return items


def corrupt_variants(stream: bytes, seed: int, count: int = 6):
    """Bit flips and truncations of a valid stream."""
    rnd = random.Random(seed)
    out = []
    for _ in range(count):
        b = bytearray(stream)
        if b:
            pos = rnd.randrange(len(b))
            b[pos] ^= 1 << rnd.randrange(8)
        out.append(bytes(b))
    if len(stream) > 2:
        out.append(stream[: rnd.randrange(1, len(stream))])
    return out


def zlib_inflate(stream: bytes):
    """(ok, bytes) per zlib 1.2.11 raw inflate."""
    try:
        return True, zlib.decompress(stream, -15)
    except zlib.error:
        return False, b""
