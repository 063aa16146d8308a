"""CPU tests of libzcrc's multi-device host path (no GPU needed): the
byte-balanced shard plan (zcrc_shard_plan, the same function zcrc32_batch /
zcrc32_checked / the drop-in use over ZCRC_DEVICES) and the reassembly of a
buffer cut at shard boundaries with the GF(2) combine.

Reference: ZIPsFS runs up to ROOTS=32 preload threads in one process
(src/ZIPsFS_async.c:468-497, src/ZIPsFS_configuration.h:110), each calling
cg_crc32 from src/ZIPsFS_preloadfileram.c:243 -- one entry per call, under
mutex_fhandle.  Piece CRCs here come from zlib (test side), the combine from
libzcrc's host-only zcrc32_combine."""
import zlib

import numpy as np
import pytest

import zipsfs_amd as z
from oracle import oracle as o


def _expected_pieces(lens, shards):
    """The plan restated: shard g covers bytes [T g / G, T (g+1) / G) of the
    concatenation; a buffer starting on a boundary opens the next shard."""
    total = int(sum(lens))
    ends = [total * (g + 1) // shards for g in range(shards)]
    ends[-1] = total
    g, pos, first, pieces = 0, 0, [], []
    for L in lens:
        while g + 1 < shards and pos >= ends[g]:
            g += 1
        first.append(g)
        off, k = 0, 0
        while True:
            take = L - off if g + 1 >= shards else min(L - off, ends[g] - pos)
            off += take
            pos += take
            k += 1
            if off == L:
                break
            g += 1
        pieces.append(k)
    return first, pieces, ends


def _config4_lens(n):
    # SURVEY 8(d) config-4 length law (the oracle's generator)
    return [int(x) for x in o.zipf_lens(n)]


@pytest.mark.parametrize("shards", [1, 2, 3, 8])
@pytest.mark.parametrize("kind", ["random", "config4", "zeros_and_huge", "single"])
def test_shard_plan_balanced_and_contiguous(shards, kind):
    rng = np.random.default_rng(shards * 7 + len(kind))
    if kind == "random":
        lens = [int(x) for x in rng.integers(0, 300_000, 500)]
    elif kind == "config4":
        lens = _config4_lens(2000)
    elif kind == "zeros_and_huge":
        lens = [0, 0, 1 << 30, 0, 5, 0, (1 << 28) + 3, 0]
    else:
        lens = [(64 << 20) + 7]
    p = z.shard_plan(lens, shards)
    first, pieces, ends = _expected_pieces(lens, shards)
    assert list(p["first"]) == first
    assert list(p["pieces"]) == pieces
    total = sum(lens)
    sb = [int(x) for x in p["shard_bytes"]]
    assert sum(sb) == total
    assert max(sb) - min(sb) <= 1  # byte-balanced
    # contiguity: a buffer's pieces open consecutive shards, in buffer order
    for i in range(1, len(lens)):
        assert first[i] >= first[i - 1] + pieces[i - 1] - 1
    assert first[-1] + pieces[-1] - 1 <= shards - 1


@pytest.mark.parametrize("shards", [2, 3, 5])
def test_reassembly_by_combine_equals_zlib(shards):
    """Piece CRCs (first piece from the buffer's seed, later pieces from 0)
    folded with zcrc32_combine give the buffer's CRC -- the host step of
    batch_host_multi (zcrc_runtime.hip)."""
    rng = np.random.default_rng(shards)
    lens = [int(x) for x in rng.integers(0, 20_000, 40)] + [100_000, 0, 3]
    seeds = [int(x) for x in rng.integers(0, 1 << 32, len(lens), dtype=np.uint64)]
    datas = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for L in lens]
    p = z.shard_plan(lens, shards)
    total = sum(lens)
    ends = [total * (g + 1) // shards for g in range(shards)]
    ends[-1] = total
    starts = [0] + ends[:-1]
    pos = 0
    cut_count = 0
    for i, (d, L, s) in enumerate(zip(datas, lens, seeds)):
        g, off, crc = int(p["first"][i]), 0, None
        for k in range(int(p["pieces"][i])):
            end = ends[g] if g + 1 < shards else total
            take = min(L - off, end - (pos + off)) if g + 1 < shards else L - off
            piece = d[off:off + take]
            if k == 0:
                crc = zlib.crc32(piece, s)
            else:
                assert pos + off == starts[g]  # a continuation opens its shard
                crc = z.crc32_combine(crc, zlib.crc32(piece), take)
                cut_count += 1
            off += take
            g += 1
        assert off == L
        assert crc == zlib.crc32(d, s), i
        pos += L
    assert cut_count >= 1


def test_device_set_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(z.ZcrcError):
        z.device_set()
