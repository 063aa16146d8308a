"""CPU checks of the kernel's decomposition (tests/kernel_model.py mirrors
zcrc_kernels.hip step by step) against the oracle, plus partition
invariants of the wave-range snapping.  No GPU needed."""
import os
import random
import zlib

import numpy as np
import pytest

import kernel_model as km
from oracle import oracle as o


def _mk_batch(rnd, mem_size, lens, seeded=True, gap=40):
    addrs, pos = [], rnd.randint(0, 15)
    for L in lens:
        addrs.append(pos)
        pos += L + rnd.randint(0, gap)
    assert pos <= mem_size
    seeds = [rnd.getrandbits(32) for _ in lens] if seeded else None
    return addrs, seeds


@pytest.mark.parametrize("num_cus", [1, 2, 256])
def test_model_matches_oracle(num_cus):
    rnd = random.Random(num_cus)
    mem = np.random.default_rng(num_cus).integers(0, 256, size=4_500_000, dtype=np.uint8)
    lens = [0, 1, 2, 3, 4, 5, 15, 16, 17, 1023, 1024, 1025, 4095, 4097, 65535, 65536, 131071, 131072,
            131073, 262145, 1_200_007] + [rnd.randint(0, 9000) for _ in range(40)] + [2_000_000]
    addrs, seeds = _mk_batch(rnd, mem.size, lens)
    b = km.Batch(mem, addrs, lens, seeds)
    got = km.run_batch(b, num_cus=num_cus)
    exp = [o.cg_crc32(mem[a:a + L], s) for a, L, s in zip(addrs, lens, seeds)]
    assert list(got) == exp


def test_model_all_empty_and_single():
    mem = np.zeros(64, dtype=np.uint8)
    b = km.Batch(mem, [0, 0, 0], [0, 0, 0], [0, 5, 0xFFFFFFFF])
    assert list(km.run_batch(b)) == [0, 5, 0xFFFFFFFF]
    b = km.Batch(mem, [3], [9], [0])
    assert list(km.run_batch(b)) == [zlib.crc32(mem[3:12].tobytes())]


def _check_partition(b, num_cus, dyn_shift=km.K_DYN_SHIFT):
    cover = {i: [] for i in range(b.n)}
    for (s0, s1, last) in km.wave_ranges(b, num_cus, dyn_shift):
        for (i, lo, hi) in km.wave_pieces(b, s0, s1, last):
            cover[i].append((lo, hi))
    for i in range(b.n):
        n = b.lens[i]
        pcs = sorted(cover[i])
        assert pcs, f"buffer {i} not visited"
        assert pcs[0][0] == 0 and pcs[-1][1] == n
        for (a0, a1), (c0, c1) in zip(pcs, pcs[1:]):
            assert a1 == c0, "pieces must tile the buffer"
        if len(pcs) > 1:
            assert n >= km.K_SPLIT_MIN, "small buffers are never split"
            for lo, hi in pcs:
                assert hi - lo >= km.K_MIN_PIECE
                assert (n - hi) % km.K_SPLIT_GRAIN == 0
        else:
            assert pcs[0] == (0, n)


@pytest.mark.parametrize("seed", range(6))
def test_partition_invariants(seed):
    rnd = random.Random(100 + seed)
    n = rnd.choice([1, 5, 300, 3000])
    kinds = [lambda: 0, lambda: rnd.randint(0, 64), lambda: rnd.randint(0, 70000),
             lambda: rnd.randint(100000, 3_000_000), lambda: 1 << 20]
    lens = [rnd.choice(kinds)() for _ in range(n)]
    mem = np.zeros(1, dtype=np.uint8)
    b = km.Batch(mem, [0] * n, lens)
    for num_cus in (1, 3, 256):
        for dyn_shift in (0, 1, 2, km.K_DYN_AUTO):
            _check_partition(b, num_cus, dyn_shift)


def test_partition_config4_shape():
    lens = [int(x) for x in o.zipf_lens(100000)]
    b = km.Batch(np.zeros(1, dtype=np.uint8), [0] * len(lens), lens)
    _check_partition(b, 256)
    _check_partition(b, 256, 0)


def test_dynamic_units_chain():
    """Static ranges and dynamic units tile [0, total) exactly, including
    totals that are not multiples of the unit; config 3 engages the dynamic
    half with one claim counter of 262144 units."""
    for total in (2**36, 2**36 + 12345, 13_123_505_587, 3 * 2**30 + 7):
        b = km.Batch(np.zeros(1, dtype=np.uint8), [0], [total])
        rs = km.wave_ranges(b, 256)
        assert sum(1 for *_, last in rs if last) == 1
        ends = sorted((s0, s1) for s0, s1, _ in rs if s1 > s0)
        assert ends[0][0] == 0 and ends[-1][1] == total
        for (a0, a1), (c0, c1) in zip(ends, ends[1:]):
            assert a1 == c0
    # config 3 (1 MiB mean): a quarter dynamic; config 4 (128 KiB mean): half
    b = km.Batch(np.zeros(1, dtype=np.uint8), [0] * 65536, [1 << 20] * 65536)
    assert len(km.wave_ranges(b, 256)) == 4096 + (2**34 >> 17)
    lens = [int(x) for x in o.zipf_lens(100000)]
    b = km.Batch(np.zeros(1, dtype=np.uint8), [0] * len(lens), lens)
    assert len(km.wave_ranges(b, 256)) == 4096 + -(-(sum(lens) >> 1) // (128 << 10))


@pytest.mark.parametrize("dyn_shift,unit", [(1, 128 << 10), (2, 128 << 10), (1, 200_000)])
def test_model_dynamic_tail_matches_oracle(dyn_shift, unit):
    rnd = random.Random(7 + dyn_shift)
    mem = np.random.default_rng(dyn_shift).integers(0, 256, size=21_000_000, dtype=np.uint8)
    lens = [0, 3, 4000, 70000, 200_001, 1 << 20, 3_000_017, 3_000_017, 5_000_011, 65536, 2, 131072,
            4_000_003] + [rnd.randint(0, 300_000) for _ in range(4)]
    rnd.shuffle(lens)
    addrs, seeds = _mk_batch(rnd, mem.size, lens)
    b = km.Batch(mem, addrs, lens, seeds)
    ranges = km.wave_ranges(b, 1, dyn_shift, unit)
    assert len(ranges) > 16, "dynamic tail must be active in this case"
    got = km.run_batch(b, num_cus=1, dyn_shift=dyn_shift, unit=unit)
    exp = [o.cg_crc32(mem[a:a + L], s) for a, L, s in zip(addrs, lens, seeds)]
    assert list(got) == exp


@pytest.mark.parametrize("shape", ["ragged_with_empties", "config4", "grid_edges"])
def test_device_search_and_first_buffer(shape):
    """The device's range search (BatchView::lower_bound_ex + snap_at) returns
    the snapped boundary, lower_bound of it and the first buffer overlapping
    it -- the values the piece walk starts from without another read.  Checked
    against the definitions (np.searchsorted, Batch.snap, the walk's own
    decrement).  grid_edges aims targets where the end-relative split grid
    puts the snap exactly on a buffer's end (q == n: its end, not inside it;
    a round-2 kernel bug complemented such buffers)."""
    M = km
    rnd = random.Random({"ragged_with_empties": 1, "config4": 2, "grid_edges": 3}[shape])
    if shape == "config4":
        lens = [M.config4_len(i) for i in range(20000)] if hasattr(M, "config4_len") else \
            [int(1024 / (1 - rnd.random() * 127 / 128) ** 2) for _ in range(20000)]
    elif shape == "grid_edges":
        lens = [rnd.choice([3 * (64 << 10) + rnd.randint(1, 5000), 1 << 20, 200_000]) for _ in range(3000)]
    else:
        lens = [rnd.choice([0, 0, 7, 4096, 130_000, 1 << 20, rnd.randint(0, 3 << 20)]) for _ in range(5000)]
    b = M.Batch(np.zeros(1, dtype=np.uint8), [0] * len(lens), lens)
    targets = [rnd.randrange(0, b.total + 1) for _ in range(600)] + [0, b.total, b.total - 1]
    if shape == "grid_edges":  # just past the last full grid cell of a buffer
        for i in rnd.sample(range(len(lens)), 300):
            b0, b1 = int(b.prefix[i]), int(b.prefix[i + 1])
            targets += [b1 - (64 << 10) + 1, b1 - 1, b0 + 1, b0 + (b1 - b0) % (64 << 10) + 1]
    for t in targets:
        t = min(max(t, 0), b.total)
        S, lb, first = M.device_snap(b, t)
        assert S == b.snap(t), t
        assert lb == b.lower_bound(S), t
        f = lb
        if 0 < f <= b.n and int(b.prefix[f]) > S:
            f -= 1
        assert first == f, (t, S, lb, first)


# ------------------------------------------------------------ small-buffer kernel model

@pytest.mark.parametrize("G,blk", [(16, 256), (8, 256), (8, 128)])
def test_small_group_model_matches_oracle(G, blk):
    """The small body's algebra (256-B blocks on MCT(x^2048), or the 8-lane
    form's 128-B blocks on MCT(x^1024); end alignment, in-lane and cross-lane
    folds, padding undone) reproduces zlib's CRC for every length 0..600 and
    the block boundaries, at every 16-B misalignment of a sample, with seeds
    and with extra leading empty blocks."""
    T = km.tables()
    rng = np.random.default_rng(G + blk)
    mem = rng.integers(0, 256, 9000 + 64, dtype=np.uint8)
    lengths = list(range(0, 601, 7)) + [255, 256, 257, 511, 512, 1023, 1024, 1025, 2048, 4095, 4096, 8191, 8192]
    for L in lengths:
        for off in (0, 3, 13):
            seed = int(rng.integers(0, 2**32)) if L % 3 else 0
            got = km.crc_small_group(mem, 16 + off, L, seed, G, T, extra_blocks=L % 2, blk=blk)
            assert got == zlib.crc32(mem[16 + off:16 + off + L].tobytes(), seed), (L, off, G, blk)


def test_split_plan_model_lists():
    """The split plan's lists: the batch kernel's buffers below 1 MiB first,
    then the others, each class in index order (round 4); the small
    list holds every buffer <= 8 KiB once, ordered by 256-B block count within
    each 8192-buffer tile (index order within a class); the split rule and the
    workgroup share follow zcrc_kernels.hip."""
    rng = np.random.default_rng(5)
    # config-4-like law: most buffers small, a few MiB-sized ones carry the bytes
    u = rng.random(20000)
    lens = np.clip(1024.0 / (1.0 - u * 127.0 / 128.0) ** 2, 1024, 16 << 20).astype(np.int64)
    p = km.split_plan(lens)
    assert p["split"] and 1 <= p["wgs"] <= 255
    assert sorted(p["large"] + p["small"]) == list(range(len(lens)))
    assert all(lens[i] > 8192 for i in p["large"])
    med = [i for i in p["large"] if lens[i] < (1 << 20)]
    assert med == sorted(med) and p["large"] == med + sorted(set(p["large"]) - set(med))
    assert 0 < len(med) < len(p["large"])
    tile = km.split_tile(len(lens))
    key = [(i // tile, (int(lens[i]) + 255) >> 8, i) for i in p["small"]]
    assert key == sorted(key)
    # all large: nothing to split; all small: every workgroup takes the small list
    assert not km.split_plan([70000] * 10000)["split"]
    q = km.split_plan([1000] * 10000)
    assert q["split"] and q["wgs"] == 256 and q["lanes"] == 8 and q["direct"]  # mode 2: no lists
    assert not km.split_plan([1000] * 10000, direct_ok=False).get("direct")
    assert not km.split_plan(list(range(100, 8100)) * 2).get("direct")  # ragged small: the class-ordered list
    # a handful of small buffers among large ones is not worth two workgroups
    few = [1 << 20] * 9000 + [100] * 5
    assert not km.split_plan(few)["split"] and km.split_plan(few, force=True)["split"]


def test_per_buffer_mode_rule_and_mapping():
    """One-launch batches: the per-buffer mode covers every buffer exactly
    once, spreads a batch of n < 16 x CUs over all CUs (at most
    ceil(n / CUs) waves per workgroup), and falls back for a buffer above
    64 KiB or more buffers than waves."""
    for n in (1, 5, 255, 256, 257, 1000, 4095, 4096):
        m = km.per_buffer_plan([65536] * n)
        assert sorted(m) == list(range(n))
        per_wg = {}
        for g, s in m.values():
            per_wg[g] = per_wg.get(g, 0) + 1
        assert max(per_wg.values()) == -(-n // 256)
        assert len(per_wg) == min(n, 256)
    assert km.per_buffer_plan([65537]) is None
    assert km.per_buffer_plan([1] * 4097) is None
    assert km.per_buffer_plan([1] * 4097, num_cus=512) is not None


def test_per_buffer_braid_build_equals_loaded_fill():
    """The per-buffer mode builds the braid in registers (no table load ahead
    of its first barrier); every one of the 32,768 LDS words must equal what
    the table fill writes from TableBlob::braid."""
    assert np.array_equal(km.braid_lds_built(), km.braid_lds_loaded())


def test_per_buffer_comb_build_equals_table_blob():
    """Round 4: the per-buffer mode also builds the 8 combine tables in
    registers (comb_gen); the 8,192-word combine area must equal
    TableBlob::comb as the other forms load it."""
    T = km.tables()
    comb = np.concatenate([t.reshape(-1) for t in T.comb])
    assert np.array_equal(km.comb_lds_built(), comb)


def test_per_buffer_flags_sit_on_zero_combine_words():
    """The round-3 per-buffer form (kPB = 3, kept for A/B in tools/) stores wave s's decision flag in the combine-area
    word 256 s: the first word of the chunk lane 0 of wave s writes (chunk
    64 s = table s >> 2, sub-table j = s & 3, v = 0), which is MCT(c)[j][0] =
    0 in every table -- so an all-clear decision leaves the tables exact."""
    T = km.tables()
    comb = np.concatenate([t.reshape(-1) for t in T.comb])  # the kernel's comb area, 8 x 1024 words
    for s in range(16):
        chunk = 64 * s
        assert 4 * chunk == 256 * s
        c, j, v = chunk >> 8, (chunk >> 6) & 3, 4 * (chunk & 63)
        assert (c, j, v) == (s >> 2, s & 3, 0)
        assert comb[256 * s] == 0 and T.comb[c][j, 0] == 0


def test_xinv8_byte_table_inverts_one_zero_byte():
    """The small body's trailing-padding step r * x^-8 = (r << 8) ^ xinv8[r >> 24]
    (zcrc_gf2.h build_xinv8_table): the top bytes of the standard table are a
    permutation, so the step is defined for every r and equals 8 exact x^-1
    steps; it undoes one zero byte fed through the register."""
    T = km.tables()
    assert sorted(int(t) >> 24 for t in T.stdtab) == list(range(256))
    rng = np.random.default_rng(3)
    for r in [0, 1, 0x80000000, 0xFFFFFFFF] + [int(x) for x in rng.integers(0, 1 << 32, 2000, dtype=np.uint64)]:
        w = ((r << 8) & 0xFFFFFFFF) ^ int(T.xinv8[r >> 24])
        b = r
        for _ in range(8):
            b = km.times_xinv(b)
        assert w == b
        fwd = (w >> 8) ^ int(T.stdtab[w & 0xFF])  # one zero byte forward
        assert fwd == r


def test_one_launch_short_buffers_per_wave_long_ones_scanned():
    """Round-4 per-buffer mode (kernel_model.run_one_launch): short buffers
    (<= 64 KiB) whole per wave, the long ones through the in-kernel scan over
    effective lengths with the short ones skipped -- every CRC equals the
    oracle's, with seeds, tiny and empty buffers, and splits of the long ones."""
    from oracle import oracle as o
    rng = np.random.default_rng(11)
    lens = [0, 1, 3, 4, 100, 65536, 65537, 300_001, 5, 200_000, 70_000, 65535, 17]
    offs = np.zeros(len(lens), dtype=np.int64)
    offs[1:] = np.cumsum(np.array(lens) + 5)[:-1]
    mem = rng.integers(0, 256, int(offs[-1] + lens[-1] + 64), dtype=np.uint8)
    seeds = [int(x) for x in rng.integers(0, 1 << 32, len(lens), dtype=np.uint64)]
    b = km.Batch(mem, offs + 3, lens, seeds)
    got = km.run_one_launch(b, num_cus=4)  # 4 CUs: the long buffers split across waves
    exp = o.crc32_batch((mem.ctypes.data + offs + 3).astype(np.uint64), np.array(lens, dtype=np.uint64),
                        np.array(seeds, dtype=np.uint32))
    np.testing.assert_array_equal(got, exp)



def test_model_constants_mirror_the_header():
    """tests/kernel_model.py's K_* constants equal zcrc_internal.h's (the
    header is parsed as text: `constexpr <type> kName = <expr>;`)."""
    import re
    src = open(os.path.join(os.path.dirname(__file__), "..", "zipsfs_amd", "csrc", "zcrc_internal.h")).read()
    vals = {}
    for name, expr in re.findall(r"constexpr\s+[\w:]+\s+(k\w+)\s*=\s*([^;]+);", src):
        e = re.sub(r"(\d+)u?ll|(\d+)u\b", lambda m: m.group(1) or m.group(2), expr)
        try:
            vals[name] = eval(e, {}, dict(vals))  # noqa: S307 -- our own header's integer expressions
        except Exception:
            pass
    pairs = {"kWaves": km.K_WAVES, "kMinRange": km.K_MIN_RANGE, "kSplitGrain": km.K_SPLIT_GRAIN,
             "kSplitMin": km.K_SPLIT_MIN, "kMinPiece": km.K_MIN_PIECE, "kDynUnit": km.K_DYN_UNIT,
             "kDynAuto": km.K_DYN_AUTO, "kDynSmallAvg": km.K_DYN_SMALL_AVG, "kSmallMax": km.K_SMALL_MAX,
             "kBigMin": km.K_BIG_MIN, "kSmallCostDefault": km.K_SMALL_COST,
             "kSplitMaxTiles": km.K_SPLIT_MAX_TILES}
    for name, model in pairs.items():
        assert vals.get(name) == model, (name, vals.get(name), model)


def test_grain_table_shift_equals_x_power():
    """The split-piece shift by whole 64 KiB grains (x8grain, at most four
    products) equals multiplying by x^(8d) bit by bit, for d across the four
    table rows (d up to 2^42 bytes, kMaxLaunchBytes)."""
    rnd = random.Random(8)
    g = km.x8grain_table()
    ds = [65536 * m for m in (1, 2, 255, 256, 257, 4577, 65535, 65536, 68664, (1 << 24) - 1, 1 << 24,
                              (1 << 26) - 1)]
    ds += [65536 * rnd.randrange(1, 1 << 26) for _ in range(20)]
    for d in ds:
        r = rnd.getrandbits(32)
        assert km.grain_shift(r, d, g) == km.gf2_mul(km.xpow8(d), r), d

