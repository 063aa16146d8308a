"""GPU parity of the small-buffer kernel (zipsfs_amd/csrc/zcrc_small_kernel.h).

Whole buffers of at most kSmallMax = 8192 bytes go to the small kernel from
the strided API, the host batch API (zcrc32_batch: direct and staged paths,
where a mixed launch is partitioned into batch-kernel and small-kernel lists)
and the device API's split plan.  Every result is compared bit-exactly with
the CPU oracle (oracle/) or zlib on the same bytes, and with the batch kernel
alone (ZCRC_SMALL=0).
"""
import random
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import zipsfs_amd as z  # noqa: E402
from oracle import oracle as o  # noqa: E402

DEV = "cuda:0"
SMALL_MAX = 8192

# every length 0..300, then the block (256 B), lane-group (2 KiB mean: 8 vs 16
# lanes) and size-limit boundaries
LENGTHS = list(range(0, 301)) + [
    511, 512, 513, 1000, 1023, 1024, 1025, 2047, 2048, 2049, 3000, 3971, 4095, 4096, 4097,
    6000, 8175, 8176, 8177, 8191, 8192, 8193, 12288, 16384]


def u32(t):
    return t.cpu().numpy().view(np.uint32)


def _seeds(rnd, n):
    s = np.array([rnd.getrandbits(32) for _ in range(n)], dtype=np.uint32)
    s[::5] = 0
    return s, torch.tensor(s.view(np.int32), device=DEV)


def _oracle(host, base_addr_offsets, lens, seeds):  # noqa: D103
    ap = np.array([host.ctypes.data + int(q) for q in base_addr_offsets], dtype=np.uint64)
    return o.crc32_batch(ap, np.asarray(lens, dtype=np.uint64), seeds, nthreads=8)


@pytest.mark.parametrize("small", ["1", "0"])
def test_strided_every_small_length(small, monkeypatch):
    """Strided batches of each length at a misaligned base and odd strides,
    with seeds; n = 37 (not a multiple of the 4 or 8 buffers per wave)."""
    monkeypatch.setenv("ZCRC_SMALL", small)
    rnd = random.Random(11)
    n = 37
    for L in LENGTHS:
        lead, stride = rnd.randrange(16), L + rnd.choice([0, 1, 3, 16, 29])
        total = lead + n * stride + 64
        mem = torch.randint(0, 256, (total,), dtype=torch.uint8, device=DEV)
        seeds_np, seeds = _seeds(rnd, n)
        got = u32(z.crc32_batch_strided(mem[lead:], stride, L, n, seeds=seeds))
        host = mem.cpu().numpy()
        exp = _oracle(host, [lead + i * stride for i in range(n)], [L] * n, seeds_np)
        np.testing.assert_array_equal(got, exp, err_msg=f"len {L}")


def test_strided_large_uniform_batches():
    """Whole-chip uniform batches (1 KiB and 4 KiB, 64 MiB each): every CRC
    against the oracle on the generator's bytes, with and without seeds."""
    for L in (1024, 4096, 3000):
        n = (64 << 20) // L
        mem = torch.empty(n * L + 64, dtype=torch.uint8, device=DEV)
        ptrs = mem.data_ptr() + torch.arange(n, dtype=torch.int64, device=DEV) * L
        lens = torch.full((n,), L, dtype=torch.int64, device=DEV)
        z.fill_synthetic(ptrs, lens, index0=5, seed=o.PAYLOAD_SEED)
        got = u32(z.crc32_batch_strided(mem, L, L, n))
        host = mem.cpu().numpy()
        exp = _oracle(host, [i * L for i in range(n)], [L] * n, np.zeros(n, np.uint32))
        np.testing.assert_array_equal(got, exp, err_msg=f"len {L}")
        seeds_np = (np.arange(n, dtype=np.uint64) * 2654435761 % (1 << 32)).astype(np.uint32)
        seeds = torch.tensor(seeds_np.view(np.int32), device=DEV)
        got = u32(z.crc32_batch_strided(mem, L, L, n, seeds=seeds))
        exp = _oracle(host, [i * L for i in range(n)], [L] * n, seeds_np)
        np.testing.assert_array_equal(got, exp, err_msg=f"len {L} seeded")


@pytest.mark.parametrize("small", ["1", "0"])
def test_host_batch_direct_and_partitioned(small, monkeypatch):
    """zcrc32_batch: all-small direct calls, mixed direct calls, and staged
    launches that mix continuation parts, large and small buffers."""
    monkeypatch.setenv("ZCRC_SMALL", small)
    rnd = random.Random(5)
    cases = [
        [rnd.choice(LENGTHS) for _ in range(300)],                            # direct, all small
        [rnd.choice(LENGTHS + [20_000, 65_536]) for _ in range(200)],         # direct, mixed
        [rnd.choice(LENGTHS + [100_000, 3_000_000]) for _ in range(3000)],    # staged, mixed
        [5, 17 << 20, 4096, 0, 3, (40 << 20) + 7, 8192, 1, 8193, 100],        # continuation parts
    ]
    for k, lens in enumerate(cases):
        bufs = [o.payload(L, 900 + k * 10_000 + i) for i, L in enumerate(lens)]
        seeds = [rnd.getrandbits(32) if i % 3 else 0 for i in range(len(bufs))]
        got = z.crc32_batch(bufs, seeds=seeds)
        exp = [zlib.crc32(b.tobytes(), s) for b, s in zip(bufs, seeds)]
        assert list(got) == exp, f"case {k}"


def test_config4_golden_through_host_batch(golden):
    """The config-4 golden sample (reference CRCs) through the host batch API,
    whose staged launches split it between the two kernels."""
    cfg = golden["cfg"]
    idx = cfg["cfg4_idx"].astype(np.int64)
    L = cfg["cfg4_len"].astype(np.int64)
    bufs = [o.payload(int(n), int(i)) for n, i in zip(L, idx)]
    got = z.crc32_batch(bufs)
    np.testing.assert_array_equal(np.asarray(got, dtype=np.uint32), cfg["cfg4"])
    assert int((L <= SMALL_MAX).sum()) > 0 and int((L > SMALL_MAX).sum()) > 0


def _device_batch(rnd, lens, max_gap=40):
    offs, pos = [], rnd.randrange(16)
    for L in lens:
        offs.append(pos)
        pos += L + rnd.randrange(max_gap)
    mem = torch.randint(0, 256, (pos + 64,), dtype=torch.uint8, device=DEV)
    ptrs = torch.tensor([mem.data_ptr() + q for q in offs], dtype=torch.int64, device=DEV)
    return mem, offs, ptrs, torch.tensor(lens, dtype=torch.int64, device=DEV)


@pytest.mark.parametrize("small", ["1", "0", "2"])
@pytest.mark.parametrize("shape", ["mixed", "all_small", "all_large", "sorted"])
def test_device_split_plan(shape, small, monkeypatch):
    """zcrc32_batch_device above kFusedMaxN buffers: the split plan sends the
    small ones to the small kernel and the rest, compacted, to the batch
    kernel (results written back through the original index), with and
    without seeds.  ZCRC_SMALL=1: split when the small list is worth two
    workgroups; 2: whenever there is a small buffer; 0: never."""
    monkeypatch.setenv("ZCRC_SMALL", small)
    rnd = random.Random(zlib.crc32(shape.encode()))
    n = {"mixed": 20_000, "all_small": 50_000, "all_large": 9_000, "sorted": 12_000}[shape]
    if shape == "all_large":
        lens = [rnd.randint(SMALL_MAX + 1, 200_000) for _ in range(n)]
    elif shape == "all_small":
        lens = [rnd.choice(LENGTHS[:-2]) for _ in range(n)]
    else:
        lens = [rnd.choice([rnd.choice(LENGTHS), rnd.randint(0, SMALL_MAX), rnd.randint(SMALL_MAX, 400_000)])
                for _ in range(n)]
        if shape == "sorted":  # long runs of small buffers, then the large ones
            lens.sort()
    mem, offs, ptrs, lt = _device_batch(rnd, lens)
    host = mem.cpu().numpy()
    seeds_np, seeds = _seeds(rnd, n)
    got = u32(z.crc32_batch_device(ptrs, lt, seeds=seeds))
    np.testing.assert_array_equal(got, _oracle(host, offs, lens, seeds_np))
    got = u32(z.crc32_batch_device(ptrs, lt))
    np.testing.assert_array_equal(got, _oracle(host, offs, lens, np.zeros(n, np.uint32)))
    # caller-owned scratch (graph-capturable entry point), same results
    scratch = torch.empty(z.scratch_bytes(n), dtype=torch.uint8, device=DEV)
    got = u32(z.crc32_batch_device_ws(ptrs, lt, scratch, seeds=seeds))
    np.testing.assert_array_equal(got, _oracle(host, offs, lens, seeds_np))


@pytest.mark.parametrize("direct", ["1", "0"])
@pytest.mark.parametrize("lens_kind", ["uniform_1k", "near_uniform", "uniform_tiny"])
def test_device_split_plan_direct_mode(lens_kind, direct, monkeypatch):
    """The split plan's mode 2 (round 4): a batch of about equal small
    buffers is walked in place by the small body (the caller's ptrs, lens and
    seeds, index order, no lists); ZCRC_SMALL_DIRECT=0 keeps the lists.
    Unaligned starts, seeds, results against the oracle."""
    monkeypatch.setenv("ZCRC_SMALL_DIRECT", direct)
    rnd = random.Random(len(lens_kind) * 11 + int(direct))
    n = 30_000
    lens = {"uniform_1k": [1024] * n, "near_uniform": [rnd.randint(900, 1200) for _ in range(n)],
            "uniform_tiny": [rnd.choice([0, 1, 2, 3, 5]) for _ in range(n)]}[lens_kind]
    mem, offs, ptrs, lt = _device_batch(rnd, lens)
    host = mem.cpu().numpy()
    seeds_np, seeds = _seeds(rnd, n)
    np.testing.assert_array_equal(u32(z.crc32_batch_device(ptrs, lt, seeds=seeds)), _oracle(host, offs, lens, seeds_np))
    np.testing.assert_array_equal(u32(z.crc32_batch_device(ptrs, lt)),
                                  _oracle(host, offs, lens, np.zeros(n, np.uint32)))


@pytest.mark.parametrize("join", [True, False])
def test_config4_golden_replicated_through_split_plan(golden, join, monkeypatch):
    """The config-4 golden sample repeated 9 times (> kFusedMaxN buffers, so
    the device split plan runs): every CRC equals the reference's -- with the
    small-list workgroups joining the dynamic part when done (the product)
    and without (ZCRC_AB_FLAGS=4, an A/B knob)."""
    if not join:
        monkeypatch.setenv("ZCRC_AB_FLAGS", "4")
    cfg = golden["cfg"]
    idx = cfg["cfg4_idx"].astype(np.int64)
    L = cfg["cfg4_len"].astype(np.int64)
    offs = np.zeros(len(L), dtype=np.int64)
    offs[1:] = np.cumsum(L + 3)[:-1]
    size = int(offs[-1] + L[-1] + 16)
    reps = 9
    mem = torch.empty(size * reps, dtype=torch.uint8, device=DEV)
    ptrs1 = mem.data_ptr() + 1 + torch.tensor(offs, device=DEV)
    lens1 = torch.tensor(L, device=DEV)
    for k in range(len(idx)):
        z.fill_synthetic(ptrs1[k:k + 1], lens1[k:k + 1], index0=int(idx[k]), seed=o.PAYLOAD_SEED)
    for r in range(1, reps):
        mem[r * size:(r + 1) * size].copy_(mem[:size])
    ptrs = torch.cat([ptrs1 + r * size for r in range(reps)])
    lens = lens1.repeat(reps)
    assert len(lens) > 8192
    got = u32(z.crc32_batch_device(ptrs, lens))
    np.testing.assert_array_equal(got, np.tile(cfg["cfg4"], reps))


def test_split_plan_graph_capture_replays():
    """The split path (plan launch, then one batch-kernel launch whose top
    workgroups run the small body on the small list) captured in a HIP graph
    and replayed after lengths and bytes change in place, so the small/large
    partition differs on every replay."""
    rnd = random.Random(17)
    n, cap = 12_000, 20_000
    mem = torch.zeros(n * cap, dtype=torch.uint8, device=DEV)
    ptrs = mem.data_ptr() + torch.arange(n, dtype=torch.int64, device=DEV) * cap
    lens = torch.zeros(n, dtype=torch.int64, device=DEV)
    out_a = torch.empty(n, dtype=torch.int32, device=DEV)
    out_b = torch.empty(n, dtype=torch.int32, device=DEV)
    scratch = torch.empty(z.scratch_bytes(n), dtype=torch.uint8, device=DEV)
    z.crc32_batch_device(ptrs, lens, out=out_a)  # warm-up outside capture
    z.crc32_batch_device_ws(ptrs, lens, scratch, out=out_b)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        z.crc32_batch_device(ptrs, lens, out=out_a)
        z.crc32_batch_device_ws(ptrs, lens, scratch, out=out_b)
    for rep in range(3):
        ln = [rnd.choice([0, rnd.randint(1, SMALL_MAX), rnd.randint(SMALL_MAX, cap)]) for _ in range(n)]
        lens.copy_(torch.tensor(ln, dtype=torch.int64))
        mem.copy_(torch.randint(0, 256, (n * cap,), dtype=torch.uint8, device=DEV))
        g.replay()
        torch.cuda.synchronize()
        host = mem.cpu().numpy()
        exp = _oracle(host, np.arange(n, dtype=np.uint64) * cap, ln, np.zeros(n, dtype=np.uint32))
        np.testing.assert_array_equal(u32(out_a), exp, err_msg=f"batch_device replay {rep}")
        np.testing.assert_array_equal(u32(out_b), exp, err_msg=f"batch_device_ws replay {rep}")


def test_profile_kinds_and_one_launch_split():
    """zcrc_profile separates the kernels: the strided path of small buffers
    times one small-kernel launch; a split device batch (small list inside
    the batch kernel's launch) times one batch-kernel launch and no other."""
    rnd = random.Random(3)
    mem = torch.randint(0, 256, (4096 * 1000,), dtype=torch.uint8, device=DEV)
    lens = [rnd.choice([100, 3000, 50_000]) for _ in range(10_000)]
    mem2, offs, ptrs, lt = _device_batch(rnd, lens)
    z.crc32_batch_strided(mem, 4096, 4096, 1000)
    z.crc32_batch_device(ptrs, lt)
    torch.cuda.synchronize()
    with z.profile() as prof:
        z.crc32_batch_strided(mem, 4096, 4096, 1000)
        torch.cuda.synchronize()
    assert (prof.launches, prof.small_launches) == (0, 1) and prof.small_ms > 0
    os_env = dict(ZCRC_SMALL="2")
    with pytest.MonkeyPatch.context() as mp:
        for k, v in os_env.items():
            mp.setenv(k, v)
        with z.profile() as prof:
            got = z.crc32_batch_device(ptrs, lt)
            torch.cuda.synchronize()
    assert (prof.launches, prof.small_launches) == (1, 0)
    np.testing.assert_array_equal(u32(got), _oracle(mem2.cpu().numpy(), offs, lens, np.zeros(len(lens), np.uint32)))
    assert "crc32_small_kernel" in z.small_kernel_name()


def test_split_batches_overlapping_on_four_streams():
    """Split-plan launches (> 8192 buffers, small-list share varying from
    none to all) from four host threads on four streams at once, each
    queueing six launches without synchronising; per-stream scratch grows
    under queued work.  Every result vs the oracle."""
    from concurrent.futures import ThreadPoolExecutor
    rnd = random.Random(321)
    total = 64 << 20
    mem = torch.randint(0, 256, (total,), dtype=torch.uint8, device=DEV)
    host = mem.cpu().numpy()
    streams = [torch.cuda.Stream(device=DEV) for _ in range(4)]
    plans = []
    for t in range(4):
        jobs = []
        for j in range(6):
            n = rnd.randint(8193, 30000)
            share = rnd.choice([0.0, 0.3, 0.9, 1.0])
            ln = [rnd.randint(0, SMALL_MAX) if rnd.random() < share else rnd.randint(SMALL_MAX + 1, 60_000)
                  for _ in range(n)]
            offs = [rnd.randrange(0, total - L) for L in ln]
            jobs.append((offs, ln))
        plans.append(jobs)

    def work(t):
        st = streams[t]
        outs = []
        with torch.cuda.stream(st):
            for offs, ln in plans[t]:
                ptrs = torch.tensor([mem.data_ptr() + q for q in offs], dtype=torch.int64, device=DEV)
                lt = torch.tensor(ln, dtype=torch.int64, device=DEV)
                outs.append((z.crc32_batch_device(ptrs, lt), ptrs, lt))
            st.synchronize()
        return [u32(o) for o, _, _ in outs]

    with ThreadPoolExecutor(4) as ex:
        res = list(ex.map(work, range(4)))
    for t in range(4):
        for j, ((offs, ln), got) in enumerate(zip(plans[t], res[t])):
            exp = _oracle(host, offs, ln, np.zeros(len(ln), dtype=np.uint32))
            np.testing.assert_array_equal(got, exp, err_msg=f"thread {t} job {j}")


def _split_lists(scratch, n):
    """The split plan's outputs in caller-owned scratch (SplitScratch,
    zcrc_runtime.hip): counts, prefix_c, oidx, and the small list's buffer
    indices (word 2 of each 16-B descriptor), pointers and lengths."""
    import kernel_model as km
    raw = scratch.cpu().numpy()
    T = -(-n // km.split_tile(n))
    prefix = 256
    tiles = prefix + 8 * (n + 1)
    tile_pre = tiles + 56 * T  # kTileWords = 7
    ptrs = tile_pre + 56 * (T + 1)
    seeds = ptrs + 8 * n
    oidx = seeds + 4 * n
    sdesc = (oidx + 4 * n + 15) // 16 * 16
    counts = raw[128:176].view(np.uint64)
    return (counts, raw[prefix:prefix + 8 * (n + 1)].view(np.uint64), raw[oidx:oidx + 4 * n].view(np.uint32),
            raw[sdesc:sdesc + 16 * n].view(np.uint32).reshape(n, 4))


@pytest.mark.parametrize("n,shape", [(20_000, "mixed"), (50_000, "all_small"), (4_200_000, "mixed"),
                                     (4_300_000, "all_small"), (20_000, "mixed_big"), (60_000, "mixed_big"),
                                     (30_000, "uniform_small"), (600_000, "near_uniform_small"),
                                     (20_000, "uniform_medium"), (20_000, "uniform_medium_but_one")])
def test_split_plan_lists_equal_the_model(n, shape):
    """The plan's decision, the compacted batch (order and byte prefix) and the
    small list (tile by tile, by size class, index order within a class) equal
    tests/kernel_model.py's split_plan; above 512 tiles (n > 4,194,304) through
    the tile-scan kernel.  Every CRC against the oracle."""
    import kernel_model as km
    rng = np.random.default_rng(n)
    top = SMALL_MAX + 1 if n < 1_000_000 else 600  # keep the 4M-buffer batches near 1 GiB
    if shape == "all_small":
        lens = rng.integers(0, min(top, 700), n)
    elif shape == "uniform_small":  # the split plan's mode 2 (direct): no lists
        lens = np.full(n, 1024)
    elif shape == "near_uniform_small":
        lens = rng.integers(1000, 1300, n)
    elif shape.startswith("uniform_medium"):  # unsplit, equal (counts[5] = 1) -- or all but the last
        lens = np.full(n, 70_001)
        if shape.endswith("one"):
            lens[-1] = 70_000
    elif shape == "mixed":  # ZIP-entry-like: most small, some large
        lens = np.where(rng.random(n) < 0.995, rng.integers(0, top, n), rng.integers(SMALL_MAX + 1, 40_000, n))
    else:  # mixed_big: medium and big (>= 1 MiB, kBigMin) batch-kernel buffers interleaved (round-4 order)
        u = rng.random(n)
        lens = np.where(u < 0.99, rng.integers(0, top, n),
                        np.where(u < 0.995, rng.integers(SMALL_MAX + 1, 1 << 20, n), rng.integers(1 << 20, 3 << 20, n)))
        lens[:3] = [1 << 20, (1 << 20) - 1, SMALL_MAX + 1]  # the class edges
    lens = lens.astype(np.int64)
    offs = np.zeros(n, dtype=np.int64)
    offs[1:] = np.cumsum(lens + 3)[:-1]
    mem = torch.randint(0, 256, (int(offs[-1] + lens[-1] + 64),), dtype=torch.uint8, device=DEV)
    ptrs = mem.data_ptr() + torch.tensor(offs, device=DEV)
    lt = torch.tensor(lens, device=DEV)
    scratch = torch.empty(z.scratch_bytes(n), dtype=torch.uint8, device=DEV)
    got = u32(z.crc32_batch_device_ws(ptrs, lt, scratch))
    counts, prefix, oidx, sdesc = _split_lists(scratch, n)
    model = km.split_plan(lens.tolist(), grid=z.device_info()["num_cus"])
    assert bool(counts[2]) == model["split"], counts
    assert (int(counts[2]) == 2) == model.get("direct", False), counts
    # every length equal and unsplit: the batch kernel's window order may apply
    assert int(counts[5]) == int(not model["split"] and len(set(lens.tolist())) == 1), counts
    if model.get("direct"):
        assert int(counts[1]) == n and int(counts[0]) == 0 and int(counts[4]) == z.device_info()["num_cus"]
    elif model["split"]:
        nl, ns = int(counts[0]), int(counts[1])
        assert (nl, ns) == (len(model["large"]), len(model["small"]))
        np.testing.assert_array_equal(oidx[:nl], np.array(model["large"], dtype=np.uint32))
        small = np.array(model["small"], dtype=np.int64)
        np.testing.assert_array_equal(sdesc[:ns, 2], small.astype(np.uint32))
        pw = sdesc[:ns, 0].astype(np.uint64) | (sdesc[:ns, 1].astype(np.uint64) << np.uint64(32))
        np.testing.assert_array_equal(pw >> np.uint64(48), lens[small].astype(np.uint64))
        np.testing.assert_array_equal(pw & np.uint64((1 << 48) - 1), (mem.data_ptr() + offs[small]).astype(np.uint64))
        large_lens = lens[model["large"]]
        np.testing.assert_array_equal(prefix[:nl + 1], np.concatenate([[0], np.cumsum(large_lens)]).astype(np.uint64))
        assert int(counts[3]) == model["lanes"] and int(counts[4]) == model["wgs"], counts
    else:
        np.testing.assert_array_equal(prefix, np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64))
    host = mem.cpu().numpy()
    exp = o.crc32_batch((host.ctypes.data + offs).astype(np.uint64), lens.astype(np.uint64), None, nthreads=16)
    np.testing.assert_array_equal(got, exp)


def _packed_batch(lead, lens, gap_rnd):
    """Buffers laid out one after another (random 0-15 B gaps, misaligned
    starts) in one device allocation: (mem, ptrs, lens tensor, offsets)."""
    offs, pos = [], lead
    for L in lens:
        offs.append(pos)
        pos += int(L) + gap_rnd.randrange(16)
    mem = torch.randint(0, 256, (pos + 64,), dtype=torch.uint8, device=DEV)
    ptrs = mem.data_ptr() + torch.tensor(offs, dtype=torch.int64, device=DEV)
    return mem, ptrs, torch.tensor([int(x) for x in lens], dtype=torch.int64, device=DEV), offs


@pytest.mark.parametrize("max_len", [1024, 2048, 4096, 8192])
def test_maxlen_hint_mixed_small_lengths(max_len):
    """zcrc32_batch_device_maxlen (round 6): a caller
    bound <= 8 KiB runs the batch in one small-kernel launch over the
    caller's arrays.  Mixed lengths 0..max_len at misaligned starts, with
    seeds, n > 8192 -- bit-exact against the oracle and against the
    unhinted call."""
    rnd = random.Random(max_len)
    n = 9000
    lens = [rnd.randrange(max_len + 1) for _ in range(n)]
    edge = [L for L in LENGTHS if L <= max_len]  # every boundary length up to the bound
    lens[:len(edge)] = edge
    mem, ptrs, lt, offs = _packed_batch(5, lens, rnd)
    seeds_np, seeds = _seeds(rnd, n)
    got = u32(z.crc32_batch_device(ptrs, lt, seeds=seeds, max_len=max_len))
    ref = u32(z.crc32_batch_device(ptrs, lt, seeds=seeds))
    exp = _oracle(mem.cpu().numpy(), offs, lens, seeds_np)
    np.testing.assert_array_equal(got, exp)
    np.testing.assert_array_equal(ref, exp)


def test_maxlen_hint_is_only_a_hint():
    """Lengths above the caller's bound (up to 300 KiB) are still exact; so
    are a bound of 0 (unknown), a bound above 8 KiB and n <= 8192 (both the
    unhinted path)."""
    rnd = random.Random(77)
    n = 10000
    lens = [rnd.randrange(1025) for _ in range(n)]
    for k in range(0, n, 997):
        lens[k] = rnd.choice([8193, 20000, 65536, 300000])
    mem, ptrs, lt, offs = _packed_batch(3, lens, rnd)
    exp = _oracle(mem.cpu().numpy(), offs, lens, np.zeros(n, np.uint32))
    for ml in (1024, 0, 65536):
        np.testing.assert_array_equal(u32(z.crc32_batch_device(ptrs, lt, max_len=ml)), exp, err_msg=f"max_len {ml}")
    np.testing.assert_array_equal(u32(z.crc32_batch_device(ptrs[:5000], lt[:5000], max_len=1024)), exp[:5000])


def test_maxlen_uniform_golden_config2_shape():
    """A whole-chip uniform 1 KiB batch (1 Mi buffers of the generator's
    payload) through the hint: equal to the strided path everywhere and to
    the oracle on a sample."""
    L, n = 1024, 1 << 20
    mem = torch.empty(n * L + 64, dtype=torch.uint8, device=DEV)
    ptrs = mem.data_ptr() + torch.arange(n, dtype=torch.int64, device=DEV) * L
    lens = torch.full((n,), L, dtype=torch.int64, device=DEV)
    z.fill_synthetic(ptrs, lens, index0=9, seed=o.PAYLOAD_SEED)
    got = u32(z.crc32_batch_device(ptrs, lens, max_len=L))
    np.testing.assert_array_equal(got, u32(z.crc32_batch_strided(mem, L, L, n)))
    sample = np.arange(0, n, 4099)
    exp = np.array([o.payload_crc(L, 9 + int(i)) for i in sample], dtype=np.uint32)
    np.testing.assert_array_equal(got[sample], exp)
