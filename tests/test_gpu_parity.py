"""GPU parity: libzcrc's HIP kernels vs the oracle / reference golden vectors.

Every test calls the product through its C ABI (ctypes over libzcrc.so) and
compares bit-exactly with (a) golden vectors produced by the reference's own
src/cg_crc32.c (tests/golden/) or (b) the CPU restatement oracle/ on the
same bytes.  Run on the MI355X box:  pytest -m gpu
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
SEED = o.PAYLOAD_SEED


def u32(t):
    return t.cpu().numpy().view(np.uint32)


def dev_buffers_from_host(chunks, align=16, gap=0, lead=0):
    """Pack host byte strings into one device allocation; return (mem, ptrs, lens, addrs)."""
    offs, pos = [], lead
    for c in chunks:
        offs.append(pos)
        pos += len(c) + gap
        pos = (pos + align - 1) // align * align if align > 1 else pos
    host = np.zeros(max(pos, 1), dtype=np.uint8)
    for off, c in zip(offs, chunks):
        host[off:off + len(c)] = np.frombuffer(c, dtype=np.uint8)
    mem = torch.from_numpy(host).to(DEV)
    base = mem.data_ptr()
    ptrs = torch.tensor([base + off for off in offs], dtype=torch.int64, device=DEV)
    lens = torch.tensor([len(c) for c in chunks], dtype=torch.int64, device=DEV)
    return mem, ptrs, lens


def test_device_visible():
    assert torch.cuda.is_available()
    info = z.device_info()
    assert info["num_cus"] >= 1


def test_kats_host_api(golden):
    for k in golden["meta"]["kats"]:
        if "text_seq" in k:
            a, b = k["text_seq"]
            data = "".join(f"{i}\n" for i in range(a, b + 1)).encode()
        else:
            data = bytes.fromhex(k["hex"])
        assert z.cg_crc32(data) == k["crc"], k["name"]
    assert z.cg_crc32(b"123456789") == 0xCBF43926
    assert z.cg_crc32(b"123456789", 4) == zlib.crc32(b"1234")
    assert z.fhandle_check_crc32(b"123456789", 0xCBF43926)
    assert not z.fhandle_check_crc32(b"123456789", 0xCBF43927)


def test_lengths_offsets_device(golden):
    """Every length 0..1100 (and a sweep to 4096) at every 16-B misalignment."""
    lo = golden["lo"]
    base = o.payload(int(lo["payload_len"]), int(lo["payload_index"]))
    mem = torch.from_numpy(np.concatenate([np.zeros(64, np.uint8), base, np.zeros(64, np.uint8)])).to(DEV)
    b0 = mem.data_ptr() + 64
    lengths = lo["lengths"].astype(np.int64)
    L = np.repeat(lengths, 16)
    off = np.tile(np.arange(16, dtype=np.int64), len(lengths))
    ptrs = torch.tensor(b0 + off, dtype=torch.int64, device=DEV)
    lens = torch.tensor(L, dtype=torch.int64, device=DEV)
    got = u32(z.crc32_batch_device(ptrs, lens)).reshape(len(lengths), 16)
    np.testing.assert_array_equal(got, lo["crc"])


def test_seeds_and_chain_splits(golden):
    chains = golden["meta"]["chains"]
    datas = [o.payload(c["len"], c["index"]).tobytes() for c in chains]
    mem, ptrs, lens = dev_buffers_from_host(datas, align=1, gap=3, lead=5)
    seeds = torch.tensor(np.array([c["seed"] for c in chains], dtype=np.uint32).view(np.int32), device=DEV)
    got = u32(z.crc32_batch_device(ptrs, lens, seeds=seeds))
    assert list(got) == [c["crc"] for c in chains]
    # chaining across two device calls: crc(tail, crc(head, seed))
    cuts = [c["cut"] for c in chains]
    heads = [d[:k] for d, k in zip(datas, cuts)]
    tails = [d[k:] for d, k in zip(datas, cuts)]
    m1, p1, l1 = dev_buffers_from_host(heads, align=1, gap=1)
    h = z.crc32_batch_device(p1, l1, seeds=seeds)
    m2, p2, l2 = dev_buffers_from_host(tails, align=1, gap=1)
    got2 = u32(z.crc32_batch_device(p2, l2, seeds=h))
    assert list(got2) == [c["crc"] for c in chains]


def _strided_fill(n, length, stride=None, index0=0, index_step=1):
    stride = stride or length
    mem = torch.empty(max(n * stride, 1), dtype=torch.uint8, device=DEV)
    ptrs = mem.data_ptr() + torch.arange(n, dtype=torch.int64, device=DEV) * stride
    lens = torch.full((n,), length, dtype=torch.int64, device=DEV)
    z.fill_synthetic(ptrs, lens, index0=index0, index_step=index_step, seed=SEED)
    return mem, ptrs, lens


def test_config2_full_bitexact(golden):
    """Config 2: 4096 x 64 KiB, every CRC vs the reference's golden vector."""
    mem, ptrs, lens = _strided_fill(4096, 65536)
    exp = golden["cfg"]["cfg2"]
    np.testing.assert_array_equal(u32(z.crc32_batch_device(ptrs, lens)), exp)
    np.testing.assert_array_equal(u32(z.crc32_batch_strided(mem, 65536, 65536, 4096)), exp)
    # the generator itself matches the CPU regeneration
    host = mem[:65536 * 3].cpu().numpy()
    for i in range(3):
        np.testing.assert_array_equal(host[i * 65536:(i + 1) * 65536], o.payload(65536, i))


def test_config1_and_config3_sample(golden):
    meta, cfg = golden["meta"], golden["cfg"]
    mem, ptrs, lens = _strided_fill(1, 1 << 20)
    assert u32(z.crc32_batch_device(ptrs, lens))[0] == meta["config1"]["crc"]
    idx = cfg["cfg3_idx"].astype(np.int64)
    n = len(idx)
    mem = torch.empty(n << 20, dtype=torch.uint8, device=DEV)
    ptrs = mem.data_ptr() + (torch.arange(n, dtype=torch.int64, device=DEV) << 20)
    lens = torch.full((n,), 1 << 20, dtype=torch.int64, device=DEV)
    for k in range(n):  # payload index per buffer
        z.fill_synthetic(ptrs[k:k + 1], lens[k:k + 1], index0=int(idx[k]), seed=SEED)
    np.testing.assert_array_equal(u32(z.crc32_batch_device(ptrs, lens)), cfg["cfg3"])


def test_config4_sample_zipf(golden):
    """Config-4 size law: ragged lengths 1 KiB..16 MiB, packed unaligned."""
    cfg = golden["cfg"]
    idx = cfg["cfg4_idx"].astype(np.int64)
    L = cfg["cfg4_len"].astype(np.int64)
    offs = np.zeros(len(L), dtype=np.int64)
    offs[1:] = np.cumsum(L + 3)[:-1]  # 3-byte gaps: starts are not 16-B aligned
    mem = torch.empty(int(offs[-1] + L[-1] + 16), dtype=torch.uint8, device=DEV)
    ptrs = mem.data_ptr() + 1 + torch.tensor(offs, device=DEV)
    lens = torch.tensor(L, device=DEV)
    for k in range(len(idx)):
        z.fill_synthetic(ptrs[k:k + 1], lens[k:k + 1], index0=int(idx[k]), seed=SEED)
    np.testing.assert_array_equal(u32(z.crc32_batch_device(ptrs, lens)), cfg["cfg4"])


@pytest.mark.parametrize("n_bytes,lead", [(64 << 20, 0), ((64 << 20) + 3, 5), (300_000_007, 11), (4_500_000_017, 3)])
def test_single_large_buffer_split_across_waves(n_bytes, lead):
    mem = torch.empty(n_bytes + 64, dtype=torch.uint8, device=DEV)
    ptrs = torch.tensor([mem.data_ptr() + lead], dtype=torch.int64, device=DEV)
    lens = torch.tensor([n_bytes], dtype=torch.int64, device=DEV)
    z.fill_synthetic(ptrs, lens, index0=42, seed=SEED)
    got = int(u32(z.crc32_batch_device(ptrs, lens))[0])
    assert got == o.payload_crc(n_bytes, 42)
    seeds = torch.tensor([0x1234567], dtype=torch.int32, device=DEV)
    got_s = int(u32(z.crc32_batch_device(ptrs, lens, seeds=seeds))[0])
    assert got_s == o.payload_crc(n_bytes, 42, crc=0x1234567)


def test_empty_and_tiny_buffers():
    datas = [b"", b"a", b"ab", b"abc", b"abcd", b"", b"\xff" * 5, b""]
    mem, ptrs, lens = dev_buffers_from_host(datas, align=1)
    seeds_np = np.array([0, 1, 0xFFFFFFFF, 7, 0, 99, 3, 0xDEADBEEF], dtype=np.uint32)
    seeds = torch.tensor(seeds_np.view(np.int32), device=DEV)
    got = u32(z.crc32_batch_device(ptrs, lens, seeds=seeds))
    assert list(got) == [zlib.crc32(d, int(s)) for d, s in zip(datas, seeds_np)]
    # a batch of only empty buffers returns the seeds
    e = torch.zeros(3, dtype=torch.int64, device=DEV)
    got = u32(z.crc32_batch_device(e + mem.data_ptr(), e, seeds=seeds[:3]))
    assert list(got) == list(seeds_np[:3])


def test_random_mixed_batches_vs_oracle():
    rnd = random.Random(7)
    for trial in range(4):
        n = rnd.choice([1, 17, 500, 3000])
        lens = [rnd.choice([rnd.randint(0, 40), rnd.randint(0, 5000), rnd.randint(0, 300_000),
                            rnd.randint(0, 3_000_000)]) for _ in range(n)]
        total = sum(lens) + 64 * n + 64
        mem = torch.randint(0, 256, (total,), dtype=torch.uint8, device=DEV)
        offs, pos = [], 0
        for L in lens:
            pos += rnd.randint(0, 48)
            offs.append(pos)
            pos += L
        ptrs = torch.tensor([mem.data_ptr() + q for q in offs], dtype=torch.int64, device=DEV)
        lt = torch.tensor(lens, dtype=torch.int64, device=DEV)
        seeds_np = np.array([rnd.getrandbits(32) for _ in lens], dtype=np.uint32)
        seeds = torch.tensor(seeds_np.view(np.int32), device=DEV)
        got = u32(z.crc32_batch_device(ptrs, lt, seeds=seeds))
        host = mem.cpu().numpy()
        ap = np.array([host.ctypes.data + q for q in offs], dtype=np.uint64)
        exp = o.crc32_batch(ap, np.array(lens, dtype=np.uint64), seeds_np, nthreads=8)
        np.testing.assert_array_equal(got, exp, err_msg=f"trial {trial}")


@pytest.mark.parametrize("shape", ["large_mean", "small_mean"])
def test_dynamic_part_mixed_batches(shape):
    """Batches big enough that the kernel's dynamic part engages: claimed
    128 KiB units cut buffers at arbitrary places, next to empty, tiny and
    unaligned buffers with random seeds, in shuffled address order.  Mean
    buffer >= 512 KiB -> a quarter of the bytes dynamic, below -> half
    (zcrc_internal.h kDynSmallAvg; tests/kernel_model.py mirrors the rule).
    Every CRC vs the oracle."""
    rnd = random.Random(2024 if shape == "large_mean" else 99)
    if shape == "large_mean":
        kinds = [lambda: 0, lambda: rnd.randint(1, 3), lambda: rnd.randint(4, 5000),
                 lambda: rnd.randint(60_000, 140_000), lambda: rnd.randint(1 << 20, 3 << 20),
                 lambda: rnd.randint(4 << 20, 12 << 20)]
        n = 2500
    else:
        kinds = [lambda: 0, lambda: rnd.randint(1, 3), lambda: rnd.randint(4, 5000),
                 lambda: rnd.randint(60_000, 140_000), lambda: rnd.randint(200_000, 400_000)]
        n = 16000
    lens = [rnd.choice(kinds)() for _ in range(n)]
    cus = z.device_info()["num_cus"]
    shift = 1 if sum(lens) // n < (512 << 10) else 2
    assert shift == (2 if shape == "large_mean" else 1)
    assert (sum(lens) >> shift) // (cus * 16) >= 128 << 10, "dynamic part must engage"
    total = sum(lens) + 64 * n
    mem = torch.randint(0, 256, (total,), dtype=torch.uint8, device=DEV)
    offs, pos = [], 0
    for L in lens:
        pos += rnd.randint(0, 60)
        offs.append(pos)
        pos += L
    order = list(range(n))
    rnd.shuffle(order)  # batch order != address order
    ptrs = torch.tensor([mem.data_ptr() + offs[i] for i in order], dtype=torch.int64, device=DEV)
    lt = torch.tensor([lens[i] for i in order], dtype=torch.int64, device=DEV)
    seeds_np = np.array([rnd.getrandbits(32) for _ in lens], dtype=np.uint32)
    seeds = torch.tensor(seeds_np.view(np.int32), device=DEV)
    got = u32(z.crc32_batch_device(ptrs, lt, seeds=seeds))
    host = mem.cpu().numpy()
    ap = np.array([host.ctypes.data + offs[i] for i in order], dtype=np.uint64)
    exp = o.crc32_batch(ap, np.array([lens[i] for i in order], dtype=np.uint64), seeds_np, nthreads=16)
    np.testing.assert_array_equal(got, exp)
    if shape == "large_mean":
        # strided form: 2100 x (1 MiB + 17) at stride +13 (2.05 GiB, a quarter dynamic)
        n, L, stride = 2100, (1 << 20) + 17, (1 << 20) + 30
        assert n * stride + 7 <= total
        got = u32(z.crc32_batch_strided(mem, stride, L, n, seeds=seeds[:n], base_offset=7))
        ap = host.ctypes.data + 7 + np.arange(n, dtype=np.uint64) * stride
        exp = o.crc32_batch(ap, np.full(n, L, dtype=np.uint64), seeds_np[:n], nthreads=16)
        np.testing.assert_array_equal(got, exp)
    del host


def test_back_to_back_launches_vs_caller_scratch_path():
    """Many zcrc32_batch_device launches queued back to back on one stream,
    each with different lengths, the reused per-stream scratch and the
    dynamic work counter, must equal zcrc32_batch_device_ws with its own
    scratch per call, and the oracle.  (Until round 1's last session this
    compared the fused plan, since removed, with the two-launch plan.)"""
    rnd = random.Random(31)
    total = 96 << 20
    mem = torch.randint(0, 256, (total,), dtype=torch.uint8, device=DEV)
    host = mem.cpu().numpy()
    cases = []
    for n in [1, 2, 63, 64, 1000, 8191, 8192, 8193, 20000] + [rnd.randint(1, 8192) for _ in range(23)]:
        cap = total // n - 64
        lens = [min(cap, rnd.choice([0, rnd.randint(1, 100), rnd.randint(100, 70_000),
                                     rnd.randint(0, 600_000)])) for _ in range(n)]
        offs = [rnd.randrange(0, total - L) for L in lens]
        ptrs = torch.tensor([mem.data_ptr() + q for q in offs], dtype=torch.int64, device=DEV)
        lt = torch.tensor(lens, dtype=torch.int64, device=DEV)
        cases.append((offs, lens, ptrs, lt))
    outs = [z.crc32_batch_device(ptrs, lt) for (_, _, ptrs, lt) in cases]  # no sync in between
    ws = []
    for (_, lens, ptrs, lt) in cases:
        scratch = torch.empty(z.scratch_bytes(len(lens)), dtype=torch.uint8, device=DEV)
        ws.append(z.crc32_batch_device_ws(ptrs, lt, scratch))
    torch.cuda.synchronize()
    for k, ((offs, lens, _, _), a, b) in enumerate(zip(cases, outs, ws)):
        ga, gb = u32(a), u32(b)
        np.testing.assert_array_equal(ga, gb, err_msg=f"case {k} n={len(lens)}")
        ap = np.array([host.ctypes.data + q for q in offs], dtype=np.uint64)
        exp = o.crc32_batch(ap, np.array(lens, dtype=np.uint64), np.zeros(len(lens), dtype=np.uint32), nthreads=8)
        np.testing.assert_array_equal(ga, exp, err_msg=f"case {k} n={len(lens)}")


def test_graph_capture_replays_with_new_data():
    """Both device entry points captured in a HIP graph (torch.cuda.graph)
    and replayed after the payload and lengths change in place: every replay
    must checksum the current bytes.  zcrc32_batch_device switches to
    stream-ordered scratch and the two-launch plan under capture (a fused
    plan's epoch would be frozen into the graph); zcrc32_batch_device_ws
    always uses the two-launch plan."""
    rnd = random.Random(5)
    n, cap = 3000, 20_000
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
        ln = [rnd.choice([0, rnd.randint(1, 64), rnd.randint(64, cap)]) for _ in range(n)]
        lens.copy_(torch.tensor(ln, dtype=torch.int64))
        mem.copy_(torch.randint(0, 256, (n * cap,), dtype=torch.uint8, device=DEV))
        g.replay()
        torch.cuda.synchronize()
        host = mem.cpu().numpy()
        exp = o.crc32_batch(host.ctypes.data + np.arange(n, dtype=np.uint64) * cap, np.array(ln, dtype=np.uint64),
                            np.zeros(n, dtype=np.uint32), nthreads=8)
        np.testing.assert_array_equal(u32(out_a), exp, err_msg=f"batch_device replay {rep}")
        np.testing.assert_array_equal(u32(out_b), exp, err_msg=f"batch_device_ws replay {rep}")


def test_strided_api_seeds_and_stride():
    n, L, stride = 300, 200_000, 200_064
    mem, ptrs, lens = _strided_fill(n, L, stride=stride, index0=1000)
    seeds_np = np.arange(n, dtype=np.uint32) * 2654435761
    seeds = torch.tensor(seeds_np.view(np.int32), device=DEV)
    got = u32(z.crc32_batch_strided(mem, stride, L, n, seeds=seeds))
    exp = [o.payload_crc(L, 1000 + i, crc=int(seeds_np[i])) for i in range(n)]
    assert list(got) == exp


def test_host_batch_api_staging_and_continuation():
    """zcrc32_batch: pinned staging, several launches, a >64 MiB buffer split
    into continuation parts (seed chained on the device)."""
    rnd = random.Random(3)
    bufs = [o.payload(L, i) for i, L in enumerate([0, 5, 70_000, 3_000_000, 100 << 20, 17, (64 << 20) - 5, 999])]
    seeds = [rnd.getrandbits(32) for _ in bufs]
    got = z.crc32_batch(bufs, seeds=seeds)
    exp = [zlib.crc32(b.tobytes(), s) for b, s in zip(bufs, seeds)]
    assert list(got) == exp
    many = [o.payload(rnd.randint(0, 3000), 50 + i) for i in range(70_000)]  # > kStageItems per launch
    got = z.crc32_batch(many)
    assert list(got) == [zlib.crc32(b.tobytes()) for b in many]


def test_tensors_helper_and_verify_entries():
    ts = [torch.randint(0, 256, (L,), dtype=torch.uint8, device=DEV) for L in (0, 10, 4096, 123457)]
    got = u32(z.crc32_tensors(ts))
    assert list(got) == [zlib.crc32(t.cpu().numpy().tobytes()) for t in ts]
    entries = [t.cpu().numpy() for t in ts]
    exp = [zlib.crc32(e.tobytes()) for e in entries]
    exp[2] ^= 1
    assert list(z.verify_entries(entries, exp)) == [True, True, False, True]


def test_profile_counts_launches():
    mem, ptrs, lens = _strided_fill(64, 65536)
    with z.profile() as p:
        z.crc32_batch_device(ptrs, lens)
        torch.cuda.synchronize()
    assert p.launches == 1 and p.total_ms > 0


def test_prefix_and_pointers_beyond_2_31_and_2_32():
    """Batch whose prefix sums cross 2^31 and 2^32 (and whose device pointers
    span > 4 GiB): 64-bit descriptor handling (readlane halves, no sign
    extension) and many whole pieces per wave."""
    from concurrent.futures import ThreadPoolExecutor
    lens_np = np.array([400 << 20] * 11 + [123_456_789, 3, 0, 1_048_577], dtype=np.int64)
    offs = np.zeros_like(lens_np)
    offs[1:] = np.cumsum(lens_np + 7)[:-1]
    mem = torch.empty(int(offs[-1] + lens_np[-1] + 64), dtype=torch.uint8, device=DEV)
    ptrs = mem.data_ptr() + 5 + torch.tensor(offs, device=DEV)
    lens = torch.tensor(lens_np, device=DEV)
    z.fill_synthetic(ptrs, lens, index0=900, seed=SEED)
    got = u32(z.crc32_batch_device(ptrs, lens))
    with ThreadPoolExecutor(16) as ex:
        exp = list(ex.map(lambda a: o.payload_crc(int(a[1]), 900 + a[0]), enumerate(lens_np)))
    assert list(got) == exp
    # same bytes as 1 MiB pieces through the strided API (many whole pieces per wave)
    n = int(lens_np[:11].sum()) >> 20
    got_s = u32(z.crc32_batch_strided(mem, 1 << 20, 1 << 20, n, base_offset=5))
    host_first = mem[5:5 + (3 << 20)].cpu().numpy()
    assert int(got_s[0]) == zlib.crc32(host_first[: 1 << 20].tobytes())
    assert int(got_s[2]) == zlib.crc32(host_first[2 << 20: 3 << 20].tobytes())


def test_stream_incremental_like_preloadram():
    """Crc32Stream over zip_fread-sized chunks (16 MiB, src/ZIPsFS_preloadfileram.c:286-306),
    ragged chunks, empty updates, intermediate final() and a seed."""
    data = o.payload((40 << 20) + 12345, 77)
    full = zlib.crc32(data.tobytes())
    with z.Crc32Stream() as s:
        for off in range(0, data.size, 16 << 20):
            s.update(data[off:off + (16 << 20)])
        assert s.final() == full
    rnd = random.Random(11)
    with z.Crc32Stream(seed=0xABCDEF01) as s:
        pos, mid_checked = 0, False
        while pos < data.size:
            step = rnd.choice([0, 1, 3, 17, 4096, 65537, 1 << 20, 20 << 20])
            s.update(data[pos:pos + step])
            pos = min(pos + step, data.size)
            if not mid_checked and pos > (5 << 20):
                assert s.final() == zlib.crc32(data[:pos].tobytes(), 0xABCDEF01)
                mid_checked = True
        assert s.final() == zlib.crc32(data.tobytes(), 0xABCDEF01)
    with z.Crc32Stream(seed=5) as s:
        assert s.final() == 5  # no data: the seed, like zlib crc32(5, NULL, 0)


@pytest.mark.parametrize("device", [True, False])
def test_zip_verify_batched(device):
    """Whole-archive verification vs the central-directory CRCs zipfile
    wrote: stored entries in one GPU CRC batch, deflated entries inflated on
    the GPU and checksummed in one more.  A flipped byte in a stored entry is
    a mismatch; one in a deflated entry is an inflate error or a mismatch."""
    import io
    import zipfile
    from zipsfs_amd import zipverify as zv
    import inflate_streams as S
    rnd = random.Random(3)
    buf = io.BytesIO()
    with zipfile.ZipFile(buf, "w", allowZip64=True) as zf:
        for i in range(300):
            n = rnd.choice([0, 1, 5, 4095, 65536, 300_000, 2_000_001])
            data = o.payload(n, i).tobytes() if i % 2 else S.text_payload(n, i)
            zf.writestr(f"e{i}", data, compress_type=zipfile.ZIP_STORED if i % 3 else zipfile.ZIP_DEFLATED,
                        compresslevel=(i % 9) + 1 if i % 3 == 0 else None)
    data = bytearray(buf.getvalue())
    res = zv.verify(bytes(data), device=device)
    assert {r.method for r in res} == {0, 8}
    assert all(r.status == zv.ZIP_OK for r in res), [(r.name, r.status, r.inflate_status) for r in res if not r.ok]
    stored = [r for r in res if r.method == 0 and r.comp_size > 1000]
    deflated = [r for r in res if r.method == 8 and r.comp_size > 1000]
    data[stored[0].data_offset + 500] ^= 0x40
    data[deflated[0].data_offset + deflated[0].comp_size // 2] ^= 0x10
    res = zv.verify(bytes(data), device=device)
    bad = {r.name: r.status for r in res if not r.ok}
    assert set(bad) == {stored[0].name, deflated[0].name}
    assert bad[stored[0].name] == zv.ZIP_MISMATCH
    assert bad[deflated[0].name] in (zv.ZIP_MISMATCH, zv.ZIP_INFLATE_ERROR)


@pytest.mark.parametrize("device", [True, False])
def test_zip_verify_crafted_zip64_sizes(device):
    """A deflated entry whose ZIP64 extra field claims 2^64 - 16 bytes
    (the arena size wrapped) is inflated into bounded room and
    reported as a mismatch -- no fault, no out-of-bounds write; an honest
    entry in the same form verifies."""
    from zipsfs_amd import zipverify as zv
    from test_zip import crafted_zip
    data = o.payload(70_000, 5).tobytes()
    res = zv.verify(crafted_zip(data, 8, usize64=0xFFFFFFFFFFFFFFF0), device=device)
    assert res[0].status == zv.ZIP_MISMATCH and res[0].inflate_status == 0
    assert res[0].crc_computed == zlib.crc32(data)  # CRC of what the stream really holds
    res = zv.verify(crafted_zip(data, 8, usize64=len(data)), device=device)
    assert res[0].status == zv.ZIP_OK and res[0].crc_computed == zlib.crc32(data)
    res = zv.verify(crafted_zip(data, 0, lho64=0xFFFFFFFFFFFFFFE2), device=device)
    assert res[0].status == zv.ZIP_BAD


def test_concurrent_host_threads_dropin():
    """ZIPsFS runs one preload thread per root (src/ZIPsFS_async.c:468); the
    drop-in must be thread-safe: many threads, each with its own staging."""
    from concurrent.futures import ThreadPoolExecutor
    bufs = [o.payload(L, 300 + i) for i, L in enumerate([1, 4096, 65537, 1 << 20, 3 << 20, 17, 0, 999_999] * 4)]
    exp = [zlib.crc32(b.tobytes()) for b in bufs]

    def work(k):
        return [z.cg_crc32(b) for b in bufs[k::4]] + list(z.crc32_batch(bufs[k::4]))

    with ThreadPoolExecutor(8) as ex:
        res = list(ex.map(work, range(4)))
    for k in range(4):
        e = exp[k::4]
        assert res[k] == e + e


@pytest.mark.parametrize("fused", ["0", "1"])
def test_concurrent_device_calls_shared_and_private_streams(fused, monkeypatch):
    """Host threads issuing zcrc32_batch_device at once, on one shared stream
    and on private streams, with growing batch sizes (the per-stream scratch
    cache grows under its lock while other threads launch): every result vs
    the oracle."""
    from concurrent.futures import ThreadPoolExecutor
    monkeypatch.setenv("ZCRC_FUSED", fused)
    rnd = random.Random(77)
    total = 64 << 20
    mem = torch.randint(0, 256, (total,), dtype=torch.uint8, device=DEV)
    host = mem.cpu().numpy()
    jobs = []
    for k in range(24):
        n = [5, 300, 2000, 8000, 12000][k % 5] + k
        ln = [rnd.randint(0, 3000) for _ in range(n)]
        offs = [rnd.randrange(0, total - L) for L in ln]
        jobs.append((offs, ln))
    shared = torch.cuda.Stream(device=DEV)
    private = [torch.cuda.Stream(device=DEV) for _ in range(4)]

    def work(k):
        offs, ln = jobs[k]
        st = shared if k % 2 == 0 else private[k % 4]
        with torch.cuda.stream(st):
            ptrs = torch.tensor([mem.data_ptr() + q for q in offs], dtype=torch.int64, device=DEV)
            lt = torch.tensor(ln, dtype=torch.int64, device=DEV)
            out = z.crc32_batch_device(ptrs, lt)
            st.synchronize()
            return u32(out)

    with ThreadPoolExecutor(8) as ex:
        res = list(ex.map(work, range(len(jobs))))
    for k, ((offs, ln), got) in enumerate(zip(jobs, res)):
        ap = np.array([host.ctypes.data + q for q in offs], dtype=np.uint64)
        exp = o.crc32_batch(ap, np.array(ln, dtype=np.uint64), np.zeros(len(ln), dtype=np.uint32), nthreads=8)
        np.testing.assert_array_equal(got, exp, err_msg=f"job {k}")


@pytest.mark.parametrize("fused", ["0", "1"])
def test_small_batches_overlapping_on_six_streams(fused, monkeypatch):
    """Small-batch launches (<= 8192 buffers) from six host threads on six
    streams at once, each queueing twelve launches without synchronising,
    so that the launches overlap on the GPU.  (Until round 1's last session
    this guarded the fused plan's cross-workgroup wait, since removed.)
    Every result vs the oracle."""
    from concurrent.futures import ThreadPoolExecutor
    monkeypatch.setenv("ZCRC_FUSED", fused)
    rnd = random.Random(123)
    total = 32 << 20
    mem = torch.randint(0, 256, (total,), dtype=torch.uint8, device=DEV)
    host = mem.cpu().numpy()
    streams = [torch.cuda.Stream(device=DEV) for _ in range(6)]
    plans = []
    for t in range(6):
        jobs = []
        for _ in range(12):
            n = rnd.randint(4000, 8192)
            ln = [rnd.randint(0, 4000) for _ in range(n)]
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

    with ThreadPoolExecutor(6) as ex:
        res = list(ex.map(work, range(6)))
    for t in range(6):
        for j, ((offs, ln), got) in enumerate(zip(plans[t], res[t])):
            ap = np.array([host.ctypes.data + q for q in offs], dtype=np.uint64)
            exp = o.crc32_batch(ap, np.array(ln, dtype=np.uint64), np.zeros(len(ln), dtype=np.uint32), nthreads=8)
            np.testing.assert_array_equal(got, exp, err_msg=f"thread {t} job {j}")


def test_wrapper_argument_validation():
    """Short or mistyped out/seeds tensors are refused before any launch
    (they let the kernel read or write past device memory)."""
    mem = torch.zeros(1 << 16, dtype=torch.uint8, device=DEV)
    ptrs = mem.data_ptr() + torch.arange(8, dtype=torch.int64, device=DEV) * 1024
    lens = torch.full((8,), 1024, dtype=torch.int64, device=DEV)
    with pytest.raises(ValueError):
        z.crc32_batch_device(ptrs, lens, out=torch.empty(7, dtype=torch.int32, device=DEV))
    with pytest.raises(ValueError):
        z.crc32_batch_device(ptrs, lens, seeds=torch.zeros(7, dtype=torch.int32, device=DEV))
    with pytest.raises(ValueError):
        z.crc32_batch_device(ptrs, lens, seeds=torch.zeros(8, dtype=torch.int64, device=DEV))
    scratch = torch.empty(z.crc32.scratch_bytes(8), dtype=torch.uint8, device=DEV)
    with pytest.raises(ValueError):
        z.crc32_batch_device_ws(ptrs, lens[:7], scratch)
    with pytest.raises(ValueError):
        z.crc32_batch_strided(mem, 1024, 1024, 8, out=torch.empty(4, dtype=torch.int32, device=DEV))
    got = u32(z.crc32_batch_device(ptrs, lens))
    assert (got == zlib.crc32(bytes(1024))).all()


@pytest.mark.parametrize("shape", ["uniform_dynamic", "ragged_split", "tiny_and_huge"])
def test_fused_small_batch_vs_two_launch_path(shape, monkeypatch):
    """n <= 8192 eager calls run ONE fused launch (the kernel scans the
    lengths; split pieces meet in self-cleaning scratch words; the claim
    counter resets itself).  Repeated launches on one stream, each vs the
    two-launch path (crc32_batch_device_ws) and the oracle on a sample."""
    monkeypatch.setenv("ZCRC_FUSED", "1")  # libzcrc reads it per call
    rnd = random.Random({"uniform_dynamic": 1, "ragged_split": 2, "tiny_and_huge": 3}[shape])
    if shape == "uniform_dynamic":  # 4 GiB in 1 MiB buffers: the dynamic part is on
        lens_l = [1 << 20] * 4096
    elif shape == "ragged_split":   # many buffers above the 128 KiB split size
        lens_l = [rnd.choice([0, 3, 4095, 65536, 200_000, 3_000_001, 9_999_999]) for _ in range(3000)]
    else:
        lens_l = [rnd.randint(0, 64) for _ in range(8190)] + [700_000_001, 123_456_789]
    n = len(lens_l)
    offs = np.zeros(n, dtype=np.int64)
    offs[1:] = np.cumsum(np.array(lens_l, dtype=np.int64) + 7)[:-1]
    mem = torch.empty(int(offs[-1] + lens_l[-1] + 64), dtype=torch.uint8, device=DEV)
    ptrs = mem.data_ptr() + 1 + torch.tensor(offs, device=DEV)
    lens = torch.tensor(lens_l, dtype=torch.int64, device=DEV)
    z.fill_synthetic(ptrs, lens, index0=5, index_step=3, seed=SEED)
    seeds_np = np.array([rnd.getrandbits(32) for _ in range(n)], dtype=np.uint32)
    seeds = torch.tensor(seeds_np.view(np.int32), device=DEV)
    scratch = torch.empty(z.crc32.scratch_bytes(n), dtype=torch.uint8, device=DEV)
    ref = u32(z.crc32_batch_device_ws(ptrs, lens, scratch, seeds=seeds))
    for rep in range(3):
        got = u32(z.crc32_batch_device(ptrs, lens, seeds=seeds))
        np.testing.assert_array_equal(got, ref, err_msg=f"{shape} launch {rep}")
        got0 = u32(z.crc32_batch_device(ptrs, lens))
        if rep == 0:
            ref0 = got0
        np.testing.assert_array_equal(got0, ref0)
    sample = sorted(set(rnd.sample(range(n), 24)) | {n - 1, n - 2})
    for i in sample:
        exp = o.payload_crc(lens_l[i], 5 + 3 * i, crc=int(seeds_np[i]))
        assert int(ref[i]) == exp, (shape, i, lens_l[i])


@pytest.mark.parametrize("n,longest", [(1, 65536), (5, 4), (255, 65536), (256, 65536), (257, 3000),
                                       (1000, 65536), (4095, 65536), (4096, 65536), (4096, 65537),
                                       (4097, 65536), (4096, 1 << 20)])
def test_per_buffer_mode_vs_oracle(n, longest, monkeypatch):
    """Default eager calls of at most 16 x CUs buffers run one launch; when no
    buffer exceeds 64 KiB the kernel gives each wave one whole buffer (no
    prefix scan, no search), otherwise it scans in-kernel (fused form).
    Ragged lengths 0..longest (tiny ones included), odd addresses, random
    seeds; vs the oracle and the two-launch path, repeated on one stream."""
    monkeypatch.delenv("ZCRC_FUSED", raising=False)
    rnd = random.Random(n * 7 + longest)
    lens_l = [rnd.choice([0, 1, 2, 3, 4, 5, 17, rnd.randint(0, longest), rnd.randint(0, longest), longest])
              for _ in range(n)]
    lens_l[-1] = longest
    offs = np.zeros(n, dtype=np.int64)
    offs[1:] = np.cumsum(np.array(lens_l, dtype=np.int64) + 3)[:-1]
    mem = torch.randint(0, 256, (int(offs[-1] + lens_l[-1] + 64),), dtype=torch.uint8, device=DEV)
    ptrs = mem.data_ptr() + 1 + torch.tensor(offs, device=DEV)
    lens = torch.tensor(lens_l, dtype=torch.int64, device=DEV)
    seeds_np = np.array([rnd.getrandbits(32) for _ in range(n)], dtype=np.uint32)
    seeds = torch.tensor(seeds_np.view(np.int32), device=DEV)
    host = mem.cpu().numpy()
    exp = o.crc32_batch(host.ctypes.data + 1 + offs.astype(np.uint64), np.array(lens_l, dtype=np.uint64),
                        seeds_np, nthreads=8)
    scratch = torch.empty(z.crc32.scratch_bytes(n), dtype=torch.uint8, device=DEV)
    np.testing.assert_array_equal(u32(z.crc32_batch_device_ws(ptrs, lens, scratch, seeds=seeds)), exp)
    for rep in range(3):
        np.testing.assert_array_equal(u32(z.crc32_batch_device(ptrs, lens, seeds=seeds)), exp,
                                      err_msg=f"n={n} launch {rep}")


@pytest.mark.parametrize("fused", ["0", "1"])
def test_fused_scratch_reuse_across_batch_sizes(fused, monkeypatch):
    """Fused launches of different n share one per-stream scratch slot.  A
    small batch leaves its prefix in the slot; a larger batch that follows
    must not read it as split-piece accumulators (round-2 bug: the
    accumulators sat at an n-dependent offset and overlapped an earlier
    prefix).  Alternating sizes with split buffers, each vs the two-launch
    path."""
    monkeypatch.setenv("ZCRC_FUSED", fused)
    rnd = random.Random(77)
    for n in [1, 3, 17, 300, 2500, 40, 8192, 2, 5000]:
        lens_l = [rnd.choice([0, 2, 1000, 65536, 300_001, 2_000_003]) for _ in range(n)]
        lens_l[0] = 2_000_003  # at least one split buffer
        offs = np.zeros(n, dtype=np.int64)
        offs[1:] = np.cumsum(np.array(lens_l, dtype=np.int64) + 5)[:-1]
        mem = torch.randint(0, 256, (int(offs[-1] + lens_l[-1] + 64),), dtype=torch.uint8, device=DEV)
        ptrs = mem.data_ptr() + torch.tensor(offs, device=DEV)
        lens = torch.tensor(lens_l, dtype=torch.int64, device=DEV)
        got = u32(z.crc32_batch_device(ptrs, lens))
        scratch = torch.empty(z.crc32.scratch_bytes(n), dtype=torch.uint8, device=DEV)
        ref = u32(z.crc32_batch_device_ws(ptrs, lens, scratch))
        np.testing.assert_array_equal(got, ref, err_msg=f"n={n}")
        host = mem.cpu().numpy()
        exp = o.crc32_batch(host.ctypes.data + offs.astype(np.uint64), np.array(lens_l, dtype=np.uint64),
                            np.zeros(n, dtype=np.uint32), nthreads=8)
        np.testing.assert_array_equal(got, exp, err_msg=f"n={n}")


@pytest.mark.parametrize("device", [True, False])
def test_zip_extract_stored(device):
    """Stored-entry extraction (the zip_fread of a method-0
    entry, src/ZIPsFS_preloadfileram.c:286-288): bytes equal zipfile's, CRCs
    equal the central directory's, every length and source alignment the
    archive produces (names of 1..40 bytes shift the data offsets); a flipped
    byte is delivered as stored and flagged ZIP_MISMATCH; deflated entries are
    not extracted."""
    import io
    import zipfile
    from zipsfs_amd import zipverify as zv
    rnd = random.Random(8)
    buf = io.BytesIO()
    payloads = {}
    with zipfile.ZipFile(buf, "w", allowZip64=True) as zf:
        for i in range(240):
            n = rnd.choice([0, 1, 2, 3, 15, 16, 17, 31, 4095, 65535, 65536, 65537, 200_003, 1_500_007])
            name = f"s{i}_" + "x" * rnd.randint(0, 40)
            payloads[name] = o.payload(n, 7000 + i).tobytes()
            zf.writestr(name, payloads[name], compress_type=zipfile.ZIP_DEFLATED if i % 7 == 0 else zipfile.ZIP_STORED)
    data = bytearray(buf.getvalue())
    res = zv.extract_stored(bytes(data), device=device)
    assert len(res) == 240
    for chk, got in res:
        if chk.method == 8:
            assert got is None and chk.status == zv.ZIP_UNVERIFIED
            continue
        assert chk.status == zv.ZIP_OK, chk
        g = got.cpu().numpy().tobytes() if device else got.tobytes()
        assert g == payloads[chk.name], chk.name
        assert chk.crc_computed == zlib.crc32(payloads[chk.name])
    big = [c for c, _ in res if c.method == 0 and c.comp_size > 100_000][0]
    data[big.data_offset + big.comp_size // 3] ^= 0x04
    res = zv.extract_stored(bytes(data), device=device)
    bad = [(c, g) for c, g in res if c.status != zv.ZIP_OK and c.method == 0]
    assert [c.name for c, _ in bad] == [big.name] and bad[0][0].status == zv.ZIP_MISMATCH
    g = bad[0][1].cpu().numpy().tobytes() if device else bad[0][1].tobytes()
    assert g == bytes(data[big.data_offset: big.data_offset + big.comp_size])
    assert bad[0][0].crc_computed == zlib.crc32(g)


@pytest.mark.parametrize("fused", ["0", "1"])
def test_scratch_growth_is_stream_ordered(fused, monkeypatch):
    """The per-stream scratch grows while launches are queued on its stream:
    the new buffer's zero fill must be ordered before the plan that follows
    on the same stream (a null-stream memset was not, and could zero a prefix
    the plan had just written).  Fresh streams, growing n, no sync between
    launches, every result vs the oracle."""
    monkeypatch.setenv("ZCRC_FUSED", fused)
    rnd = random.Random(4242)
    total = 16 << 20
    mem = torch.randint(0, 256, (total,), dtype=torch.uint8, device=DEV)
    host = mem.cpu().numpy()
    for rep in range(3):
        st = torch.cuda.Stream(device=DEV)
        jobs = []
        with torch.cuda.stream(st):
            for n in [50, 7000, 8192, 9000, 30000, 8100, 70000, 3]:
                ln = [rnd.randint(0, 300) for _ in range(n)]
                offs = [rnd.randrange(0, total - L) for L in ln]
                ptrs = torch.tensor([mem.data_ptr() + q for q in offs], dtype=torch.int64, device=DEV)
                lt = torch.tensor(ln, dtype=torch.int64, device=DEV)
                jobs.append((offs, ln, z.crc32_batch_device(ptrs, lt), ptrs, lt))
        st.synchronize()
        for offs, ln, got, _, _ in jobs:
            ap = np.array([host.ctypes.data + q for q in offs], dtype=np.uint64)
            exp = o.crc32_batch(ap, np.array(ln, dtype=np.uint64), np.zeros(len(ln), dtype=np.uint32), nthreads=8)
            np.testing.assert_array_equal(u32(got), exp, err_msg=f"rep {rep} n={len(ln)}")


@pytest.mark.parametrize("n", [20_000, 9_000])
def test_corrupted_prefix_is_caught_not_walked(n, monkeypatch):
    """A zeroed quarter of the length prefix after the plan (the round-1/2
    fault: an unordered memset over the scratch) makes the CRC kernel skip the
    inconsistent pieces (result 0) and set the scratch's fault word, instead
    of reading outside every buffer; with the hook off the same batch is
    bit-exact and reports no fault."""
    rnd = np.random.default_rng(n)
    lens = rnd.integers(9000, 300_000, n).astype(np.int64)  # no small buffers: the plain prefix
    offs = np.zeros(n, dtype=np.int64)
    offs[1:] = np.cumsum(lens + 5)[:-1]
    mem = torch.randint(0, 256, (int(offs[-1] + lens[-1] + 64),), dtype=torch.uint8, device=DEV)
    ptrs = mem.data_ptr() + torch.tensor(offs, device=DEV)
    lt = torch.tensor(lens, device=DEV)
    host = mem.cpu().numpy()  # kept alive while the oracle reads it
    exp = o.crc32_batch((host.ctypes.data + offs).astype(np.uint64), lens.astype(np.uint64), None, nthreads=16)
    got = z.crc32_batch_device(ptrs, lt).cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(got, exp)
    assert z.batch_device_faults() == 0
    monkeypatch.setenv("ZCRC_TEST_CORRUPT_PREFIX", "1")
    bad = z.crc32_batch_device(ptrs, lt).cpu().numpy().view(np.uint32)
    assert z.batch_device_faults() != 0
    assert (bad != exp).any()
    monkeypatch.delenv("ZCRC_TEST_CORRUPT_PREFIX")
    got = z.crc32_batch_device(ptrs, lt).cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(got, exp)
    assert z.batch_device_faults() == 0


@pytest.mark.parametrize("api", ["device", "strided"])
@pytest.mark.parametrize("n,L", [(16384, 1 << 20), (20011, (1 << 20) + 24)])
def test_window_order_equal_buffers(api, n, L, monkeypatch):
    """The batch kernel's window order (BatchView::wp, round 6): 16,384 equal
    1 MiB buffers -- 12 GiB static over 4,096 waves = 3 buffers per wave, so
    logical buffer i is read as physical buffer (i % 3) * 4096 + i / 3 --
    and 20,011 buffers of 1 MiB + 24 B, whose static part (three quarters)
    is not a whole number of buffers per wave: it is cut to 3 x 4,096 and
    the rest read as dynamic units from a buffer boundary; at odd addresses
    (stride L + 13) with random seeds, through the pointer API (the split
    plan finds the lengths equal) and the strided API.  Every result equal
    to the range order's (ZCRC_AB_FLAGS=8) and, on 64 sampled buffers, to
    the oracle."""
    stride = L + 13
    mem = torch.empty(n * stride + 64, dtype=torch.uint8, device=DEV)
    ptrs = mem.data_ptr() + 5 + torch.arange(n, dtype=torch.int64, device=DEV) * stride
    lens = torch.full((n,), L, dtype=torch.int64, device=DEV)
    z.fill_synthetic(ptrs, lens, index0=333, seed=SEED)
    rnd = np.random.default_rng(n)
    seeds_np = rnd.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    seeds = torch.from_numpy(seeds_np.view(np.int32)).to(DEV)

    def run():
        if api == "device":
            return u32(z.crc32_batch_device(ptrs, lens, seeds=seeds))
        return u32(z.crc32_batch_strided(mem, stride, L, n, seeds=seeds, base_offset=5))
    got = run()
    monkeypatch.setenv("ZCRC_AB_FLAGS", "8")  # the range order (A/B knob)
    ref = run()
    monkeypatch.delenv("ZCRC_AB_FLAGS")
    np.testing.assert_array_equal(got, ref)
    for i in np.concatenate([rnd.choice(n, 60, replace=False), [0, 4095, 12288, n - 1]]):
        assert int(got[i]) == o.payload_crc(L, 333 + int(i), crc=int(seeds_np[i])), i
    del mem
    torch.cuda.empty_cache()


@pytest.mark.parametrize("n,L", [(40000, 100000), (14000, 777777), (50000, 65544), (12000, (1 << 20) - 16)])
def test_window_order_cut_static_part(n, L, monkeypatch):
    """The window order with the static part cut to p x W whole buffers
    (round 6): equal lengths that are no power of two, half (mean < 512 KiB)
    or a quarter dynamic, p = 4, 2, 6 and 2 buffers per wave on 4,096 waves;
    odd addresses, random seeds, both APIs.  Every result equal to the range
    order's (ZCRC_AB_FLAGS=8) and to the other API's; the first and last
    buffers of the window, the first dynamic ones and 16 random ones equal
    to the oracle."""
    stride = L + 7
    mem = torch.empty(n * stride + 64, dtype=torch.uint8, device=DEV)
    ptrs = mem.data_ptr() + 3 + torch.arange(n, dtype=torch.int64, device=DEV) * stride
    lens = torch.full((n,), L, dtype=torch.int64, device=DEV)
    z.fill_synthetic(ptrs, lens, index0=77, seed=SEED)
    rnd = np.random.default_rng(L)
    seeds_np = rnd.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    seeds = torch.from_numpy(seeds_np.view(np.int32)).to(DEV)
    res = {}
    for flags in ("0", "8"):
        monkeypatch.setenv("ZCRC_AB_FLAGS", flags)
        res["device", flags] = u32(z.crc32_batch_device(ptrs, lens, seeds=seeds))
        res["strided", flags] = u32(z.crc32_batch_strided(mem, stride, L, n, seeds=seeds, base_offset=3))
    monkeypatch.delenv("ZCRC_AB_FLAGS")
    got = res["device", "0"]
    for k, v in res.items():
        np.testing.assert_array_equal(v, got, err_msg=str(k))
    total = n * L
    Ts = total - (total >> (1 if L < (512 << 10) else 2))
    p = Ts // (4096 * L)
    assert p >= 2
    edge = [0, 4095, 4096, p * 4096 - 1, p * 4096, p * 4096 + 1, n - 1]
    for i in np.concatenate([rnd.choice(n, 16, replace=False), edge]):
        assert int(got[i]) == o.payload_crc(L, 77 + int(i), crc=int(seeds_np[i])), i
    del mem
    torch.cuda.empty_cache()
