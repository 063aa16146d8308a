"""GPU: single buffers beyond 4 GiB -- ZIP64 entries (src/ZIPsFS.c:985-1001
reads their sizes as 64-bit; src/ZIPsFS_preloadfileram.c:243 checks whole
entries of st_size bytes).  The device API splits such a buffer into pieces
on the end-relative 64 KiB grid and moves each piece's register to the end
with 64-bit shift counts; the drop-in stages it through 16 MiB slots with
chained seeds.  Every result is compared with the oracle's streamed CRC of
the same synthetic payload (oracle_crc_payload: no host copy of the bytes)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import zipsfs_amd as z  # noqa: E402
from oracle import oracle as o  # noqa: E402

DEV = "cuda:0"
SEED = o.PAYLOAD_SEED
BIG = (5 << 30) + 3  # 5 GiB + 3: odd length, prefix and pointers past 2^32


def u32(t):
    return t.cpu().numpy().view(np.uint32)


@pytest.mark.timeout(300)
def test_device_buffer_beyond_4gib_with_neighbours_and_seeds():
    lens_np = np.array([17, BIG, 4096 + 5, 0], dtype=np.int64)
    offs = np.array([0, 64 + 5, 64 + 5 + BIG + 11, 64 + 5 + BIG + 11 + 4101 + 16], dtype=np.int64)
    mem = torch.empty(int(offs[-1] + 64), dtype=torch.uint8, device=DEV)
    ptrs = mem.data_ptr() + torch.tensor(offs, device=DEV)
    lens = torch.tensor(lens_np, device=DEV)
    z.fill_synthetic(ptrs, lens, index0=4242, seed=SEED)
    exp0 = [o.payload_crc(int(L), 4242 + i) for i, L in enumerate(lens_np)]
    assert list(u32(z.crc32_batch_device(ptrs, lens))) == exp0
    seeds = torch.tensor([0x1234, 0xDEADBEEF, 7, 0x55AA55AA], dtype=torch.int64).to(torch.int32).to(DEV)
    exp1 = [o.payload_crc(int(L), 4242 + i, crc=int(s) & 0xFFFFFFFF)
            for i, (L, s) in enumerate(zip(lens_np, [0x1234, 0xDEADBEEF, 7, 0x55AA55AA]))]
    assert list(u32(z.crc32_batch_device(ptrs, lens, seeds=seeds))) == exp1
    # the same bytes cut in two at an arbitrary point and chained: crc(A || B)
    cut = (3 << 30) + 12345
    p2 = torch.tensor([int(ptrs[1]), int(ptrs[1]) + cut], dtype=torch.int64, device=DEV)
    l2 = torch.tensor([cut, BIG - cut], dtype=torch.int64, device=DEV)
    a, b = (int(x) for x in u32(z.crc32_batch_device(p2, l2)))
    assert z.crc32_combine(a, b, BIG - cut) == exp0[1]
    del mem
    torch.cuda.empty_cache()


@pytest.mark.timeout(300)
def test_strided_chunk_beyond_4gib():
    n, stride = 2, BIG + 13
    mem = torch.empty(n * stride + 64, dtype=torch.uint8, device=DEV)
    base = mem.data_ptr() + 3
    ptrs = base + torch.arange(n, dtype=torch.int64, device=DEV) * stride
    lens = torch.full((n,), BIG, dtype=torch.int64, device=DEV)
    z.fill_synthetic(ptrs, lens, index0=99, seed=SEED)
    got = u32(z.crc32_batch_strided(mem, stride, BIG, n, base_offset=3))
    assert list(got) == [o.payload_crc(BIG, 99), o.payload_crc(BIG, 100)]
    del mem
    torch.cuda.empty_cache()


@pytest.mark.timeout(300)
def test_dropin_host_entry_beyond_4gib():
    host = o.payload(BIG, 31337)
    assert z.cg_crc32(host) == o.payload_crc(BIG, 31337)
    assert z.cg_crc32(host, crc=0xCAFEF00D) == o.payload_crc(BIG, 31337, crc=0xCAFEF00D)
