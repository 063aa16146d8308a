"""zcrc_read_sweep_device: the stream-read peak bench.py reports beside the
CRC (the loop whose bytes are counted:
src/cg_crc32.c:37-46).  It computes nothing to compare, so these check the
contract: it runs without fault on whole and ragged regions (the tail
granules), rejects a misaligned base and a short sink, reads at HBM-like
rates, and never touches the region it reads."""
import ctypes

import pytest

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    return torch


@pytest.mark.timeout(120)
def test_sweep_ragged_sizes_leave_region_unchanged():
    torch = _torch()
    import zipsfs_amd as z
    dev = torch.device("cuda:0")
    mem = torch.randint(0, 256, (64 << 20,), dtype=torch.uint8, device=dev)
    ref = mem.clone()
    sink = torch.zeros(1024, dtype=torch.int32, device=dev)
    for nbytes in (16, 4096, 65536 - 16, 65536, 65536 + 48, (1 << 20) + 12345, (64 << 20)):
        z.read_sweep_device(mem.data_ptr(), nbytes, sink)
    torch.cuda.synchronize()
    assert torch.equal(mem, ref)


@pytest.mark.timeout(120)
def test_sweep_rejects_bad_arguments():
    torch = _torch()
    import zipsfs_amd as z
    dev = torch.device("cuda:0")
    mem = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
    sink = torch.zeros(1024, dtype=torch.int32, device=dev)
    with pytest.raises(z.ZcrcError):
        z.read_sweep_device(mem.data_ptr() + 8, 4096, sink)
    with pytest.raises(ValueError):
        z.read_sweep_device(mem.data_ptr(), 4096, sink[:16])
    rc = z.lib().zcrc_read_sweep_device(ctypes.c_void_p(mem.data_ptr()), 0, None, None)
    assert rc == 0  # nothing to read: no launch


@pytest.mark.timeout(120)
def test_sweep_reads_at_hbm_rate():
    torch = _torch()
    import zipsfs_amd as z
    dev = torch.device("cuda:0")
    nbytes = 8 << 30
    mem = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    sink = torch.zeros(1024, dtype=torch.int32, device=dev)
    for _ in range(3):
        z.read_sweep_device(mem.data_ptr(), nbytes, sink)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        z.read_sweep_device(mem.data_ptr(), nbytes, sink)
    e1.record()
    torch.cuda.synchronize()
    gbs = nbytes * 10 / (e0.elapsed_time(e1) * 1e-3) / 1e9
    print(f"stream read: {gbs:.1f} GB/s")
    assert 3000.0 < gbs < 8100.0, gbs
