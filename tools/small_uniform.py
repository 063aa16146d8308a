"""tools/small_uniform.py -- uniform batches of small buffers through the
product entry points, for rocprofv3 (measurement only): two distinct 1 GiB
batches of `len`-byte buffers, `reps` calls each through
zcrc32_batch_device_strided (the small kernel) and zcrc32_batch_device (the
split plan + batch kernel launch).

  rocprofv3 --kernel-trace --stats -- python3 tools/small_uniform.py [len] [reps]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import zipsfs_amd as z  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
n = (1 << 30) // L
bat = []
for b in range(2):
    mem = torch.empty(n * L + 64, dtype=torch.uint8, device="cuda:0")
    ptrs = mem.data_ptr() + torch.arange(n, dtype=torch.int64, device="cuda:0") * L
    lens = torch.full((n,), L, dtype=torch.int64, device="cuda:0")
    z.fill_synthetic(ptrs, lens, index0=7 * b, seed=0xC0FFEE)
    bat.append((mem, ptrs, lens))
for r in range(reps):
    for mem, ptrs, lens in bat:
        a = z.crc32_batch_strided(mem, L, L, n)
for r in range(reps):
    for mem, ptrs, lens in bat:
        d = z.crc32_batch_device(ptrs, lens)
torch.cuda.synchronize()
assert torch.equal(a, d)
print(f"len {L} n {n} reps {reps}: strided and device results equal")
