"""Multi-rank sharding + results gather on CPU (gloo, world_size 2 and 3)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from zipsfs_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def fake_crc(i):
    return ((np.asarray(i, dtype=np.uint64) * np.uint64(2654435761)) & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def _worker(rank, world, port, n_total, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        idx = shard.shard_indices(n_total, rank, world)
        assert len(idx) == shard.local_count(n_total, rank, world)
        local = torch.from_numpy(fake_crc(idx).view(np.int32).copy())
        out = shard.gather_crcs(local, n_total)
        q.put((rank, out.numpy().view(np.uint32).tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_total", [(2, 10), (2, 7), (3, 1000), (2, 1)])
def test_gather_global_order(world, n_total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = fake_crc(np.arange(n_total)).tolist()
    for rank, got in res:
        assert got == exp, rank


def test_shard_partition_covers_all():
    for world in (1, 2, 3, 8):
        for n in (0, 1, 7, 1000):
            allidx = np.concatenate([shard.shard_indices(n, r, world) for r in range(world)])
            assert sorted(allidx.tolist()) == list(range(n))
