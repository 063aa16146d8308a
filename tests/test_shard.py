"""Multi-rank sharding + results gather on CPU (gloo, world_size 2, 3 and 8)."""
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


@pytest.mark.parametrize("world,n_total", [(2, 10), (2, 7), (3, 1000), (2, 1), (8, 32768), (8, 1003)])
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


# ----------------------------------------------------------- bench launcher

def _bench():
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(root, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_bench_world_resolution():
    """--gpus N without a launcher spawns N ranks; under torchrun WORLD_SIZE
    must agree with --gpus (--gpus was silently ignored)."""
    b = _bench()
    assert b.resolve_world(None, None) == (1, False)
    assert b.resolve_world(1, None) == (1, False)
    assert b.resolve_world(8, None) == (8, True)
    assert b.resolve_world(None, "4") == (4, False)
    assert b.resolve_world(4, "4") == (4, False)
    with pytest.raises(SystemExit):
        b.resolve_world(8, "2")
    with pytest.raises(SystemExit):
        b.resolve_world(0, None)
    env = b.rank_env({"X": "1"}, 3, 8, 29500)
    assert env["RANK"] == env["LOCAL_RANK"] == "3" and env["WORLD_SIZE"] == "8"
    assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29500" and env["X"] == "1"
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_bench_config5_golden_in_global_order():
    """The config-5 parity check reads the gathered CRCs in global order and
    needs >= 256 fixture samples inside the run's buffers."""
    b = _bench()
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "configs.npz"))
    n_total = 2 * 32768
    glob = np.zeros(n_total, dtype=np.uint32)
    idx = g["cfg5_idx"].astype(np.int64)
    keep = idx < n_total
    glob[idx[keep]] = g["cfg5"][keep]
    assert b.golden_check(5, glob).startswith(f"{int(keep.sum())}/{int(keep.sum())}")
    glob[idx[keep][0]] ^= 1
    with pytest.raises(SystemExit):
        b.golden_check(5, glob)
    with pytest.raises(SystemExit):  # too few samples inside a tiny run
        b.golden_check(5, np.zeros(1000, dtype=np.uint32))


def test_bench_spawn_ranks_exit_codes(tmp_path):
    """spawn_ranks starts fresh interpreters with the rank env and returns
    the first failing rank's code (script stands in for bench.py)."""
    b = _bench()
    script = tmp_path / "fake_bench.py"
    script.write_text("import os, sys\n"
                      "r = int(os.environ['RANK'])\n"
                      "open(os.path.join(sys.argv[1], f'rank{r}'), 'w').write(os.environ['WORLD_SIZE'])\n"
                      "sys.exit(int(sys.argv[2]) if r == 1 else 0)\n")
    orig = b.__file__
    try:
        b.__file__ = str(script)
        assert b.spawn_ranks(3, [str(tmp_path), "0"]) == 0
        assert sorted(p.name for p in tmp_path.glob("rank*")) == ["rank0", "rank1", "rank2"]
        assert (tmp_path / "rank2").read_text() == "3"
        assert b.spawn_ranks(2, [str(tmp_path), "7"]) == 7
    finally:
        b.__file__ = orig


def test_bench_n_gt_1_cpu_baseline_sample_and_8_rank_goldens():
    """At N > 1 rank 0 times the reference over a fixed config-5 subset,
    16 GiB by default: global buffers 0..16383 of the same payload (SURVEY
    8(d)); 8 ranks x 4096 buffers (the GPU suite's rehearsal) hold 256
    config-5 fixtures."""
    b = _bench()
    lens, idx, what = b.baseline_sample(5, 16 << 30)
    assert len(lens) == 16384 and (lens == 1 << 20).all() and (idx == np.arange(16384)).all(), what
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "configs.npz"))
    n_total = 8 * 4096
    glob = np.zeros(n_total, dtype=np.uint32)
    keep = g["cfg5_idx"] < n_total
    glob[g["cfg5_idx"][keep].astype(np.int64)] = g["cfg5"][keep]
    assert b.golden_check(5, glob) == "256/256 sampled CRCs equal the reference golden vectors"
