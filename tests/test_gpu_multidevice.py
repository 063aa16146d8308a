"""GPU: libzcrc's multi-device host path.

ZIPsFS is one process whose preload threads all call cg_crc32 from
src/ZIPsFS_preloadfileram.c:243 (src/ZIPsFS_async.c:468-497,
src/ZIPsFS_configuration.h:110).  libzcrc spreads host-memory calls over a
device set (ZCRC_DEVICES): byte-balanced shards, one per device, and a
buffer cut at a shard boundary reassembled with the GF(2) combine.  The box
has one GPU, so these tests list it twice (ZCRC_DEVICES=0,0: two logical
devices, each with its own worker thread and staging leases) and lower the
per-device minimum so that the golden batches are sharded; every CRC is
checked bit-exact against the reference-generated fixtures."""
import json
import os
import subprocess
import sys

import pytest

import dropin_util as du

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ENV2 = {"ZCRC_DEVICES": "0,0", "ZCRC_SHARD_MIN_BYTES": str(1 << 20)}


def _child(env_extra):
    env = dict(os.environ)
    env.update(env_extra)
    p = subprocess.run([sys.executable, os.path.join(HERE, "multidevice_check.py")], capture_output=True, text=True,
                       env=env, timeout=600)
    assert p.returncode == 0, p.stderr[-4000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("env", [ENV2, {"ZCRC_DEVICES": "0,0,0", "ZCRC_SHARD_MIN_BYTES": "1"}],
                         ids=["two-logical", "three-logical-tiny-shards"])
def test_host_entry_points_over_logical_devices(env):
    r = _child(env)
    n = len(env["ZCRC_DEVICES"].split(","))
    assert r["device_set"] == [0] * n
    for k in ("config2", "config4", "chains", "zip", "inflate", "concurrent"):
        assert r[k][0] == r[k][1], (k, r[k])
    assert r["checked"] and r["dropin"] and r["streams"], r
    assert r["dropin_stats"]["gpu"] == 3 and r["dropin_stats"]["fallback"] == 0, r["dropin_stats"]


def test_bad_device_list_is_reported():
    env = dict(os.environ, ZCRC_DEVICES="0,99")
    code = ("import zipsfs_amd as z\n"
            "try:\n    z.device_set()\nexcept z.ZcrcError as e:\n    print('ERR', e)\n")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=300,
                       cwd=os.path.dirname(HERE))
    assert "ERR" in p.stdout and "ZCRC_DEVICES" in p.stdout, p.stdout + p.stderr


def test_dropin_harness_over_logical_devices(tmp_path):
    """ZIPsFS's call site (fhandle_check_crc32 shape) against the drop-in with
    two logical devices: every golden entry on the GPU, large ones cut
    across both, bit-exact."""
    exe = du.build_harness(tmp_path)
    recs = du.golden_records(big=True)
    path = tmp_path / "recs.bin"
    du.write_records(path, recs)
    env = dict(ENV2, ZCRC_GPU_MIN_BYTES="0")
    rc, rows, stats, err = du.run_harness(exe, path, env)
    assert rc == 0, err
    assert [crc for _, crc, _ in rows] == [c & 0xFFFFFFFF for _, c, _ in recs]
    assert stats == {"gpu": len(recs), "host": 0, "fallback": 0}, stats
