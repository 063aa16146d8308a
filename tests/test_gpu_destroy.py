"""GPU: the device-batch scratch cache against destroyed streams, concurrent
callers and special stream handles, through
tests/dropin/destroy_release.c -- a C process linking ROCm's HIP runtime, as
ZIPsFS would (its call site: src/ZIPsFS_preloadfileram.c:243; up to 32
preload threads: src/ZIPsFS_async.c:468).

* > 2 s of batches queued on a stream that is destroyed with them queued,
  its scratch freed by zcrc_release_cached at once: every result bit-exact
  against a live-stream reference (itself checked with zlib), no fault, the
  cache empty afterwards.
* zcrc_release_cached while another thread keeps calling: returns within the
  grace plus slack (it used to wait for every later release).
* hipStreamPerThread and the null stream as the caller's stream.
* With a 1 MiB budget, 48 destroyed streams' scratch is freed by the
  library's own reaper thread while a live stream holds ~0.5 s of queued
  work, and no call waits for the device.
* Graphs captured back to back in global capture mode (torch.cuda.graph's
  default), each holding a zcrc32_batch_device_ws, next to 48 destroyed
  streams' idle scratch: below the idle budget (no trims) no capture is
  invalidated and every replay is bit-exact.  (Above it, a trim's
  synchronize and hipFree do invalidate a concurrent global-mode capture:
  measured in tools/capture_ab.sh)"""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _build(tmp_path) -> str:
    exe = os.path.join(str(tmp_path), "destroy_release")
    subprocess.run(["gcc", "-O1", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-I",
                    os.path.join(ROOT, "include"), os.path.join(HERE, "dropin", "destroy_release.c"), "-o", exe,
                    "-L", os.path.join(ROOT, "zipsfs_amd"), "-lzcrc", "-L/opt/rocm/lib", "-lamdhip64",
                    "-Wl,-rpath," + os.path.join(ROOT, "zipsfs_amd"), "-pthread", "-lz"], check=True)
    return exe


def _run(args, env_extra=None) -> dict:
    env = dict(os.environ)
    env.update(env_extra or {})
    p = subprocess.run(args, capture_output=True, text=True, env=env, timeout=150)
    assert p.returncode == 0, f"rc {p.returncode}\n{p.stdout[-2000:]}\n{p.stderr[-4000:]}"
    d = json.loads(p.stdout.strip().splitlines()[-1])
    print(json.dumps(d))
    return d


@pytest.mark.timeout(200)
def test_queued_work_outlives_grace_then_destroy_and_release(tmp_path):
    d = _run([_build(tmp_path), "destroy", "2.5"])
    assert d["queued_gpu_s"] > 2.0, d
    assert d["mismatches"] == 0 and d["checked"] == d["launches"] * 16384, d
    assert d["released_bytes"] > 0 and d["entries_after"] == 0, d
    # one deadline on entry: not every later release of the other thread
    assert d["release_while_calling_ms"] < 4000, d
    assert d["other_thread_calls"] > 0 and d["other_thread_bad"] == 0 and d["other_thread_errors"] == 0, d
    assert d["special_streams_bad"] == 0, d


@pytest.mark.timeout(200)
def test_reaper_trims_destroyed_streams_without_blocking_callers(tmp_path):
    d = _run([_build(tmp_path), "trim"], {"ZCRC_SCRATCH_CACHE_MIB": "1"})
    assert d["mismatches"] == 0, d
    assert d["bytes_after"] <= (2 << 20), d  # the reaper freed the destroyed streams' scratch by itself
    assert d["peak_entries"] > 4, d
    assert d["worst_call_ms"] < 250, d  # no call waited for the ~0.5 s queued on the live stream


@pytest.mark.timeout(200)
def test_global_mode_captures_next_to_the_cache(tmp_path):
    d = _run([_build(tmp_path), "capture", "3.5"], {"ZCRC_SCRATCH_CACHE_MIB": "2048"})
    assert d["capture_fail"] == 0 and d["replays"] == d["captures"] > 100, d
    assert d["mismatches"] == 0, d
    assert d["entries_after"] >= 48, d  # below the budget: nothing trimmed, the destroyed streams' scratch kept
