"""GPU: caller streams created and destroyed between libzcrc calls, from a C
process, in several threads at once.

tests/dropin/stream_churn.c queues device batches, one-stream inflates and
ZIP verifications on fresh HIP streams and destroys each stream with its work
still queued, so that a later stream may get the same handle back; the
library's scratch is leased per call and keyed by the stream's handle and,
where the HIP runtime has hipStreamGetId (ROCm >= 7.1, as a C process links
it), its unique id (zcrc_runtime.hip, ScratchCache), so every result must be
bit-exact (zlib is the checker).  The program waits for each destroyed
stream's work on an event recorded before the destroy: on ROCm 7.2 a
destroyed stream's last store can become visible only after hipStreamDestroy
and hipDeviceSynchronize have returned (round 6, profiles/r06/s7/).  With
ZCRC_TL_EXACT=1 every thread-local device buffer is allocated at exactly the
size asked, behind a canary the library checks after each call: an
out-of-bounds write by the split inflate, the batch inflate or the ZIP
kernels is then an error instead of landing in a reused buffer's padding.
The reference's call site: src/ZIPsFS_preloadfileram.c:243 (the CRC of the
preloaded, inflated entry)."""
import json
import os
import subprocess

import pytest

import dropin_util as du

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _build(tmp_path) -> str:
    exe = os.path.join(str(tmp_path), "stream_churn")
    subprocess.run(["gcc", "-O1", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-I",
                    os.path.join(ROOT, "include"), os.path.join(HERE, "dropin", "stream_churn.c"), "-o", exe,
                    "-L", os.path.join(ROOT, "zipsfs_amd"), "-lzcrc", "-L/opt/rocm/lib", "-lamdhip64",
                    "-Wl,-rpath," + os.path.join(ROOT, "zipsfs_amd"), "-pthread", "-lz"], check=True)
    return exe


def _run(exe, rounds, threads, env_extra=None) -> dict:
    env = dict(os.environ)
    env.update(env_extra or {})
    p = subprocess.run([exe, str(rounds), str(threads)], capture_output=True, text=True, env=env, timeout=240)
    assert p.returncode == 0, f"rc {p.returncode}\n{p.stdout[-2000:]}\n{p.stderr[-4000:]}"
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["failures"] == 0 and d["checks"] > 0, d
    print(json.dumps(d))
    return d


@pytest.mark.timeout(300)
def test_streams_destroyed_between_calls_three_threads(tmp_path):
    d = _run(_build(tmp_path), 3, 3)
    # every thread-round: 8 device batches (~64k buffers), 2 + 3 inflates, 3 x 24 ZIP entries
    assert d["checks"] >= 3 * 3 * (60000 + 5 + 72), d
    assert d["release_rc"] == 0 and d["released_bytes"] > 0, d
    # every idle entry -- those of destroyed streams included -- is freed
    assert d["entries_left"] == 0 and d["bytes_left"] == 0, d


@pytest.mark.timeout(300)
def test_streams_destroyed_with_the_reaper_trimming_throughout(tmp_path):
    """The same churn with a scratch budget of 0: every release wakes the
    library's reaper thread, which synchronizes the device and frees the idle
    scratch past its grace while three threads keep calling on fresh streams
    (round 6: the trim left the callers' path)."""
    d = _run(_build(tmp_path), 2, 3, {"ZCRC_SCRATCH_CACHE_MIB": "0"})
    assert d["release_rc"] == 0 and d["entries_left"] == 0, d


@pytest.mark.timeout(300)
def test_exact_size_thread_local_buffers_with_canaries(tmp_path):
    """The same calls with exactly sized thread-local buffers and canaries."""
    _run(_build(tmp_path), 1, 2, {"ZCRC_TL_EXACT": "1"})


@pytest.mark.timeout(300)
def test_text_entry_preload_twice_exact_allocations(tmp_path):
    """The round-4 failure's input (1 MiB text entry, seed 17, through the C
    preload harness's gpu_inflate mode) three times in one process, with
    exactly sized device buffers behind canaries."""
    import zlib
    import inflate_streams as S
    exe = du.build_preload_harness(tmp_path)
    data = S.PAYLOADS["text"](1 << 20, 17)
    path = tmp_path / "entry.deflate"
    path.write_bytes(S.deflate(data, 6))
    exp = zlib.crc32(data)
    rc, rows, stats, err = du.run_preload(exe, path, exp, 3, ["gpu_inflate"],
                                          {"ZCRC_PRELOAD_DEFLATED": str(len(data)), "ZCRC_TL_EXACT": "1",
                                           "ZCRC_SPLIT_TRACE": "1"})
    assert rc == 0, err
    r = rows["gpu_inflate"]
    assert r["ok"] and int(r["crc"], 16) == exp, r
    # The finder, the probes and the speculative decode are functions of the
    # input bytes alone: every call on the same entry must lay the stream out
    # identically.  Round 4's second call did not (its finder and probes saw
    # other bytes than its decoder: DESIGN.md 7e).
    blocks = []
    for line in err.splitlines():
        if line.startswith("[split] src"):
            blocks.append([line])
        elif line.startswith("[split]") and blocks:
            blocks[-1].append(line)
    assert len(blocks) == 3, err[-3000:]
    assert blocks[1] == blocks[0] and blocks[2] == blocks[0], (blocks[0][:3], blocks[1][:3], blocks[2][:3])
