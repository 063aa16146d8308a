// zcrc_runtime.h -- host runtime services shared by the entry points (not
// public ABI; implemented in zcrc_runtime.hip).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <functional>

#include <hip/hip_runtime.h>

namespace zcrc {

// Shards a host-memory call of `bytes` is cut into: one per logical device of
// the device set (ZCRC_DEVICES), but at least ZCRC_SHARD_MIN_BYTES (default
// 8 MiB) each; 1 when the set is empty (run_sharded then fails).
size_t host_shards(uint64_t bytes);

// Runs job(g) for g in [0, shards): g = 0 on the calling thread, the others
// on persistent per-shard workers, each with logical device (first + g) of
// the set current (first = the least loaded one) and restored afterwards.
// Returns the first negative code (its zcrc_last_error text carried over),
// else the first positive one, else 0.
int run_sharded(size_t shards, const std::function<int(size_t)> &job);

// Per-thread, per-device, grow-only device buffers for the synchronous
// calls (zcrc_inflate_batch, the ZIP verifier and extractor): hipMalloc'd once
// and reused by the thread's later calls, each of which synchronizes its
// stream before it returns -- on every exit once work is queued (SyncOnExit
// below).  Kept bytes per device are bounded (ZCRC_TL_CACHE_MIB, default
// 8 GiB); zcrc_release_cached() frees the calling thread's.  Round 4 replaced
// a per-call hipMallocAsync/hipFreeAsync pair with these after the split
// inflate's finder and probe read other bytes than its decoder on the second
// call of a C process, and one illegal-address fault followed (DESIGN.md 7e
// states what that trace does and does not show).  ZCRC_TL_EXACT=1 (tests)
// allocates exactly the size asked behind a canary that the trim checks.
enum TlBuffer { kTlInflateHost = 0, kTlZipImage, kTlZipDesc, kTlZipArena, kTlZipCopy, kTlCount };
int tl_device_buffer(int purpose, size_t bytes, void **out);
// After the call's synchronize: checks the canary (ZCRC_TL_EXACT: an error
// when an out-of-bounds write changed it), then frees the buffer when it
// holds more than keep_max bytes, when the device's kept bytes exceed the
// budget, or in exact mode.
int tl_device_trim(int purpose, size_t keep_max);
// after a failed synchronize: free the buffer (hipFree waits for the device)
void tl_device_drop(int purpose);
uint64_t tl_kept_bytes(int dev);

// Synchronizes `st` on scope exit unless disarmed: a call that returns early
// after queueing work must not leave it running on a buffer its thread's
// next call reuses.  When that synchronize fails, the thread-local
// buffer `purpose` (if >= 0) is dropped.
struct SyncOnExit {
  hipStream_t st;
  int purpose;
  bool armed = true;
  SyncOnExit(hipStream_t s, int p) : st(s), purpose(p) {}
  ~SyncOnExit() {
    if (armed && hipStreamSynchronize(st) != hipSuccess && purpose >= 0) tl_device_drop(purpose);
  }
};

// Runs fn(stream) on the HIP stream of a staging slot leased on the current
// device (waiting while none is free), returned afterwards: a persistent
// stream instead of one created per call, so the per-stream scratch caches
// are reused.
int with_lease_stream(const std::function<int(hipStream_t)> &fn);

}  // namespace zcrc
