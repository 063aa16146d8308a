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
// host-memory calls (zcrc_inflate_batch, the ZIP verifier): hipMalloc'd
// once and reused by the thread's later calls, each of which synchronizes
// before it returns.  (Round 4: a stream-ordered hipMallocAsync/hipFreeAsync
// pair per call gave the split inflate's finder stale input on the second
// call of a C process -- ROCm 7.2's runtime; torch's bundled 7.0 did not
// show it -- and one illegal-address fault: DESIGN.md section 7d.)
enum TlBuffer { kTlInflateHost = 0, kTlZipImage, kTlZipDesc, kTlZipArena, kTlZipCopy, kTlCount };
int tl_device_buffer(int purpose, size_t bytes, void **out);
// free the buffer when it holds more than keep_max bytes (large one-off arenas)
void tl_device_trim(int purpose, size_t keep_max);

// Runs fn(stream) on the HIP stream of a staging slot leased on the current
// device (waiting while none is free), returned afterwards: a persistent
// stream instead of one created per call, so the per-stream scratch caches
// are reused.
int with_lease_stream(const std::function<int(hipStream_t)> &fn);

}  // namespace zcrc
