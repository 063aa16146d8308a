// zcrc_runtime.h -- host runtime services shared by the entry points (not
// public ABI; implemented in zcrc_runtime.hip).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <functional>

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

}  // namespace zcrc
