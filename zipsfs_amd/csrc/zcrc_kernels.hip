// zcrc_kernels.hip -- instantiations of the batched CRC-32 kernel, the plan
// (prefix-scan) kernels and their launchers.  The kernel itself lives in
// zcrc_batch_kernel.h (shared with the measurement tools under tools/).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <mutex>

#include "zcrc_batch_kernel.h"
#include "zcrc_small_kernel.h"

namespace zcrc {

// ------------------------------------------------------------ plan kernels
// Exclusive prefix over lengths: prefix[0..n] (prefix[n] = total), and zero
// out[] (split pieces xor into it).  Tile = kPlanTile buffers per workgroup.

// wave_incl_scan / block_excl_scan: zcrc_batch_kernel.h

__global__ __launch_bounds__(1024) void plan_tile_sums(const uint64_t *lens, uint64_t n, uint64_t *tile_sum,
                                                       uint32_t *out) {
  __shared__ uint64_t s_tmp[16];
  const uint64_t base = (uint64_t)blockIdx.x * kPlanTile;
  uint64_t acc = 0;
  for (uint32_t k = 0; k < kPlanPerThread; k++) {
    const uint64_t idx = base + (uint64_t)k * blockDim.x + threadIdx.x;
    if (idx < n) {
      acc += lens[idx];
      out[idx] = 0u;
    }
  }
  uint64_t tot;
  (void)block_excl_scan(acc, s_tmp, &tot);
  if (threadIdx.x == 0) tile_sum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(1024) void plan_tile_scan(const uint64_t *lens, uint64_t n, const uint64_t *tile_sum,
                                                       uint64_t *prefix, uint32_t *out, int zero_out,
                                                       uint32_t *ctr) {
  __shared__ uint64_t s_tmp[16];
  __shared__ uint64_t s_off;
  if (ctr && blockIdx.x == 0 && threadIdx.x == 0) *ctr = 0u;  // the CRC kernel's work counter
  if (threadIdx.x < 64) {
    uint64_t acc = 0;
    for (uint32_t b = threadIdx.x; b < blockIdx.x; b += 64) acc += tile_sum[b];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) acc += __shfl_xor(acc, d, 64);
    if (threadIdx.x == 0) s_off = acc;
  }
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kPlanTile + (uint64_t)threadIdx.x * kPlanPerThread;
  uint64_t v[kPlanPerThread];
  uint64_t acc = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPlanPerThread; k++) {
    const uint64_t idx = base + k;
    v[k] = idx < n ? lens[idx] : 0;
    if (zero_out && idx < n) out[idx] = 0u;
    acc += v[k];
  }
  uint64_t tot;
  uint64_t run = s_off + block_excl_scan(acc, s_tmp, &tot);
#pragma unroll
  for (uint32_t k = 0; k < kPlanPerThread; k++) {
    const uint64_t idx = base + k;
    if (idx < n) prefix[idx] = run;
    run += v[k];
    if (idx + 1 == n) prefix[n] = run;
  }
  if (n == 0 && blockIdx.x == 0 && threadIdx.x == 0) prefix[0] = 0;
}

// One-tile plan (n <= kPlanTile), coalesced: wave w owns buffers
// [512w, 512w + 512) and lane l loads buffer 512w + 64k + l for k < 8, so
// every load and store of a wave covers 512 (or 256) contiguous bytes.  The
// scan runs along k with a wave-wide carry, and the 16 wave totals meet in
// LDS after the one barrier.  (plan_tile_scan gives each thread 8
// consecutive buffers: 64-B lane strides on every access, 7.6 us for
// config 2's 4096 buffers, profiles/r01/v10/rocprof_kernel_stats_config2.csv.)
__global__ __launch_bounds__(1024) void plan_one_tile(const uint64_t *lens, uint64_t n, uint64_t *prefix,
                                                      uint32_t *out, uint32_t *ctr) {
  __shared__ uint64_t s_wsum[16];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint64_t base = (uint64_t)wv * (64u * kPlanPerThread);
  if (ctr && threadIdx.x == 0) *ctr = 0u;  // the CRC kernel's work counter
  uint64_t v[kPlanPerThread];
#pragma unroll
  for (uint32_t k = 0; k < kPlanPerThread; k++) {
    const uint64_t idx = base + 64u * k + lane;
    v[k] = idx < n ? lens[idx] : 0;
    if (idx < n) out[idx] = 0u;
  }
  uint64_t carry = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPlanPerThread; k++) {
    const uint64_t inc = wave_incl_scan(v[k]);
    v[k] = carry + inc - v[k];  // exclusive within the wave's 512 buffers
    carry += __shfl(inc, 63, 64);
  }
  if (lane == 0) s_wsum[wv] = carry;
  __syncthreads();
  uint64_t off = 0, tot = 0;
  for (uint32_t j = 0; j < 16u; j++) {
    const uint64_t s = s_wsum[j];
    if (j < wv) off += s;
    tot += s;
  }
#pragma unroll
  for (uint32_t k = 0; k < kPlanPerThread; k++) {
    const uint64_t idx = base + 64u * k + lane;
    if (idx < n) prefix[idx] = off + v[k];
  }
  if (threadIdx.x == 0) prefix[n] = tot;
}

// ------------------------------------------------------------ launchers

hipError_t launch_batch(const BatchArgs &args, bool strided, int num_cus, hipStream_t stream, hipEvent_t t0,
                        hipEvent_t t1, bool fused) {
  const dim3 grid((unsigned)num_cus), block(kThreads);
  // t0/t1 (profiling): timestamps carried by the dispatch packet itself --
  // event records around the launch add ~11 us of queue bubbles per launch
  if (fused)
    hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, 0, true, false, 1, kLoadNt, true>), grid, block, 0,
                          stream, t0, t1, 0, args);
  else if (strided)
    hipExtLaunchKernelGGL((crc32_batch_kernel<true, kDepth, 0>), grid, block, 0, stream, t0, t1, 0, args);
  else
    hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, 0>), grid, block, 0, stream, t0, t1, 0, args);
  return hipGetLastError();
}

// The general-form kernel launch_batch instantiates, as rocprofv3 names it
// (bench.py reports it next to the roofline; tools/collect_profiles.sh keys
// the PMC traffic by it).
const char *product_kernel_name() {
  static char name[160];
  static std::once_flag once;
  std::call_once(once, [] {
    snprintf(name, sizeof name, "zcrc::crc32_batch_kernel<false, %uu, 0, true, false, 1, %d, false, %s>", kDepth,
             kLoadNt, kWindowed ? "true" : "false");
  });
  return name;
}

// Small whole buffers: 16 lanes per buffer with 8 blocks in flight, or 8
// lanes with 4 (same 32 VGPRs of loads, twice the buffers: pays below ~2 KiB).
hipError_t launch_small(const SmallArgs &args, bool strided, int lanes, int num_cus, hipStream_t stream,
                        hipEvent_t t0, hipEvent_t t1) {
  const dim3 grid((unsigned)num_cus), block(kThreads);
  if (strided) {
    if (lanes == 8)
      hipExtLaunchKernelGGL((crc32_small_kernel<true, 8, 4>), grid, block, 0, stream, t0, t1, 0, args);
    else
      hipExtLaunchKernelGGL((crc32_small_kernel<true, 16, 8>), grid, block, 0, stream, t0, t1, 0, args);
  } else {
    if (lanes == 8)
      hipExtLaunchKernelGGL((crc32_small_kernel<false, 8, 4>), grid, block, 0, stream, t0, t1, 0, args);
    else
      hipExtLaunchKernelGGL((crc32_small_kernel<false, 16, 8>), grid, block, 0, stream, t0, t1, 0, args);
  }
  return hipGetLastError();
}

// the general-form small kernel as rocprofv3 names it
const char *small_kernel_name(int lanes) {
  return lanes == 8 ? "zcrc::crc32_small_kernel<false, 8, 4>" : "zcrc::crc32_small_kernel<false, 16, 8>";
}

hipError_t launch_plan(const uint64_t *d_lens, uint64_t n, uint64_t *d_prefix, uint64_t *d_tile_sum,
                       uint32_t *d_out, uint32_t *d_ctr, hipStream_t stream) {
  const uint64_t tiles = n == 0 ? 1 : (n + kPlanTile - 1) / kPlanTile;
  if (tiles > 1) {
    hipLaunchKernelGGL(plan_tile_sums, dim3((unsigned)tiles), dim3(1024), 0, stream, d_lens, n, d_tile_sum, d_out);
    hipLaunchKernelGGL(plan_tile_scan, dim3((unsigned)tiles), dim3(1024), 0, stream, d_lens, n,
                       (const uint64_t *)d_tile_sum, d_prefix, d_out, 0, d_ctr);
  } else {
    static_assert(kPlanTile == 16u * 64u * kPlanPerThread, "plan_one_tile: 16 waves x 64 lanes x kPlanPerThread");
    hipLaunchKernelGGL(plan_one_tile, dim3(1), dim3(1024), 0, stream, d_lens, n, d_prefix, d_out, d_ctr);
  }
  return hipGetLastError();
}

}  // namespace zcrc
