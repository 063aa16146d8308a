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

// ------------------------------------------------------------ split plan
// Two passes like plan_tile_sums/plan_tile_scan.  Per tile: bytes of the
// buffers above kSmallMax, bytes of those at or below it, both counts packed
// (low half: above, high half: at or below) and the small buffers' size-class
// counts.  The scan decides for the whole launch (every workgroup reads all
// tile sums, so all decide alike): split when the small list is worth at
// least two of the batch kernel's workgroups (or p.force and there is any
// small buffer); otherwise it writes the plain prefix of all buffers, as
// plan_tile_scan does, and an empty small list.  The large buffers keep
// their order; the small list is ordered by size class.

__device__ __forceinline__ uint32_t size_class(uint64_t len) { return (uint32_t)((len + 255) >> 8); }  // 256-B blocks

__global__ __launch_bounds__(1024) void plan_split_sums(SplitPlan p) {
  __shared__ uint64_t s_w[16][3];
  __shared__ uint32_t s_cls[kSizeClasses];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  if (threadIdx.x < kSizeClasses) s_cls[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kPlanTile;
  uint64_t bl = 0, bs = 0, cnt = 0;
  // all loads first: with the LDS atomics between them the compiler issued
  // them one round trip at a time
  uint64_t lv[kPlanPerThread];
#pragma unroll
  for (uint32_t k = 0; k < kPlanPerThread; k++) {
    const uint64_t idx = base + (uint64_t)k * blockDim.x + threadIdx.x;
    lv[k] = idx < p.n ? p.lens[idx] : 0;
  }
#pragma unroll
  for (uint32_t k = 0; k < kPlanPerThread; k++) {
    const uint64_t idx = base + (uint64_t)k * blockDim.x + threadIdx.x;
    if (idx < p.n) {
      const uint64_t L = lv[k];
      if (L > kSmallMax) {
        bl += L, cnt += 1;
      } else {
        bs += L, cnt += 1ull << 32;
        atomicAdd(&s_cls[size_class(L)], 1u);
      }
    }
  }
  // sums only (no scan): one butterfly per wave, then the 16 wave totals
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1)
    bl += __shfl_xor(bl, d, 64), bs += __shfl_xor(bs, d, 64), cnt += __shfl_xor(cnt, d, 64);
  if (lane == 0) s_w[wv][0] = bl, s_w[wv][1] = bs, s_w[wv][2] = cnt;
  __syncthreads();
  uint64_t *t = p.tile_sum + (uint64_t)kTileWords * blockIdx.x;
  if (threadIdx.x < 3) {
    uint64_t v = 0;
    for (uint32_t w = 0; w < 16; w++) v += s_w[w][threadIdx.x];
    t[threadIdx.x] = v;
  } else if (threadIdx.x < 3 + kSizeClasses) {
    t[threadIdx.x] = s_cls[threadIdx.x - 3];
  }
}

// Thread t of a tile owns its buffers 8t .. 8t+7 (one block scan per
// quantity: a lane-contiguous layout with a wave scan per k cost 16 dependent
// 64-bit shuffle scans per thread and measured 30 us on config 4, against 12
// for plan_tile_scan).  Without a split only the byte prefix is scanned.
__global__ __launch_bounds__(1024) void plan_split_scan(SplitPlan p) {
  __shared__ uint64_t s_b[16], s_c[16];
  __shared__ uint64_t s_off[2];
  __shared__ uint32_t s_mode;
  __shared__ uint64_t s_small_bytes;
  __shared__ uint32_t s_small_wgs;
  // the small list is ordered by size class (256-B blocks), so that the
  // buffers a wave of the small body takes together run equal block counts;
  // within a class and tile the order is the LDS atomics' (any order is
  // correct: results go out by index)
  __shared__ uint64_t s_cls_prev[kSizeClasses], s_cls_all[kSizeClasses], s_cls_at[kSizeClasses];
  __shared__ uint32_t s_cls_cur[kSizeClasses];
  if (blockIdx.x == 0 && threadIdx.x == 0) *p.ctr = 0u;  // the CRC kernel's work counter
  // this thread's lengths, pointers and seeds, loaded before the tile sums
  // are read (the scatter below stores between its uses, so loads left in
  // its loop were issued one round trip at a time: 25 us per launch on
  // config 4)
  const uint64_t base = (uint64_t)blockIdx.x * kPlanTile + (uint64_t)threadIdx.x * kPlanPerThread;
  uint64_t v[kPlanPerThread];
  const uint8_t *pv[kPlanPerThread];
  uint32_t sv[kPlanPerThread];
#pragma unroll
  for (uint32_t k = 0; k < kPlanPerThread; k++) {
    const uint64_t idx = base + k;
    const bool in = idx < p.n;
    v[k] = in ? p.lens[idx] : 0;
    pv[k] = in ? p.ptrs[idx] : nullptr;
    sv[k] = in && p.seeds ? p.seeds[idx] : 0u;
  }
  // Tile sums and class counts, read in parallel (one thread summing the
  // tile words 8 at a time cost ~1 us per 8 tiles: 28 us on 1M x 1 KiB).
  // Wave w takes tile words w, w + 16, w + 32 (0..2: the sums, 3..: the class
  // counts); its lanes stride over the tiles.
  __shared__ uint64_t s_tw[3][2];
  {
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, tiles = gridDim.x;
    for (uint32_t q = wv; q < 3 + kSizeClasses; q += 16) {
      const uint32_t word = q;  // tile word: 0..2 sums, 3.. class counts
      uint64_t prev = 0, all = 0;
      for (uint32_t t = lane; t < tiles; t += 64) {
        const uint64_t x = p.tile_sum[(uint64_t)kTileWords * t + word];
        all += x;
        if (t < blockIdx.x) prev += x;
      }
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) all += __shfl_xor(all, d, 64), prev += __shfl_xor(prev, d, 64);
      if (lane == 0) {
        if (q < 3) {
          s_tw[q][0] = prev, s_tw[q][1] = all;
        } else {
          s_cls_prev[q - 3] = prev, s_cls_all[q - 3] = all, s_cls_cur[q - 3] = 0;
        }
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t pl = s_tw[0][0], ps = s_tw[1][0], pc = s_tw[2][0];  // previous tiles
    const uint64_t al = s_tw[0][1], as = s_tw[1][1], ac = s_tw[2][1];  // all tiles
    {
      // workgroups for the small list: its share of the CU time, a
      // small-list byte weighted small_cost/4 against a batch-kernel byte
      // (config 4 forced to split, one box: weight 1 -> 2.90 ms per step,
      // 1.5 -> 2.25, 2.5 -> 2.045, 3.5 -> 2.046, 5 -> 2.047, 7 -> 2.049,
      // against 2.06-2.075 unsplit; profiles/r02/small_kernel/)
      const uint64_t n_large = ac & 0xFFFFFFFFull, n_small = ac >> 32;
      const uint64_t ws = p.small_cost * as, wl = 4 * al;
      uint64_t wgs = p.grid;
      if (n_large) wgs = ws ? (p.grid * ws + ws + wl - 1) / (ws + wl) : 0;
      // split when the small list is worth at least two workgroups (a
      // workgroup given to a handful of small buffers would idle a CU)
      const uint32_t mode = n_small && (p.force || wgs >= 2);
      if (n_large) wgs = wgs < 1 ? 1 : (wgs > p.grid - 1 ? p.grid - 1 : wgs);
      s_mode = mode;
      s_small_bytes = as;
      s_small_wgs = (uint32_t)wgs;
      s_off[0] = mode ? pl : pl + ps;
      s_off[1] = pc;
    }
  }
  __syncthreads();
  const bool split = s_mode != 0;
  uint64_t bytes = 0, cnt = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPlanPerThread; k++) {
    const uint64_t idx = base + k;
    if (idx < p.n) {
      const bool large = !split || v[k] > kSmallMax;
      bytes += large ? v[k] : 0;
      cnt += large ? 1ull : 1ull << 32;
    }
  }
  uint64_t tb;
  uint64_t rb = s_off[0] + block_excl_scan(bytes, s_b, &tb);
  if (!split) {  // the plain prefix (plan_tile_scan's), counts {n, 0, 0}
#pragma unroll
    for (uint32_t k = 0; k < kPlanPerThread; k++) {
      const uint64_t idx = base + k;
      if (idx >= p.n) break;
      p.prefix_c[idx] = rb;
      p.out[idx] = 0u;  // split pieces xor into it
      rb += v[k];
      if (idx + 1 == p.n) p.prefix_c[p.n] = rb, p.counts[0] = p.n, p.counts[1] = 0, p.counts[2] = 0, p.counts[3] = 16;
    }
    return;
  }
  if (threadIdx.x == 0) {  // where this tile's entries of each class start
    uint64_t at = 0;
    for (uint32_t c = 0; c < kSizeClasses; c++) s_cls_at[c] = at + s_cls_prev[c], at += s_cls_all[c];
  }
  uint64_t tc;
  uint64_t rc = s_off[1] + block_excl_scan(cnt, s_c, &tc);  // (its barriers order s_cls_at)
#pragma unroll
  for (uint32_t k = 0; k < kPlanPerThread; k++) {
    const uint64_t idx = base + k;
    if (idx >= p.n) break;
    if (v[k] > kSmallMax) {
      const uint64_t j = rc & 0xFFFFFFFFull;
      p.prefix_c[j] = rb;
      p.ptrs_c[j] = pv[k];
      if (p.seeds) p.seeds_c[j] = sv[k];
      p.oidx[j] = (uint32_t)idx;
      p.out[idx] = 0u;
      rb += v[k];
      rc += 1;
    } else {
      const uint32_t c = size_class(v[k]);
      p.sidx[s_cls_at[c] + atomicAdd(&s_cls_cur[c], 1u)] = (uint32_t)idx;
      rc += 1ull << 32;
    }
    if (idx + 1 == p.n) {  // totals
      p.prefix_c[rc & 0xFFFFFFFFull] = rb;
      p.counts[0] = rc & 0xFFFFFFFFull;
      p.counts[1] = rc >> 32;
      p.counts[2] = 1;
      p.counts[3] = s_small_bytes <= 2048 * (rc >> 32) ? 8 : 16;  // mean small length <= 2 KiB: 8 lanes
      p.counts[4] = s_small_wgs;
    }
  }
}

hipError_t launch_plan_split(const SplitPlan &p, hipStream_t stream) {
  const uint64_t tiles = plan_tiles(p.n);
  hipLaunchKernelGGL(plan_split_sums, dim3((unsigned)tiles), dim3(1024), 0, stream, p);
  hipLaunchKernelGGL(plan_split_scan, dim3((unsigned)tiles), dim3(1024), 0, stream, p);
  return hipGetLastError();
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

// the one-launch form (launch_batch with fused = true)
const char *fused_kernel_name() {
  static char name[160];
  static std::once_flag once;
  std::call_once(once, [] {
    snprintf(name, sizeof name, "zcrc::crc32_batch_kernel<false, %uu, 0, true, false, 1, %d, true, %s>", kDepth,
             kLoadNt, kWindowed ? "true" : "false");
  });
  return name;
}

// the general-form small kernels as rocprofv3 names them
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
