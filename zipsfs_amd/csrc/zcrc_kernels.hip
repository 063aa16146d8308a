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
  if (ctr && blockIdx.x == 0 && threadIdx.x == 0) ctr[0] = 0u, ctr[kFaultByte / 4] = 0u;  // work counter, fault word
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
  if (ctr && threadIdx.x == 0) ctr[0] = 0u, ctr[kFaultByte / 4] = 0u;  // the CRC kernel's work counter, fault word
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
    carry += rdlane64(inc, 63);
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
// Two passes like plan_tile_sums/plan_tile_scan, both with plan_one_tile's
// coalesced layout at kPer buffers per thread (split_per_thread: tiles of
// 1024 kPer buffers): wave w of a tile owns its buffers [64 kPer w, 64 kPer
// (w + 1)), lane l takes 64 kPer w + 64 k + l for k < kPer.  Buffers fall into three classes: small
// (<= kSmallMax), big (>= kBigMin) and medium (between).  Per tile
// (kTileWords): medium bytes, big bytes, small bytes, the medium and big
// counts packed (low / high half), the small count and the small lengths'
// sum of squares (round 4: a batch of about equal small buffers is walked in
// place by the small body, without lists -- mode 2), and the buffers whose
// length differs from lens[0] (round 6: an unsplit batch of equal buffers
// is read in the batch kernel's window order, BatchView::wp).  The scatter decides
// for the whole launch (every workgroup reads the same tile sums, so all
// decide alike): split when the small list is worth at least two of the batch
// kernel's workgroups (or p.force and there is any small buffer); otherwise
// it writes the plain prefix of all buffers, as plan_tile_scan does, and an
// empty small list.  On a split the batch kernel's buffers are compacted
// medium first, then big, each class in index order (round 4): the batch
// kernel hands out the last bytes of its batch dynamically, in 128 KiB units,
// and with the big buffers last those units are sequential runs of one
// buffer; a unit full of medium buffers is a chain of latency-bound pieces,
// and the waves that drew such units last were config 4's ~60 us tail
// (DESIGN.md section 4).  Each tile's small buffers are listed by size class
// (256-B blocks), in index order within a class, so that the buffers a wave
// of the small body takes together run equal block counts.  The ranking is a
// counting sort by ballots -- six ballots give each lane the mask of lanes
// with its class -- with per (class, wave, k) counts scanned in LDS: no
// atomics (the LDS class atomics of the round-2 plan serialised on uniform
// batches: 25.5 us per config-4 plan, ~60 us of a 1M x 1 KiB call).

__device__ __forceinline__ uint32_t size_class(uint64_t len) { return (uint32_t)((len + 255) >> 8); }  // 256-B blocks

template <uint32_t kPer>
__global__ __launch_bounds__(1024) void plan_split_count(SplitPlan p) {
  __shared__ uint64_t s_w[16][kTileWords];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint64_t base = (uint64_t)blockIdx.x * (1024u * kPer) + 64u * kPer * wv + lane;
  uint64_t lv[kPer];
#pragma unroll
  for (uint32_t k = 0; k < kPer; k++) {
    const uint64_t idx = base + 64u * k;
    lv[k] = idx < p.n ? p.lens[idx] : ~0ull;  // ~0: absent
  }
  const uint64_t L0 = p.lens[0];  // (n > kFusedMaxN here)
  uint64_t bm = 0, bb = 0, bs = 0, cmb = 0, cs = 0, sq = 0, mis = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPer; k++) {
    const uint64_t L = lv[k];
    if (L == ~0ull) continue;
    mis += L != L0;
    if (L <= kSmallMax) bs += L, cs += 1, sq += L * L;
    else if (L >= p.big_min) bb += L, cmb += 1ull << 32;
    else bm += L, cmb += 1;
  }
  // wave totals: DPP scans, lane 63 (butterflies of __shfl_xor were LDS round trips)
  bm = rdlane64(wave_incl_scan(bm), 63);
  bb = rdlane64(wave_incl_scan(bb), 63);
  bs = rdlane64(wave_incl_scan(bs), 63);
  cmb = rdlane64(wave_incl_scan(cmb), 63);
  cs = rdlane64(wave_incl_scan(cs), 63);
  sq = rdlane64(wave_incl_scan(sq), 63);
  mis = rdlane64(wave_incl_scan(mis), 63);
  if (lane == 0)
    s_w[wv][0] = bm, s_w[wv][1] = bb, s_w[wv][2] = bs, s_w[wv][3] = cmb, s_w[wv][4] = cs, s_w[wv][5] = sq,
    s_w[wv][6] = mis;
  __syncthreads();
  if (threadIdx.x < kTileWords) {
    uint64_t v = 0;
    for (uint32_t w = 0; w < 16; w++) v += s_w[w][threadIdx.x];
    p.tile_sum[(uint64_t)kTileWords * blockIdx.x + threadIdx.x] = v;
  }
}

// Above kPlanDirectTiles tiles: one workgroup turns the tile sums into
// exclusive prefixes (tile_pre[kTileWords t + q]) and totals (tile_pre[kTileWords tiles + q]),
// so that each scatter workgroup reads 2 kTileWords words instead of every earlier
// tile's (that read grew with the square of the tile count).
__global__ __launch_bounds__(1024) void plan_split_tiles(SplitPlan p, uint32_t tiles) {
  __shared__ uint64_t s_tmp[16];
  const uint32_t per = (tiles + 1023u) / 1024u, t0 = threadIdx.x * per;
  for (uint32_t q = 0; q < kTileWords; q++) {
    uint64_t acc = 0;
    for (uint32_t t = t0; t < t0 + per && t < tiles; t++) acc += p.tile_sum[(uint64_t)kTileWords * t + q];
    uint64_t tot;
    uint64_t run = block_excl_scan(acc, s_tmp, &tot);
    for (uint32_t t = t0; t < t0 + per && t < tiles; t++) {
      const uint64_t x = p.tile_sum[(uint64_t)kTileWords * t + q];
      p.tile_pre[(uint64_t)kTileWords * t + q] = run;
      run += x;
    }
    if (threadIdx.x == 0) p.tile_pre[(uint64_t)kTileWords * tiles + q] = tot;
  }
}

template <uint32_t kPer>
__global__ __launch_bounds__(1024) void plan_split_scatter(SplitPlan p) {
  constexpr uint32_t kGroups = 16 * kPer;  // (wave, k) groups of 64 buffers per tile
  __shared__ uint64_t s_tw[kTileWords][2];           // tile words: earlier tiles, all tiles
  __shared__ uint64_t s_wb[16][2];                   // wave byte totals: medium, big
  __shared__ uint32_t s_wc[16][2];                   // wave counts: medium, big
  __shared__ uint64_t s_tmp[16];
  __shared__ uint32_t s_mode;
  __shared__ uint32_t s_cls[kSizeClasses * kGroups];  // small count per (class, group) -> exclusive position
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  const uint64_t lt = (1ull << lane) - 1;
  uint64_t st[6] = {0, 0, 0, 0, 0, 0};  // diagnostics: phase stamps (p.stamps)
  if (p.stamps) st[0] = __builtin_amdgcn_s_memrealtime();
  if (blockIdx.x == 0 && tid == 0) p.ctr[0] = 0u, p.ctr[kFaultByte / 4] = 0u;  // work counter, fault word
  const uint64_t base = (uint64_t)blockIdx.x * (1024u * kPer) + 64u * kPer * wv + lane;
  // this thread's lengths first (coalesced); pointers and seeds are loaded
  // for the stores at the end (holding them from here spilled 61 VGPRs)
  uint64_t v[kPer];
#pragma unroll
  for (uint32_t k = 0; k < kPer; k++) {
    const uint64_t idx = base + 64u * k;
    v[k] = idx < p.n ? p.lens[idx] : 0;
  }
  // earlier tiles' and all tiles' sums
  if (p.tile_pre) {
    if (tid < kTileWords) s_tw[tid][0] = p.tile_pre[(uint64_t)kTileWords * blockIdx.x + tid];
    else if (tid < 2 * kTileWords)
      s_tw[tid - kTileWords][1] = p.tile_pre[(uint64_t)kTileWords * gridDim.x + tid - kTileWords];
  } else if (wv < kTileWords) {
    uint64_t prev = 0, all = 0;
    for (uint32_t t = lane; t < gridDim.x; t += 64) {
      const uint64_t x = p.tile_sum[(uint64_t)kTileWords * t + wv];
      all += x;
      if (t < blockIdx.x) prev += x;
    }
    all = rdlane64(wave_incl_scan(all), 63);
    prev = rdlane64(wave_incl_scan(prev), 63);
    if (lane == 0) s_tw[wv][0] = prev, s_tw[wv][1] = all;
  }
  for (uint32_t i = tid; i < kSizeClasses * kGroups; i += 1024) s_cls[i] = 0u;
  __syncthreads();
  if (p.stamps) st[1] = __builtin_amdgcn_s_memrealtime();
  const uint64_t am = s_tw[0][1], ab = s_tw[1][1], as = s_tw[2][1];  // all tiles: bytes
  const uint64_t n_med = s_tw[3][1] & 0xFFFFFFFFull, n_big = s_tw[3][1] >> 32, n_small = s_tw[4][1];
  const uint64_t al = am + ab, n_large = n_med + n_big;
  if (tid == 0) {
    // workgroups for the small list: its share of the CU time, a small-list
    // byte weighted small_cost/4 against a batch-kernel byte (config 4 forced
    // to split, one box: weight 1 -> 2.90 ms per step, 1.5 -> 2.25, 2.5 ->
    // 2.045, 3.5 -> 2.046, 5 -> 2.047, 7 -> 2.049, against 2.06-2.075
    // unsplit; profiles/r02/small_kernel/)
    const uint64_t ws = p.small_cost * as, wl = 4 * al;
    uint64_t wgs = p.grid;
    if (n_large) wgs = ws ? (p.grid * ws + ws + wl - 1) / (ws + wl) : 0;
    // split when the small list is worth at least two workgroups (a
    // workgroup given to a handful of small buffers would idle a CU)
    uint32_t mode = n_small && (p.force || wgs >= 2);
    if (n_large) wgs = wgs < 1 ? 1 : (wgs > p.grid - 1 ? p.grid - 1 : wgs);
    // direct (mode 2): every buffer is small and their lengths are about equal
    // (standard deviation at most 128 B: a size class or two): the small body
    // walks the caller's arrays in index order, no lists are written (the
    // size-class order buys nothing on such a batch)
    if (mode && !n_large && p.direct_ok) {
      const double mean = (double)as / (double)n_small;
      const double var = (double)s_tw[5][1] / (double)n_small - mean * mean;
      if (var <= 128.0 * 128.0) mode = 2;
    }
    s_mode = mode;
    if (blockIdx.x == 0) {  // totals: the batch kernel's count, prefix end and the small list
      const uint64_t nl = mode ? n_large : p.n;
      p.prefix_c[nl] = mode ? al : al + as;
      p.counts[0] = nl;
      p.counts[1] = mode ? n_small : 0;
      p.counts[2] = mode;
      p.counts[3] = mode && as <= 2048 * n_small ? 8 : 16;  // mean small length <= 2 KiB: 8 lanes
      p.counts[4] = wgs;
      p.counts[5] = !mode && s_tw[6][1] == 0;  // unsplit and every length equal: the window order
    }
  }
  __syncthreads();
  if (p.stamps) st[2] = __builtin_amdgcn_s_memrealtime();
  if (s_mode == 2) return;  // direct: nothing to list (workgroup-uniform)
  const bool split = s_mode != 0;
  // byte prefixes of this tile's batch-kernel buffers, per class (without a
  // split: all of them as one class), along (k, lane) = index order, wave
  // carries; their counts from ballots.  Per (thread, k) one byte offset
  // within the wave's class and one packed word: the count offset within
  // the wave's class (bits 0-9), the size class (10-15; 63: the batch
  // kernel's), the rank within the (wave, k) group's class (16-21), big (22).
  uint64_t ex[kPer], cmry = 0, cbry = 0;
  uint32_t meta[kPer], ccm = 0, ccb = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPer; k++) {
    const bool in = base + 64u * k < p.n;
    const bool large = in && (!split || v[k] > kSmallMax);
    const bool big = large && split && v[k] >= p.big_min;
    const uint64_t xm = large && !big ? v[k] : 0, xb = big ? v[k] : 0;
    const uint64_t im = wave_incl_scan(xm), ib = wave_incl_scan(xb);
    ex[k] = big ? cbry + ib - xb : cmry + im - xm;
    cmry += rdlane64(im, 63);
    cbry += rdlane64(ib, 63);
    const uint64_t mm = __ballot(large && !big), mb = __ballot(big);
    const uint32_t cx = big ? ccb + (uint32_t)__popcll(mb & lt) : ccm + (uint32_t)__popcll(mm & lt);
    ccm += (uint32_t)__popcll(mm);
    ccb += (uint32_t)__popcll(mb);
    // small: rank among this (wave, k) group's lanes of the same class
    const uint32_t cls = in && !large ? size_class(v[k]) : 63u;
    uint32_t rank = 0;
    if (split) {  // uniform: without a split every buffer is the batch kernel's
      uint64_t match = ~0ull;
#pragma unroll
      for (int bit = 0; bit < 6; bit++) {
        const uint64_t b = __ballot((cls >> bit) & 1u);
        match &= ((cls >> bit) & 1u) ? b : ~b;
      }
      rank = (uint32_t)__popcll(match & lt);
      if (cls < kSizeClasses && rank == 0) s_cls[cls * kGroups + wv * kPer + k] = (uint32_t)__popcll(match);
    }
    meta[k] = cx | (cls << 10) | (rank << 16) | ((uint32_t)big << 22);
  }
  if (lane == 0) s_wb[wv][0] = cmry, s_wb[wv][1] = cbry, s_wc[wv][0] = ccm, s_wc[wv][1] = ccb;
  __syncthreads();
  if (p.stamps) st[3] = __builtin_amdgcn_s_memrealtime();
  uint64_t bom = 0, bob = 0;
  uint32_t com = 0, cob = 0;
  for (uint32_t j = 0; j < wv; j++) bom += s_wb[j][0], bob += s_wb[j][1], com += s_wc[j][0], cob += s_wc[j][1];
  // first position and byte of this wave's medium (or, unsplit, all) and big buffers
  const uint64_t ec = s_tw[3][0];  // earlier tiles' medium | big counts
  const uint64_t bm0 = (split ? s_tw[0][0] : s_tw[0][0] + s_tw[1][0] + s_tw[2][0]) + bom;
  const uint64_t cm0 = (split ? (ec & 0xFFFFFFFFull) : (uint64_t)blockIdx.x * (1024u * kPer)) + com;
  const uint64_t bb0 = am + s_tw[1][0] + bob;
  const uint64_t cb0 = n_med + (ec >> 32) + cob;
  if (split) {
    // exclusive positions over (class, wave, k): thread t scans kEnt consecutive entries
    constexpr uint32_t kEnt = (kSizeClasses * kGroups + 1023) / 1024;
    uint32_t loc[kEnt];
    uint64_t sum = 0;
#pragma unroll
    for (uint32_t e = 0; e < kEnt; e++) {
      const uint32_t i = tid * kEnt + e;
      loc[e] = i < kSizeClasses * kGroups ? s_cls[i] : 0u;
      sum += loc[e];
    }
    uint64_t tot;
    uint64_t run = block_excl_scan(sum, s_tmp, &tot);  // (its barriers order the reads above)
#pragma unroll
    for (uint32_t e = 0; e < kEnt; e++) {
      const uint32_t i = tid * kEnt + e;
      if (i < kSizeClasses * kGroups) s_cls[i] = (uint32_t)run;
      run += loc[e];
    }
    __syncthreads();
  }
  if (p.stamps) st[4] = __builtin_amdgcn_s_memrealtime();
  const uint64_t s0 = s_tw[4][0];  // earlier tiles' small buffers
  if (split) {  // pointers and seeds of the compacted batch and the small list
    const uint8_t *pv[kPer];
    uint32_t sv[kPer];
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
      const uint64_t idx = base + 64u * k;
      const bool in = idx < p.n;
      pv[k] = in ? p.ptrs[idx] : nullptr;
      sv[k] = in && p.seeds ? p.seeds[idx] : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
      const uint64_t idx = base + 64u * k;
      if (idx >= p.n) break;
      const uint32_t cx = meta[k] & 0x3FFu, cls = (meta[k] >> 10) & 63u, rank = (meta[k] >> 16) & 63u;
      const bool big = (meta[k] >> 22) & 1u;
      if (cls == 63u) {  // batch kernel
        const uint64_t j = big ? cb0 + cx : cm0 + cx;
        p.prefix_c[j] = (big ? bb0 : bm0) + ex[k];
        p.ptrs_c[j] = pv[k];
        if (p.seeds) p.seeds_c[j] = sv[k];
        p.oidx[j] = (uint32_t)idx;
        p.out[idx] = 0u;  // split pieces xor into it
      } else {
        // the small list's descriptor: pointer (48-bit VA) | length << 48, index, seed
        const uint64_t pw = reinterpret_cast<uint64_t>(pv[k]) | (v[k] << 48);
        p.sdesc[s0 + s_cls[cls * kGroups + wv * kPer + k] + rank] =
            make_uint4((uint32_t)pw, (uint32_t)(pw >> 32), (uint32_t)idx, sv[k]);
      }
    }
  } else {  // the plain prefix of every buffer, in index order
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
      const uint64_t idx = base + 64u * k;
      if (idx >= p.n) break;
      p.prefix_c[cm0 + (meta[k] & 0x3FFu)] = bm0 + ex[k];
      p.out[idx] = 0u;
    }
  }
  if (p.stamps && tid == 0) {
    __builtin_amdgcn_s_waitcnt(0);
    st[5] = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < 6; i++) p.stamps[8 * blockIdx.x + i] = st[i];
  }
}

template <uint32_t kPer>
hipError_t launch_plan_split_t(const SplitPlan &p, hipStream_t stream) {
  const uint64_t tiles = p.n == 0 ? 1 : (p.n + 1024u * kPer - 1) / (1024u * kPer);
  SplitPlan q = p;
  q.tile_pre = tiles > kPlanDirectTiles ? p.tile_pre : nullptr;
  hipLaunchKernelGGL(plan_split_count<kPer>, dim3((unsigned)tiles), dim3(1024), 0, stream, q);
  if (q.tile_pre) hipLaunchKernelGGL(plan_split_tiles, dim3(1), dim3(1024), 0, stream, q, (uint32_t)tiles);
  hipLaunchKernelGGL(plan_split_scatter<kPer>, dim3((unsigned)tiles), dim3(1024), 0, stream, q);
  return hipGetLastError();
}

hipError_t launch_plan_split(const SplitPlan &p, hipStream_t stream) {
  switch (split_per_thread(p.n)) {
    case 1: return launch_plan_split_t<1>(p, stream);
    case 2: return launch_plan_split_t<2>(p, stream);
    case 4: return launch_plan_split_t<4>(p, stream);
    default: return launch_plan_split_t<8>(p, stream);
  }
}

// ------------------------------------------------------------ launchers

hipError_t launch_batch(const BatchArgs &args, bool strided, int num_cus, hipStream_t stream, hipEvent_t t0,
                        hipEvent_t t1, bool fused, bool ablate) {
  const dim3 grid((unsigned)num_cus), block(kThreads);
  // t0/t1 (profiling): timestamps carried by the dispatch packet itself --
  // event records around the launch add ~11 us of queue bubbles per launch
  if (ablate) {  // the read ceiling (zcrc32_batch_device_read_ceiling): lookups replaced by one VALU op
    if (strided) return hipErrorInvalidValue;
    if (fused)
      hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, 1, true, false, 1, kLoadNt, true, kWindowed, kPerBufForm>),
                            grid, block, 0, stream, t0, t1, 0, args);
    else
      hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, 1>), grid, block, 0, stream, t0, t1, 0, args);
    return hipGetLastError();
  }
  if (fused)
    hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, 0, true, false, 1, kLoadNt, true, kWindowed, kPerBufForm>),
                          grid, block, 0, stream, t0, t1, 0, args);
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
    snprintf(name, sizeof name, "zcrc::crc32_batch_kernel<false, %uu, 0, true, false, 1, %d, false, %s, 4>", kDepth,
             kLoadNt, kWindowed ? "true" : "false");
  });
  return name;
}

// Small whole buffers: 16 lanes per buffer on 256-B blocks with 8 blocks in
// flight, or 8 lanes (twice the buffers: pays below ~2 KiB) on 128-B blocks
// with 8 in flight -- the same 32 VGPRs of loads, one 16-B chunk a lane and
// block, so 4 streams a lane and a 6-step fold instead of the 10 of 256-B
// blocks (round 5: 1 KiB 190.4 -> 183.5 us per GiB batch, 2 KiB 173.3 ->
// 171.9, same process, bit-exact; tools/ceiling_probe, profiles/r05/s15_s20/s18_ceiling_probe.txt).
hipError_t launch_small(const SmallArgs &args, bool strided, int lanes, int num_cus, hipStream_t stream,
                        hipEvent_t t0, hipEvent_t t1) {
  const dim3 grid((unsigned)num_cus), block(kThreads);
  if (strided) {
    if (lanes == 8)
      hipExtLaunchKernelGGL((crc32_small_kernel<true, 8, 8, false, false, 0, 128>), grid, block, 0, stream, t0, t1, 0,
                            args);
    else
      hipExtLaunchKernelGGL((crc32_small_kernel<true, 16, 8>), grid, block, 0, stream, t0, t1, 0, args);
  } else {
    if (lanes == 8)
      hipExtLaunchKernelGGL((crc32_small_kernel<false, 8, 8, false, false, 0, 128>), grid, block, 0, stream, t0, t1, 0,
                            args);
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
    snprintf(name, sizeof name, "zcrc::crc32_batch_kernel<false, %uu, 0, true, false, 1, %d, true, %s, %d>", kDepth,
             kLoadNt, kWindowed ? "true" : "false", kPerBufForm);
  });
  return name;
}

// the general-form small kernels as rocprofv3 names them
const char *small_kernel_name(int lanes) {
  return lanes == 8 ? "zcrc::crc32_small_kernel<false, 8, 8, false, false, 0, 128>"
                    : "zcrc::crc32_small_kernel<false, 16, 8, false, false, 0, 256>";
}

// ------------------------------------------------------- stream-read peak
// Measurement only (zcrc_read_sweep_device): the fastest plain read of a
// contiguous region found on this chip (round 5, tools/ceiling_probe part 3:
// 4-6% above every CRC-compatible wave mapping on config 3's region).  One
// 1024-thread workgroup per CU; each step a workgroup reads one 64 KiB chunk,
// four non-temporal 16-B loads per thread 16 KiB apart, chunks grid-strided.
// The ISA waits for the first load before issuing the other three, so each
// wave has 1-3 KiB in flight.  The workgroup after the last whole chunk reads
// the remaining 16-B granules; a final < 16 B is not read.  The xor of the
// bytes is stored to sink[tid] only if it equals a constant (it never needs
// to: the store keeps the loads alive).
typedef uint32_t sweep_v4u __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(1024) void read_sweep_kernel(const uint8_t *base, uint64_t bytes, uint32_t *sink) {
  typedef const __attribute__((address_space(1))) sweep_v4u *gptr;
  constexpr uint64_t kChunk = 1024u * 64u;
  const uint64_t b0 = reinterpret_cast<uint64_t>(base);
  const uint64_t full = bytes / kChunk;
  uint32_t acc = 0;
  for (uint64_t c = blockIdx.x; c < full; c += gridDim.x) {
    const uint64_t o = c * kChunk + (uint64_t)threadIdx.x * 16u;
    sweep_v4u v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) v[u] = __builtin_nontemporal_load(reinterpret_cast<gptr>(b0 + o + 16384u * u));
#pragma unroll
    for (int u = 0; u < 4; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (blockIdx.x == full % gridDim.x) {
    for (uint64_t o = full * kChunk + (uint64_t)threadIdx.x * 16u; o + 16u <= bytes; o += 1024u * 16u) {
      const sweep_v4u v = __builtin_nontemporal_load(reinterpret_cast<gptr>(b0 + o));
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x5EEDF00Du) sink[threadIdx.x] = acc;
}

hipError_t launch_read_sweep(const void *d_base, uint64_t bytes, uint32_t *d_sink, int num_cus, hipStream_t stream) {
  hipLaunchKernelGGL(read_sweep_kernel, dim3((unsigned)num_cus), dim3(1024), 0, stream,
                     static_cast<const uint8_t *>(d_base), bytes, d_sink);
  return hipGetLastError();
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
