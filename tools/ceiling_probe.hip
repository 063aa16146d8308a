// tools/ceiling_probe.hip -- pure-read ceilings for the shapes the CRC kernel
// is furthest from (VERDICT r4 missing #4, next #4/#5; measurement only).
//
// Part 1, config 2 (4096 x 64 KiB, 16 distinct 256 MiB batches rotated so
// that the 256 MB MALL cannot serve repeats), every kernel one 1024-thread
// workgroup per CU unless noted, nt 16-B loads, two groups of 4 KiB in flight:
//   pb        the per-buffer mapping (wave slot s of workgroup g reads buffer
//             s * grid + g whole), slot priorities as the product
//   grid8     grid-stride sweep, 8 workgroups of 256 per CU (c2_probe's
//             probe-grid)
//   grid16    grid-stride in 1 KiB blocks with the CRC kernel's geometry:
//             wave w of W reads blocks w, w + W, ...
//   wgc       workgroup-cooperative: workgroup g owns buffers g + grid k; its
//             16 waves interleave 1 KiB blocks over them
//   pb-desc   pb with each buffer's address and length loaded from the
//             descriptor arrays (the CRC kernel's), not computed
//   crc       the product's one-launch per-buffer CRC form (kPerBufForm)
//   abl       the product form with its table lookups replaced by one VALU
//             op (kAblate = 1: the bench line's read ceiling); -nt: no table
//             build either; -nd: no table build and no decision at the end;
//             -nl: no decision lengths (the end barriers kept); -nb: -nd
//             without the table barrier; -nf: -nb without the fold
//             (diagnostics: where the product's time over pb goes)
//   crc-18/nl/19/fm/19fm  per-buffer forms (zcrc_batch_kernel.h kPB): 18 =
//             decision after the piece; nl = no decision (right whenever no
//             buffer exceeds 64 KiB); 19 = 18 with the lengths in 16-B buffer
//             loads; fm = the fold's lane levels masked to the lanes read
//             next; results compared with crc's
// (Round-5 sessions 9-13 also measured forms 17 and the slot priorities of
// form 5 in the ablated kernel: profiles/r05/c2_bisect/.)
// Part 2, uniform small buffers (1024, 2048, 3000, 4096, 8192 B; >= 1 GiB
// per batch, two batches rotated), whole buffers in the small body's lane
// mapping (zcrc_small_kernel.h: G lanes per buffer, 256-B blocks, lane l of
// a group reads 16 B x 16/G of every block, kD blocks in flight, the next
// descriptor loaded while the current buffer runs):
//   read-G8/G16  pure reads with the product's descriptor loads
//   read-G8c     the same, 8 lanes, with lane l reading the chunks at 16 l and
//                16 l + 128 (each load covers 128 contiguous bytes per buffer)
//   crc          the product's small kernel (8 lanes on 128-B blocks up to
//                2 KiB, else 16 lanes on 256-B blocks; the split plan's
//                direct mode runs the same body inside the batch kernel)
//   crc-G8c/G16  8 lanes on 256-B blocks (coalesced), 16 lanes; crc-str:
//                the product's form with strided addressing (the strided
//                API); crc-G8cp: G8c with the pipelined walk (small_pipe);
//                results compared with crc's (session 23: the product's
//                forms with a uniform group loop and unconditional loads ran
//                1.8x slower -- the descriptor prefetch's wait moved in front
//                of the group's loads)
// (Round-5 sessions 16-18 also measured the pipelined 16-lane walk, 8 lanes
// on 128-B blocks with 4 blocks in flight, and the bodies without lookups or
// without the fold: profiles/r05/s15_s20/, DESIGN.md 7e.  Session 4 measured G4
// layouts and strided addressing of the pure reads.)
// Every launch is timed by its own dispatch packet (hipExtLaunchKernelGGL
// events); the figures are averages over the launches, in GB/s of payload.
//
//   make -C tools ceiling_probe && tools/ceiling_probe [reps [1: part 1 only | 2: part 2 only | 3: part 3 only]]
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "../zipsfs_amd/csrc/zcrc_batch_kernel.h"
#include "../zipsfs_amd/csrc/zcrc_tables.h"

#define CHECK(x)                                                                               \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));        \
      exit(1);                                                                                 \
    }                                                                                          \
  } while (0)

using namespace zcrc;

namespace {

constexpr uint64_t kN = 4096, kLen = 64u << 10, kBatchBytes = kN * kLen;
constexpr int kBatches = 16;
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t xr(v4u x) { return x[0] ^ x[1] ^ x[2] ^ x[3]; }

__device__ __forceinline__ void slot_prio(uint32_t slot) {
  if (slot >= 12) __builtin_amdgcn_s_setprio(3);
  else if (slot >= 8) __builtin_amdgcn_s_setprio(2);
  else if (slot >= 4) __builtin_amdgcn_s_setprio(1);
}

// blocks [b0, b1) of the buffer behind r, 2 x 4 KiB ping-pong
__device__ __forceinline__ uint32_t read_blocks(__amdgpu_buffer_rsrc_t r, uint32_t b0, uint32_t b1, uint32_t lane) {
  uint32_t acc = 0;
  for (uint32_t b = b0; b < b1; b += 8) {
    v4u v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) v[u] = b + u < b1 ? __builtin_amdgcn_raw_buffer_load_b128(r, 1024u * (b + u) + 16u * lane, 0, 2)
                                                   : (v4u)(0u);
#pragma unroll
    for (int u = 0; u < 8; u++) acc ^= xr(v[u]);
  }
  return acc;
}

__global__ __launch_bounds__(1024) void k_pb(const uint8_t *base, uint32_t *out) {
  const uint32_t lane = threadIdx.x & 63u, slot = threadIdx.x >> 6;
  const uint64_t w = (uint64_t)slot * gridDim.x + blockIdx.x;
  slot_prio(slot);
  if (w >= kN) return;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(base + w * kLen), (short)0, (int)kLen,
                                                                      0x00020000);
  const uint32_t acc = read_blocks(r, 0, 64, lane);
  if (acc == 0x12345678u) out[w] = acc;
}

// k_pb with the buffer's address and length loaded from the batch's
// descriptor arrays (as the CRC kernel does) instead of computed
__global__ __launch_bounds__(1024) void k_pb_desc(const uint64_t *ptrs, const uint64_t *lens, uint32_t *out) {
  const uint32_t lane = threadIdx.x & 63u, slot = threadIdx.x >> 6;
  const uint64_t w = (uint64_t)slot * gridDim.x + blockIdx.x;
  slot_prio(slot);
  if (w >= kN) return;
  const uint64_t p = uni64(ptrs[w]);  // (an int-typed readfirstlane widened with sign extension faulted here)
  const uint32_t len = (uint32_t)uni64(lens[w]);
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)p, (short)0, (int)len, 0x00020000);
  const uint32_t acc = read_blocks(r, 0, len >> 10, lane);
  if (acc == 0x12345678u) out[w] = acc;
}

// Part 3: a grid-stride sweep of `bytes` contiguous bytes with 64-bit
// global addressing (nt 16-B loads, 4 in flight per thread per step)
template <int kThr>
__global__ __launch_bounds__(kThr) void k_sweep(const uint8_t *base, uint64_t bytes, uint32_t *out) {
  typedef const __attribute__((address_space(1))) v4u *gv4u;
  uint32_t acc = 0;
  const uint64_t step = (uint64_t)gridDim.x * kThr * 64;
  for (uint64_t o = ((uint64_t)blockIdx.x * kThr * 4 + threadIdx.x) * 16; o + (uint64_t)(3 * kThr + 1) * 16 <= bytes;
       o += step) {
    v4u v[4];
#pragma unroll
    for (int u = 0; u < 4; u++)
      v[u] = __builtin_nontemporal_load(reinterpret_cast<gv4u>(reinterpret_cast<uint64_t>(base) + o + (uint64_t)u * kThr * 16));
#pragma unroll
    for (int u = 0; u < 4; u++) acc ^= xr(v[u]);
  }
  if (acc == 0x12345678u) out[threadIdx.x] = acc;
}

// Part 3: the sweep's variants -- 1024-thread workgroups, kL loads per
// thread per step; kWaveContig: a wave's kL loads are consecutive KiB (the
// workgroup still covers 16 kL KiB contiguous per step) instead of 16 KiB
// apart; the grid covers #WG x 16 kL KiB per step
template <int kL, bool kWaveContig>
__global__ __launch_bounds__(1024) void k_sweep2(const uint8_t *base, uint64_t bytes, uint32_t *out) {
  typedef const __attribute__((address_space(1))) v4u *gv4u;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint64_t wg_bytes = 16384ull * kL, step = (uint64_t)gridDim.x * wg_bytes;
  const uint64_t b0 = reinterpret_cast<uint64_t>(base);
  uint32_t acc = 0;
  for (uint64_t o = (uint64_t)blockIdx.x * wg_bytes; o + wg_bytes <= bytes; o += step) {
    v4u v[kL];
#pragma unroll
    for (int u = 0; u < kL; u++) {
      const uint64_t blk = kWaveContig ? (uint64_t)wv * kL + u : (uint64_t)u * 16 + wv;  // KiB within the WG's chunk
      v[u] = __builtin_nontemporal_load(reinterpret_cast<gv4u>(b0 + o + 1024 * blk + 16u * lane));
    }
#pragma unroll
    for (int u = 0; u < kL; u++) acc ^= xr(v[u]);
  }
  if (acc == 0x12345678u) out[threadIdx.x] = acc;
}

// Part 3 pure reads in CRC-compatible wave mappings over `bytes`: kPiece ==
// 0: wave w of W reads the contiguous range [w per, (w + 1) per) (the
// product's static ranges); kPiece > 0: wave w reads pieces w, w + W, ...
// of kPiece bytes (all waves in lockstep rows of W pieces).  1 KiB blocks,
// 8 in flight per wave.
template <uint64_t kPiece, int kLd = 8>
__global__ __launch_bounds__(1024) void k_waves(const uint8_t *base, uint64_t bytes, uint32_t *out) {
  typedef const __attribute__((address_space(1))) v4u *gv4u;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint64_t W = (uint64_t)gridDim.x * 16, w = (uint64_t)blockIdx.x * 16 + wv;
  const uint64_t b0 = reinterpret_cast<uint64_t>(base);
  uint32_t acc = 0;
  auto piece = [&](uint64_t off, uint64_t len) {
    for (uint64_t b = 0; b < len; b += 1024 * kLd) {
      v4u v[kLd];
#pragma unroll
      for (int u = 0; u < kLd; u++)
        v[u] = __builtin_nontemporal_load(reinterpret_cast<gv4u>(b0 + off + b + 1024u * u + 16u * lane));
#pragma unroll
      for (int u = 0; u < kLd; u++) acc ^= xr(v[u]);
    }
  };
  if (kPiece == 0) {
    const uint64_t per = (bytes / W) & ~(1024ull * kLd - 1);
    piece(w * per, per);
  } else {
    for (uint64_t p = w; (p + 1) * kPiece <= bytes; p += W) piece(p * kPiece, kPiece);
  }
  if (acc == 0x12345678u) out[threadIdx.x] = acc;
}

// Part 3: workgroup-cooperative ranges: workgroup g of G reads [g per,
// (g + 1) per), its wave w the 1 KiB blocks w, w + 16, w + 32, ... of it
// (kDepth blocks in flight per wave, 16 KiB apart)
template <int kDepthW>
__global__ __launch_bounds__(1024) void k_wgc_range(const uint8_t *base, uint64_t bytes, uint32_t *out) {
  typedef const __attribute__((address_space(1))) v4u *gv4u;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint64_t per = (bytes / gridDim.x) & ~((uint64_t)kDepthW * 16384 - 1);
  const uint64_t b0 = reinterpret_cast<uint64_t>(base) + (uint64_t)blockIdx.x * per + 1024u * wv + 16u * lane;
  uint32_t acc = 0;
  for (uint64_t o = 0; o < per; o += (uint64_t)kDepthW * 16384) {
    v4u v[kDepthW];
#pragma unroll
    for (int u = 0; u < kDepthW; u++) v[u] = __builtin_nontemporal_load(reinterpret_cast<gv4u>(b0 + o + 16384u * u));
#pragma unroll
    for (int u = 0; u < kDepthW; u++) acc ^= xr(v[u]);
  }
  if (acc == 0x12345678u) out[threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void k_grid8(const uint8_t *base, uint32_t *out) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, 0x7FFFFFFF, 0x00020000);
  uint32_t acc = 0;
  const uint64_t step = (uint64_t)gridDim.x * blockDim.x * 16 * 4;
  for (uint64_t o = ((uint64_t)blockIdx.x * blockDim.x * 4 + threadIdx.x) * 16; o < kBatchBytes; o += step) {
    v4u v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) v[u] = __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)(o + (uint64_t)u * blockDim.x * 16), 0, 2);
#pragma unroll
    for (int u = 0; u < 4; u++) acc ^= xr(v[u]);
  }
  if (acc == 0x12345678u) out[threadIdx.x] = acc;
}

__global__ __launch_bounds__(1024) void k_grid16(const uint8_t *base, uint32_t *out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t W = gridDim.x * 16u, w = blockIdx.x * 16u + (threadIdx.x >> 6);
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, 0x7FFFFFFF, 0x00020000);
  const uint32_t nblk = (uint32_t)(kBatchBytes >> 10);
  uint32_t acc = 0;
  for (uint32_t i = w; i < nblk; i += 8 * W) {
    v4u v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const uint32_t blk = i + (uint32_t)u * W;
      v[u] = blk < nblk ? __builtin_amdgcn_raw_buffer_load_b128(r, 1024u * blk + 16u * lane, 0, 2) : (v4u)(0u);
    }
#pragma unroll
    for (int u = 0; u < 8; u++) acc ^= xr(v[u]);
  }
  if (acc == 0x12345678u) out[w] = acc;
}

__global__ __launch_bounds__(1024) void k_wgc(const uint8_t *base, uint32_t *out) {
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, g = blockIdx.x, grid = gridDim.x;
  const uint32_t mine = (uint32_t)((kN - g + grid - 1) / grid);  // buffers g, g + grid, ...
  const uint32_t nblk = mine * 64u;
  uint32_t acc = 0;
  for (uint32_t i = wv; i < nblk; i += 8 * 16) {
    v4u v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const uint32_t j = i + 16u * u;
      if (j < nblk) {
        const uint64_t buf = g + (uint64_t)grid * (j >> 6);
        v[u] = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(base + buf * kLen + 1024u * (j & 63u) + 16u * lane));
      } else {
        v[u] = (v4u)(0u);
      }
    }
#pragma unroll
    for (int u = 0; u < 8; u++) acc ^= xr(v[u]);
  }
  if (acc == 0x12345678u) out[g * 16 + wv] = acc;
}

// Per-CU queue: workgroup g owns buffers g + grid k (k < 16), cut into
// quarters of 16 KiB; wave s reads quarter 0 of its own buffer, then claims
// the other 48 quarters (quarter-major) from an LDS counter -- the waves of a
// CU that the SIMDs serve first take more pieces (within-CU balance, no
// global atomics)
template <uint32_t kParts>
__global__ __launch_bounds__(1024) void k_pb_lds(const uint8_t *base, uint32_t *out) {
  __shared__ uint32_t next;
  const uint32_t lane = threadIdx.x & 63u, slot = threadIdx.x >> 6, g = blockIdx.x, grid = gridDim.x;
  constexpr uint32_t kPart = 64u / kParts;  // blocks per piece
  if (threadIdx.x == 0) next = 16u;
  __syncthreads();
  slot_prio(slot);
  uint32_t acc = 0;
  uint32_t piece = slot;  // piece p: buffer p % 16 of the workgroup, part p / 16
  for (uint32_t guard = 0; guard < 1024; guard++) {
    const uint64_t buf = g + (uint64_t)grid * (piece & 15u);
    const uint32_t part = piece >> 4;
    if (buf < kN) {
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(base + buf * kLen), (short)0,
                                                                          (int)kLen, 0x00020000);
      acc ^= read_blocks(r, kPart * part, kPart * (part + 1), lane);
    }
    uint32_t t = 0;
    if (lane == 0) t = atomicAdd(&next, 1u);
    piece = (uint32_t)__builtin_amdgcn_readfirstlane((int)t);
    if (piece >= 16u * kParts) break;
  }
  if (acc == 0x12345678u) out[g * 16 + slot] = acc;
}

// ---------------------------------------------------------------- part 2

// the small body's mapping (zcrc_small_kernel.h small_body), loads only
template <int G, int kD, bool kDesc, bool kCoal = false>
__global__ __launch_bounds__(1024) void k_small_read(const uint64_t *ptrs, const uint64_t *lens, const uint8_t *base,
                                                     uint64_t stride, uint64_t len, uint64_t n, uint32_t *out) {
  constexpr int C = 16 / G;
  constexpr uint32_t BPW = 64 / G;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, g = lane / G, lg = lane % G;
  const uint64_t waves = (uint64_t)gridDim.x * 16;
  const uint64_t nq = (n + BPW - 1) / BPW;
  uint64_t q = (uint64_t)blockIdx.x * 16 + (tid >> 6);
  auto desc = [&](uint64_t j, uint64_t &p, uint64_t &l) {
    if (kDesc) {
      p = ptrs[j];
      l = lens[j];
    } else {
      p = reinterpret_cast<uint64_t>(base) + j * stride;
      l = len;
    }
  };
  uint64_t nx_p = 0, nx_l = 0;
  if (BPW * q + g < n) desc(BPW * q + g, nx_p, nx_l);
  uint32_t acc = 0;
  for (; q < nq; q += waves) {
    const uint64_t bi = BPW * q + g;
    const bool active = bi < n;
    const uint64_t pstart = nx_p;
    const uint32_t l = active ? (uint32_t)nx_l : 0u;
    if (bi + BPW * waves < n) desc(bi + BPW * waves, nx_p, nx_l);
    const uint64_t astart = pstart & ~(uint64_t)15;
    const int32_t rs = (int32_t)(pstart & 15u), re = rs + (int32_t)l, span = (re + 15) & ~15;
    const uint32_t kq = (active && l) ? (uint32_t)(span + 255) >> 8 : 0u;
    const uint32_t kmax = (uint32_t)__builtin_amdgcn_readfirstlane(__reduce_max_sync(0xFFFFFFFFFFFFFFFFull, kq));
    int32_t rel0 = kq ? span - 256 * (int32_t)kmax + (kCoal ? 16 : 16 * C) * (int32_t)lg : -(1 << 30);
    for (uint32_t k = 0; k < kmax; k += kD) {
      v4u d[kD][C];
#pragma unroll
      for (int b = 0; b < kD; b++)
#pragma unroll
        for (int c = 0; c < C; c++) {
          const int32_t rel = rel0 + 256 * b + (kCoal ? 16 * G : 16) * c;
          d[b][c] = (v4u)(0u);
          if (k + b < kmax && rel >= 0) d[b][c] = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(astart + (uint32_t)rel));
        }
#pragma unroll
      for (int b = 0; b < kD; b++)
#pragma unroll
        for (int c = 0; c < C; c++) acc ^= xr(d[b][c]);
      rel0 += 256 * kD;
    }
  }
  if (acc == 0x12345678u) out[tid] = acc;
}

double pct(std::vector<double> v, double p) {
  std::sort(v.begin(), v.end());
  return v[(size_t)(p * (v.size() - 1))];
}

}  // namespace

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 24;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  static TableBlob tb;
  build_tables(tb);
  TableBlob *d_tab;
  CHECK(hipMalloc(&d_tab, sizeof(TableBlob)));
  CHECK(hipMemcpy(d_tab, &tb, sizeof(TableBlob), hipMemcpyHostToDevice));
  uint32_t *out, *scratch;
  CHECK(hipMalloc(&out, 4u << 20));
  CHECK(hipMalloc(&scratch, 1 << 20));
  CHECK(hipMemset(scratch, 0, 1 << 20));
  std::vector<hipEvent_t> ev(2 * kBatches);  // one pair per batch: a variant's launches go back to back
  for (auto &e : ev) CHECK(hipEventCreate(&e));
  // launch(b, e0, e1) for b < nb back to back on the null stream (each timed by
  // its own dispatch packet, as c2_probe), one synchronize, then the times;
  // progress on stderr: a launch that never ends names itself
  auto timed = [&](const char *name, bool first, int nb, auto launch, std::vector<double> &into) {
    if (first) fprintf(stderr, "  %s ...", name);
    for (int b = 0; b < nb; b++) launch(b, ev[2 * b], ev[2 * b + 1]);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    for (int b = 0; b < nb; b++) {
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, ev[2 * b], ev[2 * b + 1]));
      into.push_back(ms);
      if (first && b == 0) fprintf(stderr, " %.1f us\n", ms * 1e3);
    }
  };

  // ---------------------------------------------------------------- part 1
  if (!(argc > 2 && atoi(argv[2]) >= 2)) {  // (2: part 2 only)
    uint8_t *data;
    CHECK(hipMalloc(&data, kBatchBytes * kBatches));
    std::vector<uint64_t> hp(kN * kBatches), hl(kN * kBatches, kLen);
    for (uint64_t i = 0; i < kN * kBatches; i++) hp[i] = (uint64_t)(data + i * kLen);
    uint64_t *dp, *dl, *dpre;
    CHECK(hipMalloc(&dp, 8 * kN * kBatches));
    CHECK(hipMalloc(&dl, 8 * kN * kBatches));
    CHECK(hipMalloc(&dpre, 8 * (kFusedMaxN + 1)));
    CHECK(hipMemcpy(dp, hp.data(), 8 * kN * kBatches, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dl, hl.data(), 8 * kN * kBatches, hipMemcpyHostToDevice));
    CHECK(launch_fill_synthetic(dp, dl, kN * kBatches, 0, 1, 0xC0FFEE, 0));
    CHECK(hipDeviceSynchronize());
    // v >= 8: per-buffer kernel forms; the real ones (v >= kReal) write their
    // results to ov, compared with crc's below
    const char *names[] = {"pb",     "grid8",  "grid16", "wgc",    "pb-desc", "crc",    "pb-lds4",
                           "pb-lds8", "abl",    "abl-nt", "abl-nd", "abl-nl",  "abl-nb", "abl-nf",
                           "crc-18", "crc-nl", "crc-19", "crc-fm", "crc-19fm"};
    constexpr int kV = 19, kReal = 14;
    uint32_t *ov;
    CHECK(hipMalloc(&ov, (kV - kReal) * 4 * kN));
    std::vector<std::vector<double>> t(kV);
    for (int r = 0; r < reps; r++)
      for (int v = 0; v < kV; v++)
        timed(names[v], r == 0, kBatches, [&](int b, hipEvent_t a, hipEvent_t z) {
          const uint8_t *base = data + (uint64_t)b * kBatchBytes;
          switch (v) {
            case 0: hipExtLaunchKernelGGL(k_pb, dim3(cus), dim3(1024), 0, 0, a, z, 0, base, out); break;
            case 1: hipExtLaunchKernelGGL(k_grid8, dim3(cus * 8), dim3(256), 0, 0, a, z, 0, base, out); break;
            case 2: hipExtLaunchKernelGGL(k_grid16, dim3(cus), dim3(1024), 0, 0, a, z, 0, base, out); break;
            case 3: hipExtLaunchKernelGGL(k_wgc, dim3(cus), dim3(1024), 0, 0, a, z, 0, base, out); break;
            case 4:
              hipExtLaunchKernelGGL(k_pb_desc, dim3(cus), dim3(1024), 0, 0, a, z, 0, dp + (uint64_t)b * kN,
                                    dl + (uint64_t)b * kN, out);
              break;
            case 6: hipExtLaunchKernelGGL(k_pb_lds<4>, dim3(cus), dim3(1024), 0, 0, a, z, 0, base, out); break;
            case 7: hipExtLaunchKernelGGL(k_pb_lds<8>, dim3(cus), dim3(1024), 0, 0, a, z, 0, base, out); break;
            default: {
              BatchArgs x{};
              x.ptrs = reinterpret_cast<const uint8_t *const *>(dp + (uint64_t)b * kN);
              x.lens = dl + (uint64_t)b * kN;
              x.prefix = dpre;
              // the ablated forms' results are not CRCs
              x.out = v >= kReal ? ov + (v - kReal) * kN : v >= 8 ? scratch + 65536 : out;
              x.n = kN;
              x.tab = d_tab;
              x.ctr = scratch + 2048;
              x.done = scratch + 2049;
              x.acc = reinterpret_cast<uint64_t *>(scratch + 4096);
              x.dyn_shift = kDynAuto;
#define ZCRC_PB(abl, form)                                                                                \
  hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, abl, true, false, 1, kLoadNt, true, kWindowed, form>), \
                        dim3(cus), dim3(kThreads), 0, 0, a, z, 0, x)
              switch (v) {
                case 8: ZCRC_PB(1, kPerBufForm); break;
                case 9: ZCRC_PB(1, 1000 + kPerBufForm); break;
                case 10: ZCRC_PB(1, 2000 + kPerBufForm); break;
                case 11: ZCRC_PB(1, 3000 + kPerBufForm); break;
                case 12: ZCRC_PB(1, 4000 + kPerBufForm); break;
                case 13: ZCRC_PB(1, 5000 + kPerBufForm); break;
                case 14: ZCRC_PB(0, 18); break;
                case 15: ZCRC_PB(0, 3000 + kPerBufForm); break;  // right whenever no buffer exceeds kPerBufMax
                case 16: ZCRC_PB(0, 19); break;
                case 17: ZCRC_PB(0, 6000 + kPerBufForm); break;
                case 18: ZCRC_PB(0, 6019); break;
                default: ZCRC_PB(0, kPerBufForm);
              }
#undef ZCRC_PB
            }
          }
        }, t[v]);
    printf("ceiling_probe part 1: config 2 (4096 x 64 KiB), %d CUs, %d batches rotated, %d reps\n", cus, kBatches,
           reps);
    for (int v = 0; v < kV; v++) {
      double sum = 0;
      for (double x : t[v]) sum += x;
      const double avg = sum / t[v].size();
      printf("  %-8s avg %7.2f us  p10 %7.2f  p50 %7.2f  %7.1f GB/s (avg)\n", names[v], avg * 1e3, pct(t[v], 0.1) * 1e3,
             pct(t[v], 0.5) * 1e3, kBatchBytes / (avg * 1e-3) / 1e9);
    }
    {  // the real forms against crc (all ran batch 15 last)
      std::vector<uint32_t> h0(kN), h1((kV - kReal) * kN);
      CHECK(hipMemcpy(h0.data(), out, 4 * kN, hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(h1.data(), ov, (kV - kReal) * 4 * kN, hipMemcpyDeviceToHost));
      for (int k = 0; k < kV - kReal; k++) {
        uint64_t bad = 0;
        for (uint64_t i = 0; i < kN; i++) bad += h0[i] != h1[k * kN + i];
        printf("  %s results: %s (%llu of %llu differ from crc)\n", names[kReal + k], bad ? "DIFFER" : "equal",
               (unsigned long long)bad, (unsigned long long)kN);
      }
    }
    fflush(stdout);
    CHECK(hipFree(ov));
    CHECK(hipFree(data));
    CHECK(hipFree(dp));
    CHECK(hipFree(dl));
    CHECK(hipFree(dpre));
  }

  // ---------------------------------------------------------------- part 3
  // (3: part 3 only) the sustained read of config 3's and config 4's payload
  // regions as one contiguous sweep -- the bound for any mapping of their
  // buffers (config 4: the bench's layout, 16-B aligned bounded power law)
  if (argc > 2 && atoi(argv[2]) == 3) {
    const uint64_t c3 = 65536ull << 20;
    uint64_t c4 = 0;
    {
      // bench.py zipf_lens: the same mix64 hash and bounded power law
      for (uint64_t i = 0; i < 100000; i++) {
        uint64_t z = 0x5A1F5EEDull ^ ((i + 1) * 0xD1B54A32D192ED03ull);
        z += 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        const double u = (double)(z >> 11) * (1.0 / 9007199254740992.0);
        const double t = 1.0 - u * 127.0 / 128.0;
        double L = 1024.0 / (t * t);
        L = L < 1024 ? 1024 : (L > (1 << 24) ? (1 << 24) : L);
        c4 += ((uint64_t)L + 15) & ~15ull;
      }
    }
    uint8_t *mem;
    CHECK(hipMalloc(&mem, c3));
    CHECK(hipMemset(mem, 1, c3));
    CHECK(hipDeviceSynchronize());
    // crc-c3 / abl-c3: the product's batch kernel on config 3 in its strided
    // form (65,536 x 1 MiB; static ranges per wave, then dynamic units) and
    // its read-ceiling form, launched as zcrc32_batch_device_strided does
    const char *nm[] = {"sweep8-c3", "sweep16-c3", "sweep8-c4", "sweep16-c4", "crc-c3",  "abl-c3",
                        "range-c3",  "range2-c3",  "range4-c3", "crc-d2-c3",  "abl-d2-c3"};
    constexpr int kV3 = 11;
    uint32_t *o3;
    CHECK(hipMalloc(&o3, 4 * 65536));
    std::vector<std::vector<double>> t(kV3);
    for (int r = 0; r < reps; r++)
      for (int v = 0; v < kV3; v++) {
        if (v == 4 || v == 5 || v >= 9) {
          CHECK(hipMemsetAsync(o3, 0, 4 * 65536, 0));
          CHECK(hipMemsetAsync(scratch + 2048, 0, 64, 0));
        }
        timed(nm[v], r == 0, 1, [&](int, hipEvent_t a, hipEvent_t z) {
          const uint64_t bytes = v < 2 ? c3 : c4;
          const uint8_t *base = v < 2 ? mem : mem + (r & 1) * (c3 / 2);  // config 4: two distinct regions
          if (v == 4 || v == 5 || v >= 9) {
            BatchArgs x{};
            x.base = mem;
            x.stride = 1u << 20;
            x.len = 1u << 20;
            x.n = 65536;
            x.out = o3;
            x.tab = d_tab;
            x.ctr = scratch + 2048;
            x.dyn_shift = kDynAuto;
            if (v == 4)
              hipExtLaunchKernelGGL((crc32_batch_kernel<true, kDepth, 0>), dim3(cus), dim3(kThreads), 0, 0, a, z, 0, x);
            else if (v == 5)
              hipExtLaunchKernelGGL((crc32_batch_kernel<true, kDepth, 1>), dim3(cus), dim3(kThreads), 0, 0, a, z, 0, x);
            else if (v == 9)
              hipExtLaunchKernelGGL((crc32_batch_kernel<true, 2, 0>), dim3(cus), dim3(kThreads), 0, 0, a, z, 0, x);
            else
              hipExtLaunchKernelGGL((crc32_batch_kernel<true, 2, 1>), dim3(cus), dim3(kThreads), 0, 0, a, z, 0, x);
          } else if (v >= 6 && v <= 8) {
            switch (v) {
              case 6: hipExtLaunchKernelGGL((k_waves<0>), dim3(cus), dim3(1024), 0, 0, a, z, 0, mem, c3, out); break;
              case 7: hipExtLaunchKernelGGL((k_waves<0, 2>), dim3(cus), dim3(1024), 0, 0, a, z, 0, mem, c3, out); break;
              case 8: hipExtLaunchKernelGGL((k_waves<0, 4>), dim3(cus), dim3(1024), 0, 0, a, z, 0, mem, c3, out); break;
            }
          } else if (v % 2 == 0) {
            hipExtLaunchKernelGGL((k_sweep<256>), dim3(cus * 8), dim3(256), 0, 0, a, z, 0, base, bytes, out);
          } else {
            hipExtLaunchKernelGGL((k_sweep<1024>), dim3(cus), dim3(1024), 0, 0, a, z, 0, base, bytes, out);
          }
        }, t[v]);
      }
    printf("ceiling_probe part 3: contiguous sweeps, config 3 (%llu B) and config 4 (%llu B) regions, %d reps\n",
           (unsigned long long)c3, (unsigned long long)c4, reps);
    for (int v = 0; v < kV3; v++) {
      double sum = 0;
      for (double x : t[v]) sum += x;
      const double avg = sum / t[v].size();
      const uint64_t bytes = v == 2 || v == 3 ? c4 : c3;
      printf("  %-10s avg %9.3f ms  %7.1f GB/s (avg)  %7.1f GB/s (best)\n", nm[v], avg, bytes / (avg * 1e-3) / 1e9,
             bytes / (pct(t[v], 0) * 1e-3) / 1e9);
    }
    CHECK(hipFree(mem));
    CHECK(hipFree(o3));
    return 0;
  }

  // ---------------------------------------------------------------- part 2
  if (argc > 2 && atoi(argv[2]) == 1) return 0;  // part 1 only
  const uint64_t sizes[] = {1024, 2048, 3000, 4096, 8192};
  fprintf(stderr, "part 2\n");
  printf("ceiling_probe part 2: uniform small buffers, 2 batches of >= 1 GiB rotated, %d reps\n", reps);
  for (uint64_t L : sizes) {
    const uint64_t stride = (L + 15) & ~15ull;
    const uint64_t n = (1ull << 30) / L;
    uint8_t *data;
    CHECK(hipMalloc(&data, 2 * n * stride + 256));
    uint64_t *dp, *dl;
    uint32_t *o1, *o2;  // "crc" and the other CRC forms (compared below)
    CHECK(hipMalloc(&dp, 16 * n));
    CHECK(hipMalloc(&dl, 16 * n));
    CHECK(hipMalloc(&o1, 4 * n));
    CHECK(hipMalloc(&o2, 4 * n));
    std::vector<uint64_t> hp(2 * n), hl(2 * n, L);
    for (uint64_t i = 0; i < 2 * n; i++) hp[i] = (uint64_t)(data + i * stride);
    CHECK(hipMemcpy(dp, hp.data(), 16 * n, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dl, hl.data(), 16 * n, hipMemcpyHostToDevice));
    CHECK(launch_fill_synthetic(dp, dl, 2 * n, 0, 1, 0xC0FFEE, 0));
    CHECK(hipDeviceSynchronize());
    const char *names[] = {"read-G8", "read-G16", "read-G8c", "crc", "crc-G8c", "crc-G16", "crc-str", "crc-G8cp"};
    constexpr int kV = 8, kCmp = 8;  // forms below kCmp: results compared with crc's
    std::vector<std::vector<double>> t(kV);
    const int lanes = L <= 2048 ? 8 : 16;  // the product's choice (small_lanes)
    auto crc_launch = [&](int v, const uint64_t *p, const uint64_t *l, const uint8_t *base, uint32_t *o, hipEvent_t a,
                          hipEvent_t z) {
      SmallArgs sa{};
      sa.ptrs = reinterpret_cast<const uint8_t *const *>(p);
      sa.lens = l;
      sa.n = n;
      sa.tab = d_tab;
      sa.out = o;
      // 3 ("crc"): the product's form (8 lanes on 128-B blocks up to 2 KiB,
      // else 16 on 256-B blocks); 4: 8 lanes on 256-B blocks, coalesced; 5:
      // 16 lanes; 6: the product's form, strided addressing; 7: 4 with the
      // pipelined walk
      if (v == 6) {
        sa.base = base;
        sa.stride = stride;
        sa.len = L;
        if (lanes == 8)
          hipExtLaunchKernelGGL((crc32_small_kernel<true, 8, 8, false, false, 0, 128>), dim3(cus), dim3(1024), 0, 0, a,
                                z, 0, sa);
        else
          hipExtLaunchKernelGGL((crc32_small_kernel<true, 16, 8>), dim3(cus), dim3(1024), 0, 0, a, z, 0, sa);
        return;
      }
      const int form = v == 3 ? (lanes == 8 ? 10 : 5) : v;
      if (form == 4)
        hipExtLaunchKernelGGL((crc32_small_kernel<false, 8, 4, true>), dim3(cus), dim3(1024), 0, 0, a, z, 0, sa);
      else if (form == 5)
        hipExtLaunchKernelGGL((crc32_small_kernel<false, 16, 8>), dim3(cus), dim3(1024), 0, 0, a, z, 0, sa);
      else if (form == 7)
        hipExtLaunchKernelGGL((crc32_small_kernel<false, 8, 4, true, true>), dim3(cus), dim3(1024), 0, 0, a, z, 0, sa);
      else
        hipExtLaunchKernelGGL((crc32_small_kernel<false, 8, 8, false, false, 0, 128>), dim3(cus), dim3(1024), 0, 0, a,
                              z, 0, sa);
    };
    for (int r = 0; r < reps; r++)
      for (int v = 0; v < kV; v++)
        timed(names[v], r == 0, 2, [&](int b, hipEvent_t a, hipEvent_t z) {
          const uint64_t *p = dp + (uint64_t)b * n, *l = dl + (uint64_t)b * n;
          const uint8_t *base = data + (uint64_t)b * n * stride;
          switch (v) {
            case 0: hipExtLaunchKernelGGL((k_small_read<8, 4, true>), dim3(cus), dim3(1024), 0, 0, a, z, 0, p, l, base, stride, L, n, out); break;
            case 1: hipExtLaunchKernelGGL((k_small_read<16, 8, true>), dim3(cus), dim3(1024), 0, 0, a, z, 0, p, l, base, stride, L, n, out); break;
            case 2: hipExtLaunchKernelGGL((k_small_read<8, 4, true, true>), dim3(cus), dim3(1024), 0, 0, a, z, 0, p, l, base, stride, L, n, out); break;
            default: crc_launch(v, p, l, base, v == 3 ? o1 : o2, a, z);
          }
        }, t[v]);
    printf("  L %5llu  n %8llu per batch\n", (unsigned long long)L, (unsigned long long)n);
    for (int v = 0; v < kV; v++) {
      double sum = 0;
      for (double x : t[v]) sum += x;
      const double avg = sum / t[v].size();
      printf("    %-9s avg %8.2f us  %7.1f GB/s (avg)  %7.1f GB/s (best)\n", names[v], avg * 1e3,
             n * L / (avg * 1e-3) / 1e9, n * L / (pct(t[v], 0) * 1e-3) / 1e9);
    }
    {  // every CRC form against "crc" (whose last launch ran batch 1), on batch 1
      std::vector<uint32_t> h1(n), h2(n);
      CHECK(hipMemcpy(h1.data(), o1, 4 * n, hipMemcpyDeviceToHost));
      for (int v = 4; v < kCmp; v++) {
        CHECK(hipMemset(o2, 0, 4 * n));
        crc_launch(v, dp + n, dl + n, data + n * stride, o2, ev[0], ev[1]);
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemcpy(h2.data(), o2, 4 * n, hipMemcpyDeviceToHost));
        uint64_t bad = 0;
        for (uint64_t i = 0; i < n; i++) bad += h1[i] != h2[i];
        printf("    %s results: %s (%llu of %llu differ from crc)\n", names[v], bad ? "DIFFER" : "equal",
               (unsigned long long)bad, (unsigned long long)n);
      }
    }
    fflush(stdout);
    CHECK(hipFree(data));
    CHECK(hipFree(dp));
    CHECK(hipFree(dl));
    CHECK(hipFree(o1));
    CHECK(hipFree(o2));
  }
  return 0;
}
