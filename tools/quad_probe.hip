// tools/quad_probe.hip -- prototype of a separate small-buffer kernel
// (measurement only): four whole buffers per wave, one per 16-lane quarter,
// on the batch kernel's braided table.  Compares it with the product kernel
// on uniform batches of small buffers (2 x 1 GiB rotated) and checks that
// both give the same CRCs.
//
// Lane l of quarter g reads the 16-B chunks at 256 j + 16 l (j < 4) of every
// 1 KiB block of buffer g, so each of its 16 dword streams advances exactly
// 1 KiB per block and MCT(x^(8*1024)) serves it; the fold is 15 in-lane and
// 4 cross-lane levels for four buffers.  All four are aligned to their own
// 16-B-aligned ends and run max(K) blocks (blocks before a shorter buffer's
// start load nothing: leading zeros are free in the raw domain).
//
//   make -C tools quad_probe && tools/quad_probe [reps]
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

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

struct QuadArgs {
  const uint64_t *ptrs;
  const uint64_t *lens;  // every length in [4, 16 KiB]
  uint32_t *out;
  uint64_t n;
  const TableBlob *tab;
};

__device__ __forceinline__ uint64_t pick4(uint32_t g, uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
  return g == 0 ? a : (g == 1 ? b : (g == 2 ? c : d));
}

template <int kMaxK>
__global__ __launch_bounds__(1024) void quad_kernel(QuadArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t s_lds[kLdsBytes / 4];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, g = lane >> 4, l16 = lane & 15u;
  {  // LDS tables, as the batch kernel fills them
    uint4 *dst = reinterpret_cast<uint4 *>(s_lds);
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t o = 16u * (tid + 1024u * k);
      const uint32_t v = a.tab->braid[(((o >> 16) << 1) | ((o >> 7) & 1u)) * 256u + ((o >> 8) & 255u)];
      dst[tid + 1024u * k] = make_uint4(v, v, v, v);
    }
    const uint4 *cs = reinterpret_cast<const uint4 *>(a.tab->comb);
    uint4 *cd = reinterpret_cast<uint4 *>(s_lds + kLdsCombDword);
    cd[tid] = cs[tid];
    cd[tid + 1024u] = cs[tid + 1024u];
  }
  __syncthreads();
  const uint32_t lo0 = (lane & 31u) * 4u;
  const uint32_t o0 = lo0, o1 = lo0 + 128u, o2 = lo0 + 65536u, o3 = lo0 + 65536u + 128u;
  const uint64_t waves = (uint64_t)gridDim.x * 16u;
  const uint64_t nq = (a.n + 3) / 4;
  for (uint64_t q = (uint64_t)blockIdx.x * 16u + (tid >> 6); q < nq; q += waves) {
    const uint64_t bi = 4 * q + g;
    const bool active = bi < a.n;
    const uint64_t pstart = active ? a.ptrs[bi] : 0;
    const uint32_t len = active ? (uint32_t)a.lens[bi] : 0u;
    const uint64_t astart = pstart & ~(uint64_t)15;
    const int32_t rs = (int32_t)(pstart & 15u), re = rs + (int32_t)len, span = (re + 15) & ~15;
    const uint32_t inj = 0xFFFFFFFFu;  // seed 0
    const uint32_t kq = active ? (uint32_t)(span + 1023) >> 10 : 0u;
    const uint32_t kmax = __reduce_max_sync(0xFFFFFFFFFFFFFFFFull, kq);
    uint32_t s[16];
#pragma unroll
    for (int t = 0; t < 16; t++) s[t] = 0u;
    int32_t rel0 = active ? span - 1024 * (int32_t)kmax + 16 * (int32_t)l16 : -(1 << 30);
    for (uint32_t k = 0; k < kmax; k++, rel0 += 1024) {
      v4u d[4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int32_t rel = rel0 + 256 * j;
        d[j] = (v4u)(0u);
        if (rel >= 0) d[j] = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(astart + (uint32_t)rel));
      }
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int32_t rel = rel0 + 256 * j;
        uint4 w = make_uint4(d[j].x, d[j].y, d[j].z, d[j].w);
        if (rel >= 0 && (rel < rs + 4 || rel + 16 > re))
          w = fix_chunk(w, clamp_rel(rs - rel), clamp_rel(re - rel), clamp_rel(rs - rel), inj);
        s[4 * j + 0] = braid_step(s_lds, s[4 * j + 0] ^ w.x, o0, o1, o2, o3);
        s[4 * j + 1] = braid_step(s_lds, s[4 * j + 1] ^ w.y, o0, o1, o2, o3);
        s[4 * j + 2] = braid_step(s_lds, s[4 * j + 2] ^ w.z, o0, o1, o2, o3);
        s[4 * j + 3] = braid_step(s_lds, s[4 * j + 3] ^ w.w, o0, o1, o2, o3);
      }
    }
    // fold: stream (l16, j, q) sits at aend + 256 j + 16 l16 + 4 q
    uint32_t rj[4];
#pragma unroll
    for (int j = 0; j < 4; j++)
      rj[j] = (s[4 * j] ^ comb_apply(s_lds, 0, s[4 * j + 1])) ^
              comb_apply(s_lds, 1, s[4 * j + 2] ^ comb_apply(s_lds, 0, s[4 * j + 3]));
    uint32_t r = (rj[0] ^ comb_apply(s_lds, 6, rj[1])) ^ comb_apply(s_lds, 7, rj[2] ^ comb_apply(s_lds, 6, rj[3]));
#pragma unroll
    for (int j = 0; j < 4; j++) r ^= __shfl_down(comb_apply(s_lds, 2 + j, r), 1u << j, 64);
    const uint32_t tpad = (uint32_t)(span - re), a4 = tpad >> 2;
    if (a4 & 2u) r = comb_apply(s_lds, 1, r);
    if (a4 & 1u) r = comb_apply(s_lds, 0, r);
    const uint32_t nbits = 8u * (tpad & 3u);
    for (uint32_t b = 0; b < 24u; b++)
      if (b < nbits) r = gf2_times_xinv(r);
    if (active && l16 == 0) a.out[bi] = ~r;
  }
}

// 256-B blocks: lane l of quarter g reads the 16-B chunk at 16 l of every
// 256-B block of buffer g; its 4 dword streams advance 256 B per block, so the
// braided table is MCT(x^(8*256)) (a.b256, same LDS layout as the batch
// kernel's) and the fold is 3 in-lane + 4 cross-lane combines (combs 0..5).
// Loads of up to kD blocks are in flight before their braid steps.
template <int kD, bool kPf, bool kAbl = false>
__global__ __launch_bounds__(1024) void quad256_kernel(QuadArgs a, const uint32_t *b256) {
  __shared__ __attribute__((aligned(16))) uint32_t s_lds[kLdsBytes / 4];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, g = lane >> 4, l16 = lane & 15u;
  {
    uint4 *dst = reinterpret_cast<uint4 *>(s_lds);
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t o = 16u * (tid + 1024u * k);
      const uint32_t v = b256[(((o >> 16) << 1) | ((o >> 7) & 1u)) * 256u + ((o >> 8) & 255u)];
      dst[tid + 1024u * k] = make_uint4(v, v, v, v);
    }
    const uint4 *cs = reinterpret_cast<const uint4 *>(a.tab->comb);
    uint4 *cd = reinterpret_cast<uint4 *>(s_lds + kLdsCombDword);
    cd[tid] = cs[tid];
    cd[tid + 1024u] = cs[tid + 1024u];
  }
  __syncthreads();
  const uint32_t lo0 = (lane & 31u) * 4u;
  const uint32_t o0 = lo0, o1 = lo0 + 128u, o2 = lo0 + 65536u, o3 = lo0 + 65536u + 128u;
  const uint64_t waves = (uint64_t)gridDim.x * 16u;
  const uint64_t nq = (a.n + 3) / 4;
  uint64_t q = (uint64_t)blockIdx.x * 16u + (tid >> 6);
  uint64_t nx_p = 0, nx_l = 0;
  if (kPf && 4 * q + g < a.n) nx_p = a.ptrs[4 * q + g], nx_l = a.lens[4 * q + g];
  for (; q < nq; q += waves) {
    const uint64_t bi = 4 * q + g;
    const bool active = bi < a.n;
    uint64_t pstart, len64;
    if (kPf) {
      pstart = nx_p, len64 = nx_l;
      const uint64_t bn = bi + 4 * waves;
      if (bn < a.n) nx_p = a.ptrs[bn], nx_l = a.lens[bn];
    } else {
      pstart = active ? a.ptrs[bi] : 0;
      len64 = active ? a.lens[bi] : 0;
    }
    const uint32_t len = active ? (uint32_t)len64 : 0u;
    const uint64_t astart = pstart & ~(uint64_t)15;
    const int32_t rs = (int32_t)(pstart & 15u), re = rs + (int32_t)len, span = (re + 15) & ~15;
    const uint32_t inj = 0xFFFFFFFFu;
    const uint32_t kq = active ? (uint32_t)(span + 255) >> 8 : 0u;
    const uint32_t kmax = __reduce_max_sync(0xFFFFFFFFFFFFFFFFull, kq);
    uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    int32_t rel0 = active ? span - 256 * (int32_t)kmax + 16 * (int32_t)l16 : -(1 << 30);
    for (uint32_t k = 0; k < kmax; k += kD) {
      v4u d[kD];
#pragma unroll
      for (int j = 0; j < kD; j++) {
        const int32_t rel = rel0 + 256 * j;
        d[j] = (v4u)(0u);
        if (k + j < kmax && rel >= 0)
          d[j] = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(astart + (uint32_t)rel));
      }
#pragma unroll
      for (int j = 0; j < kD; j++) {
        if (k + j < kmax) {
          const int32_t rel = rel0 + 256 * j;
          uint4 w = make_uint4(d[j].x, d[j].y, d[j].z, d[j].w);
          if (rel >= 0 && (rel < rs + 4 || rel + 16 > re))
            w = fix_chunk(w, clamp_rel(rs - rel), clamp_rel(re - rel), clamp_rel(rs - rel), inj);
          if (kAbl) {
            s0 = __builtin_amdgcn_alignbit(s0 ^ w.x, s0 ^ w.x, 5), s1 = __builtin_amdgcn_alignbit(s1 ^ w.y, s1, 3);
            s2 ^= w.z, s3 ^= w.w;
          } else {
            s0 = braid_step(s_lds, s0 ^ w.x, o0, o1, o2, o3);
            s1 = braid_step(s_lds, s1 ^ w.y, o0, o1, o2, o3);
            s2 = braid_step(s_lds, s2 ^ w.z, o0, o1, o2, o3);
            s3 = braid_step(s_lds, s3 ^ w.w, o0, o1, o2, o3);
          }
        }
      }
      rel0 += 256 * kD;
    }
    uint32_t r;
    if (kAbl) {
      r = s0 ^ s1 ^ s2 ^ s3;
#pragma unroll
      for (int j = 0; j < 4; j++) r ^= __shfl_down(r, 1u << j, 64);
    } else {
      r = (s0 ^ comb_apply(s_lds, 0, s1)) ^ comb_apply(s_lds, 1, s2 ^ comb_apply(s_lds, 0, s3));
#pragma unroll
      for (int j = 0; j < 4; j++) r ^= __shfl_down(comb_apply(s_lds, 2 + j, r), 1u << j, 64);
    }
    const uint32_t tpad = (uint32_t)(span - re), a4 = tpad >> 2;
    if (a4 & 2u) r = comb_apply(s_lds, 1, r);
    if (a4 & 1u) r = comb_apply(s_lds, 0, r);
    const uint32_t nbits = 8u * (tpad & 3u);
    for (uint32_t b = 0; b < 24u; b++)
      if (b < nbits) r = gf2_times_xinv(r);
    if (active && l16 == 0) a.out[bi] = ~r;
  }
}

// G lanes per buffer (64/G buffers per wave), 256-B blocks: lane l of a group
// reads C = 16/G consecutive 16-B chunks at 16 C l of every block, so each of
// its 4C dword streams advances 256 B per block (MCT(x^2048)).  In-lane fold
// over 4C dwords (combs 0..log2(4C)-1), cross-lane over G lanes (the next
// log2(G) combs): 16 C lanes-stride .. 128 B.
template <int G, int kD>
__global__ __launch_bounds__(1024) void group_kernel(QuadArgs a, const uint32_t *b256) {
  constexpr int C = 16 / G, NS = 4 * C, LOG_NS = NS == 4 ? 2 : (NS == 8 ? 3 : 4), LOG_G = G == 4 ? 2 : (G == 8 ? 3 : 4);
  constexpr uint32_t BPW = 64 / G;
  __shared__ __attribute__((aligned(16))) uint32_t s_lds[kLdsBytes / 4];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, g = lane / G, lg = lane % G;
  {
    uint4 *dst = reinterpret_cast<uint4 *>(s_lds);
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t o = 16u * (tid + 1024u * k);
      const uint32_t v = b256[(((o >> 16) << 1) | ((o >> 7) & 1u)) * 256u + ((o >> 8) & 255u)];
      dst[tid + 1024u * k] = make_uint4(v, v, v, v);
    }
    const uint4 *cs = reinterpret_cast<const uint4 *>(a.tab->comb);
    uint4 *cd = reinterpret_cast<uint4 *>(s_lds + kLdsCombDword);
    cd[tid] = cs[tid];
    cd[tid + 1024u] = cs[tid + 1024u];
  }
  __syncthreads();
  const uint32_t lo0 = (lane & 31u) * 4u;
  const uint32_t o0 = lo0, o1 = lo0 + 128u, o2 = lo0 + 65536u, o3 = lo0 + 65536u + 128u;
  const uint64_t waves = (uint64_t)gridDim.x * 16u;
  const uint64_t nq = (a.n + BPW - 1) / BPW;
  uint64_t q = (uint64_t)blockIdx.x * 16u + (tid >> 6);
  uint64_t nx_p = 0, nx_l = 0;
  if (BPW * q + g < a.n) nx_p = a.ptrs[BPW * q + g], nx_l = a.lens[BPW * q + g];
  for (; q < nq; q += waves) {
    const uint64_t bi = BPW * q + g;
    const bool active = bi < a.n;
    const uint64_t pstart = nx_p;
    const uint32_t len = active ? (uint32_t)nx_l : 0u;
    {
      const uint64_t bn = bi + BPW * waves;
      if (bn < a.n) nx_p = a.ptrs[bn], nx_l = a.lens[bn];
    }
    const uint64_t astart = pstart & ~(uint64_t)15;
    const int32_t rs = (int32_t)(pstart & 15u), re = rs + (int32_t)len, span = (re + 15) & ~15;
    const uint32_t inj = 0xFFFFFFFFu;
    const uint32_t kq = active ? (uint32_t)(span + 255) >> 8 : 0u;
    const uint32_t kmax = __reduce_max_sync(0xFFFFFFFFFFFFFFFFull, kq);
    uint32_t s[NS];
#pragma unroll
    for (int t = 0; t < NS; t++) s[t] = 0u;
    int32_t rel0 = active ? span - 256 * (int32_t)kmax + 16 * C * (int32_t)lg : -(1 << 30);
    for (uint32_t k = 0; k < kmax; k += kD) {
      v4u d[kD][C];
#pragma unroll
      for (int j = 0; j < kD; j++)
#pragma unroll
        for (int c = 0; c < C; c++) {
          const int32_t rel = rel0 + 256 * j + 16 * c;
          d[j][c] = (v4u)(0u);
          if (k + j < kmax && rel >= 0)
            d[j][c] = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(astart + (uint32_t)rel));
        }
#pragma unroll
      for (int j = 0; j < kD; j++) {
        if (k + j < kmax) {
#pragma unroll
          for (int c = 0; c < C; c++) {
            const int32_t rel = rel0 + 256 * j + 16 * c;
            uint4 w = make_uint4(d[j][c].x, d[j][c].y, d[j][c].z, d[j][c].w);
            if (rel >= 0 && (rel < rs + 4 || rel + 16 > re))
              w = fix_chunk(w, clamp_rel(rs - rel), clamp_rel(re - rel), clamp_rel(rs - rel), inj);
            s[4 * c + 0] = braid_step(s_lds, s[4 * c + 0] ^ w.x, o0, o1, o2, o3);
            s[4 * c + 1] = braid_step(s_lds, s[4 * c + 1] ^ w.y, o0, o1, o2, o3);
            s[4 * c + 2] = braid_step(s_lds, s[4 * c + 2] ^ w.z, o0, o1, o2, o3);
            s[4 * c + 3] = braid_step(s_lds, s[4 * c + 3] ^ w.w, o0, o1, o2, o3);
          }
        }
      }
      rel0 += 256 * kD;
    }
#pragma unroll
    for (int t = 0; t < LOG_NS; t++)
#pragma unroll
      for (int m = 0; m < NS; m += 2 << t) s[m] ^= comb_apply(s_lds, t, s[m + (1 << t)]);
    uint32_t r = s[0];
#pragma unroll
    for (int j = 0; j < LOG_G; j++) r ^= __shfl_down(comb_apply(s_lds, LOG_NS + j, r), 1u << j, 64);
    const uint32_t tpad = (uint32_t)(span - re), a4 = tpad >> 2;
    if (a4 & 2u) r = comb_apply(s_lds, 1, r);
    if (a4 & 1u) r = comb_apply(s_lds, 0, r);
    const uint32_t nbits = 8u * (tpad & 3u);
    for (uint32_t b = 0; b < 24u; b++)
      if (b < nbits) r = gf2_times_xinv(r);
    if (active && lg == 0) a.out[bi] = ~r;
  }
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  static TableBlob tb;
  build_tables(tb);
  TableBlob *d_tab;
  CHECK(hipMalloc(&d_tab, sizeof(TableBlob)));
  CHECK(hipMemcpy(d_tab, &tb, sizeof(TableBlob), hipMemcpyHostToDevice));
  static uint32_t h256[4 * 256];
  {
    XPowTable xp;
    build_xpow_table(xp);
    build_mct(gf2_xpow8(xp, 256), h256);
  }
  uint32_t *d256;
  CHECK(hipMalloc(&d256, sizeof h256));
  CHECK(hipMemcpy(d256, h256, sizeof h256, hipMemcpyHostToDevice));
  uint32_t *d_ctr;
  CHECK(hipMalloc(&d_ctr, 256));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  printf("quad_probe: %d CUs, %d reps\n", cus, reps);
  for (uint64_t L : {1024ull, 3000ull, 4096ull, 8192ull, 16384ull}) {
    const uint64_t n = (1ull << 30) / L;
    uint8_t *data[2];
    uint64_t *dp[2], *dl, *dpre;
    uint32_t *o1, *o2;
    std::vector<uint64_t> lens(n, L), pre(n + 1, 0);
    for (uint64_t i = 0; i < n; i++) pre[i + 1] = pre[i] + L;
    const uint64_t stride = (L + 15) & ~15ull;
    CHECK(hipMalloc(&dl, 8 * n));
    CHECK(hipMalloc(&dpre, 8 * (n + 1)));
    CHECK(hipMalloc(&o1, 4 * n));
    CHECK(hipMalloc(&o2, 4 * n));
    CHECK(hipMemcpy(dl, lens.data(), 8 * n, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dpre, pre.data(), 8 * (n + 1), hipMemcpyHostToDevice));
    for (int b = 0; b < 2; b++) {
      CHECK(hipMalloc(&data[b], n * stride + 64));
      std::vector<uint64_t> hp(n);
      for (uint64_t i = 0; i < n; i++) hp[i] = (uint64_t)(data[b] + i * stride + (i % 7));
      CHECK(hipMalloc(&dp[b], 8 * n));
      CHECK(hipMemcpy(dp[b], hp.data(), 8 * n, hipMemcpyHostToDevice));
      CHECK(launch_fill_synthetic(dp[b], dl, n, 11 * b, 1, 0xC0FFEE, 0));
    }
    CHECK(hipDeviceSynchronize());
    auto run_main = [&](int b, uint32_t *o, bool timed) -> float {
      BatchArgs a{};
      a.ptrs = reinterpret_cast<const uint8_t *const *>(dp[b]);
      a.prefix = dpre;
      a.out = o;
      a.n = n;
      a.tab = d_tab;
      a.ctr = d_ctr;
      a.dyn_shift = kDynAuto;
      CHECK(hipMemsetAsync(o, 0, 4 * n, 0));
      CHECK(hipMemsetAsync(d_ctr, 0, 4, 0));
      hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, 0>), dim3(cus), dim3(kThreads), 0, 0,
                            timed ? e0 : nullptr, timed ? e1 : nullptr, 0, a);
      CHECK(hipDeviceSynchronize());
      float ms = 0;
      if (timed) CHECK(hipEventElapsedTime(&ms, e0, e1));
      return ms;
    };
    auto run_quad = [&](int b, uint32_t *o, bool timed) -> float {
      QuadArgs a{dp[b], dl, o, n, d_tab};
      hipExtLaunchKernelGGL((quad_kernel<17>), dim3(cus), dim3(1024), 0, 0, timed ? e0 : nullptr,
                            timed ? e1 : nullptr, 0, a);
      CHECK(hipGetLastError());
      CHECK(hipDeviceSynchronize());
      float ms = 0;
      if (timed) CHECK(hipEventElapsedTime(&ms, e0, e1));
      return ms;
    };
    auto run_q256 = [&](int b, uint32_t *o, bool timed, int v) -> float {
      QuadArgs a{dp[b], dl, o, n, d_tab};
      static void (*const ks[])(QuadArgs, const uint32_t *) = {
          quad256_kernel<8, true>, group_kernel<16, 8>, group_kernel<8, 4>, group_kernel<8, 8>, group_kernel<4, 2>,
          group_kernel<4, 4>};
      auto k = ks[v];
      hipExtLaunchKernelGGL(k, dim3(cus), dim3(1024), 0, 0, timed ? e0 : nullptr,
                            timed ? e1 : nullptr, 0, a, (const uint32_t *)d256);
      CHECK(hipGetLastError());
      CHECK(hipDeviceSynchronize());
      float ms = 0;
      if (timed) CHECK(hipEventElapsedTime(&ms, e0, e1));
      return ms;
    };
    uint64_t bad = 0, bad2 = 0;
    std::vector<uint32_t> h1(n), h2(n);
    for (int b = 0; b < 2; b++) {
      run_main(b, o1, false);
      run_quad(b, o2, false);
      CHECK(hipMemcpy(h1.data(), o1, 4 * n, hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(h2.data(), o2, 4 * n, hipMemcpyDeviceToHost));
      for (uint64_t i = 0; i < n; i++) bad += h1[i] != h2[i];
      CHECK(hipMemsetAsync(o2, 0, 4 * n, 0));
      for (int v = 0; v < 6; v++) {
        CHECK(hipMemsetAsync(o2, 0, 4 * n, 0));
        run_q256(b, o2, false, v);
        CHECK(hipMemcpy(h2.data(), o2, 4 * n, hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < n; i++) bad2 += h1[i] != h2[i];
      }
    }
    double tm = 0, tq = 0, t2[6] = {0, 0, 0, 0, 0, 0};
    for (int r = 0; r < reps; r++)
      for (int b = 0; b < 2; b++) {
        tm += run_main(b, o1, true), tq += run_quad(b, o2, true);
        for (int v = 0; v < 6; v++) t2[v] += run_q256(b, o2, true, v);
      }
    tm /= 2 * reps, tq /= 2 * reps;
    for (int v = 0; v < 6; v++) t2[v] /= 2 * reps;
    printf("L %6llu n %8llu  batch kernel %.3f ms %7.1f GB/s | quad kernel %.3f ms %7.1f GB/s | %s\n",
           (unsigned long long)L, (unsigned long long)n, tm, n * L / (tm * 1e-3) / 1e9, tq,
           n * L / (tq * 1e-3) / 1e9, bad ? "MISMATCH" : "equal");
    const char *vn[6] = {"q256 D8 pf", "G16 D8", "G8 D4", "G8 D8", "G4 D2", "G4 D4"};
    for (int v = 0; v < 6; v++)
      printf("           %-10s %.3f ms %7.1f GB/s\n", vn[v], t2[v], n * L / (t2[v] * 1e-3) / 1e9);
    printf("           q256 variants %s\n", bad2 ? "MISMATCH" : "equal");
    fflush(stdout);
    for (int b = 0; b < 2; b++) {
      CHECK(hipFree(data[b]));
      CHECK(hipFree(dp[b]));
    }
    CHECK(hipFree(dl));
    CHECK(hipFree(dpre));
    CHECK(hipFree(o1));
    CHECK(hipFree(o2));
  }
  return 0;
}
