// tools/waves_probe.hip -- config 3 with fewer, deeper CRC streams per CU?
// (measurement only; round 6)
//
// tools/phase_probe's pure reads of config 3's 64 GiB in the product's shape
// (per-wave contiguous ranges, buffers rotated, two groups in flight) read
// 1.2% faster with 8 waves per CU than with the product's 16 (10.00 against
// 10.13 ms; the sweep 9.77): fewer streams and half the bytes in flight
// chip-wide.  Does the CRC keep that with half the waves to hide its LDS
// lookups?  A plain CRC kernel for equal, 16-B aligned 1 MiB buffers (each
// wave whole buffers of its range: the product's hot loop, table layout and
// fold, no edge fix-ups), kWv waves per workgroup, kG-block register groups,
// one workgroup per CU, against the product kernel and the sweep in one
// process; every variant's 65,536 CRCs are compared with the product's.
//
//   make -C tools waves_probe && tools/waves_probe [reps]
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

constexpr uint64_t kN = 65536, kLen = 1u << 20, kBytes = kN * kLen;

template <int kWv, int kG, bool kRR = false>
__global__ __launch_bounds__(kWv * 64) void simple_crc(const uint8_t *base, const TableBlob *tab, uint32_t *out) {
  __shared__ __attribute__((aligned(16))) uint32_t s_lds[kLdsBytes / 4];
  constexpr uint32_t kT = kWv * 64;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = uni32(tid >> 6);
  // the product's layout: braided x32 (byte o holds braid[j][v], j = 2 (o >> 16)
  // + ((o >> 7) & 1), v = (o >> 8) & 255), then the 8 combine tables
  for (uint32_t d = tid; d < kLdsCombDword; d += kT) {
    const uint32_t o = 4u * d;
    s_lds[d] = tab->braid[(((o >> 16) << 1) | ((o >> 7) & 1u)) * 256u + ((o >> 8) & 255u)];
  }
  for (uint32_t d = tid; d < 8u * 1024u; d += kT) s_lds[kLdsCombDword + d] = tab->comb[d];
  __syncthreads();
  const uint32_t lo0 = (lane & 31u) * 4u;
  const uint32_t o0 = lo0, o1 = lo0 + 128u, o2 = lo0 + 65536u, o3 = lo0 + 65536u + 128u;
  const uint32_t W = gridDim.x * kWv, w = blockIdx.x * kWv + wv;
  const uint32_t nb = (uint32_t)(kN / W);  // buffers per wave
  const uint32_t rot = hash32(w) % nb;
  for (uint32_t k = 0; k < nb; k++) {
    // kRR: round-robin buffers (wave w: buffers w, w + W, ...): the waves'
    // current buffers form one contiguous window (tools/region_probe)
    const uint32_t bi = kRR ? k * W + w : w * nb + (k + rot) % nb;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)(base + (uint64_t)bi * kLen), (short)0, (int)kLen, 0x00020000);
    uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0, q0 = 0, q1 = 0, q2 = 0, q3 = 0;
    uint4 ga[kG], gb[kG];
    auto ld = [&](uint4 *G, uint32_t g) {
#pragma unroll
      for (uint32_t u = 0; u < kG; u++) {
        auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, 1024u * (g * kG + u) + 16u * lane, 0, kLoadNt);
        G[u] = make_uint4(v[0], v[1], v[2], v[3]);
      }
    };
    auto use = [&](const uint4 *G) {
#pragma unroll
      for (uint32_t u = 0; u < kG; u++) {
        braid_step2(s_lds, s0, q0, G[u].x, o0, o1, o2, o3);
        braid_step2(s_lds, s1, q1, G[u].y, o0, o1, o2, o3);
        braid_step2(s_lds, s2, q2, G[u].z, o0, o1, o2, o3);
        braid_step2(s_lds, s3, q3, G[u].w, o0, o1, o2, o3);
      }
    };
    constexpr uint32_t ng = (uint32_t)(kLen / 1024 / kG);
    ld(ga, 0);
    ld(gb, 1);
    if (lane == 0) ga[0].x ^= 0xFFFFFFFFu;  // seed 0: ~0 into the buffer's first word
    for (uint32_t g = 0; g + 2 < ng; g += 2) {
      use(ga);
      ld(ga, g + 2);
      use(gb);
      if (g + 3 < ng) ld(gb, g + 3);
    }
    use(ga);
    use(gb);
    s0 ^= q0, s1 ^= q1, s2 ^= q2, s3 ^= q3;
    uint32_t r = (s0 ^ comb_apply(s_lds, 0, s1)) ^ comb_apply(s_lds, 1, s2 ^ comb_apply(s_lds, 0, s3));
    r ^= row_shl<1>(comb_apply(s_lds, 2, r));
    r ^= row_shl<2>(comb_apply(s_lds, 3, r));
    r ^= row_shl<4>(comb_apply(s_lds, 4, r));
    r ^= row_shl<8>(comb_apply(s_lds, 5, r));
    const uint32_t r0 = uni32(r);
    const uint32_t r16 = (uint32_t)__builtin_amdgcn_readlane((int)r, 16);
    const uint32_t r32 = (uint32_t)__builtin_amdgcn_readlane((int)r, 32);
    const uint32_t r48 = (uint32_t)__builtin_amdgcn_readlane((int)r, 48);
    r = uni32(r0 ^ comb_apply(s_lds, 6, r16) ^ comb_apply(s_lds, 7, r32 ^ comb_apply(s_lds, 6, r48)));
    if (lane == 0) out[bi] = ~r;
  }
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 8;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  static TableBlob tb;
  build_tables(tb);
  TableBlob *d_tab;
  CHECK(hipMalloc(&d_tab, sizeof(TableBlob)));
  CHECK(hipMemcpy(d_tab, &tb, sizeof(TableBlob), hipMemcpyHostToDevice));
  uint8_t *mem;
  CHECK(hipMalloc(&mem, kBytes));
  {
    std::vector<uint64_t> hp(kN), hl(kN, kLen);
    for (uint64_t i = 0; i < kN; i++) hp[i] = (uint64_t)(mem + i * kLen);
    uint64_t *dp, *dl;
    CHECK(hipMalloc(&dp, 8 * kN));
    CHECK(hipMalloc(&dl, 8 * kN));
    CHECK(hipMemcpy(dp, hp.data(), 8 * kN, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dl, hl.data(), 8 * kN, hipMemcpyHostToDevice));
    CHECK(launch_fill_synthetic(dp, dl, kN, 0, 1, 0xC0FFEE, 0));
    CHECK(hipDeviceSynchronize());
    CHECK(hipFree(dp));
    CHECK(hipFree(dl));
  }
  uint32_t *o_ref, *o_new, *scratch;
  CHECK(hipMalloc(&o_ref, 4 * kN));
  CHECK(hipMalloc(&o_new, 4 * kN));
  CHECK(hipMalloc(&scratch, 1 << 16));
  auto product = [&](hipEvent_t e0, hipEvent_t e1) {
    BatchArgs x{};
    x.base = mem;
    x.stride = kLen;
    x.len = kLen;
    x.n = kN;
    x.out = o_ref;
    x.tab = d_tab;
    x.ctr = scratch;
    x.dyn_shift = kDynAuto;
    CHECK(hipMemsetAsync(o_ref, 0, 4 * kN, 0));
    CHECK(hipMemsetAsync(scratch, 0, 256, 0));
    hipExtLaunchKernelGGL((crc32_batch_kernel<true, kDepth, 0>), dim3(cus), dim3(kThreads), 0, 0, e0, e1, 0, x);
    CHECK(hipGetLastError());
  };
  const char *nm[] = {"product", "simple-16w-2K", "simple-8w-2K", "simple-8w-4K", "simple-4w-4K", "simple-16w-1K"};
  constexpr int kV = 6;
  auto launch = [&](int v, hipEvent_t e0, hipEvent_t e1) {
    switch (v) {
      case 0: product(e0, e1); return;
      case 1: hipExtLaunchKernelGGL((simple_crc<16, 2>), dim3(cus), dim3(1024), 0, 0, e0, e1, 0, mem, d_tab, o_new); break;
      case 2: hipExtLaunchKernelGGL((simple_crc<8, 2>), dim3(cus), dim3(512), 0, 0, e0, e1, 0, mem, d_tab, o_new); break;
      case 3: hipExtLaunchKernelGGL((simple_crc<8, 4>), dim3(cus), dim3(512), 0, 0, e0, e1, 0, mem, d_tab, o_new); break;
      case 4: hipExtLaunchKernelGGL((simple_crc<4, 4>), dim3(cus), dim3(256), 0, 0, e0, e1, 0, mem, d_tab, o_new); break;
      case 5: hipExtLaunchKernelGGL((simple_crc<16, 1>), dim3(cus), dim3(1024), 0, 0, e0, e1, 0, mem, d_tab, o_new); break;
    }
    CHECK(hipGetLastError());
  };
  launch(0, nullptr, nullptr);
  CHECK(hipDeviceSynchronize());
  std::vector<uint32_t> ref(kN), got(kN);
  CHECK(hipMemcpy(ref.data(), o_ref, 4 * kN, hipMemcpyDeviceToHost));
  bool all_eq = true;
  for (int v = 1; v < kV; v++) {
    CHECK(hipMemset(o_new, 0, 4 * kN));
    launch(v, nullptr, nullptr);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(got.data(), o_new, 4 * kN, hipMemcpyDeviceToHost));
    uint64_t bad = 0;
    for (uint64_t i = 0; i < kN; i++) bad += got[i] != ref[i];
    printf("parity %-14s %s (%llu differ)\n", nm[v], bad ? "DIFFER" : "equal", (unsigned long long)bad);
    all_eq = all_eq && !bad;
  }
  fflush(stdout);
  hipEvent_t a, z;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&z));
  std::vector<std::vector<double>> t(kV);
  for (int r = 0; r < reps; r++)
    for (int v = 0; v < kV; v++) {
      launch(v, a, z);
      CHECK(hipEventSynchronize(z));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, a, z));
      if (r > 0) t[v].push_back(ms);
    }
  printf("waves_probe: config 3 (%llu B), %d CUs, %d reps (first dropped)\n", (unsigned long long)kBytes, cus, reps);
  for (int v = 0; v < kV; v++) {
    double s = 0;
    for (double x : t[v]) s += x;
    const double avg = s / t[v].size();
    printf("  %-14s avg %8.3f ms  %7.1f GB/s   best %8.3f\n", nm[v], avg, kBytes / (avg * 1e-3) / 1e9,
           *std::min_element(t[v].begin(), t[v].end()));
  }
  return all_eq ? 0 : 1;
}
