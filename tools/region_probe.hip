// tools/region_probe.hip -- is a box's config-3 rate a property of the box or
// of where its 64 GiB landed?  (measurement only; round 6)
//
// (Below: the kernels of tools/waves_probe.hip, which this probe reuses.)
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
#include <string>
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
    // current buffers form one contiguous window
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

__global__ __launch_bounds__(1024) void k_sweep(const uint8_t *base, uint64_t bytes, uint32_t *out) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  typedef const __attribute__((address_space(1))) v4u *gv4u;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint64_t step = (uint64_t)gridDim.x * 65536;
  const uint64_t b0 = reinterpret_cast<uint64_t>(base);
  uint32_t acc = 0;
  for (uint64_t o = (uint64_t)blockIdx.x * 65536; o + 65536 <= bytes; o += step) {
    v4u v[4];
    v[0] = __builtin_nontemporal_load(reinterpret_cast<gv4u>(b0 + o + 1024u * wv + 16u * lane));
    __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
    for (int u = 1; u < 4; u++)
      v[u] = __builtin_nontemporal_load(reinterpret_cast<gv4u>(b0 + o + 1024u * (16u * u + wv) + 16u * lane));
#pragma unroll
    for (int u = 0; u < 4; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x12345678u) out[threadIdx.x] = acc;
}

// Pure reads in CRC-compatible mappings (16 waves per CU, 2 KiB groups, two
// in flight, 1 MiB buffers), kMap: 0 per-wave contiguous ranges, buffers
// rotated (the product's static partition); 1 round-robin buffers (wave w:
// buffers w, w + W, ...: the waves' current buffers form one contiguous
// window); 2 workgroup-cooperative (the 16 waves of a workgroup share its
// current buffer, wave s reading blocks s, s + 16, ...; workgroup g: buffers
// g, g + G, ...); 3 per-wave ranges, but the waves of one XCD (workgroups
// x, x + 8, ...) own adjacent ranges (one eighth of the region per XCD)
template <int kMap>
__global__ __launch_bounds__(1024) void k_map(const uint8_t *base, uint64_t bytes, uint32_t *out) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  typedef const __attribute__((address_space(1))) v4u *gv4u;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t G = gridDim.x, W = G * 16u;
  const uint32_t nbuf = (uint32_t)(bytes / kLen);
  uint32_t w = blockIdx.x * 16u + wv;
  if (kMap == 3) {  // XCD-compact: workgroup g runs on XCD g % 8
    const uint32_t x = blockIdx.x % 8u, k = blockIdx.x / 8u;
    w = (x * (G / 8u) + k) * 16u + wv;
  }
  const uint64_t b0 = reinterpret_cast<uint64_t>(base);
  uint32_t acc = 0;
  auto buffer_of = [&](uint32_t j) -> uint64_t {  // the wave's j-th buffer
    if (kMap == 0 || kMap == 3) {
      const uint32_t per = nbuf / W, rot = hash32(w) % per;
      return (uint64_t)w * per + (j + rot) % per;
    }
    if (kMap == 1) return (uint64_t)j * W + w;
    return (uint64_t)j * G + blockIdx.x;  // kMap 2: the workgroup's j-th buffer
  };
  const uint32_t nj = kMap == 2 ? nbuf / G : nbuf / W;
  // per buffer: kMap 2 reads 64 blocks (s, s+16, ...), the others 1024 blocks
  const uint32_t blocks = kMap == 2 ? 64u : 1024u;
  auto blk = [&](uint32_t i) -> uint32_t { return kMap == 2 ? i * 16u + wv : i; };
  const uint32_t ng = nj * (blocks / 2u);
  auto addr = [&](uint32_t g) -> uint64_t {  // group g of the walk: 2 blocks
    const uint32_t j = g / (blocks / 2u), i = (g % (blocks / 2u)) * 2u;
    return b0 + buffer_of(j) * kLen + 1024ull * blk(i);
  };
  auto addr2 = [&](uint32_t g) -> uint64_t {
    const uint32_t j = g / (blocks / 2u), i = (g % (blocks / 2u)) * 2u + 1u;
    return b0 + buffer_of(j) * kLen + 1024ull * blk(i);
  };
  v4u ga[2], gb[2];
  auto ld = [&](v4u *X, uint32_t g) {
    X[0] = __builtin_nontemporal_load(reinterpret_cast<gv4u>(addr(g) + 16u * lane));
    X[1] = __builtin_nontemporal_load(reinterpret_cast<gv4u>(addr2(g) + 16u * lane));
  };
  ld(ga, 0);
  ld(gb, 1);
  for (uint32_t g = 0; g + 2 < ng; g += 2) {
    acc ^= ga[0].x ^ ga[0].y ^ ga[0].z ^ ga[0].w ^ ga[1].x ^ ga[1].y ^ ga[1].z ^ ga[1].w;
    ld(ga, g + 2);
    acc ^= gb[0].x ^ gb[0].y ^ gb[0].z ^ gb[0].w ^ gb[1].x ^ gb[1].y ^ gb[1].z ^ gb[1].w;
    if (g + 3 < ng) ld(gb, g + 3);
  }
  acc ^= ga[0].x ^ ga[1].x ^ gb[0].x ^ gb[1].x;
  if (acc == 0x12345678u) out[threadIdx.x] = acc;
}

// Mode "regions" (default): three 64 GiB regions (each its own hipMalloc, the
// second and third after 1 GiB and 7 GiB spacers), each filled with the
// synthetic payload; per region the stream-read sweep, the product's strided
// config-3 kernel and the plain 16-wave CRC (waves_probe's simple_crc<16, 2>),
// reps interleaved.  Mode "offsets": ONE allocation of 64 GiB + 64 MiB, the
// same kernels over the 64 GiB window starting at several byte offsets into
// it (the same physical pages, shifted).
int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 6;
  const bool offsets = argc > 2 && argv[2][0] == 'o';
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  static TableBlob tb;
  build_tables(tb);
  TableBlob *d_tab;
  CHECK(hipMalloc(&d_tab, sizeof(TableBlob)));
  CHECK(hipMemcpy(d_tab, &tb, sizeof(TableBlob), hipMemcpyHostToDevice));
  std::vector<uint8_t *> mem;
  std::vector<uint64_t> offs;
  std::vector<std::string> label;
  uint64_t *dp, *dl;
  CHECK(hipMalloc(&dp, 8 * kN));
  CHECK(hipMalloc(&dl, 8 * kN));
  auto fill = [&](uint8_t *p) {
    std::vector<uint64_t> hp(kN), hl(kN, kLen);
    for (uint64_t i = 0; i < kN; i++) hp[i] = (uint64_t)(p + i * kLen);
    CHECK(hipMemcpy(dp, hp.data(), 8 * kN, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dl, hl.data(), 8 * kN, hipMemcpyHostToDevice));
    CHECK(launch_fill_synthetic(dp, dl, kN, 0, 1, 0xC0FFEE, 0));
    CHECK(hipDeviceSynchronize());
  };
  if (!offsets) {
    for (int r = 0; r < 3; r++) {
      uint8_t *sp = nullptr, *p = nullptr;
      if (r > 0) CHECK(hipMalloc(&sp, r == 1 ? (1ull << 30) : (7ull << 30)));
      CHECK(hipMalloc(&p, kBytes));
      fill(p);
      mem.push_back(p);
      char b[64];
      snprintf(b, sizeof b, "region %d", r);
      label.push_back(b);
      printf("region %d at %p (mod 64 MiB: %llu KiB)\n", r, (void *)p,
             (unsigned long long)(((uint64_t)p & ((64ull << 20) - 1)) >> 10));
    }
  } else {
    uint8_t *p = nullptr;
    CHECK(hipMalloc(&p, kBytes + (64ull << 20)));
    printf("allocation at %p (mod 64 MiB: %llu KiB)\n", (void *)p,
           (unsigned long long)(((uint64_t)p & ((64ull << 20) - 1)) >> 10));
    const uint64_t o[] = {0, 64ull << 10, 512ull << 10, 1ull << 20, 2ull << 20, 4ull << 20, 6ull << 20, 8ull << 20,
                          16ull << 20, 32ull << 20};
    for (uint64_t x : o) {
      mem.push_back(p + x);
      char b[64];
      snprintf(b, sizeof b, "+%6llu KiB", (unsigned long long)(x >> 10));
      label.push_back(b);
    }
    fill(p);  // (the offsets' windows read the payload of shifted buffers: rates only)
  }
  const int kR = (int)mem.size();
  uint32_t *o_ref, *o_new, *scratch;
  CHECK(hipMalloc(&o_ref, 4 * kN));
  CHECK(hipMalloc(&o_new, 4 * kN));
  CHECK(hipMalloc(&scratch, 1 << 16));
  hipEvent_t a, z;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&z));
  constexpr int kVv = 8;
  std::vector<std::vector<double>> t(kR * kVv);
  for (int rep = 0; rep < reps; rep++)
    for (int r = 0; r < kR; r++)
      for (int v = 0; v < kVv; v++) {
        if (v == 0) {
          hipExtLaunchKernelGGL(k_sweep, dim3(cus), dim3(1024), 0, 0, a, z, 0, mem[r], kBytes, o_new);
        } else if (v == 1) {
          BatchArgs x{};
          x.base = mem[r];
          x.stride = kLen;
          x.len = kLen;
          x.n = kN;
          x.out = o_ref;
          x.tab = d_tab;
          x.ctr = scratch;
          x.dyn_shift = kDynAuto;
          CHECK(hipMemsetAsync(o_ref, 0, 4 * kN, 0));
          CHECK(hipMemsetAsync(scratch, 0, 256, 0));
          hipExtLaunchKernelGGL((crc32_batch_kernel<true, kDepth, 0>), dim3(cus), dim3(kThreads), 0, 0, a, z, 0, x);
        } else if (v == 2) {
          hipExtLaunchKernelGGL((simple_crc<16, 2>), dim3(cus), dim3(1024), 0, 0, a, z, 0, mem[r], d_tab, o_new);
        } else if (v == 3) {
          hipExtLaunchKernelGGL((k_map<0>), dim3(cus), dim3(1024), 0, 0, a, z, 0, mem[r], kBytes, o_new);
        } else if (v == 4) {
          hipExtLaunchKernelGGL((k_map<1>), dim3(cus), dim3(1024), 0, 0, a, z, 0, mem[r], kBytes, o_new);
        } else if (v == 5) {
          hipExtLaunchKernelGGL((k_map<2>), dim3(cus), dim3(1024), 0, 0, a, z, 0, mem[r], kBytes, o_new);
        } else if (v == 6) {
          hipExtLaunchKernelGGL((k_map<3>), dim3(cus), dim3(1024), 0, 0, a, z, 0, mem[r], kBytes, o_new);
        } else {
          hipExtLaunchKernelGGL((simple_crc<16, 2, true>), dim3(cus), dim3(1024), 0, 0, a, z, 0, mem[r], d_tab, o_new);
        }
        CHECK(hipGetLastError());
        CHECK(hipEventSynchronize(z));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, z));
        if (rep > 0) t[r * kVv + v].push_back(ms);
      }
  std::vector<uint32_t> h1(kN), h2(kN);
  CHECK(hipMemcpy(h1.data(), o_ref, 4 * kN, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(h2.data(), o_new, 4 * kN, hipMemcpyDeviceToHost));
  printf("region_probe (%s): config 3 (%llu B) x %d windows, %d CUs, %d reps (first dropped); product == plain: %s\n",
         offsets ? "offsets" : "regions", (unsigned long long)kBytes, kR, cus, reps, h1 == h2 ? "yes" : "NO");
  const char *nm[kVv] = {"sweep", "product", "plain-16w", "rd-ranges", "rd-roundrob", "rd-wgcoop", "rd-xcdcompact", "plain-rr"};
  for (int r = 0; r < kR; r++)
    for (int v = 0; v < kVv; v++) {
      const std::vector<double> &x = t[r * kVv + v];
      double s = 0;
      for (double y : x) s += y;
      const double avg = s / x.size();
      printf("  %-12s %-13s avg %8.3f ms  %7.1f GB/s   min %8.3f  max %8.3f\n", label[r].c_str(), nm[v], avg,
             kBytes / (avg * 1e-3) / 1e9, *std::min_element(x.begin(), x.end()), *std::max_element(x.begin(), x.end()));
    }
  return h1 == h2 ? 0 : 1;
}
