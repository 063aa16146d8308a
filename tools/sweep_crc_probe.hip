// tools/sweep_crc_probe.hip -- would a CRC in the stream-read sweep's mapping
// keep the sweep's rate?  (measurement only; round 6)
//
// The sweep (zcrc_read_sweep_device) reads config 3's region 3-4% faster
// than the CRC's own mappings.  A CRC can follow the sweep's mapping: wave w
// of a workgroup takes the 1 KiB blocks w, w + 16, ... of each chunk its
// workgroup owns, each dword stream advancing 16 KiB per block (one braided
// table for x^(8*16384) instead of x^(8*1024)), and the wave folds its streams
// and xors the chunk's share into the buffer's result at the end of every
// chunk.  This probe runs that cost -- the braid steps on LDS lookups, the
// fold, one atomicXor per wave and chunk -- over the sweep's loads (the CRC
// values are not the real ones: the cost, not the result, is measured), next
// to the plain sweep, interleaved in one process.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I zipsfs_amd/csrc tools/sweep_crc_probe.hip -o tools/sweep_crc_probe
//   tools/sweep_crc_probe [reps] [GiB]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "zcrc_batch_kernel.h"

using namespace zcrc;

#define CHECK(x)                                                                          \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

typedef uint32_t p_v4u __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) p_v4u *p_gptr;

// kB: 1 KiB blocks per wave and chunk (a chunk is 16 kB KiB); kCost 0: xor
// only (the pure read of the mapping), 1: braid steps + fold + atomicXor per
// chunk; kOrder 1: each group of 4 loads as the sweep issues them (first
// alone, a wait, then three), 0: all kB loads at once
template <int kB, int kCost, int kOrder>
__global__ __launch_bounds__(1024) void k_sweep_crc(const uint8_t *base, uint64_t bytes, uint32_t *out) {
  __shared__ __attribute__((aligned(16))) uint32_t s_lds[kLdsBytes / 4];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  if (kCost) {
    for (uint32_t i = tid; i < kLdsBytes / 4; i += 1024) s_lds[i] = i * 0x9E3779B1u;
    __syncthreads();
  }
  const uint32_t lo0 = (lane & 31u) * 4u;
  const uint32_t o0 = lo0, o1 = lo0 + 128u, o2 = lo0 + 65536u, o3 = lo0 + 65536u + 128u;
  constexpr uint64_t kChunk = 16384ull * kB;
  const uint64_t b0 = reinterpret_cast<uint64_t>(base);
  const uint64_t full = bytes / kChunk;
  uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0, q0 = 0, q1 = 0, q2 = 0, q3 = 0, acc = 0;
  for (uint64_t c = blockIdx.x; c < full; c += gridDim.x) {
    const uint64_t o = b0 + c * kChunk + (uint64_t)wv * 1024u + 16u * lane;
#pragma unroll
    for (int g = 0; g < kB; g += 4) {
      p_v4u v[4];
      v[0] = __builtin_nontemporal_load(reinterpret_cast<p_gptr>(o + 16384u * g));
      if (kOrder) __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
      for (int u = 1; u < 4; u++) v[u] = __builtin_nontemporal_load(reinterpret_cast<p_gptr>(o + 16384u * (g + u)));
#pragma unroll
      for (int u = 0; u < 4; u++) {
        if (kCost) {
          braid_step2(s_lds, s0, q0, v[u].x, o0, o1, o2, o3);
          braid_step2(s_lds, s1, q1, v[u].y, o0, o1, o2, o3);
          braid_step2(s_lds, s2, q2, v[u].z, o0, o1, o2, o3);
          braid_step2(s_lds, s3, q3, v[u].w, o0, o1, o2, o3);
        } else {
          acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
        }
      }
    }
    if (kCost) {  // the product's fold, a shift to the buffer end, one atomicXor
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
      r = comb_apply(s_lds, 3, comb_apply(s_lds, 4, r));  // the shift to the buffer end (~2 table products)
      if (lane == 0) atomicXor(out + ((c * kChunk) >> 20), r);
      s0 = s1 = s2 = s3 = q0 = q1 = q2 = q3 = 0;
    }
  }
  if (!kCost && acc == 0x5EEDF00Du) out[tid] = acc;
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 8;
  const uint64_t gib = argc > 2 ? strtoull(argv[2], nullptr, 0) : 64;
  const uint64_t bytes = gib << 30;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint8_t *mem;
  uint32_t *out;
  CHECK(hipMalloc(&mem, bytes));
  CHECK(hipMalloc(&out, 4u << 20));
  CHECK(hipMemset(mem, 0x5A, bytes));
  CHECK(hipMemset(out, 0, 4u << 20));
  CHECK(hipDeviceSynchronize());
  struct V {
    const char *name;
    void (*k)(const uint8_t *, uint64_t, uint32_t *);
  };
  const V vs[] = {
      {"read-b4-order", k_sweep_crc<4, 0, 1>},   // = the stream-read sweep
      {"read-b4-all", k_sweep_crc<4, 0, 0>},     // its loads issued at once
      {"crc-b4-order", k_sweep_crc<4, 1, 1>},    // CRC cost, fold per 4 KiB per wave
      {"crc-b4-all", k_sweep_crc<4, 1, 0>},
      {"read-b16-order", k_sweep_crc<16, 0, 1>}, // 256 KiB chunks
      {"crc-b16-order", k_sweep_crc<16, 1, 1>},  // fold per 16 KiB per wave
      {"crc-b16-all", k_sweep_crc<16, 1, 0>},
  };
  constexpr int kV = sizeof(vs) / sizeof(vs[0]);
  hipEvent_t a, z;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&z));
  std::vector<std::vector<double>> t(kV);
  for (int r = 0; r < reps; r++)
    for (int v = 0; v < kV; v++) {
      if (r == 0) fprintf(stderr, "  %s ...\n", vs[v].name);
      CHECK(hipEventRecord(a, 0));
      hipLaunchKernelGGL(vs[v].k, dim3(cus), dim3(1024), 0, 0, mem, bytes, out);
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(z, 0));
      CHECK(hipEventSynchronize(z));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, a, z));
      t[v].push_back(ms);
    }
  printf("sweep_crc_probe: %llu GiB region, %d reps interleaved, %d CUs\n", (unsigned long long)gib, reps, cus);
  for (int v = 0; v < kV; v++) {
    double sum = 0, best = 1e30;
    for (size_t i = 1; i < t[v].size(); i++) sum += t[v][i], best = best < t[v][i] ? best : t[v][i];
    const double avg = sum / (t[v].size() - 1);
    printf("  %-16s avg %8.3f ms  %7.1f GB/s   best %8.3f ms\n", vs[v].name, avg, bytes / (avg * 1e-3) / 1e9, best);
  }
  CHECK(hipFree(mem));
  CHECK(hipFree(out));
  return 0;
}
