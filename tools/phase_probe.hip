// tools/phase_probe.hip -- config 3's read: does the waves' phase inside their
// buffers cost the per-wave mapping its distance to the stream-read sweep?
// (measurement only; round 6)
//
// The product gives each of the 4,096 waves a contiguous 16 MiB range of
// config 3's 64 GiB (16 buffers of 1 MiB), visits the buffers in a hashed
// rotation (walk_rotation) and reads each buffer from its first byte, two
// 2 KiB register groups in flight.  All waves start together and progress at
// about the same rate, so at any moment their addresses agree in the bits
// below 20 (the offset inside the current buffer).  The sweep reads a
// contiguous 16 MiB window, every address bit below 24 covered at once, and
// reads 2-5% faster.  Pure reads (xor of the loaded words), same region,
// interleaved reps, dispatch-packet timestamps:
//   sweep          zcrc_read_sweep_device's k_sweep<1024>
//   wave-inorder   per-wave contiguous range, buffers in order, from offset 0
//   wave-bufrot    + buffers visited in the product's hashed rotation
//   wave-phase64K  + each wave enters every buffer at its own 64 KiB-aligned
//                  offset (hash of the wave) and wraps: the phase spread over
//                  the buffer (a CRC would pay one extra fold + combine per
//                  buffer for it)
//   wave-phase4K   the same at 4 KiB granularity
//   wave-rangephase range entered at a hashed 64 KiB offset of the whole 16
//                  MiB range, wrapping (buffers in order from there)
//   deep-Nw-GK     N waves per CU (one workgroup), each a contiguous range,
//                  buffers rotated, G KiB groups, two in flight: fewer,
//                  deeper streams (deep-16w-2K is the product's shape)
//
//   make -C tools phase_probe && tools/phase_probe [reps]
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CHECK(x)                                                                               \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));        \
      exit(1);                                                                                 \
    }                                                                                          \
  } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) v4u *gv4u;

__device__ __forceinline__ uint32_t xr(v4u v) { return v.x ^ v.y ^ v.z ^ v.w; }

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  return x ^ (x >> 16);
}

constexpr uint64_t kBuf = 1u << 20;

__global__ __launch_bounds__(1024) void k_sweep(const uint8_t *base, uint64_t bytes, uint32_t *out) {
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
    for (int u = 0; u < 4; u++) acc ^= xr(v[u]);
  }
  if (acc == 0x12345678u) out[threadIdx.x] = acc;
}

// kMode 0: in order; 1: buffers rotated; 2: + in-buffer phase 64 KiB; 3: +
// in-buffer phase 4 KiB; 4: range phase 64 KiB
template <int kMode>
__global__ __launch_bounds__(1024) void k_wave(const uint8_t *base, uint64_t bytes, uint32_t *out) {
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t w = blockIdx.x * 16u + wv, W = gridDim.x * 16u;
  const uint64_t per = bytes / W;  // 16 MiB at config 3
  const uint32_t nbuf = (uint32_t)(per / kBuf);
  const uint64_t b0 = reinterpret_cast<uint64_t>(base) + (uint64_t)w * per;
  const uint32_t h = hash32(w * 0x9E3779B1u + 7u);
  const uint32_t rot = kMode >= 1 && kMode <= 3 ? h % nbuf : 0u;
  const uint32_t ph = kMode == 2 ? ((h >> 8) % 16u) * 65536u : kMode == 3 ? ((h >> 8) % 256u) * 4096u : 0u;
  const uint64_t rph = kMode == 4 ? (uint64_t)((h >> 8) % (uint32_t)(per / 65536)) * 65536u : 0u;
  uint32_t acc = 0;
  // the wave's stream of 2 KiB groups: group g of the walk -> address
  const uint32_t gpb = (uint32_t)(kBuf / 2048);  // groups per buffer
  const uint32_t ng = nbuf * gpb;
  auto addr = [&](uint32_t g) -> uint64_t {
    if (kMode == 4) return (rph + 2048ull * g) % per;
    const uint32_t bi = (g / gpb + rot) % nbuf;
    const uint32_t off = (uint32_t)((ph + 2048u * (g % gpb)) % kBuf);
    return (uint64_t)bi * kBuf + off;
  };
  v4u ga[2], gb[2];
  auto ld = [&](v4u *G, uint32_t g) {
    const uint64_t a = b0 + addr(g) + 16u * lane;
#pragma unroll
    for (int u = 0; u < 2; u++) G[u] = __builtin_nontemporal_load(reinterpret_cast<gv4u>(a + 1024u * u));
  };
  ld(ga, 0);
  ld(gb, 1);
  for (uint32_t g = 0; g + 2 < ng; g += 2) {
    acc ^= xr(ga[0]) ^ xr(ga[1]);
    ld(ga, g + 2);
    acc ^= xr(gb[0]) ^ xr(gb[1]);
    if (g + 3 < ng) ld(gb, g + 3);
  }
  acc ^= xr(ga[0]) ^ xr(ga[1]) ^ xr(gb[0]) ^ xr(gb[1]);
  if (acc == 0x12345678u) out[threadIdx.x] = acc;
}

// fewer, deeper streams: kWv waves per workgroup (one workgroup per CU), each
// a contiguous range of bytes / (CUs * kWv), buffers rotated as the product,
// groups of kG KiB, two groups in flight
template <int kWv, int kG>
__global__ __launch_bounds__(kWv * 64) void k_deep(const uint8_t *base, uint64_t bytes, uint32_t *out) {
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t w = blockIdx.x * kWv + wv, W = gridDim.x * kWv;
  const uint64_t per = bytes / W;
  const uint32_t nbuf = (uint32_t)(per / kBuf);
  const uint64_t b0 = reinterpret_cast<uint64_t>(base) + (uint64_t)w * per;
  const uint32_t rot = hash32(w * 0x9E3779B1u + 7u) % nbuf;
  constexpr uint32_t gb_bytes = 1024u * kG;
  const uint32_t gpb = (uint32_t)(kBuf / gb_bytes), ng = nbuf * gpb;
  auto addr = [&](uint32_t g) -> uint64_t {
    return (uint64_t)((g / gpb + rot) % nbuf) * kBuf + (uint64_t)(g % gpb) * gb_bytes;
  };
  uint32_t acc = 0;
  v4u ga[kG], gb[kG];
  auto ld = [&](v4u *G, uint32_t g) {
    const uint64_t a = b0 + addr(g) + 16u * lane;
#pragma unroll
    for (int u = 0; u < kG; u++) G[u] = __builtin_nontemporal_load(reinterpret_cast<gv4u>(a + 1024u * u));
  };
  auto use = [&](const v4u *G) {
#pragma unroll
    for (int u = 0; u < kG; u++) acc ^= xr(G[u]);
  };
  ld(ga, 0);
  ld(gb, 1);
  for (uint32_t g = 0; g + 2 < ng; g += 2) {
    use(ga);
    ld(ga, g + 2);
    use(gb);
    if (g + 3 < ng) ld(gb, g + 3);
  }
  use(ga);
  use(gb);
  if (acc == 0x12345678u) out[threadIdx.x] = acc;
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 8;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t bytes = 65536ull << 20;  // config 3
  uint8_t *mem;
  uint32_t *out;
  CHECK(hipMalloc(&mem, bytes));
  CHECK(hipMalloc(&out, 1 << 20));
  CHECK(hipMemset(mem, 1, bytes));
  CHECK(hipDeviceSynchronize());
  const char *nm[] = {"sweep", "wave-inorder", "wave-bufrot", "wave-phase64K", "wave-phase4K", "wave-rangephase",
                      "deep-16w-2K", "deep-8w-4K", "deep-4w-8K", "deep-8w-2K", "deep-4w-4K"};
  constexpr int kV = 11;
  std::vector<std::vector<double>> t(kV);
  hipEvent_t a, z;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&z));
  for (int r = 0; r < reps; r++)
    for (int v = 0; v < kV; v++) {
      switch (v) {
        case 0: hipExtLaunchKernelGGL(k_sweep, dim3(cus), dim3(1024), 0, 0, a, z, 0, mem, bytes, out); break;
        case 1: hipExtLaunchKernelGGL(k_wave<0>, dim3(cus), dim3(1024), 0, 0, a, z, 0, mem, bytes, out); break;
        case 2: hipExtLaunchKernelGGL(k_wave<1>, dim3(cus), dim3(1024), 0, 0, a, z, 0, mem, bytes, out); break;
        case 3: hipExtLaunchKernelGGL(k_wave<2>, dim3(cus), dim3(1024), 0, 0, a, z, 0, mem, bytes, out); break;
        case 4: hipExtLaunchKernelGGL(k_wave<3>, dim3(cus), dim3(1024), 0, 0, a, z, 0, mem, bytes, out); break;
        case 5: hipExtLaunchKernelGGL(k_wave<4>, dim3(cus), dim3(1024), 0, 0, a, z, 0, mem, bytes, out); break;
        case 6: hipExtLaunchKernelGGL((k_deep<16, 2>), dim3(cus), dim3(1024), 0, 0, a, z, 0, mem, bytes, out); break;
        case 7: hipExtLaunchKernelGGL((k_deep<8, 4>), dim3(cus), dim3(512), 0, 0, a, z, 0, mem, bytes, out); break;
        case 8: hipExtLaunchKernelGGL((k_deep<4, 8>), dim3(cus), dim3(256), 0, 0, a, z, 0, mem, bytes, out); break;
        case 9: hipExtLaunchKernelGGL((k_deep<8, 2>), dim3(cus), dim3(512), 0, 0, a, z, 0, mem, bytes, out); break;
        case 10: hipExtLaunchKernelGGL((k_deep<4, 4>), dim3(cus), dim3(256), 0, 0, a, z, 0, mem, bytes, out); break;
      }
      CHECK(hipGetLastError());
      CHECK(hipEventSynchronize(z));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, a, z));
      if (r > 0) t[v].push_back(ms);
    }
  printf("phase_probe: config 3 region (%llu B), %d CUs, %d reps (first dropped)\n", (unsigned long long)bytes, cus,
         reps);
  for (int v = 0; v < kV; v++) {
    double sum = 0, best = 1e30;
    for (double x : t[v]) sum += x, best = std::min(best, x);
    const double avg = sum / t[v].size();
    printf("  %-16s avg %8.3f ms  %7.1f GB/s   best %8.3f ms\n", nm[v], avg, bytes / (avg * 1e-3) / 1e9, best);
  }
  CHECK(hipFree(mem));
  CHECK(hipFree(out));
  return 0;
}
