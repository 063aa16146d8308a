// tools/piece_probe.hip -- how much HBM rate do short pieces cost a
// streaming wave, and does keeping loads in flight across piece boundaries
// win it back?  (measurement only: pure reads, no CRC)
//
// One 1024-thread workgroup per CU, as the CRC kernel.  Wave w reads pieces
// w, w + W, w + 2W, ... of a batch of equal pieces of L bytes laid end to end
// (L a power of two >= 4 KiB; 4 GiB in all), in 4 KiB groups (one 16-B nt load
// per lane per KiB, 4 per group), `kG` groups in flight:
//   restart   each piece starts with an empty pipeline (the batch kernel's
//             piece_raw: issue kG groups, then consume one / issue one)
//   carry     the next piece's first groups are issued while the current
//             piece's last ones are consumed (the pipeline never drains
//             between pieces)
// Prints GB/s per (L, kG, form), best of `reps`, so that the per-piece cost
// of a restart can be set against config 4's medium buffers (8 KiB-1 MiB).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o piece_probe piece_probe.hip
//   piece_probe [reps]
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// group q of the wave's stream: piece p = w + W * (q / gpp), group q % gpp
// (gpp = groups per piece)
template <int kG, bool kCarry>
__global__ __launch_bounds__(1024) void piece_read(const uint8_t *base, uint64_t L, uint64_t npieces,
                                                   uint32_t *out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t W = (uint64_t)gridDim.x * 16u;
  const uint64_t w = (uint64_t)(threadIdx.x >> 6) * gridDim.x + blockIdx.x;
  const uint64_t gpp = L >> 12;  // groups per piece (a power of two)
  const uint32_t sh = (uint32_t)__builtin_ctzll(gpp);
  const uint64_t mine = w < npieces ? (npieces - w + W - 1) / W : 0;
  uint32_t acc = 0;
  auto addr = [&](uint64_t q) -> const v4u * {
    const uint64_t p = w + W * (q >> sh), g = q & (gpp - 1);
    return reinterpret_cast<const v4u *>(base + p * L + (g << 12) + 16u * lane);
  };
  auto load = [&](v4u *dst, uint64_t q) {
    const v4u *a = addr(q);
#pragma unroll
    for (int u = 0; u < 4; u++) dst[u] = __builtin_nontemporal_load(a + 64 * u);
  };
  auto use = [&](const v4u *src) {
#pragma unroll
    for (int u = 0; u < 4; u++) acc ^= src[u].x ^ src[u].y ^ src[u].z ^ src[u].w;
  };
  v4u ring[kG][4];
  if (kCarry) {
    const uint64_t total = mine * gpp;
    // one pipeline over all the wave's groups, piece boundaries ignored
#pragma unroll
    for (int s = 0; s < kG; s++)
      if ((uint64_t)s < total) load(ring[s], s);
    for (uint64_t q = 0; q < total; q += kG) {
#pragma unroll
      for (int s = 0; s < kG; s++) {
        if (q + s < total) {
          use(ring[s]);
          if (q + s + kG < total) load(ring[s], q + s + kG);
        }
      }
    }
  } else {
    for (uint64_t k = 0; k < mine; k++) {
      const uint64_t q0 = k * gpp;
#pragma unroll
      for (int s = 0; s < kG; s++)
        if ((uint64_t)s < gpp) load(ring[s], q0 + s);
      for (uint64_t q = 0; q < gpp; q += kG) {
#pragma unroll
        for (int s = 0; s < kG; s++) {
          if (q + s < gpp) {
            use(ring[s]);
            if (q + s + kG < gpp) load(ring[s], q0 + q + s + kG);
          }
        }
      }
      acc = (uint32_t)__builtin_amdgcn_readfirstlane((int)acc) + lane;  // the piece's end: a fold-like dependency
    }
  }
  if (acc == 0x12345678u) out[threadIdx.x] = acc;
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 5;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t bytes = 4ull << 30;
  uint8_t *base;
  uint32_t *out;
  CK(hipMalloc(&base, bytes));
  CK(hipMalloc(&out, 4096));
  CK(hipMemset(base, 0x5A, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("piece_probe: %d CUs, 4 GiB of equal pieces, 4 KiB groups, best of %d\n", cus, reps);
  printf("%10s %10s  %9s %9s %9s  %9s %9s %9s  (GB/s)\n", "piece", "pieces", "restart2", "restart3", "restart4",
         "carry2", "carry3", "carry4");
  for (uint64_t L : {8192ull, 16384ull, 32768ull, 65536ull, 262144ull, 1048576ull}) {
    const uint64_t np = bytes / L;
    double gbs[6];
    for (int v = 0; v < 6; v++) {
      double best = 1e30;
      for (int r = 0; r < reps + 1; r++) {
        switch (v) {
          case 0: hipExtLaunchKernelGGL((piece_read<2, false>), dim3(cus), dim3(1024), 0, 0, e0, e1, 0, base, L, np, out); break;
          case 1: hipExtLaunchKernelGGL((piece_read<3, false>), dim3(cus), dim3(1024), 0, 0, e0, e1, 0, base, L, np, out); break;
          case 2: hipExtLaunchKernelGGL((piece_read<4, false>), dim3(cus), dim3(1024), 0, 0, e0, e1, 0, base, L, np, out); break;
          case 3: hipExtLaunchKernelGGL((piece_read<2, true>), dim3(cus), dim3(1024), 0, 0, e0, e1, 0, base, L, np, out); break;
          case 4: hipExtLaunchKernelGGL((piece_read<3, true>), dim3(cus), dim3(1024), 0, 0, e0, e1, 0, base, L, np, out); break;
          default: hipExtLaunchKernelGGL((piece_read<4, true>), dim3(cus), dim3(1024), 0, 0, e0, e1, 0, base, L, np, out); break;
        }
        CK(hipGetLastError());
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r) best = std::min(best, (double)ms);  // the first launch warms up
      }
      gbs[v] = bytes / (best * 1e-3) / 1e9;
    }
    printf("%10llu %10llu  %9.0f %9.0f %9.0f  %9.0f %9.0f %9.0f\n", (unsigned long long)L, (unsigned long long)np,
           gbs[0], gbs[1], gbs[2], gbs[3], gbs[4], gbs[5]);
  }
  return 0;
}
