// tools/atomic_probe.hip -- how fast can the batch kernel's waves claim
// dynamic units?  (measurement only)
//
// Every wave of a 256 x 1024 launch (one workgroup per CU, as the CRC
// kernel) takes `claims` values from device-scope atomicAdd counters, one
// claim after another (each waits for its result, as a claim does), with
// lane 0 issuing.  Counters: 1 (the product's one claim counter), or P
// partitions `stride` bytes apart, wave w using partition (w's workgroup) %
// P.  Prints the launch time and the claims per microsecond, so that the
// per-address throughput of the claim atomic can be set against config 4's
// ~50k claims per 1.95 ms launch.
//
//   hipcc --offload-arch=gfx950 -O3 -o atomic_probe atomic_probe.hip
//   atomic_probe [claims_per_wave]
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

__global__ __launch_bounds__(1024) void claim_kernel(uint32_t *ctr, uint32_t parts, uint32_t stride_words,
                                                     uint32_t claims, uint32_t *sink) {
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t *c = ctr + (blockIdx.x % parts) * stride_words;
  uint32_t acc = 0;
  for (uint32_t k = 0; k < claims; k++) {
    uint32_t v = 0;
    if (lane == 0) v = atomicAdd(c, 1u);
    v = (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
    acc += v;  // the next claim depends on this one (as a claim does)
    if (acc == 0xFFFFFFFFu) break;
  }
  if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

int main(int argc, char **argv) {
  const uint32_t claims = argc > 1 ? (uint32_t)atoi(argv[1]) : 12;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t *ctr, *sink;
  CK(hipMalloc(&ctr, 1 << 20));
  CK(hipMalloc(&sink, 4096));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct Cfg {
    uint32_t parts, stride_bytes;
  } cfgs[] = {{1, 256}, {2, 256}, {8, 256}, {8, 4096}, {16, 256}, {64, 256}};
  printf("atomic_probe: %d workgroups x 16 waves, %u claims per wave (%u in all)\n", cus, claims,
         (uint32_t)cus * 16u * claims);
  for (int round = 0; round < 2; round++) {
    for (const Cfg &c : cfgs) {
      CK(hipMemset(ctr, 0, 1 << 20));
      hipExtLaunchKernelGGL(claim_kernel, dim3(cus), dim3(1024), 0, 0, e0, e1, 0, ctr, c.parts, c.stride_bytes / 4,
                            claims, sink);
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      uint32_t sum = 0, h[64 * 1024];
      CK(hipMemcpy(h, ctr, sizeof h, hipMemcpyDeviceToHost));
      for (uint32_t p = 0; p < c.parts; p++) sum += h[p * (c.stride_bytes / 4)];
      const double total = (double)cus * 16 * claims;
      printf("parts %2u stride %5u B: %8.1f us, %7.1f claims/us, %6.1f ns per claim per address, count %s\n",
             c.parts, c.stride_bytes, ms * 1e3, total / (ms * 1e3), ms * 1e6 / (total / c.parts),
             sum == (uint32_t)total ? "ok" : "WRONG");
    }
  }
  return 0;
}
