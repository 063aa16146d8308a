// tools/crc_variants.hip -- A/B timing of batched CRC kernel variants
// (measurement only; the product instantiates one variant in libzcrc).
// Interleaves variants in one process (guide 5.4 rule 24).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../zipsfs_amd/csrc/zcrc_batch_kernel.h"
#include "../zipsfs_amd/csrc/zcrc_tables.h"

#define CHECK(x)                                                                               \
  do {                                                                                         \
    hipError_t e = (x);                                                                        \
    if (e != hipSuccess) {                                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));         \
      exit(1);                                                                                 \
    }                                                                                          \
  } while (0)

using namespace zcrc;
typedef void (*kfn)(BatchArgs);

static float time_it(kfn k, const BatchArgs &a, int cus, int reps) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k, dim3(cus), dim3(kThreads), 0, 0, a);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k, dim3(cus), dim3(kThreads), 0, 0, a);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main(int argc, char **argv) {
  const uint64_t nbuf = argc > 1 ? strtoull(argv[1], 0, 0) : 16384;
  const uint64_t len = argc > 2 ? strtoull(argv[2], 0, 0) : (1u << 20);
  const int reps = argc > 3 ? atoi(argv[3]) : 10;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint8_t *data;
  uint32_t *out, *ref;
  TableBlob *d_tab;
  static TableBlob tb;
  build_tables(tb);
  CHECK(hipMalloc(&data, nbuf * len));
  CHECK(hipMalloc(&out, nbuf * 4));
  CHECK(hipMalloc(&ref, nbuf * 4));
  CHECK(hipMalloc(&d_tab, sizeof(TableBlob)));
  CHECK(hipMemcpy(d_tab, &tb, sizeof(TableBlob), hipMemcpyHostToDevice));
  // payload: any non-trivial bytes will do for timing
  uint64_t *hp = (uint64_t *)malloc(nbuf * 8), *hl = (uint64_t *)malloc(nbuf * 8);
  for (uint64_t i = 0; i < nbuf; i++) hp[i] = (uint64_t)(data + i * len), hl[i] = len;
  uint64_t *dp, *dl;
  CHECK(hipMalloc(&dp, nbuf * 8));
  CHECK(hipMalloc(&dl, nbuf * 8));
  CHECK(hipMemcpy(dp, hp, nbuf * 8, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dl, hl, nbuf * 8, hipMemcpyHostToDevice));
  CHECK(launch_fill_synthetic(dp, dl, nbuf, 0, 1, 0xC0FFEE, 0));
  CHECK(hipDeviceSynchronize());
  BatchArgs a{};
  a.base = data;
  a.stride = len;
  a.len = len;
  a.n = nbuf;
  a.tab = d_tab;
  const double bytes = (double)nbuf * len;
  printf("crc_variants: %llu x %llu B (%.1f GiB), %d CUs, %d reps\n", (unsigned long long)nbuf,
         (unsigned long long)len, bytes / (1 << 30), cus, reps);
  struct V {
    const char *name;
    kfn k;
    bool check;
  } vs[] = {
      {"D=4", crc32_batch_kernel<true, 4, 0, true>, true},
      {"D=3", crc32_batch_kernel<true, 3, 0, true>, true},
      {"D=4 ablate", crc32_batch_kernel<true, 4, 1, true>, false},
  };
  const uint64_t ranges[] = {16384, 32768, 65536, 262144};
  a.out = ref;
  hipLaunchKernelGGL((crc32_batch_kernel<true, 4, 0, false>), dim3(cus), dim3(kThreads), 0, 0, a);
  CHECK(hipDeviceSynchronize());
  uint32_t *h_ref = (uint32_t *)malloc(nbuf * 4), *h_out = (uint32_t *)malloc(nbuf * 4);
  CHECK(hipMemcpy(h_ref, ref, nbuf * 4, hipMemcpyDeviceToHost));
  a.out = out;
  for (int round = 0; round < 2; round++) {
    for (uint64_t mr : ranges)
    for (auto &v : vs) {
      a.min_range = mr;
      const float ms = time_it(v.k, a, cus, reps);
      int bad = 0;
      if (v.check) {
        CHECK(hipMemcpy(h_out, out, nbuf * 4, hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < nbuf; i++) bad += h_out[i] != h_ref[i];
      }
      printf("round %d  min_range %7llu  %-12s %8.3f ms  %8.1f GB/s  %s\n", round, (unsigned long long)mr, v.name, ms, bytes / (ms * 1e-3) / 1e9,
             v.check ? (bad ? "MISMATCH" : "ok") : "-");
      fflush(stdout);
    }
  }
  return 0;
}
