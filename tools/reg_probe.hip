// tools/reg_probe.hip -- measurement tooling (not product): what it costs to
// get a ZIPsFS preload segment (an anonymous mmap filled by read(),
// src/ZIPsFS_preloadfileram.c:284-306) to the GPU.
//   * hipHostRegister / hipHostUnregister of the segment, before or after it
//     is filled, and the H2D DMA rate straight from it;
//   * memcpy into pinned staging (one core) + H2D from the pinned copy;
//   * hipMemcpy from pageable memory (the runtime's own staging).
// One JSON line per (size, rep).   hipcc --offload-arch=gfx950 -O2 -o reg_probe reg_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>

static double now_us() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

static char *seg_new(size_t n) {
  void *p = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) exit(1);
  return static_cast<char *>(p);
}

static void fill(char *p, size_t n, int v) {
  for (size_t o = 0; o < n; o += 16u << 20) memset(p + o, v, (n - o) < (16u << 20) ? (n - o) : (16u << 20));
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 3;
  const size_t sizes[] = {4u << 20, 16u << 20, 64u << 20, 256u << 20};
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  void *d = nullptr;
  CK(hipMalloc(&d, 256u << 20));
  char *pinned = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void **>(&pinned), 256u << 20, hipHostMallocDefault));
  memset(pinned, 1, 256u << 20);
  CK(hipMemcpy(d, pinned, 1 << 20, hipMemcpyHostToDevice));  // warm
  for (size_t n : sizes) {
    for (int r = 0; r < reps; r++) {
      // (a) filled segment, then register / DMA / unregister
      char *s = seg_new(n);
      double t = now_us();
      fill(s, n, r + 1);
      const double fill_us = now_us() - t;
      t = now_us();
      CK(hipHostRegister(s, n, hipHostRegisterDefault));
      const double reg_us = now_us() - t;
      t = now_us();
      CK(hipMemcpyAsync(d, s, n, hipMemcpyHostToDevice, st));
      CK(hipStreamSynchronize(st));
      const double dma_reg_us = now_us() - t;
      t = now_us();
      CK(hipHostUnregister(s));
      const double unreg_us = now_us() - t;
      // (b) register the untouched segment first (at open), then fill it
      char *s2 = seg_new(n);
      t = now_us();
      CK(hipHostRegister(s2, n, hipHostRegisterDefault));
      const double reg_empty_us = now_us() - t;
      t = now_us();
      fill(s2, n, r + 2);
      const double fill_after_reg_us = now_us() - t;
      t = now_us();
      CK(hipMemcpyAsync(d, s2, n, hipMemcpyHostToDevice, st));
      CK(hipStreamSynchronize(st));
      const double dma_reg2_us = now_us() - t;
      CK(hipHostUnregister(s2));
      munmap(s2, n);
      // (c) one-core memcpy into pinned staging, then DMA from it
      t = now_us();
      memcpy(pinned, s, n);
      const double memcpy_us = now_us() - t;
      t = now_us();
      CK(hipMemcpyAsync(d, pinned, n, hipMemcpyHostToDevice, st));
      CK(hipStreamSynchronize(st));
      const double dma_pinned_us = now_us() - t;
      // (d) pageable source: the runtime stages it
      t = now_us();
      CK(hipMemcpyAsync(d, s, n, hipMemcpyHostToDevice, st));
      CK(hipStreamSynchronize(st));
      const double dma_pageable_us = now_us() - t;
      munmap(s, n);
      printf("{\"mib\": %zu, \"rep\": %d, \"fill_us\": %.1f, \"register_filled_us\": %.1f, \"dma_registered_us\": %.1f, "
             "\"unregister_us\": %.1f, \"register_empty_us\": %.1f, \"fill_after_register_us\": %.1f, "
             "\"dma_registered_at_open_us\": %.1f, \"memcpy_to_pinned_us\": %.1f, \"dma_pinned_us\": %.1f, "
             "\"dma_pageable_us\": %.1f}\n",
             n >> 20, r, fill_us, reg_us, dma_reg_us, unreg_us, reg_empty_us, fill_after_reg_us, dma_reg2_us, memcpy_us,
             dma_pinned_us, dma_pageable_us);
      fflush(stdout);
    }
  }
  return 0;
}
