// tools/small_probe.hip -- same-process A/B of the batched CRC kernel on
// small-buffer shapes (measurement only): uniform batches of 1..64 KiB
// buffers and the SURVEY 8(d) config-4 Zipf batch: piece descriptors read
// per piece against 64 at a time (kWin, zcrc_batch_kernel.h).  Two distinct >= 1 GiB batches per shape are rotated so the
// MALL cannot serve repeats; every launch is timed by its own dispatch packet
// (hipExtLaunchKernelGGL events); results of every variant are compared with
// the first variant (itself pinned by the GPU parity tests).
//
//   make -C tools small_probe && tools/small_probe [reps]
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
typedef void (*kfn)(BatchArgs);

struct Variant {
  const char *name;
  kfn k;
};
static const Variant kVariants[] = {
    {"per-piece", crc32_batch_kernel<false, kDepth, 0, true, false, 1, kLoadNt, false, false>},
    {"window", crc32_batch_kernel<false, kDepth, 0, true, false, 1, kLoadNt, false, true>},
};
constexpr int kNumV = sizeof(kVariants) / sizeof(kVariants[0]);

static uint64_t zipf_len(uint64_t i) {  // SURVEY 8(d) config-4 law
  uint64_t z = (0x5A1F5EEDull ^ ((i + 1) * 0xD1B54A32D192ED03ull)) + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  const double u = (double)(z >> 11) * (1.0 / 9007199254740992.0), t = 1.0 - u * 127.0 / 128.0;
  double L = 1024.0 / (t * t);
  L = L < 1024.0 ? 1024.0 : (L > 16777216.0 ? 16777216.0 : L);
  return (uint64_t)L;
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
  uint32_t *d_ctr;
  CHECK(hipMalloc(&d_ctr, 256));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  printf("small_probe: %d CUs, %d reps per variant per batch, 2 batches per shape\n", cus, reps);
  const uint64_t shapes[] = {1024, 3000, 4096, 8192, 16384, 65536, 0};  // 0 = config 4
  for (uint64_t L : shapes) {
    std::vector<uint64_t> lens;
    if (L == 0) {
      for (uint64_t i = 0; i < 100000; i++) lens.push_back(zipf_len(i));
    } else {
      const uint64_t n = (1ull << 30) / L;
      lens.assign(n, L);
    }
    const uint64_t n = lens.size();
    uint64_t bytes = 0, padded = 0;
    for (uint64_t x : lens) bytes += x, padded += (x + 15) & ~15ull;
    uint8_t *data[2];
    uint64_t *dp[2], *dpre, *dl;
    uint32_t *out, *ref;
    std::vector<uint64_t> pre(n + 1, 0);
    for (uint64_t i = 0; i < n; i++) pre[i + 1] = pre[i] + lens[i];
    CHECK(hipMalloc(&dpre, 8 * (n + 1)));
    CHECK(hipMalloc(&dl, 8 * n));
    CHECK(hipMalloc(&out, 4 * n));
    CHECK(hipMalloc(&ref, 4 * n));
    CHECK(hipMemcpy(dpre, pre.data(), 8 * (n + 1), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dl, lens.data(), 8 * n, hipMemcpyHostToDevice));
    for (int b = 0; b < 2; b++) {
      CHECK(hipMalloc(&data[b], padded + 64));
      std::vector<uint64_t> hp(n);
      // odd start offsets: misaligned buffers as in real archives
      for (uint64_t i = 0, off = 0; i < n; i++) hp[i] = (uint64_t)(data[b] + off + (i % 7)), off += (lens[i] + 15) & ~15ull;
      // keep every buffer inside the allocation despite the offset
      CHECK(hipMalloc(&dp[b], 8 * n));
      CHECK(hipMemcpy(dp[b], hp.data(), 8 * n, hipMemcpyHostToDevice));
      CHECK(launch_fill_synthetic(dp[b], dl, n, 7 * b, 1, 0xC0FFEE, 0));
    }
    CHECK(hipDeviceSynchronize());
    auto run = [&](int v, int b, uint32_t *o, bool timed) -> float {
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
      hipExtLaunchKernelGGL(kVariants[v].k, dim3(cus), dim3(kThreads), 0, 0, timed ? e0 : nullptr,
                            timed ? e1 : nullptr, 0, a);
      CHECK(hipGetLastError());
      CHECK(hipDeviceSynchronize());
      float ms = 0;
      if (timed) CHECK(hipEventElapsedTime(&ms, e0, e1));
      return ms;
    };
    std::vector<double> sum(kNumV, 0);
    std::vector<int> bad(kNumV, 0);
    std::vector<uint32_t> h_ref(n), h_out(n);
    for (int b = 0; b < 2; b++) {
      run(0, b, ref, false);
      CHECK(hipMemcpy(h_ref.data(), ref, 4 * n, hipMemcpyDeviceToHost));
      for (int v = 0; v < kNumV; v++) {
        run(v, b, out, false);
        CHECK(hipMemcpy(h_out.data(), out, 4 * n, hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < n; i++) bad[v] += h_out[i] != h_ref[i];
      }
    }
    for (int r = 0; r < reps; r++)
      for (int v = 0; v < kNumV; v++)
        for (int b = 0; b < 2; b++) sum[v] += run(v, b, out, true);
    for (int v = 0; v < kNumV; v++) {
      const double ms = sum[v] / (2 * reps);
      printf("%-9s %-10s n %7llu  %8.3f ms  %7.1f GB/s  %s\n", L ? "uniform" : "config4", kVariants[v].name,
             (unsigned long long)n, ms, bytes / (ms * 1e-3) / 1e9, bad[v] ? "MISMATCH" : "equal");
      fflush(stdout);
    }
    for (int b = 0; b < 2; b++) {
      CHECK(hipFree(data[b]));
      CHECK(hipFree(dp[b]));
    }
    CHECK(hipFree(dpre));
    CHECK(hipFree(dl));
    CHECK(hipFree(out));
    CHECK(hipFree(ref));
  }
  return 0;
}
