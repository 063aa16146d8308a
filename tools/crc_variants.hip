// tools/crc_variants.hip -- A/B timing of batched CRC kernel variants
// (measurement only; the product instantiates one variant in libzcrc).
// Interleaves variants in one process (guide 5.4 rule 24).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "../zipsfs_amd/csrc/zcrc_batch_kernel.h"
#include "../zipsfs_amd/csrc/zcrc_tables.h"
#include "ab/kernel_v1.h"  // generated: tools/ab/make_v1.sh (make -C tools crc_variants)

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
  const uint64_t nb = a.n;
  CHECK(hipMemsetAsync(a.out, 0, nb * 4, 0));
  if (a.ctr) CHECK(hipMemsetAsync(a.ctr, 0, 4, 0));
  hipLaunchKernelGGL(k, dim3(cus), dim3(kThreads), 0, 0, a);
  CHECK(hipDeviceSynchronize());
  float total = 0;
  for (int r = 0; r < reps; r++) {
    // per-launch reset of the work counter and of out[] (split pieces xor into
    // it); the memsets are outside the timed interval
    CHECK(hipMemsetAsync(a.out, 0, nb * 4, 0));
    if (a.ctr) CHECK(hipMemsetAsync(a.ctr, 0, 4, 0));
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k, dim3(cus), dim3(kThreads), 0, 0, a);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    total += ms;
  }
  return total / reps;
  CHECK(hipEventRecord(e0, 0));
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
  const bool zipf = (len == 0);
  std::vector<uint64_t> zl(nbuf);
  uint64_t tot = 0;
  for (uint64_t i = 0; i < nbuf; i++) {
    if (zipf) {  // SURVEY 8(d) config-4 law
      uint64_t z = (0x5A1F5EEDull ^ ((i + 1) * 0xD1B54A32D192ED03ull)) + 0x9E3779B97F4A7C15ull;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      z ^= z >> 31;
      const double u = (double)(z >> 11) * (1.0 / 9007199254740992.0), t = 1.0 - u * 127.0 / 128.0;
      double L = 1024.0 / (t * t);
      L = L < 1024.0 ? 1024.0 : (L > 16777216.0 ? 16777216.0 : L);
      zl[i] = (uint64_t)L;
    } else {
      zl[i] = len;
    }
    tot += (zl[i] + 15) & ~15ull;
  }
  CHECK(hipMalloc(&data, tot));
  CHECK(hipMalloc(&out, nbuf * 4));
  CHECK(hipMalloc(&ref, nbuf * 4));
  CHECK(hipMalloc(&d_tab, sizeof(TableBlob)));
  CHECK(hipMemcpy(d_tab, &tb, sizeof(TableBlob), hipMemcpyHostToDevice));
  // payload: any non-trivial bytes will do for timing
  uint64_t *hp = (uint64_t *)malloc(nbuf * 8), *hl = (uint64_t *)malloc(nbuf * 8);
  for (uint64_t i = 0, off = 0; i < nbuf; i++) hp[i] = (uint64_t)(data + off), hl[i] = zl[i], off += (zl[i] + 15) & ~15ull;
  uint64_t *dp, *dl;
  CHECK(hipMalloc(&dp, nbuf * 8));
  CHECK(hipMalloc(&dl, nbuf * 8));
  CHECK(hipMemcpy(dp, hp, nbuf * 8, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dl, hl, nbuf * 8, hipMemcpyHostToDevice));
  CHECK(launch_fill_synthetic(dp, dl, nbuf, 0, 1, 0xC0FFEE, 0));
  CHECK(hipDeviceSynchronize());
  // general (pointer-array) form with a host-computed prefix, like
  // zcrc32_batch_device after its plan kernel
  std::vector<uint64_t> hprefix(nbuf + 1, 0);
  for (uint64_t i = 0; i < nbuf; i++) hprefix[i + 1] = hprefix[i] + hl[i];
  uint64_t *dprefix;
  CHECK(hipMalloc(&dprefix, (nbuf + 1) * 8));
  CHECK(hipMemcpy(dprefix, hprefix.data(), (nbuf + 1) * 8, hipMemcpyHostToDevice));
  BatchArgs a{};
  a.ptrs = reinterpret_cast<const uint8_t *const *>(dp);
  a.prefix = dprefix;
  a.n = nbuf;
  a.tab = d_tab;
  const double bytes = (double)hprefix[nbuf];
  printf("crc_variants: %llu buffers, %.2f GiB (%s), %d CUs, %d reps\n", (unsigned long long)nbuf,
         bytes / (1 << 30), zipf ? "zipf" : "uniform", cus, reps);
  struct V {
    const char *name;
    kfn k;
    bool check;
    uint32_t dyn;
    uint64_t unit;
  } vs[] = {
      {"static-dflt", crc32_batch_kernel<false, 4, 0, true, false, 0, 0>, true, 0, 0},
      {"product-dflt", crc32_batch_kernel<false, 4, 0, true, false, 1, 0>, true, kDynShift, kDynUnit},
      {"static", crc32_batch_kernel<false, 4, 0, true, false, 0>, true, 0, 0},
      {"prio", crc32_batch_kernel<false, 4, 0, true, false, 1>, true, 0, 0},
      {"product", crc32_batch_kernel<false, 4, 0, true, false, 1>, true, kDynShift, kDynUnit},
      {"product+sc1nt", crc32_batch_kernel<false, 4, 0, true, false, 1, 18>, true, kDynShift, kDynUnit},
      {"prod-u256k", crc32_batch_kernel<false, 4, 0, true, false, 1>, true, kDynShift, 256u << 10},
      {"prod-u512k", crc32_batch_kernel<false, 4, 0, true, false, 1>, true, kDynShift, 512u << 10},
      {"prod-q", crc32_batch_kernel<false, 4, 0, true, false, 1>, true, 2, kDynUnit},
      {"prod-q-u512k", crc32_batch_kernel<false, 4, 0, true, false, 1>, true, 2, 512u << 10},
      {"prod-8th", crc32_batch_kernel<false, 4, 0, true, false, 1>, true, 3, kDynUnit},
  };
  uint32_t *d_counter;
  CHECK(hipMalloc(&d_counter, 32));
  CHECK(hipMemset(d_counter, 0, 32));
  a.ctr = d_counter;

  const uint64_t ranges[] = {65536};
  uint32_t *h_ref = (uint32_t *)malloc(nbuf * 4), *h_out = (uint32_t *)malloc(nbuf * 4);
  a.out = ref;
  CHECK(hipMemset(ref, 0, nbuf * 4));
  CHECK(hipMemset(d_counter, 0, 32));
  hipLaunchKernelGGL((crc32_batch_kernel<false, 4, 0, true, false, 0>), dim3(cus), dim3(kThreads), 0, 0, a);
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(h_ref, ref, nbuf * 4, hipMemcpyDeviceToHost));
  a.out = out;
  // stamp runs: per-wave wall-clock begin/end (100 MHz)
  auto stamp_run = [&](const char *name, kfn k, uint32_t dyn, uint64_t unit) {
    a.dyn_shift = dyn;
    a.dyn_unit = unit;
    const uint64_t nw = (uint64_t)cus * kWaves;
    uint64_t *dst;
    CHECK(hipMalloc(&dst, nw * 64));
    CHECK(hipMemset(dst, 0, nw * 64));
    CHECK(hipMemset(d_counter, 0, 32));
    a.stamps = dst;
    hipLaunchKernelGGL(k, dim3(cus), dim3(kThreads), 0, 0, a);
    CHECK(hipDeviceSynchronize());
    std::vector<uint64_t> st8(nw * 8), st(nw * 4);
    CHECK(hipMemcpy(st8.data(), dst, nw * 64, hipMemcpyDeviceToHost));
    for (uint64_t w = 0; w < nw; w++)
      for (int k = 0; k < 4; k++) st[4 * w + k] = st8[8 * w + k];
    {  // prologue: kernel entry -> range search done -> LDS written + barrier
      uint64_t e0 = ~0ull, e1 = 0, b0 = ~0ull;
      std::vector<double> fill, srch;  // search (table loads in flight), then LDS writes + barrier
      for (uint64_t w = 0; w < nw; w++)
        if (st8[8 * w + 1]) {
          e0 = std::min(e0, st8[8 * w + 4]), e1 = std::max(e1, st8[8 * w + 4]), b0 = std::min(b0, st8[8 * w]);
          srch.push_back((st8[8 * w + 5] - st8[8 * w + 4]) * 1e-2);
          fill.push_back((st8[8 * w + 0] - st8[8 * w + 5]) * 1e-2);
        }
      std::sort(fill.begin(), fill.end());
      std::sort(srch.begin(), srch.end());
      {
        double us = 0, mx = 0;
        uint64_t cnt = 0;
        for (uint64_t w = 0; w < nw; w++)
          if (st8[8 * w + 1]) us += st8[8 * w + 6] * 1e-2, mx = std::max(mx, st8[8 * w + 6] * 1e-2), cnt++;
        double dr = 0;
        for (uint64_t w = 0; w < nw; w++)
          if (st8[8 * w + 1]) dr += st8[8 * w + 7] * 1e-2;
        double tl = 0;
        for (uint64_t w = 0; w < nw; w++)
          if (st8[8 * w + 1]) tl += st8[8 * w + 3] * 1e-2;
        printf("unit searches %-8s mean %.1f us per wave, max %.1f us; draining stores first %.1f us per wave; "
               "padding MCTs %.1f us per wave\n",
               name, us / (cnt ? cnt : 1), mx, dr / (cnt ? cnt : 1), tl / (cnt ? cnt : 1));
      }
      printf("prologue %-8s entry spread %.1f us | first entry->first begin %.1f us | search us p50 %.1f p100 %.1f | "
             "LDS fill us p50 %.1f p100 %.1f\n", name, (e1 - e0) * 1e-2, (b0 - e0) * 1e-2, srch[srch.size() / 2],
             srch.back(), fill[fill.size() / 2], fill.back());
    }
    uint64_t t0 = ~0ull, t1 = 0;
    for (uint64_t w = 0; w < nw; w++)
      if (st[4 * w + 1]) t0 = std::min(t0, st[4 * w]), t1 = std::max(t1, st[4 * w + 1]);
    std::vector<double> dur, endt;
    double c2 = 0, c3 = 0;
    for (uint64_t w = 0; w < nw; w++)
      if (st[4 * w + 1]) {
        dur.push_back((st[4 * w + 1] - st[4 * w]) * 1e-2);
        endt.push_back((st[4 * w + 1] - t0) * 1e-2);
        c2 += st[4 * w + 2];
        c3 += st[4 * w + 3];
      }
    std::sort(dur.begin(), dur.end());
    std::sort(endt.begin(), endt.end());
    auto pct = [](const std::vector<double> &v, double p) { return v[(size_t)(p * (v.size() - 1))]; };
    printf("stamps %-8s waves %zu span %.1f us | wave us p0 %.1f p10 %.1f p50 %.1f p90 %.1f p100 %.1f | end us p10 %.1f p50 %.1f p90 %.1f | w2 %.1f w3 %.1f\n",
           name, dur.size(), (t1 - t0) * 1e-2, pct(dur, 0), pct(dur, .1), pct(dur, .5), pct(dur, .9), pct(dur, 1),
           pct(endt, .1), pct(endt, .5), pct(endt, .9), c2 / dur.size(), c3 / dur.size());
    // where does the spread live?  by wave slot inside the WG, by XCD, and
    // within-WG spread vs spread of WG means
    {
      double slot[kWaves] = {0}, xcd[8] = {0};
      int nslot[kWaves] = {0}, nxcd[8] = {0};
      std::vector<double> wg_mean, wg_spread;
      for (uint64_t g = 0; g < (uint64_t)cus; g++) {
        double s = 0, mn = 1e30, mx = 0;
        int c = 0;
        for (uint32_t w = 0; w < kWaves; w++) {
          const uint64_t i = g * kWaves + w;
          if (!st[4 * i + 1]) continue;
          const double e = (st[4 * i + 1] - t0) * 1e-2;
          slot[w] += e, nslot[w]++;
          xcd[g % 8] += e, nxcd[g % 8]++;
          s += e, c++, mn = std::min(mn, e), mx = std::max(mx, e);
        }
        if (c) wg_mean.push_back(s / c), wg_spread.push_back(mx - mn);
      }
      printf("  end us by wave slot:");
      for (uint32_t w = 0; w < kWaves; w++) printf(" %.0f", nslot[w] ? slot[w] / nslot[w] : 0.0);
      printf("\n  end us by xcd:");
      for (int x = 0; x < 8; x++) printf(" %.0f", nxcd[x] ? xcd[x] / nxcd[x] : 0.0);
      std::sort(wg_mean.begin(), wg_mean.end());
      std::sort(wg_spread.begin(), wg_spread.end());
      printf("\n  WG mean end us p0 %.0f p50 %.0f p100 %.0f | within-WG spread us p10 %.0f p50 %.0f p90 %.0f\n",
             wg_mean.front(), pct(wg_mean, .5), wg_mean.back(), pct(wg_spread, .1), pct(wg_spread, .5),
             pct(wg_spread, .9));
    }
    a.stamps = nullptr;
    CHECK(hipFree(dst));
  };
  if (getenv("CRC_VARIANTS_STAMPS")) {
    stamp_run("static", crc32_batch_kernel<false, 4, 0, true, true, 0>, 0, 0);
    stamp_run("product", crc32_batch_kernel<false, 4, 0, true, true, 1>, kDynShift, kDynUnit);
  }
  for (int round = 0; round < 2; round++) {
    for (uint64_t mr : ranges)
    for (auto &v : vs) {
      a.min_range = mr;
      a.dyn_shift = v.dyn;
      a.dyn_unit = v.unit;
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
