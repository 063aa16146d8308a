// crc_ab.hip -- same-process A/B of two versions of the batched CRC kernel
// (measurement tooling).  Box-to-box and run-to-run drift on MI355X is a few
// percent, larger than the differences worth measuring, so the two builds
// are compiled into one binary (tools/ab/va_body.h, vb_body.h from
// tools/ab/make_body.sh) and timed interleaved on the same buffers.
//
//   tools/ab/make_body.sh <rev> tools/ab/va_body.h && tools/ab/make_body.sh WT tools/ab/vb_body.h
//   make -C tools crc_ab && tools/crc_ab <nbuf> <len|0=zipf> <rounds>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "../zipsfs_amd/csrc/zcrc_gf2.h"
#include "../zipsfs_amd/csrc/zcrc_internal.h"
#include "../zipsfs_amd/csrc/zcrc_tables.h"

namespace va {
using namespace ::zcrc;
#include "ab/va_body.h"
}  // namespace va
namespace vb {
using namespace ::zcrc;
#include "ab/vb_body.h"
}  // namespace vb

namespace zcrc {
hipError_t launch_fill_synthetic(const uint64_t *d_ptrs, const uint64_t *d_lens, uint64_t n, uint64_t index0,
                                 uint64_t index_step, uint64_t seed, hipStream_t stream);
}
using namespace zcrc;

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

typedef void (*kfn)(BatchArgs);

static float time_one(kfn k, BatchArgs a, int cus) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipMemsetAsync(a.out, 0, a.n * 4, 0));
  CHECK(hipMemsetAsync(a.ctr, 0, 4, 0));
  CHECK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL(k, dim3(cus), dim3(kThreads), 0, 0, a);
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return ms;
}

int main(int argc, char **argv) {
  const uint64_t nbuf = argc > 1 ? strtoull(argv[1], 0, 0) : 65536;
  const uint64_t len = argc > 2 ? strtoull(argv[2], 0, 0) : (1u << 20);
  const int rounds = argc > 3 ? atoi(argv[3]) : 8;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  static TableBlob tb;
  build_tables(tb);
  std::vector<uint64_t> zl(nbuf);
  uint64_t tot = 0;
  for (uint64_t i = 0; i < nbuf; i++) {
    if (len == 0) {  // SURVEY 8(d) config-4 law
      uint64_t z = (0x5A1F5EEDull ^ ((i + 1) * 0xD1B54A32D192ED03ull)) + 0x9E3779B97F4A7C15ull;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      z ^= z >> 31;
      const double u = (double)(z >> 11) * (1.0 / 9007199254740992.0), t = 1.0 - u * 127.0 / 128.0;
      double L = 1024.0 / (t * t);
      zl[i] = (uint64_t)(L < 1024.0 ? 1024.0 : (L > 16777216.0 ? 16777216.0 : L));
    } else {
      zl[i] = len;
    }
    tot += (zl[i] + 15) & ~15ull;
  }
  uint8_t *data;
  uint32_t *outa, *outb, *ctr;
  TableBlob *d_tab;
  CHECK(hipMalloc(&data, tot));
  CHECK(hipMalloc(&outa, nbuf * 4));
  CHECK(hipMalloc(&outb, nbuf * 4));
  CHECK(hipMalloc(&ctr, 256));
  CHECK(hipMalloc(&d_tab, sizeof(TableBlob)));
  CHECK(hipMemcpy(d_tab, &tb, sizeof(TableBlob), hipMemcpyHostToDevice));
  std::vector<uint64_t> hp(nbuf), prefix(nbuf + 1, 0);
  for (uint64_t i = 0, off = 0; i < nbuf; i++) hp[i] = (uint64_t)(data + off), off += (zl[i] + 15) & ~15ull;
  for (uint64_t i = 0; i < nbuf; i++) prefix[i + 1] = prefix[i] + zl[i];
  uint64_t *dp, *dl, *dpre;
  CHECK(hipMalloc(&dp, nbuf * 8));
  CHECK(hipMalloc(&dl, nbuf * 8));
  CHECK(hipMalloc(&dpre, (nbuf + 1) * 8));
  CHECK(hipMemcpy(dp, hp.data(), nbuf * 8, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dl, zl.data(), nbuf * 8, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dpre, prefix.data(), (nbuf + 1) * 8, hipMemcpyHostToDevice));
  CHECK(launch_fill_synthetic(dp, dl, nbuf, 0, 1, 0xC0FFEE, 0));
  CHECK(hipDeviceSynchronize());
  BatchArgs a{};
  a.ptrs = reinterpret_cast<const uint8_t *const *>(dp);
  a.prefix = dpre;
  a.lens = dl;  // round 3: the kernel checks each piece's prefix bounds against the lengths
  a.n = nbuf;
  a.tab = d_tab;
  a.ctr = ctr;
  a.dyn_shift = kDynShift;
  uint64_t *acc;
  uint32_t *done;
  CHECK(hipMalloc(&acc, 8 * kFusedMaxN));
  CHECK(hipMalloc(&done, 256));
  CHECK(hipMemset(acc, 0, 8 * kFusedMaxN));
  CHECK(hipMemset(done, 0, 256));
  a.acc = acc;  // fused form only (AB_FUSED): split-piece cells and the finished-wave counter
  a.done = done;
  const double bytes = (double)prefix[nbuf];
  printf("crc_ab: %llu buffers, %.2f GiB (%s), %d CUs, %d rounds\n", (unsigned long long)nbuf, bytes / (1 << 30),
         len ? "uniform" : "zipf", cus, rounds);
  // AB_B_NOWIN: B is the working tree's kernel with the piece-descriptor
  // windows off (kWin = false)
#if defined(AB_FUSED)
  // AB_FUSED: both one-launch kernels (n <= 16 x CUs; the per-buffer mode
  // when no buffer exceeds 64 KiB, else the in-kernel scan)
  kfn ka = va::crc32_batch_kernel<false, 4u, 0, true, false, 1, 2, true>;
  kfn kb = vb::crc32_batch_kernel<false, 4u, 0, true, false, 1, 2, true>;
#elif defined(AB_B_NOWIN)
  kfn ka = va::crc32_batch_kernel<false, 4u, 0, true, false, 1, 2>;
  kfn kb = vb::crc32_batch_kernel<false, 4u, 0, true, false, 1, 2, false, false>;
#else
  kfn ka = va::crc32_batch_kernel<false, 4u, 0, true, false, 1, 2>;
  kfn kb = vb::crc32_batch_kernel<false, 4u, 0, true, false, 1, 2>;
#endif
  BatchArgs aa = a, ab = a;
  aa.out = outa;
  ab.out = outb;
  (void)time_one(ka, aa, cus);
  (void)time_one(kb, ab, cus);
  std::vector<float> ta, tb2;
  for (int r = 0; r < rounds; r++) {  // A B B A ... cancels drift
    if (r & 1) {
      tb2.push_back(time_one(kb, ab, cus));
      ta.push_back(time_one(ka, aa, cus));
    } else {
      ta.push_back(time_one(ka, aa, cus));
      tb2.push_back(time_one(kb, ab, cus));
    }
  }
  std::vector<uint32_t> ha(nbuf), hb(nbuf);
  CHECK(hipMemcpy(ha.data(), outa, nbuf * 4, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(hb.data(), outb, nbuf * 4, hipMemcpyDeviceToHost));
  uint64_t bad = 0;
  for (uint64_t i = 0; i < nbuf; i++) bad += ha[i] != hb[i];
  auto med = [](std::vector<float> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
  auto mean = [](const std::vector<float> &v) { double s = 0; for (float x : v) s += x; return s / v.size(); };
  printf("A: median %.3f ms mean %.3f ms (%.1f GB/s)\n", med(ta), mean(ta), bytes / (med(ta) * 1e-3) / 1e9);
  printf("B: median %.3f ms mean %.3f ms (%.1f GB/s)\n", med(tb2), mean(tb2), bytes / (med(tb2) * 1e-3) / 1e9);
  printf("B/A median %.4f  outputs %s\n", med(tb2) / med(ta), bad ? "DIFFER" : "equal");
  return 0;
}
