// tools/plan_probe.hip -- measurement tooling (not product): the split plan
// (plan_split_count + plan_split_scatter, zcrc_kernels.hip) alone, on
// config-4 lengths or uniform ones: GPU time per plan over back-to-back
// launches (events around the loop), then one launch with the scatter's
// diagnostic phase stamps (SplitPlan::stamps, s_memrealtime at 100 MHz):
// loads + tile sums | decision | scans and ballots | class scan | stores.
// One JSON line per tile size (1024 x per buffers per workgroup, per = 8, 4,
// 2, 1; the product's is kSplitPerThread), interleaved over `rounds`.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o plan_probe plan_probe.hip
//   plan_probe [n] [len|0=config-4 law] [reps] [rounds]
#include "../zipsfs_amd/csrc/zcrc_kernels.hip"

#include <vector>

using namespace zcrc;

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

static uint64_t zipf_len(uint64_t i) {
  uint64_t z = (0x5A1F5EEDull ^ ((i + 1) * 0xD1B54A32D192ED03ull)) + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  const double u = (double)(z >> 11) * (1.0 / 9007199254740992.0), t = 1.0 - u * 127.0 / 128.0;
  const double L = 1024.0 / (t * t);
  return (uint64_t)(L < 1024.0 ? 1024.0 : (L > 16777216.0 ? 16777216.0 : L));
}

int main(int argc, char **argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 0) : 100000;
  const uint64_t len = argc > 2 ? strtoull(argv[2], 0, 0) : 0;
  const int reps = argc > 3 ? atoi(argv[3]) : 50;
  const int rounds = argc > 4 ? atoi(argv[4]) : 1;
  std::vector<uint64_t> lens(n), ptrs(n);
  uint64_t off = 0;
  for (uint64_t i = 0; i < n; i++) {
    lens[i] = len ? len : zipf_len(i);
    ptrs[i] = 0x100000000ull + off;  // never dereferenced by the plan
    off += (lens[i] + 15) & ~15ull;
  }
  const uint64_t tiles = n == 0 ? 1 : (n + 1023) / 1024;  // the most tiles (per = 1): scratch and stamps
  uint64_t *d_lens, *d_ptrs, *d_stamps;
  uint8_t *scratch;
  uint32_t *d_out;
  const size_t sbytes = 256 + 8 * (n + 1) + 8 * kTileWords * tiles + 8 * kTileWords * (tiles + 1) + 32 * n + 16;
  CK(hipMalloc(&d_lens, 8 * n));
  CK(hipMalloc(&d_ptrs, 8 * n));
  CK(hipMalloc(&scratch, sbytes));
  CK(hipMalloc(&d_out, 4 * n));
  CK(hipMalloc(&d_stamps, 64 * tiles));
  CK(hipMemcpy(d_lens, lens.data(), 8 * n, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_ptrs, ptrs.data(), 8 * n, hipMemcpyHostToDevice));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  SplitPlan p{};
  const size_t prefix = 256, tl = prefix + 8 * (n + 1), tp = tl + 8 * kTileWords * tiles,
               pc = tp + 8 * kTileWords * (tiles + 1), sc = pc + 8 * n, oi = sc + 4 * n, si = (oi + 4 * n + 15) & ~size_t(15);
  p.ptrs = reinterpret_cast<const uint8_t *const *>(d_ptrs);
  p.lens = d_lens;
  p.n = n;
  p.tile_sum = reinterpret_cast<uint64_t *>(scratch + tl);
  p.tile_pre = reinterpret_cast<uint64_t *>(scratch + tp);
  p.prefix_c = reinterpret_cast<uint64_t *>(scratch + prefix);
  p.ptrs_c = reinterpret_cast<const uint8_t **>(scratch + pc);
  p.seeds_c = reinterpret_cast<uint32_t *>(scratch + sc);
  p.oidx = reinterpret_cast<uint32_t *>(scratch + oi);
  p.sdesc = reinterpret_cast<uint4 *>(scratch + si);
  p.out = d_out;
  p.counts = reinterpret_cast<uint64_t *>(scratch + 128);
  p.ctr = reinterpret_cast<uint32_t *>(scratch);
  p.grid = (uint32_t)cus;
  p.small_cost = kSmallCostDefault;
  p.big_min = kBigMin;
  p.direct_ok = getenv("ZCRC_SMALL_DIRECT") == nullptr || getenv("ZCRC_SMALL_DIRECT")[0] != '0';
  auto run = [&](int per) {
    auto launch = [&]() {
      switch (per) {
        case 8: CK(launch_plan_split_t<8>(p, 0)); break;
        case 4: CK(launch_plan_split_t<4>(p, 0)); break;
        case 2: CK(launch_plan_split_t<2>(p, 0)); break;
        default: CK(launch_plan_split_t<1>(p, 0)); break;
      }
    };
    const uint64_t nt = n == 0 ? 1 : (n + 1024u * per - 1) / (1024u * per);
    p.stamps = nullptr;
    for (int r = 0; r < 5; r++) launch();
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; r++) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    p.stamps = d_stamps;
    launch();
    CK(hipDeviceSynchronize());
    std::vector<uint64_t> st(8 * nt);
    CK(hipMemcpy(st.data(), d_stamps, 64 * nt, hipMemcpyDeviceToHost));
    uint64_t t0 = ~0ull, tend = 0;
    double ph[5] = {0, 0, 0, 0, 0};
    for (uint64_t b = 0; b < nt; b++) {
      t0 = std::min(t0, st[8 * b]);
      tend = std::max(tend, st[8 * b + 5]);
      for (int i = 0; i < 5; i++) ph[i] += (double)(st[8 * b + i + 1] - st[8 * b + i]) * 0.01 / nt;  // 100 MHz -> us
    }
    uint64_t counts[5];
    CK(hipMemcpy(counts, scratch + 128, 40, hipMemcpyDeviceToHost));
    printf("{\"n\": %llu, \"len\": %llu, \"per\": %d, \"tiles\": %llu, \"plan_us\": %.2f, \"split\": %llu, "
           "\"n_large\": %llu, \"n_small\": %llu, \"scatter_span_us\": %.2f, \"phase_us\": {\"loads_tiles\": %.2f, "
           "\"decision\": %.2f, \"scans_ballots\": %.2f, \"class_scan\": %.2f, \"stores\": %.2f}}\n",
           (unsigned long long)n, (unsigned long long)len, per, (unsigned long long)nt, ms * 1e3 / reps,
           (unsigned long long)counts[2], (unsigned long long)counts[0], (unsigned long long)counts[1],
           (double)(tend - t0) * 0.01, ph[0], ph[1], ph[2], ph[3], ph[4]);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
  };
  for (int r = 0; r < rounds; r++)
    for (int per : {8, 4, 2, 1}) run(per);
  return 0;
}
