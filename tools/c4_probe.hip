// tools/c4_probe.hip -- where does a config-4 step (100k ZIP-entry-like
// buffers, 13.1 GB, the split plan + one batch-kernel launch) spend its
// time, and which waves make its tail?  (measurement only)
//
// Same buffers as bench.py --config 4 (zipf law, 16-B aligned, payload from
// fill_synthetic).  Per variant, interleaved rounds: the step (plan + CRC
// launch, events around `steps` back-to-back steps), the plan alone, and the
// CRC launch alone (its dispatch packet's timestamps).  Variants move the
// split's knobs: the small-list workgroups' cost weight (small_cost), the big
// class edge (big_min), the dynamic unit and A/B flags (ab_flags).  Then one stamped launch
// (kStamp build, s_memrealtime at 100 MHz): batch waves' entry, static
// range end and end, small-list waves' end, percentiles; the last 24 waves
// to finish with their pieces, dynamic units and static bytes; end p50 per
// wave slot.  Parity: every variant's CRCs equal, and 64 sampled buffers
// equal a bitwise host CRC.
//
//   make -C tools c4_probe && tools/c4_probe [rounds] [steps] [all|big|medium|nosmall]
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../zipsfs_amd/csrc/zcrc_kernels.hip"
#include "../zipsfs_amd/csrc/zcrc_tables.h"

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

using namespace zcrc;

static uint64_t zipf_len(uint64_t i) {  // bench.py zipf_lens
  uint64_t z = (0x5A1F5EEDull ^ ((i + 1) * 0xD1B54A32D192ED03ull)) + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  const double u = (double)(z >> 11) * (1.0 / 9007199254740992.0), t = 1.0 - u * 127.0 / 128.0;
  const double L = 1024.0 / (t * t);
  return (uint64_t)(L < 1024.0 ? 1024.0 : (L > 16777216.0 ? 16777216.0 : L));
}

static uint32_t crc_bitwise(const uint8_t *p, uint64_t n) {
  uint32_t c = 0xFFFFFFFFu;
  for (uint64_t i = 0; i < n; i++) {
    c ^= p[i];
    for (int b = 0; b < 8; b++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
  }
  return ~c;
}

static double pct(std::vector<double> v, double p) {
  if (v.empty()) return 0.0;
  std::sort(v.begin(), v.end());
  return v[(size_t)(p * (v.size() - 1))];
}

struct Variant {
  const char *name;
  uint32_t small_cost;
  uint64_t big_min;
  uint64_t dyn_unit;  // 0: kDynUnit
  uint32_t ab_flags;  // BatchArgs::ab_flags
};

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 3;
  const int steps = argc > 2 ? atoi(argv[2]) : 20;
  // argv[3]: which of config 4's buffers (all / big: >= 1 MiB / medium: 8 KiB <
  // len < 1 MiB / nosmall: > 8 KiB), or uniform1m (config 3's 1 MiB buffers,
  // ~13 GB), to see which class streams below config 3
  const std::string cls = argc > 3 ? argv[3] : "all";
  std::vector<uint64_t> law;
  for (uint64_t i = 0; i < 100000; i++) {
    const uint64_t L = zipf_len(i);
    const bool keep = cls == "all" || (cls == "big" && L >= (1u << 20)) ||
                      (cls == "medium" && L > 8192 && L < (1u << 20)) || (cls == "nosmall" && L > 8192);
    if (keep) law.push_back(L);
  }
  if (cls == "uniform1m") law.assign(12516, 1ull << 20);  // config 3's buffers, config 4's byte count
  const uint64_t n = law.size();
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  static TableBlob tb;
  build_tables(tb);
  TableBlob *d_tab;
  CK(hipMalloc(&d_tab, sizeof(TableBlob)));
  CK(hipMemcpy(d_tab, &tb, sizeof(TableBlob), hipMemcpyHostToDevice));

  std::vector<uint64_t> lens(n), offs(n), ptrs(n);
  uint64_t off = 0, total = 0;
  for (uint64_t i = 0; i < n; i++) {
    lens[i] = law[i];
    offs[i] = off;
    off += (lens[i] + 15) & ~15ull;
    total += lens[i];
  }
  uint8_t *data;
  CK(hipMalloc(&data, off + 16));
  for (uint64_t i = 0; i < n; i++) ptrs[i] = (uint64_t)(data + offs[i]);
  const uint64_t tiles = split_tiles(n);
  uint64_t *d_lens, *d_ptrs, *d_stamps;
  uint8_t *scratch;
  uint32_t *d_out;
  const size_t prefix = 256, tl = prefix + 8 * (n + 1), tp = tl + 8 * kTileWords * tiles,
               pc = tp + 8 * kTileWords * (tiles + 1), sc = pc + 8 * n, oi = sc + 4 * n,
               si = (oi + 4 * n + 15) & ~size_t(15), sbytes = si + 16 * n;
  const uint64_t nw = (uint64_t)cus * kWaves;
  CK(hipMalloc(&d_lens, 8 * n));
  CK(hipMalloc(&d_ptrs, 8 * n));
  CK(hipMalloc(&scratch, sbytes));
  CK(hipMalloc(&d_out, 4 * n));
  CK(hipMalloc(&d_stamps, 64 * nw));
  CK(hipMemset(scratch, 0, sbytes));
  CK(hipMemcpy(d_lens, lens.data(), 8 * n, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_ptrs, ptrs.data(), 8 * n, hipMemcpyHostToDevice));
  for (uint64_t k = 0; k < n; k += 4096)  // payload index = buffer index (bench.py, one rank)
    CK(launch_fill_synthetic(d_ptrs + k, d_lens + k, std::min<uint64_t>(4096, n - k), k, 1, 0xC0FFEEull, 0));
  CK(hipDeviceSynchronize());

  SplitPlan p{};
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
  p.direct_ok = 1;
  BatchArgs a{};
  a.ptrs = p.ptrs;
  a.ptrs_split = p.ptrs_c;
  a.prefix = p.prefix_c;
  a.out = d_out;
  a.n = n;
  a.n_dev = p.counts;
  a.oidx = p.oidx;
  a.lens = d_lens;
  a.sdesc = p.sdesc;
  a.tab = d_tab;
  a.ctr = p.ctr;
  a.dyn_shift = kDynAuto;
  a.fault = reinterpret_cast<uint32_t *>(scratch + kFaultByte);

  const Variant vs[] = {
      {"default", kSmallCostDefault, kBigMin, 0, 0},
      {"nojoin", kSmallCostDefault, kBigMin, 0, 4},
      {"cost28", 28, kBigMin, 0, 0},
      {"cost7", 7, kBigMin, 0, 0},
  };
  const int nv = (int)(sizeof vs / sizeof vs[0]);
  auto set = [&](const Variant &v) {
    p.small_cost = v.small_cost;
    p.big_min = v.big_min;
    a.dyn_unit = v.dyn_unit;
    a.ab_flags = v.ab_flags;
  };
  hipEvent_t e0, e1, k0, k1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&k0));
  CK(hipEventCreate(&k1));
  const dim3 grid((unsigned)cus), block(kThreads);
  std::vector<std::vector<double>> step_ms(nv), plan_ms(nv), kern_ms(nv);
  std::vector<uint32_t> ref(n), got(n);
  bool parity = true;
  for (int r = 0; r < rounds; r++) {
    for (int vi = 0; vi < nv; vi++) {
      set(vs[vi]);
      for (int s = 0; s < 3; s++) {  // warm
        CK(launch_plan_split(p, 0));
        CK(launch_batch(a, false, cus, 0, nullptr, nullptr, false));
      }
      CK(hipEventRecord(e0, 0));
      for (int s = 0; s < steps; s++) {
        CK(launch_plan_split(p, 0));
        CK(launch_batch(a, false, cus, 0, nullptr, nullptr, false));
      }
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      step_ms[vi].push_back(ms / steps);
      CK(hipEventRecord(e0, 0));
      for (int s = 0; s < steps; s++) CK(launch_plan_split(p, 0));
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      plan_ms[vi].push_back(ms / steps);
      double ksum = 0;
      for (int s = 0; s < 5; s++) {
        CK(launch_plan_split(p, 0));
        CK(launch_batch(a, false, cus, 0, k0, k1, false));
        CK(hipEventSynchronize(k1));
        CK(hipEventElapsedTime(&ms, k0, k1));
        ksum += ms;
      }
      kern_ms[vi].push_back(ksum / 5);
      CK(hipMemcpy(vi == 0 && r == 0 ? ref.data() : got.data(), d_out, 4 * n, hipMemcpyDeviceToHost));
      if (vi || r) parity = parity && got == ref;
    }
  }
  std::vector<uint8_t> hb;
  int host_ok = 0;
  for (int k = 0; k < 64; k++) {
    const uint64_t i = (uint64_t)k * 1553 % n;
    hb.resize(lens[i]);
    CK(hipMemcpy(hb.data(), data + offs[i], lens[i], hipMemcpyDeviceToHost));
    host_ok += crc_bitwise(hb.data(), lens[i]) == ref[i];
  }
  uint64_t counts[5];
  CK(hipMemcpy(counts, scratch + 128, 40, hipMemcpyDeviceToHost));
  printf("c4_probe (%s): %d CUs, n %llu, %.3f GB, rounds %d x %d steps; variants agree: %s; host CRC 64 sampled: "
         "%d/64\n",
         cls.c_str(), cus, (unsigned long long)n, total / 1e9, rounds, steps, parity ? "yes" : "NO", host_ok);
  for (int vi = 0; vi < nv; vi++) {
    std::string sm, pm, km;
    char b[32];
    for (double x : step_ms[vi]) snprintf(b, sizeof b, " %.4f", x), sm += b;
    for (double x : plan_ms[vi]) snprintf(b, sizeof b, " %.2f", x * 1e3), pm += b;
    for (double x : kern_ms[vi]) snprintf(b, sizeof b, " %.4f", x), km += b;
    printf("%-9s step ms%s | plan us%s | kernel ms%s | %.0f GB/s (best step)\n", vs[vi].name, sm.c_str(),
           pm.c_str(), km.c_str(), total / (*std::min_element(step_ms[vi].begin(), step_ms[vi].end()) * 1e-3) / 1e9);
  }

  // ---- stamped launches
  auto stamped = [&](const Variant &sv) {
    set(sv);
    CK(launch_plan_split(p, 0));
    CK(hipMemcpy(counts, scratch + 128, 40, hipMemcpyDeviceToHost));
    CK(hipMemset(d_stamps, 0, 64 * nw));
    BatchArgs as = a;
    as.stamps = d_stamps;
    hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, 0, true, true>), grid, block, 0, 0, k0, k1, 0, as);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    float ms;
    CK(hipEventElapsedTime(&ms, k0, k1));
    CK(hipMemcpy(got.data(), d_out, 4 * n, hipMemcpyDeviceToHost));
    std::vector<uint64_t> st(8 * nw);
    CK(hipMemcpy(st.data(), d_stamps, 64 * nw, hipMemcpyDeviceToHost));
    uint64_t t0 = ~0ull;
    for (uint64_t w = 0; w < nw; w++)
      if (st[8 * w + 1]) t0 = std::min(t0, st[8 * w + 4]);
    const uint32_t nsm = (uint32_t)counts[4];
    std::vector<double> entry, search, begin, send, end, s_begin, s_end, j_start, j_end, j_units;
    std::vector<double> slot_end[kWaves];
    struct Row {
      double end, send, search, claim;
      uint64_t w, pieces, dyn;
    };
    std::vector<double> searches, claims;
    std::vector<Row> rows;
    for (uint64_t w = 0; w < nw; w++) {
      if (!st[8 * w + 1]) continue;
      const double e = (st[8 * w + 1] - t0) * 1e-2;
      if (st[8 * w + 2] == ~0ull) {
        s_begin.push_back((st[8 * w + 0] - t0) * 1e-2);
        s_end.push_back(e);
        continue;
      }
      if (st[8 * w + 2] >> 63) {  // a small-list wave that joined the dynamic part
        s_begin.push_back((st[8 * w + 4] - t0) * 1e-2);
        j_start.push_back((st[8 * w + 3] - t0) * 1e-2);
        j_end.push_back(e);
        j_units.push_back((double)((st[8 * w + 2] >> 32) & 0x7FFFFFFFull));
        continue;
      }
      entry.push_back((st[8 * w + 4] - t0) * 1e-2);
      search.push_back((st[8 * w + 5] - t0) * 1e-2);
      begin.push_back((st[8 * w + 0] - t0) * 1e-2);
      const double se = st[8 * w + 3] ? (st[8 * w + 3] - t0) * 1e-2 : e;
      send.push_back(se);
      end.push_back(e);
      slot_end[w % kWaves].push_back(e);
      rows.push_back({e, se, st[8 * w + 6] * 1e-2, st[8 * w + 7] * 1e-2, w, st[8 * w + 2] & 0xFFFFFFFFull,
                      st[8 * w + 2] >> 32});
      searches.push_back(st[8 * w + 6] * 1e-2);
      claims.push_back(st[8 * w + 7] * 1e-2);
    }
    printf("stamped launch (%s): %.2f us (events), CRCs %s; split %llu: %llu batch buffers, %llu small on %u workgroups "
           "(%u lanes each)\n",
           sv.name, ms * 1e3, got == ref ? "equal" : "DIFFER", (unsigned long long)counts[2], (unsigned long long)counts[0],
           (unsigned long long)counts[1], nsm, (unsigned)counts[3]);
    printf("us after first entry      p0      p10     p50     p90     p99    p100\n");
    auto row = [&](const char *k, const std::vector<double> &v) {
      printf("  %-20s %7.1f %7.1f %7.1f %7.1f %7.1f %7.1f\n", k, pct(v, 0), pct(v, .1), pct(v, .5), pct(v, .9),
             pct(v, .99), pct(v, 1));
    };
    row("batch entry", entry);
    row("batch search", search);
    row("batch begin", begin);
    row("batch static end", send);
    row("batch end", end);
    row("small begin", s_begin);
    row("small end", s_end);
    row("joined at", j_start);
    row("joined: end", j_end);
    row("joined: units", j_units);
    row("unit searches (sum)", searches);
    row("claim waits (sum)", claims);
    std::sort(rows.begin(), rows.end(), [](const Row &x, const Row &y) { return x.end > y.end; });
    printf("last waves: w (cu, slot) end | static end | pieces dyn_units | unit searches, claim waits (us)\n");
    for (size_t i = 0; i < rows.size() && i < 24; i++)
      printf("  %5llu (%3llu,%2llu) %7.1f | %7.1f | %5llu %3llu | %6.1f %6.1f\n", (unsigned long long)rows[i].w,
             (unsigned long long)(rows[i].w / kWaves), (unsigned long long)(rows[i].w % kWaves), rows[i].end,
             rows[i].send, (unsigned long long)rows[i].pieces, (unsigned long long)rows[i].dyn, rows[i].search,
             rows[i].claim);
    printf("end p50 by wave slot:");
    for (int s = 0; s < kWaves; s++) printf(" %.0f", pct(slot_end[s], .5));
    printf("\n");
  };
  stamped(vs[0]);
  stamped(vs[1]);
  return 0;
}
