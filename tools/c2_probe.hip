// tools/c2_probe.hip -- where does a config-2 launch (4096 x 64 KiB) spend
// its time?  (measurement only)
//
// 16 distinct 256 MiB batches are rotated so that the 256 MB MALL cannot
// serve repeats.  Every launch is timed by the timestamps of
// its own dispatch packet (hipExtLaunchKernelGGL), so the figures are kernel
// durations without queue gaps.  Variants:
//   probe-wave   pure-read kernel in the CRC kernel's shape: one 1024-thread
//                workgroup per CU, wave w reads buffer w (nt 16-B loads,
//                two groups of 4 KiB in flight), xor into one word
//   probe-grid   pure-read grid-stride sweep, 8 workgroups of 256 per CU
//   probe-pb     pure read in the per-buffer mode's mapping and 2 x 4 KiB
//                ping-pong, slot priorities as the product; -rot: each wave
//                starts at a hashed block of its buffer and wraps; -np:
//                no slot priorities; -fat: ~600 VALU before the first load
//   crc          the product kernel (prefix precomputed: the plan's output)
//   crc-fused    the one-launch kernel, per-buffer form 4 (tables built in
//                registers, the batch decided after the work)
//   crc-fused-r3 the round-3 per-buffer form (tables and lengths in front of
//                its one barrier)
//   crc-fused-N  per-buffer form N (crc32_batch_kernel's kPB): 5 = first
//                payload loads ahead of the table build; +10 priority by
//                progress, +20 none (instead of by wave slot); +100 / +200
//                6- / 8-block register groups.  15 is the product's form.
// and one stamped launch of each CRC form (s_memrealtime, 100 MHz) printed
// as a timeline: kernel entry, range search done, LDS fill + barrier done,
// wave end -- percentiles over all waves, relative to the first entry.  The
// per-buffer mode (crc-fused) stamps entry, its one barrier ("begin") and
// its buffer's CRC stored ("end").
//
//   make -C tools c2_probe && tools/c2_probe [reps]
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

constexpr uint64_t kN = 4096, kLen = 64u << 10, kBatchBytes = kN * kLen;
constexpr int kBatches = 16;

// wave w of the grid reads [w * per, (w + 1) * per) bytes of `base`
__global__ __launch_bounds__(1024) void probe_wave(const uint8_t *base, uint64_t per, uint32_t *out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t w = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(base + w * per), (short)0, (int)per, 0x00020000);
  uint32_t acc = 0;
  const uint32_t blocks = (uint32_t)(per >> 10);
  for (uint32_t b = 0; b < blocks; b += 8) {
    uint32_t v[8][4];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      auto x = __builtin_amdgcn_raw_buffer_load_b128(r, 1024u * (b + u) + 16u * lane, 0, 2);
      v[u][0] = x[0], v[u][1] = x[1], v[u][2] = x[2], v[u][3] = x[3];
    }
#pragma unroll
    for (int u = 0; u < 8; u++) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  if (acc == 0x12345678u) out[w] = acc;  // keep the loads
}

// The per-buffer mode's mapping (wave slot s of workgroup g reads buffer
// s * grid + g), 2 x 4 KiB ping-pong like the CRC loop; kRot: each wave
// starts at a hashed block of its buffer and wraps (the pure-read cost of a
// de-phased visit order)
// kFat: ~kFat straight-line VALU instructions (no memory) before the first
// load -- does a long prologue of code alone delay a launch's first loads
// (instruction fetch from a cold instruction cache)?
template <bool kRot, bool kPrio = true, int kFat = 0>
__global__ __launch_bounds__(1024) void probe_pb(const uint8_t *base, uint64_t per, uint32_t *out) {
  const uint32_t lane = threadIdx.x & 63u, slot = threadIdx.x >> 6;
  const uint64_t w = (uint64_t)slot * gridDim.x + blockIdx.x;
  uint32_t fat = lane;
#pragma unroll
  for (int f = 0; f < kFat; f++) fat = __builtin_amdgcn_alignbit(fat, fat ^ (uint32_t)(0x9E3779B9u * (f + 1)), 7);
  if (kFat && fat == 0x12345678u) out[w ^ 1] = fat;  // keep it
  if (kPrio) {
    if (slot >= 12) __builtin_amdgcn_s_setprio(3);
    else if (slot >= 8) __builtin_amdgcn_s_setprio(2);
    else if (slot >= 4) __builtin_amdgcn_s_setprio(1);
  }
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(base + w * per), (short)0, (int)per, 0x00020000);
  const uint32_t blocks = (uint32_t)(per >> 10);
  const uint32_t rot = kRot ? (uint32_t)((w * 0x9E3779B1u) >> 7) % blocks & ~3u : 0u;
  uint32_t acc = 0;
  uint32_t ga[4][4], gb[4][4];
  auto ld = [&](uint32_t (*G)[4], uint32_t g) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint32_t blk = (rot + 4 * g + u) % blocks;
      auto x = __builtin_amdgcn_raw_buffer_load_b128(r, 1024u * blk + 16u * lane, 0, 2);
      G[u][0] = x[0], G[u][1] = x[1], G[u][2] = x[2], G[u][3] = x[3];
    }
  };
  auto use = [&](uint32_t (*G)[4]) {
#pragma unroll
    for (int u = 0; u < 4; u++) acc ^= G[u][0] ^ G[u][1] ^ G[u][2] ^ G[u][3];
  };
  const uint32_t ng = blocks / 4;
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
  if (acc == 0x12345678u) out[w] = acc;  // keep the loads
}

__global__ __launch_bounds__(256) void probe_grid(const uint8_t *base, uint64_t bytes, uint32_t *out) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, 0x7FFFFFFF, 0x00020000);
  uint32_t acc = 0;
  const uint64_t step = (uint64_t)gridDim.x * blockDim.x * 16 * 4;
  for (uint64_t o = ((uint64_t)blockIdx.x * blockDim.x * 4 + threadIdx.x) * 16; o < bytes; o += step) {
    uint32_t v[4][4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      auto x = __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)(o + (uint64_t)u * blockDim.x * 16), 0, 2);
      v[u][0] = x[0], v[u][1] = x[1], v[u][2] = x[2], v[u][3] = x[3];
    }
#pragma unroll
    for (int u = 0; u < 4; u++) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  if (acc == 0x12345678u) out[threadIdx.x] = acc;
}

static double pct(std::vector<double> v, double p) {
  std::sort(v.begin(), v.end());
  return v[(size_t)(p * (v.size() - 1))];
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 64;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  static TableBlob tb;
  build_tables(tb);
  TableBlob *d_tab;
  CHECK(hipMalloc(&d_tab, sizeof(TableBlob)));
  CHECK(hipMemcpy(d_tab, &tb, sizeof(TableBlob), hipMemcpyHostToDevice));
  uint8_t *data;
  CHECK(hipMalloc(&data, kBatchBytes * kBatches));
  std::vector<uint64_t> hp(kN * kBatches), hl(kN * kBatches, kLen), pre(kN + 1);
  for (uint64_t i = 0; i < kN * kBatches; i++) hp[i] = (uint64_t)(data + i * kLen);
  for (uint64_t i = 0; i <= kN; i++) pre[i] = i * kLen;
  uint64_t *dp, *dl, *dpre, *dpre_f, *stamps;
  uint32_t *out, *scratch;
  CHECK(hipMalloc(&dp, 8 * kN * kBatches));
  CHECK(hipMalloc(&dl, 8 * kN * kBatches));
  CHECK(hipMalloc(&dpre, 8 * (kN + 1)));
  CHECK(hipMalloc(&dpre_f, 8 * (kFusedMaxN + 1) * kBatches));
  CHECK(hipMalloc(&out, 4 * kN * kBatches));
  CHECK(hipMalloc(&scratch, 1 << 20));
  CHECK(hipMalloc(&stamps, 64 * (uint64_t)cus * kWaves));
  CHECK(hipMemset(scratch, 0, 1 << 20));
  CHECK(hipMemcpy(dp, hp.data(), 8 * kN * kBatches, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dl, hl.data(), 8 * kN * kBatches, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dpre, pre.data(), 8 * (kN + 1), hipMemcpyHostToDevice));
  CHECK(launch_fill_synthetic(dp, dl, kN * kBatches, 0, 1, 0xC0FFEE, 0));
  CHECK(hipDeviceSynchronize());

  auto crc_args = [&](int b, bool fused) {
    BatchArgs a{};
    a.ptrs = reinterpret_cast<const uint8_t *const *>(dp + b * kN);
    a.prefix = fused ? dpre_f + b * (kFusedMaxN + 1) : dpre;
    a.lens = dl + b * kN;
    a.out = out + b * kN;
    a.n = kN;
    a.tab = d_tab;
    a.ctr = scratch;
    a.done = scratch + 1;
    a.acc = reinterpret_cast<uint64_t *>(scratch + 64);
    a.dyn_shift = kDynAuto;
    return a;
  };
  std::vector<hipEvent_t> ev(2 * kBatches);
  for (auto &e : ev) CHECK(hipEventCreate(&e));
  enum { kProbeWave, kProbeGrid, kCrc, kCrcFused, kCrcFusedR3, kCrcFused5, kProbePb, kProbePbRot, kProbePbNoPrio,
         kProbePbFat, kCrcFused14, kCrcFused24, kCrcFused15, kCrcFused104, kCrcFused204, kCrcFused105, kNumV };
  const char *names[kNumV] = {"probe-wave", "probe-grid", "crc", "crc-fused", "crc-fused-r3", "crc-fused-5", "probe-pb",
                              "probe-pb-rot", "probe-pb-np", "probe-pb-fat", "crc-fused-14", "crc-fused-24",
                              "crc-fused-15", "crc-fused-104", "crc-fused-204", "crc-fused-105"};
  auto launch = [&](int v, int b, hipEvent_t e0, hipEvent_t e1) {
    const uint8_t *base = data + b * kBatchBytes;
    switch (v) {
      case kProbeWave:
        hipExtLaunchKernelGGL(probe_wave, dim3(cus), dim3(1024), 0, 0, e0, e1, 0, base, kLen, out);
        break;
      case kProbeGrid:
        hipExtLaunchKernelGGL(probe_grid, dim3(cus * 8), dim3(256), 0, 0, e0, e1, 0, base, kBatchBytes, out);
        break;
      case kProbePb:
        hipExtLaunchKernelGGL(probe_pb<false>, dim3(cus), dim3(1024), 0, 0, e0, e1, 0, base, kLen, out);
        break;
      case kProbePbRot:
        hipExtLaunchKernelGGL(probe_pb<true>, dim3(cus), dim3(1024), 0, 0, e0, e1, 0, base, kLen, out);
        break;
      case kProbePbNoPrio:
        hipExtLaunchKernelGGL((probe_pb<false, false>), dim3(cus), dim3(1024), 0, 0, e0, e1, 0, base, kLen, out);
        break;
      case kProbePbFat:  // ~600 instructions (~5 KB of code) in front of the loads
        hipExtLaunchKernelGGL((probe_pb<false, true, 600>), dim3(cus), dim3(1024), 0, 0, e0, e1, 0, base, kLen, out);
        break;
      case kCrc:
        hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, 0>), dim3(cus), dim3(kThreads), 0, 0, e0, e1, 0,
                              crc_args(b, false));
        break;
      case kCrcFused:
        hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, 0, true, false, 1, kLoadNt, true>), dim3(cus),
                              dim3(kThreads), 0, 0, e0, e1, 0, crc_args(b, true));
        break;
      case kCrcFused5:
        hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, 0, true, false, 1, kLoadNt, true, kWindowed, 5>),
                              dim3(cus), dim3(kThreads), 0, 0, e0, e1, 0, crc_args(b, true));
        break;
      case kCrcFusedR3:
        hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, 0, true, false, 1, kLoadNt, true, kWindowed, 3>),
                              dim3(cus), dim3(kThreads), 0, 0, e0, e1, 0, crc_args(b, true));
        break;
      case kCrcFused14:
        hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, 0, true, false, 1, kLoadNt, true, kWindowed, 14>),
                              dim3(cus), dim3(kThreads), 0, 0, e0, e1, 0, crc_args(b, true));
        break;
      case kCrcFused24:
        hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, 0, true, false, 1, kLoadNt, true, kWindowed, 24>),
                              dim3(cus), dim3(kThreads), 0, 0, e0, e1, 0, crc_args(b, true));
        break;
      case kCrcFused104:
        hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, 0, true, false, 1, kLoadNt, true, kWindowed, 104>),
                              dim3(cus), dim3(kThreads), 0, 0, e0, e1, 0, crc_args(b, true));
        break;
      case kCrcFused204:
        hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, 0, true, false, 1, kLoadNt, true, kWindowed, 204>),
                              dim3(cus), dim3(kThreads), 0, 0, e0, e1, 0, crc_args(b, true));
        break;
      case kCrcFused105:
        hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, 0, true, false, 1, kLoadNt, true, kWindowed, 105>),
                              dim3(cus), dim3(kThreads), 0, 0, e0, e1, 0, crc_args(b, true));
        break;
      case kCrcFused15:
        hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, 0, true, false, 1, kLoadNt, true, kWindowed, 15>),
                              dim3(cus), dim3(kThreads), 0, 0, e0, e1, 0, crc_args(b, true));
        break;
    }
    CHECK(hipGetLastError());
  };
  std::vector<double> sum(kNumV, 0.0), best(kNumV, 1e30);
  for (int r = 0; r < reps; r++) {
    for (int v = 0; v < kNumV; v++) {
      for (int b = 0; b < kBatches; b++) launch(v, b, ev[2 * b], ev[2 * b + 1]);
      CHECK(hipDeviceSynchronize());
      for (int b = 0; b < kBatches; b++) {
        float ms;
        CHECK(hipEventElapsedTime(&ms, ev[2 * b], ev[2 * b + 1]));
        sum[v] += ms;
        best[v] = std::min(best[v], (double)ms);
      }
    }
  }
  // parity of the two CRC forms (same payload): batch 0
  std::vector<uint32_t> o1(kN), o2(kN);
  launch(kCrc, 0, nullptr, nullptr);
  CHECK(hipMemcpy(o1.data(), out, 4 * kN, hipMemcpyDeviceToHost));
  launch(kCrcFused, 0, nullptr, nullptr);
  CHECK(hipMemcpy(o2.data(), out, 4 * kN, hipMemcpyDeviceToHost));
  std::vector<uint32_t> o3(kN), o4(kN);
  launch(kCrcFusedR3, 0, nullptr, nullptr);
  CHECK(hipMemcpy(o3.data(), out, 4 * kN, hipMemcpyDeviceToHost));
  launch(kCrcFused5, 0, nullptr, nullptr);
  CHECK(hipMemcpy(o4.data(), out, 4 * kN, hipMemcpyDeviceToHost));
  bool eq = o1 == o2 && o1 == o3 && o1 == o4;
  for (int v : {kCrcFused14, kCrcFused24, kCrcFused15, kCrcFused104, kCrcFused204, kCrcFused105}) {
    launch(v, 0, nullptr, nullptr);
    CHECK(hipMemcpy(o4.data(), out, 4 * kN, hipMemcpyDeviceToHost));
    eq = eq && o1 == o4;
  }
  printf("c2_probe: %d CUs, 16 x 256 MiB batches rotated, %d reps; crc forms %s\n", cus, reps,
         eq ? "equal" : "DIFFER");
  for (int v = 0; v < kNumV; v++) {
    const double avg = sum[v] / (reps * kBatches);
    printf("%-11s avg %7.2f us  best %7.2f us  %7.1f GB/s (avg)\n", names[v], avg * 1e3, best[v] * 1e3,
           kBatchBytes / (avg * 1e-3) / 1e9);
  }
  // stamped timelines (one cold batch each)
  auto timeline = [&](const char *name, bool fused, int b, int pb = 4) {
    BatchArgs a = crc_args(b, fused);
    a.stamps = stamps;
    CHECK(hipMemset(stamps, 0, 64 * (uint64_t)cus * kWaves));
    if (fused && pb == 5)
      hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, 0, true, true, 1, kLoadNt, true, kWindowed, 5>),
                            dim3(cus), dim3(kThreads), 0, 0, ev[0], ev[1], 0, a);
    else if (fused && pb == 14)
      hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, 0, true, true, 1, kLoadNt, true, kWindowed, 14>),
                            dim3(cus), dim3(kThreads), 0, 0, ev[0], ev[1], 0, a);
    else if (fused && pb == 204)
      hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, 0, true, true, 1, kLoadNt, true, kWindowed, 204>),
                            dim3(cus), dim3(kThreads), 0, 0, ev[0], ev[1], 0, a);
    else if (fused && pb == 24)
      hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, 0, true, true, 1, kLoadNt, true, kWindowed, 24>),
                            dim3(cus), dim3(kThreads), 0, 0, ev[0], ev[1], 0, a);
    else if (fused && pb == 3)
      hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, 0, true, true, 1, kLoadNt, true, kWindowed, 3>),
                            dim3(cus), dim3(kThreads), 0, 0, ev[0], ev[1], 0, a);
    else if (fused)
      hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, 0, true, true, 1, kLoadNt, true>), dim3(cus),
                            dim3(kThreads), 0, 0, ev[0], ev[1], 0, a);
    else
      hipExtLaunchKernelGGL((crc32_batch_kernel<false, kDepth, 0, true, true, 1, kLoadNt, false>), dim3(cus),
                            dim3(kThreads), 0, 0, ev[0], ev[1], 0, a);
    CHECK(hipDeviceSynchronize());
    float ms;
    CHECK(hipEventElapsedTime(&ms, ev[0], ev[1]));
    const uint64_t nw = (uint64_t)cus * kWaves;
    std::vector<uint64_t> st(8 * nw);
    CHECK(hipMemcpy(st.data(), stamps, 64 * nw, hipMemcpyDeviceToHost));
    uint64_t t0 = ~0ull;
    for (uint64_t w = 0; w < nw; w++)
      if (st[8 * w + 1]) t0 = std::min(t0, st[8 * w + 4]);
    std::vector<double> entry, search, begin, end, lens;
    std::vector<double> slot_end[kWaves];
    for (uint64_t w = 0; w < nw; w++) {
      if (!st[8 * w + 1]) continue;
      entry.push_back((st[8 * w + 4] - t0) * 1e-2);
      if (fused && st[8 * w + 6]) lens.push_back((st[8 * w + 6] - t0) * 1e-2);  // per-buffer mode: lengths in
      search.push_back((st[8 * w + 5] - t0) * 1e-2);
      begin.push_back((st[8 * w + 0] - t0) * 1e-2);
      end.push_back((st[8 * w + 1] - t0) * 1e-2);
      slot_end[w % kWaves].push_back((st[8 * w + 1] - t0) * 1e-2);
    }
    printf("timeline %-9s kernel %.2f us (events) | us after first entry, p0/p50/p100:\n", name, ms * 1e3);
    auto row = [&](const char *k, const std::vector<double> &v) {
      printf("  %-7s %6.2f %6.2f %6.2f\n", k, pct(v, 0), pct(v, .5), pct(v, 1));
    };
    row("entry", entry);
    if (fused) {  // per-buffer mode: round 3 -- lengths in, tables built and batch decided at its one barrier;
                  // round 4 -- tables written (the barrier waits for them alone)
      if (!lens.empty()) row(pb == 3 ? "lengths" : "tables", lens);
      row("begin", begin);
      row("end", end);
    } else {
      row("search", search);
      row("begin", begin);
      row("end", end);
    }
    printf("  end p50 by wave slot:");
    for (int s = 0; s < kWaves; s++) printf(" %.1f", slot_end[s].empty() ? 0.0 : pct(slot_end[s], .5));
    printf("\n");
  };
  timeline("crc", false, 3);
  timeline("crc-fused", true, 5);
  timeline("crc-fused-r3", true, 7, 3);
  timeline("crc-fused-5", true, 9, 5);
  timeline("crc-fused-14", true, 11, 14);
  timeline("crc-fused-24", true, 13, 24);
  timeline("crc-fused-204", true, 15, 204);
  return 0;
}
