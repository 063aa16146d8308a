// tools/stream_reuse_probe.hip -- what HIP does with a caller stream that is
// destroyed with work still queued (measurement only; the library's scratch
// cache is keyed on what this shows, zcrc_runtime.hip ScratchCache).
//
// For each of `rounds`: a bounded spin kernel (~`ms` ms of wall clock) is
// queued on a fresh non-blocking stream, the stream is destroyed at once and a
// new one created.  Prints how long hipStreamDestroy took, whether the new
// stream got the same handle, both hipStreamGetId values, and whether the spin
// kernel's completion flag was set when hipDeviceSynchronize returned.
//
//   hipcc --offload-arch=gfx950 -O2 tools/stream_reuse_probe.hip -o tools/stream_reuse_probe
//   tools/stream_reuse_probe [rounds] [ms]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                 \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

// one wave spins until `ticks` of the 100 MHz wall clock have passed (bounded
// by construction), then stores `tag`
__global__ void spin(unsigned *flag, unsigned tag, unsigned long long ticks) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
  if (threadIdx.x == 0) flag[0] = tag;
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 4;
  const double ms = argc > 2 ? atof(argv[2]) : 50.0;
  int khz = 0;
  CHK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  const unsigned long long ticks = (unsigned long long)(ms * khz);
  unsigned *flag = nullptr;
  CHK(hipMalloc(&flag, 4));
  CHK(hipMemset(flag, 0, 4));
  CHK(hipDeviceSynchronize());
  hipStream_t s = nullptr;
  CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int r = 1; r <= rounds; r++) {
    unsigned long long id_old = 0, id_new = 0;
    CHK(hipStreamGetId(s, &id_old));
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, flag, (unsigned)r, ticks);
    CHK(hipGetLastError());
    const auto t0 = std::chrono::steady_clock::now();
    CHK(hipStreamDestroy(s));
    const auto t1 = std::chrono::steady_clock::now();
    hipStream_t old = s;
    CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CHK(hipStreamGetId(s, &id_new));
    unsigned before = 0, after = 0;
    // a host read through the null stream would order against the spin only
    // if destroy or the null stream waited; read it with a device synchronize
    // in between instead, and once before on a fresh stream (no wait)
    CHK(hipMemcpyAsync(&before, flag, 4, hipMemcpyDeviceToHost, s));
    CHK(hipStreamSynchronize(s));
    const auto t2 = std::chrono::steady_clock::now();
    CHK(hipDeviceSynchronize());
    const auto t3 = std::chrono::steady_clock::now();
    CHK(hipMemcpy(&after, flag, 4, hipMemcpyDeviceToHost));
    auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    printf("{\"round\": %d, \"spin_ms\": %.1f, \"destroy_us\": %.1f, \"same_handle\": %d, \"id_old\": %llu, "
           "\"id_new\": %llu, \"flag_on_new_stream\": %u, \"device_sync_us\": %.1f, \"flag_after_sync\": %u}\n",
           r, ms, us(t0, t1), old == s, id_old, id_new, before, us(t2, t3), after);
    fflush(stdout);
  }
  CHK(hipStreamDestroy(s));
  CHK(hipFree(flag));
  return 0;
}
