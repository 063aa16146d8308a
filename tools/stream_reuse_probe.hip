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
//   tools/stream_reuse_probe [rounds] [ms] [threads] [launches per stream] [realloc]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <unistd.h>

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
  if (threadIdx.x == 0 && tag) flag[0] = tag;  // (tag 0: a chain member that stores nothing)
}

// Threaded form (argv[3] = threads > 0): each thread, `rounds` times, queues
// one spin kernel of 1..ms ms on a fresh stream, destroys the stream at once,
// calls hipDeviceSynchronize and reads its flag.  Counts the reads that came
// back before the kernel's store ("early"): work of a destroyed stream that
// neither the destroy nor the device synchronize waited for.
#include <atomic>
#include <thread>
#include <vector>
static std::atomic<long> g_early{0}, g_total{0};
// round 6: a wrong first read is read again 200 ms later
// -- its own tag then: the store arrived late; another thread's tag: the
// allocation was re-used and written; still the memset's 0: never written
static std::atomic<long> g_late{0}, g_foreign{0}, g_never{0}, g_other{0};
static std::atomic<long long> g_destroy_max_us{0};

static int g_chain = 1, g_realloc = 0;

static void thread_rounds(int t, int rounds, double ms, int khz) {
  unsigned *flag = nullptr;
  CHK(hipMalloc(&flag, 4));
  for (int r = 1; r <= rounds; r++) {
    if (g_realloc) {  // a fresh allocation per round (the library-level repro needed it)
      CHK(hipFree(flag));
      CHK(hipMalloc(&flag, 4));
    }
    const unsigned tag = (unsigned)(t << 16 | r);
    CHK(hipMemset(flag, 0, 4));
    CHK(hipDeviceSynchronize());
    hipStream_t s = nullptr;
    CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const double this_ms = 1.0 + (ms - 1.0) * (double)((r * 7919 + t * 104729) % 97) / 96.0;
    // g_chain launches of this_ms / g_chain each; only the last stores the tag
    for (int k = 0; k < g_chain; k++) {
      hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, flag, k + 1 == g_chain ? tag : 0u,
                         (unsigned long long)(this_ms / g_chain * khz));
      CHK(hipGetLastError());
    }
    const auto t0 = std::chrono::steady_clock::now();
    CHK(hipStreamDestroy(s));
    const long long us =
        (long long)std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    long long m = g_destroy_max_us.load();
    while (us > m && !g_destroy_max_us.compare_exchange_weak(m, us)) {
    }
    CHK(hipDeviceSynchronize());
    unsigned got = 0;
    CHK(hipMemcpy(&got, flag, 4, hipMemcpyDeviceToHost));
    g_total++;
    if (got != tag) {
      g_early++;
      usleep(200 * 1000);
      unsigned again = 0;
      CHK(hipMemcpy(&again, flag, 4, hipMemcpyDeviceToHost));
      if (again == tag) g_late++;
      else if (again == 0) g_never++;
      else if ((again >> 16) != (unsigned)t) g_foreign++;
      else g_other++;
      fprintf(stderr, "thread %d round %d: tag %08x, first read %08x, 200 ms later %08x\n", t, r, tag, got, again);
    }
  }
  CHK(hipDeviceSynchronize());
  CHK(hipFree(flag));
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 4;
  const double ms = argc > 2 ? atof(argv[2]) : 50.0;
  const int threads = argc > 3 ? atoi(argv[3]) : 0;
  g_chain = argc > 4 ? atoi(argv[4]) : 1;
  g_realloc = argc > 5 ? atoi(argv[5]) : 0;
  if (g_chain < 1) g_chain = 1;
  if (threads > 0) {
    int khz0 = 0;
    CHK(hipDeviceGetAttribute(&khz0, hipDeviceAttributeWallClockRate, 0));
    std::vector<std::thread> th;
    for (int t = 0; t < threads && t < 16; t++) th.emplace_back(thread_rounds, t, rounds, ms, khz0);
    for (auto &x : th) x.join();
    printf("{\"threads\": %d, \"rounds\": %d, \"max_spin_ms\": %.1f, \"launches_per_stream\": %d, "
           "\"realloc\": %d, \"reads\": %ld, \"early\": %ld, \"late\": %ld, \"foreign\": %ld, "
           "\"never\": %ld, \"other\": %ld, \"destroy_max_us\": %lld}\n",
           threads, rounds, ms, g_chain, g_realloc, g_total.load(), g_early.load(), g_late.load(), g_foreign.load(),
           g_never.load(), g_other.load(), g_destroy_max_us.load());
    return 0;
  }
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
  {  // host cost of hipStreamGetId (the library calls it once per leased call)
    unsigned long long id = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 100000; i++) CHK(hipStreamGetId(s, &id));
    const double ns = std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count() / 1e5;
    printf("{\"hipStreamGetId_ns\": %.1f}\n", ns);
  }
  CHK(hipStreamDestroy(s));
  CHK(hipFree(flag));
  return 0;
}
