/* destroy_release.c -- the scratch cache against destroyed streams and
 * concurrent callers, from a C process
 * linking ROCm's own HIP runtime, as ZIPsFS would.
 *
 * Mode "destroy" (default):
 *   1. > `seconds` of zcrc32_batch_device launches (16 GiB split-plan
 *      batches, each into its own result array) queued on a fresh stream,
 *      an event recorded, the stream destroyed with the launches queued and
 *      zcrc_release_cached() called at once -- it frees that stream's scratch
 *      after its grace and a device synchronize.  Then every launch's results
 *      are compared with a reference computed on a live stream (itself
 *      checked with zlib on sampled buffers), and the cache must be empty.
 *   2. zcrc_release_cached() while another thread keeps calling
 *      zcrc32_batch_device on its own stream: it must return within the
 *      grace plus slack (it used to wait for every later release), and the
 *      other thread's results stay right.
 *   3. hipStreamPerThread and the null stream as the caller's stream.
 * Mode "trim" (run with ZCRC_SCRATCH_CACHE_MIB=1): one live stream holds
 *   ~0.5 s of queued batches while 48 fresh streams each run a batch and are
 *   destroyed; the library's reaper must free their idle scratch by itself,
 *   and no call may wait for the device (each returns in milliseconds).
 * Mode "capture": 48 fresh streams each run a batch and are destroyed, 30 ms
 *   apart; then, for `seconds` (default 3.5, past the scratch grace), the
 *   main thread captures graphs back to back in GLOBAL capture mode
 *   (torch.cuda.graph's default) -- each a memset and a
 *   zcrc32_batch_device_ws with caller scratch, the capture held open 4 ms --
 *   and replays them.  Counts the captures that fail (a synchronize or
 *   hipFree of another thread invalidates a global-mode capture), checks
 *   every replay.  With ZCRC_SCRATCH_CACHE_MIB=1 the reaper trims the
 *   destroyed streams' scratch some 30 times during the loop
 *   (tools/capture_ab.sh); with the default budget it never trims.
 * Output: one JSON line; exit status 1 on any mismatch or error.  The
 * reference's call site: src/ZIPsFS_preloadfileram.c:243 (ZIPsFS runs up to
 * 32 preload threads, src/ZIPsFS_async.c:468). */
#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>
#include <zlib.h>

#include "zcrc.h"

#define DIE(...)                          \
  do {                                    \
    fprintf(stderr, __VA_ARGS__);         \
    fputc('\n', stderr);                  \
    exit(1);                              \
  } while (0)
#define HIPCHK(x)                                                                           \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) DIE("%s:%d %s -> %s", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
  } while (0)
#define ZCHK(x)                                                                                  \
  do {                                                                                           \
    int r_ = (x);                                                                                \
    if (r_) DIE("%s:%d %s -> %d (%s)", __FILE__, __LINE__, #x, r_, zcrc_last_error());           \
  } while (0)

static double now_ms(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

/* n buffers of len bytes at d_mem, filled with the synthetic payload (index i) */
typedef struct {
  uint8_t *mem;
  uint64_t *ptrs, *lens;  /* device arrays */
  size_t n;
  uint64_t len;
  uint32_t *ref;  /* device: reference CRCs */
  uint32_t *href; /* host copy */
} Batch;

static void batch_make(Batch *b, size_t n, uint64_t len, hipStream_t s) {
  b->n = n;
  b->len = len;
  HIPCHK(hipMalloc((void **)&b->mem, n * len));
  HIPCHK(hipMalloc((void **)&b->ptrs, 8 * n));
  HIPCHK(hipMalloc((void **)&b->lens, 8 * n));
  HIPCHK(hipMalloc((void **)&b->ref, 4 * n));
  uint64_t *hp = malloc(8 * n), *hl = malloc(8 * n);
  b->href = malloc(4 * n);
  for (size_t i = 0; i < n; i++) hp[i] = (uint64_t)(uintptr_t)(b->mem + i * len), hl[i] = len;
  HIPCHK(hipMemcpy(b->ptrs, hp, 8 * n, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(b->lens, hl, 8 * n, hipMemcpyHostToDevice));
  ZCHK(zcrc_fill_synthetic(b->ptrs, b->lens, n, 0, 1, 0xC0FFEE, s));
  ZCHK(zcrc32_batch_device((const void *const *)b->ptrs, b->lens, NULL, b->ref, n, s));
  HIPCHK(hipStreamSynchronize(s));
  HIPCHK(hipMemcpy(b->href, b->ref, 4 * n, hipMemcpyDeviceToHost));
  /* zlib on sampled buffers: the reference itself is right */
  uint8_t *h = malloc(len);
  for (size_t k = 0; k < 6; k++) {
    const size_t i = k * (n - 1) / 5;
    HIPCHK(hipMemcpy(h, b->mem + i * len, len, hipMemcpyDeviceToHost));
    const uint32_t z = (uint32_t)crc32(0L, h, (uInt)len);
    if (z != b->href[i]) DIE("reference CRC of buffer %zu: %08x, zlib %08x", i, b->href[i], z);
  }
  free(h);
  free(hp);
  free(hl);
}

static size_t count_bad(const uint32_t *got, const uint32_t *exp, size_t n) {
  size_t bad = 0;
  for (size_t i = 0; i < n; i++) bad += got[i] != exp[i];
  return bad;
}

/* ------------------------------------------------------------ part 2 */
typedef struct {
  Batch *b;
  volatile int stop;
  long calls, bad, errors;
} Caller;

static void *caller_main(void *arg) {
  Caller *c = arg;
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
    c->errors++;
    return NULL;
  }
  uint32_t *d_out = NULL, *h = malloc(4 * c->b->n);
  if (hipMalloc((void **)&d_out, 4 * c->b->n) != hipSuccess) c->errors++;
  while (!c->stop && !c->errors) {
    for (int k = 0; k < 8; k++) {
      if (zcrc32_batch_device((const void *const *)c->b->ptrs, c->b->lens, NULL, d_out, c->b->n, s)) c->errors++;
      c->calls++;
    }
    if (hipStreamSynchronize(s) != hipSuccess ||
        hipMemcpy(h, d_out, 4 * c->b->n, hipMemcpyDeviceToHost) != hipSuccess)
      c->errors++;
    c->bad += (long)count_bad(h, c->b->href, c->b->n);
  }
  (void)hipStreamSynchronize(s);
  (void)hipStreamDestroy(s);
  (void)hipFree(d_out);
  free(h);
  return NULL;
}

static int mode_destroy(double seconds) {
  hipStream_t s0;
  HIPCHK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  Batch big, mid;
  batch_make(&big, 16384, 1u << 20, s0); /* 16 GiB, the split plan's scratch */
  batch_make(&mid, 8192, 65536, s0);     /* 512 MiB */

  /* 1. > seconds of launches on a stream destroyed with them queued */
  hipEvent_t a, z;
  HIPCHK(hipEventCreate(&a));
  HIPCHK(hipEventCreate(&z));
  HIPCHK(hipEventRecord(a, s0));
  for (int k = 0; k < 5; k++) ZCHK(zcrc32_batch_device((const void *const *)big.ptrs, big.lens, NULL, big.ref, big.n, s0));
  HIPCHK(hipEventRecord(z, s0));
  HIPCHK(hipEventSynchronize(z));
  float ms5 = 0;
  HIPCHK(hipEventElapsedTime(&ms5, a, z));
  const double per = ms5 / 5.0;
  size_t K = (size_t)(seconds * 1e3 / per) + 1;
  if (K > 6000) K = 6000;
  uint32_t *d_outs = NULL;
  HIPCHK(hipMalloc((void **)&d_outs, 4 * big.n * K));
  HIPCHK(hipMemset(d_outs, 0xEE, 4 * big.n * K));
  HIPCHK(hipDeviceSynchronize());
  hipStream_t s1;
  HIPCHK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  const double t0 = now_ms();
  for (size_t k = 0; k < K; k++)
    ZCHK(zcrc32_batch_device((const void *const *)big.ptrs, big.lens, NULL, d_outs + k * big.n, big.n, s1));
  hipEvent_t ev;
  HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  HIPCHK(hipEventRecord(ev, s1));
  const double t1 = now_ms();
  HIPCHK(hipStreamDestroy(s1));
  const double t2 = now_ms();
  uint64_t freed = 0;
  ZCHK(zcrc_release_cached(&freed));
  const double t3 = now_ms();
  HIPCHK(hipEventSynchronize(ev));
  HIPCHK(hipDeviceSynchronize());
  const double t4 = now_ms();
  uint32_t *h = malloc(4 * big.n * K);
  HIPCHK(hipMemcpy(h, d_outs, 4 * big.n * K, hipMemcpyDeviceToHost));
  size_t bad1 = 0;
  for (size_t k = 0; k < K; k++) bad1 += count_bad(h + k * big.n, big.href, big.n);
  free(h);
  HIPCHK(hipFree(d_outs));
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  uint64_t entries1 = 0, bytes1 = 0;
  ZCHK(zcrc_cache_info(dev, &entries1, &bytes1, NULL));

  /* 2. release while another thread keeps calling */
  Caller c = {&mid, 0, 0, 0, 0};
  pthread_t th;
  pthread_create(&th, NULL, caller_main, &c);
  usleep(300 * 1000);
  const double r0 = now_ms();
  uint64_t freed2 = 0;
  ZCHK(zcrc_release_cached(&freed2));
  const double r1 = now_ms();
  usleep(300 * 1000);
  c.stop = 1;
  pthread_join(th, NULL);

  /* 3. special stream handles */
  uint32_t *d_o = NULL, *h3 = malloc(4 * mid.n);
  HIPCHK(hipMalloc((void **)&d_o, 4 * mid.n));
  size_t bad3 = 0;
  hipStream_t specials[2] = {hipStreamPerThread, NULL};
  for (int k = 0; k < 2; k++) {
    HIPCHK(hipMemset(d_o, 0, 4 * mid.n));
    HIPCHK(hipDeviceSynchronize());
    ZCHK(zcrc32_batch_device((const void *const *)mid.ptrs, mid.lens, NULL, d_o, mid.n, specials[k]));
    uint32_t faults = 7;
    ZCHK(zcrc32_batch_device_faults(NULL, specials[k], &faults));
    if (faults) DIE("faults %u on special stream %d", faults, k);
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(h3, d_o, 4 * mid.n, hipMemcpyDeviceToHost));
    bad3 += count_bad(h3, mid.href, mid.n);
  }
  free(h3);
  HIPCHK(hipFree(d_o));

  printf("{\"mode\": \"destroy\", \"launch_ms\": %.3f, \"launches\": %zu, \"queued_gpu_s\": %.2f, "
         "\"queue_ms\": %.1f, \"destroy_ms\": %.1f, \"release_ms\": %.1f, \"released_bytes\": %llu, "
         "\"wait_after_release_ms\": %.1f, \"mismatches\": %zu, \"checked\": %zu, \"entries_after\": %llu, "
         "\"release_while_calling_ms\": %.1f, \"other_thread_calls\": %ld, \"other_thread_bad\": %ld, "
         "\"other_thread_errors\": %ld, \"special_streams_bad\": %zu}\n",
         per, K, K * per / 1e3, t1 - t0, t2 - t1, t3 - t2, (unsigned long long)freed, t4 - t3, bad1, K * big.n,
         (unsigned long long)entries1, r1 - r0, c.calls, c.bad, c.errors, bad3);
  return bad1 || c.bad || c.errors || bad3 ? 1 : 0;
}

static int mode_trim(void) {
  hipStream_t sl;
  HIPCHK(hipStreamCreateWithFlags(&sl, hipStreamNonBlocking));
  Batch big, mid;
  batch_make(&big, 16384, 1u << 20, sl);
  batch_make(&mid, 8192, 65536, sl);
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  /* ~0.5 s queued on the live stream: a device synchronize would wait for it */
  uint32_t *d_o = NULL;
  HIPCHK(hipMalloc((void **)&d_o, 4 * big.n));
  const double q0 = now_ms();
  for (int k = 0; k < 200; k++)
    ZCHK(zcrc32_batch_device((const void *const *)big.ptrs, big.lens, NULL, d_o, big.n, sl));
  const double q1 = now_ms();
  uint32_t *d_m = NULL, *h = malloc(4 * mid.n);
  HIPCHK(hipMalloc((void **)&d_m, 4 * mid.n * 48));
  double worst = 0;
  uint64_t peak_entries = 0;
  for (int i = 0; i < 48; i++) {
    hipStream_t s;
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const double c0 = now_ms();
    ZCHK(zcrc32_batch_device((const void *const *)mid.ptrs, mid.lens, NULL, d_m + (size_t)i * mid.n, mid.n, s));
    const double c1 = now_ms();
    if (c1 - c0 > worst) worst = c1 - c0;
    hipEvent_t ev;
    HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    HIPCHK(hipEventRecord(ev, s));
    HIPCHK(hipStreamDestroy(s));
    HIPCHK(hipEventSynchronize(ev));
    HIPCHK(hipEventDestroy(ev));
    uint64_t e = 0;
    ZCHK(zcrc_cache_info(dev, &e, NULL, NULL));
    if (e > peak_entries) peak_entries = e;
  }
  /* the reaper frees entries once their grace has passed: wait it out */
  uint64_t entries = 0, bytes = 0;
  double waited = 0;
  const double w0 = now_ms();
  for (int k = 0; k < 100; k++) {
    usleep(100 * 1000);
    ZCHK(zcrc_cache_info(dev, &entries, &bytes, NULL));
    waited = now_ms() - w0;
    if (bytes <= (2u << 20)) break; /* within the 1 MiB budget plus the live stream's entry */
  }
  HIPCHK(hipDeviceSynchronize());
  size_t bad = 0;
  for (int i = 0; i < 48; i++) {
    HIPCHK(hipMemcpy(h, d_m + (size_t)i * mid.n, 4 * mid.n, hipMemcpyDeviceToHost));
    bad += count_bad(h, mid.href, mid.n);
  }
  HIPCHK(hipMemcpy(h, d_o, 4 * mid.n, hipMemcpyDeviceToHost));
  bad += count_bad(h, big.href, mid.n);
  free(h);
  printf("{\"mode\": \"trim\", \"queue_live_ms\": %.1f, \"worst_call_ms\": %.2f, \"peak_entries\": %llu, "
         "\"entries_after\": %llu, \"bytes_after\": %llu, \"reaper_wait_ms\": %.0f, \"mismatches\": %zu}\n",
         q1 - q0, worst, (unsigned long long)peak_entries, (unsigned long long)entries, (unsigned long long)bytes,
         waited, bad);
  return bad ? 1 : 0;
}

static int mode_capture(double seconds) {
  hipStream_t s0;
  HIPCHK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  Batch mid;
  batch_make(&mid, 8192, 65536, s0);
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  uint32_t *d_m = NULL, *h = malloc(4 * mid.n);
  HIPCHK(hipMalloc((void **)&d_m, 4 * mid.n * 48));
  /* 48 destroyed streams' scratch, released 30 ms apart: their graces end
     one after another inside the capture loop below, so the reaper trims
     (device synchronize + hipFree) some 30 times while graphs are captured */
  for (int i = 0; i < 48; i++) {
    hipStream_t s;
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    ZCHK(zcrc32_batch_device((const void *const *)mid.ptrs, mid.lens, NULL, d_m + (size_t)i * mid.n, mid.n, s));
    hipEvent_t ev;
    HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    HIPCHK(hipEventRecord(ev, s));
    HIPCHK(hipStreamDestroy(s));
    HIPCHK(hipEventSynchronize(ev));
    HIPCHK(hipEventDestroy(ev));
    usleep(30 * 1000);
  }
  uint64_t bytes_before = 0;
  ZCHK(zcrc_cache_info(dev, NULL, &bytes_before, NULL));
  /* graphs captured back to back in global mode while the reaper works */
  const size_t sb = zcrc32_batch_device_scratch_bytes(mid.n);
  void *d_scr = NULL;
  uint32_t *d_g = NULL;
  HIPCHK(hipMalloc(&d_scr, sb));
  HIPCHK(hipMalloc((void **)&d_g, 4 * mid.n));
  hipStream_t sc;
  HIPCHK(hipStreamCreateWithFlags(&sc, hipStreamNonBlocking));
  long captures = 0, capture_fail = 0, replays = 0;
  size_t bad = 0;
  double trimmed_at = -1, first_fail_at = -1;
  hipError_t first_err = hipSuccess;
  const char *first_what = "";
  const double t0 = now_ms();
  while (now_ms() - t0 < seconds * 1e3) {
    hipGraph_t g = NULL;
    hipGraphExec_t ge = NULL;
    const hipError_t eb = hipStreamBeginCapture(sc, hipStreamCaptureModeGlobal);
    if (eb != hipSuccess) {
      captures++, capture_fail++;
      if (first_fail_at < 0) first_fail_at = now_ms() - t0, first_err = eb, first_what = "begin";
      (void)hipGetLastError();
      hipGraph_t gx = NULL;
      (void)hipStreamEndCapture(sc, &gx);
      (void)hipGetLastError();
      if (gx) (void)hipGraphDestroy(gx);
      (void)hipStreamDestroy(sc);
      HIPCHK(hipStreamCreateWithFlags(&sc, hipStreamNonBlocking));
      continue;
    }
    const hipError_t em = hipMemsetAsync(d_g, 0, 4 * mid.n, sc);
    const int zr = zcrc32_batch_device_ws((const void *const *)mid.ptrs, mid.lens, NULL, d_g, mid.n, d_scr, sb, sc);
    usleep(4000); /* the capture stays open most of the loop's time */
    const hipError_t ee = hipStreamEndCapture(sc, &g);
    captures++;
    if (em != hipSuccess || zr || ee != hipSuccess || !g) {
      capture_fail++;
      if (first_fail_at < 0) {
        first_fail_at = now_ms() - t0;
        first_err = em != hipSuccess ? em : ee;
        first_what = em != hipSuccess ? "memset" : zr ? zcrc_last_error() : "end";
      }
      (void)hipGetLastError();
      if (g) (void)hipGraphDestroy(g);
      continue;
    }
    HIPCHK(hipGraphInstantiate(&ge, g, NULL, NULL, 0));
    HIPCHK(hipGraphLaunch(ge, sc));
    HIPCHK(hipStreamSynchronize(sc));
    HIPCHK(hipMemcpy(h, d_g, 4 * mid.n, hipMemcpyDeviceToHost));
    bad += count_bad(h, mid.href, mid.n);
    replays++;
    HIPCHK(hipGraphExecDestroy(ge));
    HIPCHK(hipGraphDestroy(g));
    uint64_t b = 0;
    ZCHK(zcrc_cache_info(dev, NULL, &b, NULL));
    if (trimmed_at < 0 && b <= (2u << 20)) trimmed_at = now_ms() - t0;
  }
  const double loop_ms = now_ms() - t0;
  /* the reaper may have had to wait for a gap between captures: let it finish */
  uint64_t entries = 0, bytes = 0;
  for (int k = 0; k < 60; k++) {
    ZCHK(zcrc_cache_info(dev, &entries, &bytes, NULL));
    if (bytes <= (2u << 20)) break;
    usleep(100 * 1000);
  }
  HIPCHK(hipDeviceSynchronize());
  for (int i = 0; i < 48; i++) {
    HIPCHK(hipMemcpy(h, d_m + (size_t)i * mid.n, 4 * mid.n, hipMemcpyDeviceToHost));
    bad += count_bad(h, mid.href, mid.n);
  }
  free(h);
  printf("{\"mode\": \"capture\", \"loop_ms\": %.0f, \"captures\": %ld, \"capture_fail\": %ld, "
         "\"first_fail_ms\": %.0f, \"first_error\": \"%s\", \"first_fail_in\": \"%s\", \"replays\": %ld, \"bytes_before\": %llu, "
         "\"trimmed_during_loop_ms\": %.0f, \"bytes_after\": %llu, \"entries_after\": %llu, \"mismatches\": %zu}\n",
         loop_ms, captures, capture_fail, first_fail_at, hipGetErrorName(first_err), first_what, replays,
         (unsigned long long)bytes_before, trimmed_at, (unsigned long long)bytes, (unsigned long long)entries, bad);
  return bad || capture_fail ? 1 : 0;
}

int main(int argc, char **argv) {
  const char *mode = argc > 1 ? argv[1] : "destroy";
  if (!strcmp(mode, "trim")) return mode_trim();
  if (!strcmp(mode, "capture")) return mode_capture(argc > 2 ? atof(argv[2]) : 3.5);
  return mode_destroy(argc > 2 ? atof(argv[2]) : 2.5);
}
