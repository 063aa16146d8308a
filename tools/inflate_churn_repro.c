/* tools/inflate_churn_repro.c -- the part of tests/dropin/stream_churn.c
 * that failed intermittently (round 5), alone and under switches
 * (measurement tooling).
 *
 * Each of `threads` threads inflates, `reps` times, entry 1 of part B (1 MiB:
 * half text, half incompressible -> ~600 KB of raw DEFLATE) with
 * zcrc_inflate_device on a stream, then checks the result.  Switches:
 *   fresh   1: a fresh non-blocking stream per call, destroyed after it
 *           0: one stream per thread, kept
 *   presync 1: hipStreamSynchronize before the destroy (or before the check)
 *   zero    1: a second, tiny entry (entry 0 of part B) goes first on its own
 *           fresh stream, as the test does
 *   host    1: after each check, zcrc_inflate_batch (host memory) of entries
 *           0, 1, 0, as the test's part B does next
 *   realloc 1: the device buffers are allocated anew for every repetition
 * A failure is re-read after a 200 ms sleep and another device synchronize:
 * "late" = the results arrived afterwards (the first read raced the decode),
 * "lost" = still never written.
 *
 *   tools/inflate_churn_repro threads reps fresh presync zero host realloc
 * Output: one JSON line per setting. */
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

static int g_reps = 10, g_fresh = 1, g_presync = 0, g_zero = 1, g_host = 0, g_realloc = 0;
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static long g_ok = 0, g_late = 0, g_lost = 0, g_wrong = 0, g_err = 0, g_host_bad = 0;
static double g_destroy_us_max = 0;

static uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static void rnd_bytes(uint8_t *p, size_t n, uint64_t seed) {
  for (size_t i = 0; i < n; i += 8) {
    const uint64_t v = mix(seed ^ (i >> 3));
    memcpy(p + i, &v, n - i < 8 ? n - i : 8);
  }
}

static void words(uint8_t *p, size_t n, uint64_t seed) {
  static const char *w[] = {"spectrum ", "peak ", "retention ", "intensity ", "mass ", "charge ",
                            "scan ", "0.0125 ", "1337 ", "\n", "zip ", "entry ", "crc "};
  for (size_t i = 0; i < n;) {
    seed = mix(seed);
    const char *x = w[seed % 13];
    const size_t l = strlen(x);
    memcpy(p + i, x, n - i < l ? n - i : l);
    i += l;
  }
}

static uint8_t *raw_deflate(const uint8_t *in, size_t n, size_t *out_n) {
  z_stream zs;
  memset(&zs, 0, sizeof zs);
  if (deflateInit2(&zs, 6, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return NULL;
  const size_t cap = deflateBound(&zs, n) + 16;
  uint8_t *out = malloc(cap);
  zs.next_in = (Bytef *)in;
  zs.avail_in = (uInt)n;
  zs.next_out = out;
  zs.avail_out = (uInt)cap;
  const int ok = deflate(&zs, Z_FINISH) == Z_STREAM_END;
  *out_n = cap - zs.avail_out;
  deflateEnd(&zs);
  if (!ok) free(out);
  return ok ? out : NULL;
}

static double now_us(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec / 1e3;
}

typedef struct {
  size_t n, clen;
  uint8_t *raw, *comp;
  void *d_src, *d_dst;
  uint64_t *d_olen;
  int32_t *d_st;
} entry_t;

static int entry_alloc(entry_t *e) {
  if (hipMalloc(&e->d_src, e->clen) || hipMemcpy(e->d_src, e->comp, e->clen, hipMemcpyHostToDevice) ||
      hipMalloc(&e->d_dst, e->n) || hipMalloc((void **)&e->d_olen, 8) || hipMalloc((void **)&e->d_st, 4))
    return -1;
  return 0;
}

static void entry_unalloc(entry_t *e) {
  hipFree(e->d_src), hipFree(e->d_dst), hipFree(e->d_olen), hipFree(e->d_st);
}

/* zcrc_inflate_batch of one entry from host memory: 0 ok */
static int host_inflate(entry_t *e, uint8_t *back) {
  const void *src[1] = {e->comp};
  const size_t sl[1] = {e->clen}, cap[1] = {e->n};
  void *dst[1] = {back};
  size_t olen[1] = {0};
  int32_t st[1] = {-1};
  uint32_t crc[1] = {0};
  if (zcrc_inflate_batch(src, sl, dst, cap, olen, st, crc, 1, 0)) return -1;
  const int ok = st[0] == 0 && olen[0] == e->n && !memcmp(back, e->raw, e->n) &&
                 crc[0] == (uint32_t)crc32(0L, e->raw, (uInt)e->n);
  if (!ok) fprintf(stderr, "zcrc_inflate_batch (%zu bytes): status %d, %zu bytes\n", e->n, st[0], olen[0]);
  return ok ? 0 : 1;
}

static int entry_make(entry_t *e, int which, uint64_t seed) {
  e->n = which ? 1 << 20 : 256 << 10;
  e->raw = malloc(e->n);
  if (which) {
    words(e->raw, e->n / 2, seed + 99);
    rnd_bytes(e->raw + e->n / 2, e->n - e->n / 2, seed + 98);
  } else {
    words(e->raw, e->n, seed);
  }
  e->comp = raw_deflate(e->raw, e->n, &e->clen);
  if (!e->comp) return -1;
  return entry_alloc(e);
}

static void entry_free(entry_t *e) {
  entry_unalloc(e);
  free(e->raw), free(e->comp);
}

/* 0 ok, 1 results never written, 2 wrong */
static int entry_check(entry_t *e, uint8_t *back) {
  uint64_t olen = 0;
  int32_t st = 0;
  if (hipMemcpy(&olen, e->d_olen, 8, hipMemcpyDeviceToHost) || hipMemcpy(&st, e->d_st, 4, hipMemcpyDeviceToHost) ||
      hipMemcpy(back, e->d_dst, e->n, hipMemcpyDeviceToHost))
    return 3;
  if (st == (int32_t)0xEEEEEEEE && olen == 0xEEEEEEEEEEEEEEEEull) return 1;
  return st == 0 && olen == e->n && !memcmp(back, e->raw, e->n) ? 0 : 2;
}

static int run_one(hipStream_t *keep, entry_t *e) {
  if (hipMemset(e->d_olen, 0xEE, 8) || hipMemset(e->d_st, 0xEE, 4) || hipDeviceSynchronize()) return -1;
  hipStream_t s = *keep;
  if (g_fresh && hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) return -1;
  if (zcrc_inflate_device(e->d_src, e->clen, e->d_dst, e->n, e->d_olen, e->d_st, 0, s)) {
    fprintf(stderr, "zcrc_inflate_device: %s\n", zcrc_last_error());
    return -1;
  }
  if (g_presync && hipStreamSynchronize(s)) return -1;
  if (g_fresh) {
    const double t0 = now_us();
    if (hipStreamDestroy(s)) return -1;
    const double dt = now_us() - t0;
    pthread_mutex_lock(&g_mu);
    if (dt > g_destroy_us_max) g_destroy_us_max = dt;
    pthread_mutex_unlock(&g_mu);
  }
  return 0;
}

static void *worker(void *arg) {
  const uint64_t t = (uint64_t)(uintptr_t)arg;
  hipStream_t keep = NULL;
  if (!g_fresh && hipStreamCreateWithFlags(&keep, hipStreamNonBlocking)) return NULL;
  entry_t e0, e1;
  if (entry_make(&e0, 0, 1000 * t + 1) || entry_make(&e1, 1, 1000 * t + 1)) {
    pthread_mutex_lock(&g_mu);
    g_err++;
    pthread_mutex_unlock(&g_mu);
    return NULL;
  }
  uint8_t *back = malloc(1 << 20);
  for (int r = 0; r < g_reps; r++) {
    if (g_realloc && r > 0) {
      entry_unalloc(&e0), entry_unalloc(&e1);
      if (entry_alloc(&e0) || entry_alloc(&e1)) {
        pthread_mutex_lock(&g_mu);
        g_err++;
        pthread_mutex_unlock(&g_mu);
        break;
      }
    }
    if (g_host) {
      const int h = host_inflate(&e0, back) | host_inflate(&e1, back) | host_inflate(&e0, back);
      pthread_mutex_lock(&g_mu);
      if (h < 0) g_err++;
      else g_host_bad += h;
      pthread_mutex_unlock(&g_mu);
    }
    if ((g_zero && run_one(&keep, &e0)) || run_one(&keep, &e1) || hipDeviceSynchronize()) {
      pthread_mutex_lock(&g_mu);
      g_err++;
      pthread_mutex_unlock(&g_mu);
      break;
    }
    int c = entry_check(&e1, back);
    if (c == 1 || c == 2) {
      usleep(200000);
      (void)hipDeviceSynchronize();
      const int c2 = entry_check(&e1, back);
      pthread_mutex_lock(&g_mu);
      if (c2 == 0) g_late++;
      else if (c == 1 && c2 == 1) g_lost++;
      else g_wrong++;
      pthread_mutex_unlock(&g_mu);
      continue;
    }
    pthread_mutex_lock(&g_mu);
    if (c == 0) g_ok++;
    else g_err++;
    pthread_mutex_unlock(&g_mu);
  }
  free(back);
  entry_free(&e0);
  entry_free(&e1);
  if (keep) hipStreamDestroy(keep);
  return NULL;
}

int main(int argc, char **argv) {
  const int threads = argc > 1 ? atoi(argv[1]) : 3;
  g_reps = argc > 2 ? atoi(argv[2]) : 10;
  g_fresh = argc > 3 ? atoi(argv[3]) : 1;
  g_presync = argc > 4 ? atoi(argv[4]) : 0;
  g_zero = argc > 5 ? atoi(argv[5]) : 1;
  g_host = argc > 6 ? atoi(argv[6]) : 0;
  g_realloc = argc > 7 ? atoi(argv[7]) : 0;
  if (threads < 1 || threads > 16 || g_reps < 1) return 2;
  pthread_t th[16];
  for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, worker, (void *)(uintptr_t)t);
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  printf("{\"threads\": %d, \"reps\": %d, \"fresh\": %d, \"presync\": %d, \"zero\": %d, \"host\": %d, "
         "\"realloc\": %d, \"ok\": %ld, \"late\": %ld, \"lost\": %ld, \"wrong\": %ld, \"host_bad\": %ld, "
         "\"errors\": %ld, \"destroy_us_max\": %.0f}\n",
         threads, g_reps, g_fresh, g_presync, g_zero, g_host, g_realloc, g_ok, g_late, g_lost, g_wrong, g_host_bad,
         g_err, g_destroy_us_max);
  return g_err ? 1 : 0;
}
