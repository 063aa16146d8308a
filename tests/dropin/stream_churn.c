/* stream_churn.c -- caller streams created and destroyed between libzcrc calls
 * (VERDICT r4 next #2), from a C process (ROCm's own HIP runtime, as ZIPsFS
 * would link it), in several threads at once.
 *
 * Every round of every thread:
 *   A. device batches: a batch on a fresh stream s1, s1 destroyed with the
 *      launches still queued, then another batch (other buffers, other
 *      lengths) on a fresh stream s2 -- which may get s1's handle back --
 *      and so on for the one-launch (n <= 16 x CUs), two-launch and split-plan
 *      forms; results checked against zlib once events recorded before
 *      each destroy have completed (destroy_queued);
 *   B. one-stream inflate (zcrc_inflate_device) of two different deflated
 *      entries on two fresh streams, the first destroyed before the second is
 *      queued; then the host-memory inflate (zcrc_inflate_batch) of entries
 *      A, B, A (its thread-local device buffers reused with other bytes, then
 *      the same ones); outputs compared byte for byte, CRCs with zlib;
 *   C. ZIP: an archive of stored and deflated entries built here, verified
 *      from host memory (zcrc_zip_verify_host), from device memory on a fresh
 *      stream (zcrc_zip_verify_device) and extracted on another
 *      (zcrc_zip_extract_stored_device), each stream destroyed afterwards.
 * zlib is the checker here (crc32(), deflate()); the reference's call site is
 * src/ZIPsFS_preloadfileram.c:243 (the CRC after the preload, which libzip's
 * inflate produced).
 *
 * Usage: stream_churn <rounds> <threads>   (STREAM_CHURN_PARTS=abc: parts run)
 * Output: one JSON line; exit status 1 on any mismatch or error. */
#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

#include "zcrc.h"

static int g_rounds = 3;
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static long g_checks = 0, g_fail = 0;

#define FAILF(...)                                   \
  do {                                               \
    pthread_mutex_lock(&g_mu);                       \
    g_fail++;                                        \
    fprintf(stderr, __VA_ARGS__);                    \
    fputc('\n', stderr);                             \
    pthread_mutex_unlock(&g_mu);                     \
  } while (0)
#define LOGF(...)                \
  do {                           \
    pthread_mutex_lock(&g_mu);   \
    fprintf(stderr, __VA_ARGS__); \
    fputc('\n', stderr);         \
    pthread_mutex_unlock(&g_mu); \
  } while (0)
#define HIPCHK(x)                                                             \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      FAILF("%s:%d %s -> %s", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return -1;                                                              \
    }                                                                         \
  } while (0)
#define ZCHK(x)                                                                   \
  do {                                                                            \
    int r_ = (x);                                                                 \
    if (r_) {                                                                     \
      FAILF("%s:%d %s -> %d (%s)", __FILE__, __LINE__, #x, r_, zcrc_last_error()); \
      return -1;                                                                  \
    }                                                                             \
  } while (0)

/* Destroy a stream with its work still queued, after recording `ev` on it.
 * The checks wait on the event, not on hipDeviceSynchronize: on ROCm 7.2 a
 * destroyed stream's last store can become visible only after
 * hipStreamDestroy and a later hipDeviceSynchronize have returned (round 6:
 * the right value 200 ms later, never another thread's;
 * profiles/r06/s7/). */
static int destroy_queued(hipStream_t s, hipEvent_t *ev) {
  if (hipEventCreateWithFlags(ev, hipEventDisableTiming) != hipSuccess) return -1;
  if (hipEventRecord(*ev, s) != hipSuccess) return -1;
  return hipStreamDestroy(s) == hipSuccess ? 0 : -1;
}

static int wait_queued(hipEvent_t *ev, int n) {
  int rc = 0;
  for (int k = 0; k < n; k++) {
    rc |= hipEventSynchronize(ev[k]) != hipSuccess;
    rc |= hipEventDestroy(ev[k]) != hipSuccess;
  }
  return rc ? -1 : 0;
}

static void count(long ok, long bad) {
  pthread_mutex_lock(&g_mu);
  g_checks += ok + bad;
  g_fail += bad;
  pthread_mutex_unlock(&g_mu);
}

static uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static void fill_random(uint8_t *p, size_t n, uint64_t seed) {
  for (size_t i = 0; i < n; i += 8) {
    const uint64_t v = mix64(seed ^ (i >> 3));
    memcpy(p + i, &v, n - i < 8 ? n - i : 8);
  }
}

/* compressible, text-like bytes (dynamic-Huffman blocks, the split path) */
static void fill_text(uint8_t *p, size_t n, uint64_t seed) {
  static const char *w[] = {"spectrum ", "peak ", "retention ", "intensity ", "mass ", "charge ",
                            "scan ", "0.0125 ", "1337 ", "\n", "zip ", "entry ", "crc "};
  size_t i = 0;
  uint64_t s = seed;
  while (i < n) {
    s = mix64(s);
    const char *x = w[s % 13];
    const size_t l = strlen(x);
    memcpy(p + i, x, n - i < l ? n - i : l);
    i += l;
  }
}

/* raw DEFLATE (no zlib header), as a ZIP method-8 entry holds */
static uint8_t *deflate_raw(const uint8_t *in, size_t n, size_t *out_n) {
  z_stream zs;
  memset(&zs, 0, sizeof zs);
  if (deflateInit2(&zs, 6, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return NULL;
  const size_t cap = deflateBound(&zs, n) + 16;
  uint8_t *out = malloc(cap);
  zs.next_in = (Bytef *)in;
  zs.avail_in = (uInt)n;
  zs.next_out = out;
  zs.avail_out = (uInt)cap;
  if (deflate(&zs, Z_FINISH) != Z_STREAM_END) {
    free(out);
    deflateEnd(&zs);
    return NULL;
  }
  *out_n = cap - zs.avail_out;
  deflateEnd(&zs);
  return out;
}

static uint32_t zcrc(const uint8_t *p, size_t n) { return (uint32_t)crc32(0L, p, (uInt)n); }

/* ---------------------------------------------------------------- A */

typedef struct {
  size_t n;
  uint8_t *h;       /* host bytes */
  uint64_t *lens;   /* host lengths */
  uint32_t *exp;
  void *d_arena;
  uint64_t *d_ptrs, *d_lens;
  uint32_t *d_out;
} batch_t;

static int batch_make(batch_t *b, size_t n, size_t max_len, uint64_t seed) {
  memset(b, 0, sizeof *b);
  b->n = n;
  b->lens = malloc(8 * n);
  b->exp = malloc(4 * n);
  uint64_t *offs = malloc(8 * n), tot = 0;
  for (size_t i = 0; i < n; i++) {
    b->lens[i] = mix64(seed * 7919 + i) % (max_len + 1);
    offs[i] = tot;
    tot += (b->lens[i] + 15) & ~15ull;
  }
  b->h = malloc(tot + 16);
  fill_random(b->h, tot + 16, seed);
  for (size_t i = 0; i < n; i++) b->exp[i] = zcrc(b->h + offs[i], b->lens[i]);
  HIPCHK(hipMalloc(&b->d_arena, tot + 16));
  HIPCHK(hipMemcpy(b->d_arena, b->h, tot + 16, hipMemcpyHostToDevice));
  uint64_t *ptrs = malloc(8 * n);
  for (size_t i = 0; i < n; i++) ptrs[i] = (uint64_t)(uintptr_t)b->d_arena + offs[i];
  HIPCHK(hipMalloc((void **)&b->d_ptrs, 8 * n));
  HIPCHK(hipMalloc((void **)&b->d_lens, 8 * n));
  HIPCHK(hipMalloc((void **)&b->d_out, 4 * n));
  HIPCHK(hipMemcpy(b->d_ptrs, ptrs, 8 * n, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(b->d_lens, b->lens, 8 * n, hipMemcpyHostToDevice));
  HIPCHK(hipMemset(b->d_out, 0, 4 * n));
  free(ptrs);
  free(offs);
  return 0;
}

static int batch_check(batch_t *b, const char *what) {
  uint32_t *got = malloc(4 * b->n);
  HIPCHK(hipMemcpy(got, b->d_out, 4 * b->n, hipMemcpyDeviceToHost));
  long bad = 0;
  for (size_t i = 0; i < b->n; i++)
    if (got[i] != b->exp[i]) {
      if (!bad) LOGF("%s: buffer %zu of %zu: %08x, expected %08x", what, i, b->n, got[i], b->exp[i]);
      bad++;
    }
  count((long)b->n - bad, bad);
  free(got);
  return 0;
}

static void batch_free(batch_t *b) {
  hipFree(b->d_arena);
  hipFree(b->d_ptrs);
  hipFree(b->d_lens);
  hipFree(b->d_out);
  free(b->h);
  free(b->lens);
  free(b->exp);
}

static int part_a(uint64_t seed) {
  /* (n, max length): one-launch form, two-launch form, split plan (small list) */
  const size_t shapes[4][2] = {{200, 96 << 10}, {3000, 300 << 10}, {9000, 12 << 10}, {20000, 40 << 10}};
  batch_t b[8];
  for (int k = 0; k < 8; k++)
    if (batch_make(&b[k], shapes[k % 4][0], shapes[k % 4][1], seed * 16 + (uint64_t)k)) return -1;
  hipEvent_t ev[8];
  for (int k = 0; k < 8; k++) {
    hipStream_t s;
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    ZCHK(zcrc32_batch_device((const void *const *)b[k].d_ptrs, b[k].d_lens, NULL, b[k].d_out, b[k].n, s));
    /* launches still queued: the next stream may get this handle */
    if (destroy_queued(s, &ev[k])) FAILF("destroy_queued");
  }
  if (wait_queued(ev, 8)) FAILF("wait_queued");
  for (int k = 0; k < 8; k++) batch_check(&b[k], "device batch on a churned stream");
  for (int k = 0; k < 8; k++) batch_free(&b[k]);
  return 0;
}

/* ---------------------------------------------------------------- B */

static int part_b(uint64_t seed) {
  const size_t n = 1 << 20;
  uint8_t *raw[2];
  size_t clen[2];
  uint8_t *comp[2];
  for (int e = 0; e < 2; e++) {
    raw[e] = malloc(n);
    if (e == 0) fill_text(raw[e], n, seed);
    else { /* half text, half incompressible */
      fill_text(raw[e], n / 2, seed + 99);
      fill_random(raw[e] + n / 2, n - n / 2, seed + 98);
    }
    comp[e] = deflate_raw(raw[e], n, &clen[e]);
    if (!comp[e]) {
      FAILF("deflate failed");
      return -1;
    }
  }
  /* one-stream inflate on churned streams */
  void *d_src[2], *d_dst[2];
  uint64_t *d_olen[2];
  int32_t *d_st[2];
  /* the results start as 0xEE sentinels and the output has a 4 KiB canary of
   * 0xEE behind it: a failure then tells "never written" from "overwritten",
   * and an overrun of the output from a short one */
  const size_t canary = 4096;
  for (int e = 0; e < 2; e++) {
    HIPCHK(hipMalloc(&d_src[e], clen[e]));
    HIPCHK(hipMemcpy(d_src[e], comp[e], clen[e], hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&d_dst[e], n + canary));
    HIPCHK(hipMemset((uint8_t *)d_dst[e] + n, 0xEE, canary));
    HIPCHK(hipMalloc((void **)&d_olen[e], 8));
    HIPCHK(hipMalloc((void **)&d_st[e], 4));
    HIPCHK(hipMemset(d_olen[e], 0xEE, 8));
    HIPCHK(hipMemset(d_st[e], 0xEE, 4));
  }
  HIPCHK(hipDeviceSynchronize());
  hipEvent_t ev[2];
  for (int e = 0; e < 2; e++) {
    hipStream_t s;
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    ZCHK(zcrc_inflate_device(d_src[e], clen[e], d_dst[e], n, d_olen[e], d_st[e], 0, s));
    if (destroy_queued(s, &ev[e])) FAILF("destroy_queued");
  }
  if (wait_queued(ev, 2)) FAILF("wait_queued");
  uint8_t *back = malloc(n + canary);
  for (int e = 0; e < 2; e++) {
    uint64_t olen = 0;
    int32_t st = -1;
    HIPCHK(hipMemcpy(&olen, d_olen[e], 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&st, d_st[e], 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(back, d_dst[e], n + canary, hipMemcpyDeviceToHost));
    size_t canary_bad = 0;
    for (size_t i = n; i < n + canary; i++) canary_bad += back[i] != 0xEE;
    const int ok = st == 0 && olen == n && !memcmp(back, raw[e], n) && !canary_bad;
    if (!ok) {
      size_t first = n, ndiff = 0;
      for (size_t i = 0; i < n; i++)
        if (back[i] != raw[e][i]) ndiff++, first = first < i ? first : i;
      LOGF("zcrc_inflate_device entry %d (seed %llu, %zu compressed bytes): status %d%s, %llu bytes%s, %zu bytes "
           "differ (first at %zu), %zu canary bytes overwritten",
           e, (unsigned long long)seed, clen[e], st, st == (int32_t)0xEEEEEEEE ? " (never written)" : "",
           (unsigned long long)olen, olen == 0xEEEEEEEEEEEEEEEEull ? " (never written)" : "", ndiff, first,
           canary_bad);
    }
    count(ok, !ok);
    hipFree(d_src[e]);
    hipFree(d_dst[e]);
    hipFree(d_olen[e]);
    hipFree(d_st[e]);
  }
  /* host-memory inflate: A, B, A (thread-local buffers reused with other bytes) */
  const int order[3] = {0, 1, 0};
  for (int k = 0; k < 3; k++) {
    const int e = order[k];
    const void *src[1] = {comp[e]};
    const size_t sl[1] = {clen[e]}, cap[1] = {n};
    void *dst[1] = {back};
    size_t olen[1] = {0};
    int32_t st[1] = {-1};
    uint32_t crc[1] = {0};
    memset(back, 0, n);
    ZCHK(zcrc_inflate_batch(src, sl, dst, cap, olen, st, crc, 1, 0));
    const int ok = st[0] == 0 && olen[0] == n && !memcmp(back, raw[e], n) && crc[0] == zcrc(raw[e], n);
    if (!ok) LOGF("zcrc_inflate_batch call %d (entry %d): status %d, %zu bytes, crc %08x vs %08x", k, e, st[0],
                   olen[0], crc[0], zcrc(raw[e], n));
    count(ok, !ok);
  }
  free(back);
  for (int e = 0; e < 2; e++) free(raw[e]), free(comp[e]);
  return 0;
}

/* ---------------------------------------------------------------- C */

static void put16(uint8_t *p, uint16_t v) { p[0] = (uint8_t)v, p[1] = (uint8_t)(v >> 8); }
static void put32(uint8_t *p, uint32_t v) { put16(p, (uint16_t)v), put16(p + 2, (uint16_t)(v >> 16)); }

/* An archive of `m` entries, even ones stored, odd ones deflated. */
static uint8_t *zip_build(int m, uint64_t seed, size_t *len) {
  size_t cap = 64 << 20, at = 0;
  uint8_t *a = malloc(cap), *cd = malloc(1 << 20);
  size_t cdl = 0;
  for (int i = 0; i < m; i++) {
    const size_t n = 1000 + (size_t)(mix64(seed + (uint64_t)i) % (600 << 10));
    uint8_t *raw = malloc(n);
    if (i % 3) fill_text(raw, n, seed * 31 + (uint64_t)i);
    else fill_random(raw, n, seed * 31 + (uint64_t)i);
    size_t cl = n;
    uint8_t *data = raw;
    const int deflated = i & 1;
    if (deflated) data = deflate_raw(raw, n, &cl);
    char name[32];
    const int nl = snprintf(name, sizeof name, "e%04d.bin", i);
    const uint32_t crc = zcrc(raw, n);
    uint8_t *h = a + at;
    memset(h, 0, 30);
    put32(h, 0x04034b50);
    put16(h + 4, 20);
    put16(h + 8, deflated ? 8 : 0);
    put32(h + 14, crc);
    put32(h + 18, (uint32_t)cl);
    put32(h + 22, (uint32_t)n);
    put16(h + 26, (uint16_t)nl);
    memcpy(h + 30, name, (size_t)nl);
    memcpy(h + 30 + nl, data, cl);
    uint8_t *c = cd + cdl;
    memset(c, 0, 46);
    put32(c, 0x02014b50);
    put16(c + 4, 20);
    put16(c + 6, 20);
    put16(c + 10, deflated ? 8 : 0);
    put32(c + 16, crc);
    put32(c + 20, (uint32_t)cl);
    put32(c + 24, (uint32_t)n);
    put16(c + 28, (uint16_t)nl);
    put32(c + 42, (uint32_t)at);
    memcpy(c + 46, name, (size_t)nl);
    cdl += 46 + (size_t)nl;
    at += 30 + (size_t)nl + cl;
    if (deflated) free(data);
    free(raw);
  }
  memcpy(a + at, cd, cdl);
  uint8_t *e = a + at + cdl;
  memset(e, 0, 22);
  put32(e, 0x06054b50);
  put16(e + 8, (uint16_t)m);
  put16(e + 10, (uint16_t)m);
  put32(e + 12, (uint32_t)cdl);
  put32(e + 16, (uint32_t)at);
  *len = at + cdl + 22;
  free(cd);
  return a;
}

static int zip_count(const zcrc_zip_entry *E, size_t n, const char *what, int want_extracted) {
  long bad = 0;
  for (size_t i = 0; i < n; i++) {
    const int expect = want_extracted && E[i].method != 0 ? ZCRC_ZIP_UNVERIFIED : ZCRC_ZIP_OK;
    if (E[i].status != expect) {
      if (!bad) LOGF("%s: entry %zu method %u status %d (expected %d) crc %08x/%08x", what, i, E[i].method,
                      E[i].status, expect, E[i].crc_computed, E[i].crc_expected);
      bad++;
    }
  }
  count((long)n - bad, bad);
  return 0;
}

static int part_c(uint64_t seed) {
  size_t len = 0;
  const int m = 24;
  uint8_t *a = zip_build(m, seed, &len);
  zcrc_zip_entry E[64];
  size_t n = 0;
  ZCHK(zcrc_zip_scan(a, len, E, 64, &n));
  if (n != (size_t)m) {
    FAILF("zip scan: %zu entries, expected %d", n, m);
    return -1;
  }
  zcrc_zip_entry H[64];
  memcpy(H, E, sizeof(zcrc_zip_entry) * n);
  ZCHK(zcrc_zip_verify_host(a, len, H, n));
  zip_count(H, n, "zcrc_zip_verify_host", 0);
  void *d = NULL;
  HIPCHK(hipMalloc(&d, len));
  HIPCHK(hipMemcpy(d, a, len, hipMemcpyHostToDevice));
  hipStream_t s;
  HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  memcpy(H, E, sizeof(zcrc_zip_entry) * n);
  ZCHK(zcrc_zip_verify_device(d, len, H, n, s));
  HIPCHK(hipStreamDestroy(s));
  zip_count(H, n, "zcrc_zip_verify_device", 0);
  /* stored extraction into device buffers on another fresh stream */
  void *dst[64];
  size_t cap[64];
  for (size_t i = 0; i < n; i++) {
    cap[i] = E[i].comp_size;
    HIPCHK(hipMalloc(&dst[i], cap[i] ? cap[i] : 1));
  }
  HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  memcpy(H, E, sizeof(zcrc_zip_entry) * n);
  ZCHK(zcrc_zip_extract_stored_device(d, len, H, dst, cap, n, s));
  HIPCHK(hipStreamDestroy(s));
  zip_count(H, n, "zcrc_zip_extract_stored_device", 1);
  for (size_t i = 0; i < n; i++) hipFree(dst[i]);
  hipFree(d);
  free(a);
  return 0;
}

static const char *g_parts = "abc"; /* STREAM_CHURN_PARTS: which parts each round runs */

static void *worker(void *arg) {
  const uint64_t t = (uint64_t)(uintptr_t)arg;
  for (int r = 0; r < g_rounds; r++) {
    const uint64_t seed = 1000 * t + (uint64_t)r + 1;
    if ((strchr(g_parts, 'a') && part_a(seed)) || (strchr(g_parts, 'b') && part_b(seed)) ||
        (strchr(g_parts, 'c') && part_c(seed)))
      break;
  }
  return NULL;
}

int main(int argc, char **argv) {
  g_rounds = argc > 1 ? atoi(argv[1]) : 3;
  const int threads = argc > 2 ? atoi(argv[2]) : 2;
  if (g_rounds < 1 || threads < 1 || threads > 16) return 2;
  if (getenv("STREAM_CHURN_PARTS")) g_parts = getenv("STREAM_CHURN_PARTS");
  pthread_t th[16];
  for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, worker, (void *)(uintptr_t)t);
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  uint64_t entries = 0, bytes = 0, tl = 0;
  zcrc_cache_info(0, &entries, &bytes, &tl);
  uint64_t freed = 0;
  const int rrc = zcrc_release_cached(&freed);
  uint64_t left = 0, left_bytes = 0;
  zcrc_cache_info(0, &left, &left_bytes, NULL);
  printf("{\"rounds\": %d, \"threads\": %d, \"checks\": %ld, \"failures\": %ld, \"scratch_entries\": %llu, "
         "\"scratch_bytes\": %llu, \"thread_local_bytes\": %llu, \"release_rc\": %d, \"released_bytes\": %llu, "
         "\"entries_left\": %llu, \"bytes_left\": %llu}\n",
         g_rounds, threads, g_checks, g_fail, (unsigned long long)entries, (unsigned long long)bytes,
         (unsigned long long)tl, rrc, (unsigned long long)freed, (unsigned long long)left,
         (unsigned long long)left_bytes);
  return g_fail ? 1 : 0;
}
