/*
 * oracle/zlib_baseline.c -- TEST INFRASTRUCTURE ONLY.
 *
 * The CPU baseline for the GPU inflate: the system zlib (1.2.11 in this
 * image), which is what ZIPsFS's libzip calls under zip_fread()
 * (src/ZIPsFS.c:2016-2019, src/ZIPsFS_preloadfileram.c:286-306), run as raw
 * inflate over a batch of streams with a pthread pool.  bench/tools report it
 * as cpu_baseline kind "reference" (the reference's own inflate library).
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <zlib.h>

typedef struct {
  const uint8_t *const *src;
  const uint64_t *src_len;
  uint8_t *const *dst;
  const uint64_t *cap;
  uint64_t *out_len;
  int32_t *status;
  size_t n;
  int nthreads, tid;
} zjob;

static void *zworker(void *p) {
  zjob *j = (zjob *)p;
  z_stream zs;
  memset(&zs, 0, sizeof(zs));
  if (inflateInit2(&zs, -15) != Z_OK) return NULL;
  for (size_t i = (size_t)j->tid; i < j->n; i += (size_t)j->nthreads) {
    inflateReset(&zs);
    zs.next_in = (Bytef *)j->src[i];
    zs.avail_in = (uInt)j->src_len[i];
    zs.next_out = j->dst[i];
    zs.avail_out = (uInt)j->cap[i];
    const int rc = inflate(&zs, Z_FINISH);
    j->status[i] = rc == Z_STREAM_END ? 0 : 1;
    j->out_len[i] = zs.total_out;
  }
  inflateEnd(&zs);
  return NULL;
}

int oracle_zlib_inflate_batch(const uint8_t *const *src, const uint64_t *src_len, uint8_t *const *dst,
                              const uint64_t *cap, uint64_t *out_len, int32_t *status, size_t n, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  zjob jobs[256];
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (zjob){src, src_len, dst, cap, out_len, status, n, nthreads, t};
    if (pthread_create(&th[t], NULL, zworker, &jobs[t]) != 0) return -1;
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  return 0;
}
