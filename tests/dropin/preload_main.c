/*
 * tests/dropin/preload_main.c -- preloadram_now's read loop
 * (src/ZIPsFS_preloadfileram.c:262-328) with the CRC check of
 * fhandle_check_crc32 (:237-250), compiled against the drop-in
 * (zipsfs_amd/cg_crc32.c -> libzcrc) and libzcrc's stream API.
 *
 * The entry is read with read(fd, dst + already, min(16 MiB, st_size -
 * already)) (:284-306, PRELOADRAM_READ_BYTES_NUM) into one segment that is
 * mmap'd above THRESHOLD_MALLOC_MMAP = 128 KiB and malloc'd below
 * (ZIPsFS_configuration.h:113, cg_textbuffer.c:103-106).  After the last
 * read the CRC is checked while mutex_fhandle is held (:309-321), which
 * every other FUSE reader waits on; hold_us is that time.
 *
 * Modes (argv[3..]):
 *   dropin  as ZIPsFS with the drop-in: cg_crc32(dst, st_size, 0, &mutex)
 *           after the loop (GPU at or above the drop-in threshold)
 *   stream  SURVEY 8(f) rank 1: zcrc32_stream_update() per chunk inside the
 *           loop (the GPU checksums chunk k while chunk k+1 is read), and
 *           zcrc32_stream_final() after it; open_us/close_us per entry
 *   ref     the reference's own cg_crc32 (src/cg_crc32.c, built -O0 as
 *           shipped into oracle/_ref by oracle/Makefile; test
 *           infrastructure, loaded with dlopen from $ZCRC_REF_LIB)
 *   stream_reg  as stream, but the segment is registered when the stream is
 *           opened (zcrc32_stream_open_registered, open_us includes the
 *           registration, close_us the unregistration): the chunks are DMA'd
 *           from it, update() copies nothing
 *   none    the loop with no CRC at all (its loop_ms is the baseline)
 *
 * Deflated entries (ZCRC_PRELOAD_DEFLATED=<uncompressed size> in the
 * environment; the entry file then holds the entry's raw DEFLATE data, as
 * libzip reads it after the local header).  ZIPsFS inflates with
 * zip_fread() (src/ZIPsFS.c:2016-2019: libzip over zlib) in the same 16 MiB
 * pieces and checks the CRC after the loop; the compressed bytes are read
 * into memory first in every mode (libzip's own reads).  Modes:
 *   zlib_ref     zlib raw inflate in 16 MiB output pieces, then the
 *                reference's cg_crc32 (-O0) under the lock (what ZIPsFS does)
 *   zlib_dropin  the same loop, then the drop-in cg_crc32 under the lock
 *   gpu_inflate  one zcrc_inflate_batch call: inflate + CRC on the GPU, the
 *                bytes copied into the segment; under the lock only the
 *                compare of the CRC it returned
 * Usage: preload_main <entry file> <expected crc hex> <reps> mode...
 * Output: one JSON line per mode with the median over reps.
 */
#include "cg_crc32.c"

#include <dlfcn.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>
#include <zlib.h>

#define PRELOADRAM_READ_BYTES_NUM (16L << 20)
#define THRESHOLD_MALLOC_MMAP (128L << 10)

static pthread_mutex_t mutex_fhandle = PTHREAD_MUTEX_INITIALIZER;
static pthread_mutex_t mutex_crc = PTHREAD_MUTEX_INITIALIZER;
typedef uint32_t (*ref_fn)(const void *, size_t, uint32_t);

static double now_us(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static int cmp_d(const void *a, const void *b) {
  const double x = *(const double *)a, y = *(const double *)b;
  return x < y ? -1 : x > y;
}

static double median(const double *v, int n) {
  double t[1000];
  memcpy(t, v, sizeof(double) * (size_t)n);
  qsort(t, n, sizeof(double), cmp_d);
  return t[n / 2];
}

typedef struct {
  uint32_t crc;
  double loop_ms, hold_us, open_us, close_us;
} result_t;

/* a deflated entry (ZCRC_PRELOAD_DEFLATED): mode 5 zlib_ref, 6 zlib_dropin,
 * 7 gpu_inflate.  st_size = the uncompressed size (central directory). */
static int preload_deflated_once(const char *path, off_t st_size, int mode, ref_fn ref, result_t *r) {
  const int fd = open(path, O_RDONLY);
  if (fd < 0) return -1;
  struct stat st;
  if (fstat(fd, &st)) return -1;
  const size_t clen = (size_t)st.st_size;
  const int use_mmap = st_size > THRESHOLD_MALLOC_MMAP;
  char *dst = use_mmap ? mmap(NULL, st_size ? st_size : 1, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0)
                       : malloc(st_size ? st_size : 1);
  if (!dst || dst == MAP_FAILED) return -1;
  r->open_us = r->close_us = 0;
  const double t0 = now_us();
  unsigned char *comp = malloc(clen ? clen : 1);
  if (!comp) return -1;
  for (size_t got = 0; got < clen;) {  /* the compressed bytes, as libzip reads them */
    const ssize_t n = read(fd, comp + got, clen - got);
    if (n <= 0) return -1;
    got += (size_t)n;
  }
  off_t already = 0;
  uint32_t gpu_crc = 0;
  if (mode == 5 || mode == 6) {
    z_stream zs;
    memset(&zs, 0, sizeof zs);
    if (inflateInit2(&zs, -15) != Z_OK) return -1;
    zs.next_in = comp;
    zs.avail_in = (uInt)clen;
    int zr = Z_OK;
    while (st_size > already && zr != Z_STREAM_END) {  /* zip_fread(zf, dst + already, n_max) (:288) */
      const off_t n_max = st_size - already < PRELOADRAM_READ_BYTES_NUM ? st_size - already : PRELOADRAM_READ_BYTES_NUM;
      zs.next_out = (unsigned char *)dst + already;
      zs.avail_out = (uInt)n_max;
      while (zs.avail_out && zr == Z_OK) zr = inflate(&zs, Z_NO_FLUSH);
      if (zr != Z_OK && zr != Z_STREAM_END) return -1;
      pthread_mutex_lock(&mutex_fhandle);
      already += n_max - (off_t)zs.avail_out;
      pthread_mutex_unlock(&mutex_fhandle);
    }
    inflateEnd(&zs);
  } else {
    const void *src[1] = {comp};
    const size_t src_len[1] = {clen}, cap[1] = {(size_t)st_size};
    void *dsts[1] = {dst};
    size_t out_len[1] = {0};
    int32_t status[1] = {-1};
    const int irc = zcrc_inflate_batch(src, src_len, dsts, cap, out_len, status, &gpu_crc, 1, 0);
    if (irc || status[0] != 0) {
      fprintf(stderr, "zcrc_inflate_batch: rc %d, status %d, out_len %zu of %zu (%s)\n", irc, (int)status[0],
              out_len[0], (size_t)st_size, zcrc_last_error());
      return -1;
    }
    pthread_mutex_lock(&mutex_fhandle);
    already = (off_t)out_len[0];
    pthread_mutex_unlock(&mutex_fhandle);
  }
  r->loop_ms = (now_us() - t0) * 1e-3;
  free(comp);
  if (already != st_size) return -1;
  pthread_mutex_lock(&mutex_fhandle); /* LOCK(mutex_fhandle, ok_crc=fhandle_check_crc32(d)) (:313) */
  const double h = now_us();
  uint32_t crc = 0;
  if (mode == 5) crc = ref(dst, st_size, 0);
  if (mode == 6) crc = cg_crc32(dst, st_size, 0, &mutex_crc);
  if (mode == 7) crc = gpu_crc;
  r->hold_us = now_us() - h;
  pthread_mutex_unlock(&mutex_fhandle);
  r->crc = crc;
  if (!use_mmap) free(dst);
  else munmap(dst, st_size ? st_size : 1);
  close(fd);
  return 0;
}

/* one preload of the entry; mode: 0 dropin, 1 stream, 2 ref, 3 stream_reg, 4 none */
static int preload_once(const char *path, int mode, ref_fn ref, result_t *r) {
  const int fd = open(path, O_RDONLY);
  if (fd < 0) return -1;
  struct stat st;
  if (fstat(fd, &st)) return -1;
  const off_t st_size = st.st_size;
  const int use_mmap = st_size > THRESHOLD_MALLOC_MMAP;
  /* ZCRC_PRELOAD_REUSE=1 (diagnostics): one segment for every repetition,
   * never unmapped in between */
  static char *kept = NULL;
  const int reuse = getenv("ZCRC_PRELOAD_REUSE") && use_mmap;
  char *dst = reuse && kept ? kept
              : use_mmap ? mmap(NULL, st_size ? st_size : 1, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0)
                         : malloc(st_size ? st_size : 1);
  if (reuse) kept = dst;
  if (!dst || dst == MAP_FAILED) return -1;
  zcrc32_stream *s = NULL;
  r->open_us = r->close_us = 0;
  if (mode == 1 || mode == 3) {
    const double t = now_us();
    s = mode == 1 ? zcrc32_stream_open(0) : zcrc32_stream_open_registered(0, dst, (size_t)st_size);
    r->open_us = now_us() - t;
    if (!s) return -1;
  }
  const double t0 = now_us();
  off_t already = 0;
  for (; st_size > already;) {
    const off_t n_max = st_size - already < PRELOADRAM_READ_BYTES_NUM ? st_size - already : PRELOADRAM_READ_BYTES_NUM;
    const ssize_t n = read(fd, dst + already, n_max);
    if (n <= 0) break;
    if (s && zcrc32_stream_update(s, dst + already, (size_t)n)) return -1;
    pthread_mutex_lock(&mutex_fhandle); /* the loop's bookkeeping under the lock (:293-303) */
    already += n;
    pthread_mutex_unlock(&mutex_fhandle);
  }
  r->loop_ms = (now_us() - t0) * 1e-3;
  if (already != st_size) return -1;
  pthread_mutex_lock(&mutex_fhandle); /* LOCK(mutex_fhandle, ok_crc=fhandle_check_crc32(d)) (:313) */
  const double h = now_us();
  uint32_t crc = 0;
  if (mode == 0) crc = cg_crc32(dst, st_size, 0, &mutex_crc);
  if ((mode == 1 || mode == 3) && zcrc32_stream_final(s, &crc)) return -1;
  if (mode == 2) crc = ref(dst, st_size, 0);
  if (mode == 4) crc = r->crc;  /* no CRC: reported as the expected value */
  r->hold_us = now_us() - h;
  pthread_mutex_unlock(&mutex_fhandle);
  r->crc = crc;
  if (s) {
    const double t = now_us();
    zcrc32_stream_close(s);
    r->close_us = now_us() - t;
  }
  if (!use_mmap) free(dst);
  else if (!reuse) munmap(dst, st_size ? st_size : 1);
  close(fd);
  return 0;
}

int main(int argc, char **argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s entry expected_crc_hex reps mode...\n", argv[0]);
    return 2;
  }
  const char *path = argv[1];
  const uint32_t expected = (uint32_t)strtoul(argv[2], NULL, 16);
  const int reps = atoi(argv[3]);
  if (reps < 1 || reps > 1000) return 2;
  /* as ZIPsFS would at startup, outside any lock: device
   * init and staging slots, which the drop-in never creates under
   * mutex_fhandle; without a GPU it fails and the drop-in answers on the host */
  (void)zcrc32_prewarm(2);
  const char *defl = getenv("ZCRC_PRELOAD_DEFLATED");
  const off_t usize = defl ? (off_t)strtoll(defl, NULL, 10) : -1;
  int bad = 0;
  for (int a = 4; a < argc; a++) {
    const char *m = argv[a];
    const int mode = !strcmp(m, "dropin")        ? 0
                     : !strcmp(m, "stream")      ? 1
                     : !strcmp(m, "ref")         ? 2
                     : !strcmp(m, "stream_reg")  ? 3
                     : !strcmp(m, "none")        ? 4
                     : !strcmp(m, "zlib_ref")    ? 5
                     : !strcmp(m, "zlib_dropin") ? 6
                     : !strcmp(m, "gpu_inflate") ? 7
                                                 : -1;
    if (mode < 0 || (mode >= 5) != (usize >= 0)) return 2;  /* deflated modes need ZCRC_PRELOAD_DEFLATED */
    ref_fn ref = NULL;
    if (mode == 2 || mode == 5) {
      const char *lib = getenv("ZCRC_REF_LIB");
      void *h = lib ? dlopen(lib, RTLD_NOW | RTLD_LOCAL) : NULL;
      ref = h ? (ref_fn)dlsym(h, "ref_cg_crc32") : NULL;
      if (!ref) {
        printf("{\"mode\": \"%s\", \"skipped\": \"ZCRC_REF_LIB not loadable\"}\n", m);
        continue;
      }
    }
    double loop[1000], hold[1000], op[1000], cl[1000];
    uint32_t crc = 0;
    int ok = 1;
    for (int k = 0; k < reps; k++) {
      result_t r = {expected, 0, 0, 0, 0};
      if (mode >= 5 ? preload_deflated_once(path, usize, mode, ref, &r) : preload_once(path, mode, ref, &r)) {
        fprintf(stderr, "%s: preload failed (%s)\n", argv[a], zcrc_last_error());
        return 1;
      }
      loop[k] = r.loop_ms, hold[k] = r.hold_us, op[k] = r.open_us, cl[k] = r.close_us;
      crc = r.crc;
      ok &= r.crc == expected;
    }
    if (!ok) fprintf(stderr, "crc32-mismatch!  ZIP: %x != computed: %x (%s)\n", expected, crc, argv[a]);
    bad += !ok;
    char holds[8192];
    size_t hl = 0;
    for (int k = 0; k < reps && hl + 32 < sizeof holds; k++)
      hl += (size_t)snprintf(holds + hl, sizeof holds - hl, "%s%.1f", k ? ", " : "", hold[k]);
    printf("{\"mode\": \"%s\", \"crc\": \"%08x\", \"ok\": %s, \"reps\": %d, \"loop_ms\": %.3f, \"hold_us\": %.1f, "
           "\"open_us\": %.1f, \"close_us\": %.1f, \"hold_all_us\": [%s]}\n",
           argv[a], crc, ok ? "true" : "false", reps, median(loop, reps), median(hold, reps), median(op, reps),
           median(cl, reps), holds);
  }
  uint64_t gpu = 0, host = 0, fallback = 0;
  zcrc32_dropin_stats(&gpu, &host, &fallback);
  printf("{\"stats\": {\"gpu\": %llu, \"host\": %llu, \"fallback\": %llu}}\n", (unsigned long long)gpu,
         (unsigned long long)host, (unsigned long long)fallback);
  return bad ? 1 : 0;
}
