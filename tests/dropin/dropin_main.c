/*
 * tests/dropin/dropin_main.c -- ZIPsFS's call site of cg_crc32, compiled
 * against the drop-in (zipsfs_amd/cg_crc32.c -> libzcrc).
 *
 * check_entry() has the shape of fhandle_check_crc32
 * (src/ZIPsFS_preloadfileram.c:237-250): CRC of a fully preloaded entry with
 * seed 0, compared with the central-directory CRC, "crc32-mismatch" on
 * stderr and false when they differ.  Input: a file of records
 * [u64 len][u32 expected][u32 seed][len bytes]; a nonzero seed checks the
 * chaining form cg_crc32(data, n, seed) instead.  Output: one line per record
 * "<index> <computed crc hex> ok|mismatch", then the drop-in's path counters.
 */
#include "cg_crc32.c"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static pthread_mutex_t mutex_crc = PTHREAD_MUTEX_INITIALIZER;

static bool check_entry(const void *buf, size_t st_size, uint32_t seed, uint32_t zipcrc32, uint32_t *computed) {
  const uint32_t crc32 = cg_crc32(buf, st_size, seed, &mutex_crc);
  *computed = crc32;
  if (crc32 != zipcrc32) {
    fprintf(stderr, "crc32-mismatch!  ZIP: %x != computed: %x size=%zu\n", zipcrc32, crc32, st_size);
    return false;
  }
  return true;
}

int main(int argc, char **argv) {
  if (argc != 2) {
    fprintf(stderr, "usage: %s records.bin\n", argv[0]);
    return 2;
  }
  FILE *f = fopen(argv[1], "rb");
  if (!f) return 2;
  /* as ZIPsFS would at startup, outside any lock: device
   * init and staging slots, which the drop-in never creates under
   * mutex_fhandle; without a GPU it fails and the drop-in answers on the host */
  (void)zcrc32_prewarm(2);
  int bad = 0;
  for (int i = 0;; i++) {
    uint64_t len;
    uint32_t expected, seed;
    if (fread(&len, 8, 1, f) != 1) break;
    if (fread(&expected, 4, 1, f) != 1 || fread(&seed, 4, 1, f) != 1) return 2;
    unsigned char *buf = (unsigned char *)malloc(len ? len : 1);
    if (!buf || fread(buf, 1, len, f) != len) return 2;
    uint32_t got = 0;
    const bool ok = check_entry(buf, len, seed, expected, &got);
    printf("%d %08x %s\n", i, got, ok ? "ok" : "mismatch");
    bad += !ok;
    free(buf);
  }
  fclose(f);
  uint64_t gpu = 0, host = 0, fallback = 0;
  zcrc32_dropin_stats(&gpu, &host, &fallback);
  printf("stats gpu=%llu host=%llu fallback=%llu\n", (unsigned long long)gpu, (unsigned long long)host,
         (unsigned long long)fallback);
  return bad ? 1 : 0;
}
