/*
 * oracle/ref_shim.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Compiles the reference's own src/cg_crc32.c where it lies under
 * /root/reference (included by path via -I, never copied into this repo)
 * and exports its static cg_crc32() under a linkable name, so that
 * tests/golden/gen_golden.py can generate golden vectors from the reference
 * itself and bench.py can time it as the CPU baseline ("kind": "reference").
 * Output goes to oracle/_ref/ only (git-ignored).
 */
#include <pthread.h>
#include <stdint.h>
#include <stddef.h>
#include "cg_crc32.c" /* /root/reference/src/cg_crc32.c:26 static cg_crc32 */

static pthread_mutex_t ref_init_mutex = PTHREAD_MUTEX_INITIALIZER;

uint32_t ref_cg_crc32(const void *data, size_t n_bytes, uint32_t crc) {
  return cg_crc32(data, n_bytes, crc, &ref_init_mutex);
}
