/*
 * zipsfs_amd/cg_crc32.c -- drop-in replacement for ZIPsFS src/cg_crc32.c.
 *
 * ZIPsFS textually includes "cg_crc32.c" (src/ZIPsFS_preloadfileram.c:11)
 * and calls the static function below once per fully preloaded ZIP entry
 * (fhandle_check_crc32, src/ZIPsFS_preloadfileram.c:243).  This file keeps
 * the reference's include guard (src/cg_crc32.c:1-2) and the exact static
 * signature (src/cg_crc32.c:26) and forwards to libzcrc, which computes the
 * CRC (zlib crc32 semantics, bit-exact to the reference): on the MI355X for
 * entries of at least the GPU threshold, on libzcrc's host CRC below it.
 *
 * Build change on the ZIPsFS side: put this directory
 * before src/ on the include path, add -I<repo>/include and
 * -L<repo>/zipsfs_amd -lzcrc -Wl,-rpath,<repo>/zipsfs_amd to the link line.
 *
 * `mutex` only guarded the reference's lazy table initialisation
 * (src/cg_crc32.c:31-36); libzcrc initialises its device tables once per
 * process internally, so the argument is accepted and unused.
 * Like the reference, this never fails: zcrc32() answers from libzcrc's
 * host CRC when the GPU cannot (include/zcrc.h, "Drop-in contract").
 */
#ifndef _cg_crc32_dot_c
#define _cg_crc32_dot_c

#include <inttypes.h>
#include <stddef.h>
#include <pthread.h>
#include <stdbool.h>

#include "zcrc.h"

static uint32_t cg_crc32(const void *data, size_t n_bytes, uint32_t crc, pthread_mutex_t *mutex) {
  (void)mutex;
  return zcrc32(data, n_bytes, crc);
}
#endif  // _cg_crc32_dot_c
