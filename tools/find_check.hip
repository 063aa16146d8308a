// tools/find_check.hip -- host build of the block-parallel inflate's block-
// start test (zipsfs_amd/csrc/zcrc_inflate_find.h) for the CPU test
// tests/test_inflate_find.py: flags[q] = quick filter (head_ok && cl_ok) | full_ok << 1 for
// every bit position q of a stream, with the stream staged as the finder
// kernel stages it (little-endian words, zeros past the end).  Test tooling.
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../zipsfs_amd/csrc/zcrc_inflate_find.h"

extern "C" int find_flags(const uint8_t *data, size_t n, uint8_t *flags) {
  std::vector<uint32_t> w((n + 3) / 4 + 8, 0u);
  memcpy(w.data(), data, n);
  uint8_t sorted[20];
  for (size_t q = 0; q < 8 * n; q++) {
    const size_t i = q >> 5;
    uint32_t x0, x1, x2;
    zcrc::find::window96(w[i], w[i + 1], w[i + 2], w[i + 3], (uint32_t)(q & 31), x0, x1, x2);
    const bool a = zcrc::find::head_ok(x0) && zcrc::find::cl_ok(x0, x1, x2);
    const bool b = a && zcrc::find::full_ok(w.data(), (uint32_t)q, (uint32_t)(8 * n - q), sorted);
    flags[q] = (uint8_t)(a | (b << 1));
  }
  return 0;
}
