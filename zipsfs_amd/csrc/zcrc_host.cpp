// zcrc_host.cpp -- libzcrc's own host CRC-32, for the drop-in's contract.
//
// the function ZIPsFS calls, cg_crc32 (src/cg_crc32.c:26-49),
// has no error path and runs while mutex_fhandle is held
// (src/ZIPsFS_preloadfileram.c:309-321).  Its replacement zcrc32() must
// therefore answer even when the GPU cannot (no device, a HIP error) and
// should not pay a PCIe round trip for an entry a core checksums faster.
// This file is that answer, written for this library: carry-less-multiply
// folding (PCLMULQDQ, eight 128-bit lanes) for long inputs, slicing-by-16
// tables for short inputs, tails and CPUs without PCLMUL.  The batched and
// device-resident entry points never use it (include/zcrc.h).
//
// Folding, in the reflected domain the CRC works in (bit i of a 128-bit
// block <-> coefficient of x^(127-i)): a lane A = A_hi x^64 + A_lo moved F
// bits forward is A_hi x^(64+F) + A_lo x^F, congruent mod P to
// clmul(A_hi, x^(63+F) mod P) ^ clmul(A_lo, x^(F-1) mod P): a reflected
// 64x64 product lands one bit low, hence the exponents one below.  The last
// 128-bit residue R satisfies R == message (mod P), so the CRC register is
// the table CRC of R's 16 bytes from register 0, continued over the tail.
#include <stdint.h>
#include <string.h>

#include <mutex>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

#include "zcrc_internal.h"

namespace zcrc {
namespace {

constexpr uint32_t kPolyRefl = 0xEDB88320u;  // x^32 + ... + 1, bit-reversed, x^32 implicit

struct HostTables {
  uint32_t t[16][256];   // t[k][b]: register after byte b then k zero bytes, from 0
  uint64_t fold[8][2];   // fold[k-1] = {x^(128k+63), x^(128k-1)} mod P, reflected-64
};

HostTables g_tab;
bool g_pclmul = false;

// x^m mod P, reflected 32-bit form (bit i <-> coefficient of x^(31-i))
uint32_t xpow_mod(uint32_t m) {
  uint32_t r = 0x80000000u;  // x^0
  for (uint32_t i = 0; i < m; i++) r = (r >> 1) ^ ((r & 1u) ? kPolyRefl : 0u);
  return r;
}

void init_tables() {
  for (uint32_t b = 0; b < 256; b++) {
    uint32_t c = b;
    for (int k = 0; k < 8; k++) c = (c >> 1) ^ ((c & 1u) ? kPolyRefl : 0u);
    g_tab.t[0][b] = c;
  }
  for (int k = 1; k < 16; k++)
    for (uint32_t b = 0; b < 256; b++) {
      const uint32_t c = g_tab.t[k - 1][b];
      g_tab.t[k][b] = (c >> 8) ^ g_tab.t[0][c & 0xFFu];
    }
  // reflected-32 (degree d at bit 31-d) -> reflected-64 (degree d at bit 63-d)
  for (uint32_t k = 1; k <= 8; k++) {
    g_tab.fold[k - 1][0] = (uint64_t)xpow_mod(128 * k + 63) << 32;
    g_tab.fold[k - 1][1] = (uint64_t)xpow_mod(128 * k - 1) << 32;
  }
#if defined(__x86_64__)
  __builtin_cpu_init();
  g_pclmul = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse2");
#endif
}

const HostTables &tables() {
  static std::once_flag once;
  std::call_once(once, init_tables);
  return g_tab;
}

inline uint32_t load_le32(const uint8_t *p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;  // little-endian host (x86-64, as the reference assumes)
}

// register update (no pre/post inversion) over n bytes, slicing by 16
uint32_t update_tables(const HostTables &T, uint32_t reg, const uint8_t *p, size_t n) {
  while (n >= 16) {
    const uint32_t a = load_le32(p) ^ reg, b = load_le32(p + 4), c = load_le32(p + 8), d = load_le32(p + 12);
    reg = T.t[15][a & 0xFF] ^ T.t[14][(a >> 8) & 0xFF] ^ T.t[13][(a >> 16) & 0xFF] ^ T.t[12][a >> 24] ^
          T.t[11][b & 0xFF] ^ T.t[10][(b >> 8) & 0xFF] ^ T.t[9][(b >> 16) & 0xFF] ^ T.t[8][b >> 24] ^
          T.t[7][c & 0xFF] ^ T.t[6][(c >> 8) & 0xFF] ^ T.t[5][(c >> 16) & 0xFF] ^ T.t[4][c >> 24] ^
          T.t[3][d & 0xFF] ^ T.t[2][(d >> 8) & 0xFF] ^ T.t[1][(d >> 16) & 0xFF] ^ T.t[0][d >> 24];
    p += 16;
    n -= 16;
  }
  while (n--) reg = T.t[0][(reg ^ *p++) & 0xFF] ^ (reg >> 8);
  return reg;
}

#if defined(__x86_64__)
constexpr size_t kLanes = 8;
constexpr size_t kFoldMin = 256;  // below: tables (setup + lane merge cost more than they save)

__attribute__((target("pclmul,sse2"))) inline __m128i fold(__m128i a, __m128i k) {
  return _mm_xor_si128(_mm_clmulepi64_si128(a, k, 0x00), _mm_clmulepi64_si128(a, k, 0x11));
}

__attribute__((target("pclmul,sse2"))) uint32_t update_clmul(const HostTables &T, uint32_t reg, const uint8_t *p,
                                                             size_t n) {
  __m128i x[kLanes];
  for (size_t j = 0; j < kLanes; j++) x[j] = _mm_loadu_si128(reinterpret_cast<const __m128i *>(p + 16 * j));
  x[0] = _mm_xor_si128(x[0], _mm_cvtsi32_si128((int)reg));  // register enters as the first 32 bits
  p += 16 * kLanes;
  n -= 16 * kLanes;
  const __m128i k8 = _mm_loadu_si128(reinterpret_cast<const __m128i *>(T.fold[kLanes - 1]));
  while (n >= 16 * kLanes) {
    for (size_t j = 0; j < kLanes; j++)
      x[j] = _mm_xor_si128(fold(x[j], k8), _mm_loadu_si128(reinterpret_cast<const __m128i *>(p + 16 * j)));
    p += 16 * kLanes;
    n -= 16 * kLanes;
  }
  // lane j sits 128 * (7 - j) bits ahead of the last lane
  __m128i r = x[kLanes - 1];
  for (size_t j = 0; j + 1 < kLanes; j++)
    r = _mm_xor_si128(r, fold(x[j], _mm_loadu_si128(reinterpret_cast<const __m128i *>(T.fold[kLanes - 2 - j]))));
  const __m128i k1 = _mm_loadu_si128(reinterpret_cast<const __m128i *>(T.fold[0]));
  while (n >= 16) {
    r = _mm_xor_si128(fold(r, k1), _mm_loadu_si128(reinterpret_cast<const __m128i *>(p)));
    p += 16;
    n -= 16;
  }
  alignas(16) uint8_t res[16];
  _mm_store_si128(reinterpret_cast<__m128i *>(res), r);
  return update_tables(T, update_tables(T, 0u, res, 16), p, n);
}
#endif

}  // namespace

uint32_t host_crc32(const void *data, size_t n, uint32_t crc) {
  const HostTables &T = tables();
  const uint8_t *p = static_cast<const uint8_t *>(data);
  uint32_t reg = ~crc;
#if defined(__x86_64__)
  if (g_pclmul && n >= kFoldMin) return ~update_clmul(T, reg, p, n);
#endif
  return ~update_tables(T, reg, p, n);
}

bool host_crc32_uses_clmul() {
  (void)tables();
  return g_pclmul;
}

}  // namespace zcrc
