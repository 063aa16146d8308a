// zcrc_gf2.h -- GF(2) algebra for CRC-32/ISO-HDLC (zlib crc32), host + device.
//
// Everything here works on the *raw* CRC register in the reflected bit order
// used by zlib and by ZIPsFS's src/cg_crc32.c (reflected polynomial
// 0xEDB88320, src/cg_crc32.c:11).  A register value r stands for the
// polynomial R(x) = sum_b bit_b(r) * x^(31-b), so the constant 1 is
// 0x80000000 and "feed k zero bits" is multiplication by x^k mod P.
//
// zlib semantics that the engine reproduces:
//   crc32(seed, M) = ~( (~seed) * x^(8|M|)  xor  raw(M) )
// where raw(M) is the register after feeding M from a zero register.  For
// |M| >= 4 the (~seed) term is the same as xoring ~seed into M's first four
// bytes, which is how the kernels inject the seed.
//
// Two primitives carry the whole engine:
//   * gf2_mul(a,b)           -- a*b mod P (bit-serial, used off the hot loop)
//   * MCT(c)[j][v]           -- "multiply-by-constant" byte tables:
//                               r*c = xor_j MCT(c)[j][byte_j(r)]
// The braided slice-by-4 table of the hot loop is MCT(x^(8*1024)): feeding a
// 4-byte word followed by 1020 zero bytes (see zcrc_kernels.hip).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define ZCRC_HD __host__ __device__ inline
#else
#define ZCRC_HD inline
#endif

namespace zcrc {

constexpr uint32_t kPolyReflected = 0xEDB88320u;  // src/cg_crc32.c:11
constexpr uint32_t kOne = 0x80000000u;            // x^0 in reflected order

// r * x (one zero bit through the register).
ZCRC_HD constexpr uint32_t gf2_times_x(uint32_t r) { return (r >> 1) ^ (kPolyReflected & (0u - (r & 1u))); }

// r * x^-1.  Exact because P(0) = 1: the reflected polynomial has bit 31 set,
// so a set bit 31 after the forward step can only come from the reduction.
ZCRC_HD uint32_t gf2_times_xinv(uint32_t r) {
  return (r & 0x80000000u) ? (((r ^ kPolyReflected) << 1) | 1u) : (r << 1);
}

// a * b mod P.
ZCRC_HD constexpr uint32_t gf2_mul(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
  for (int i = 0; i < 32; i++) {
    p ^= b & (0u - ((a >> (31 - i)) & 1u));
    b = gf2_times_x(b);
  }
  return p;
}

// x^(2^k) for k = 0..66 is built once on the host; x^n by square-and-multiply.
struct XPowTable {
  uint32_t x2k[67];  // x2k[k] = x^(2^k) mod P
};

inline void build_xpow_table(XPowTable &t) {
  uint32_t v = kOne >> 1;  // x^1
  t.x2k[0] = v;
  for (int k = 1; k < 67; k++) {
    v = gf2_mul(v, v);
    t.x2k[k] = v;
  }
}

// x^(8*nbytes) mod P  (multiplier that moves a register over nbytes zeros).
inline uint32_t gf2_xpow8(const XPowTable &t, uint64_t nbytes) {
  uint32_t acc = kOne;
  int k = 3;  // 8*nbytes = nbytes << 3
  while (nbytes) {
    if (nbytes & 1u) acc = gf2_mul(acc, t.x2k[k]);
    nbytes >>= 1;
    k++;
  }
  return acc;
}

// x^(-8*nbytes) mod P, for small nbytes (table construction only).
inline uint32_t gf2_xinvpow8_small(uint32_t nbytes) {
  uint32_t r = kOne;
  for (uint32_t i = 0; i < 8u * nbytes; i++) r = gf2_times_xinv(r);
  return r;
}

// MCT(c): table[j*256 + v] = (v << 8j) * c.
inline void build_mct(uint32_t c, uint32_t *table /* 4*256 */) {
  for (int j = 0; j < 4; j++)
    for (uint32_t v = 0; v < 256; v++) table[j * 256 + v] = gf2_mul(c, v << (8 * j));
}

// Compile-time products for building an MCT in registers (the per-buffer
// mode's braid, zcrc_batch_kernel.h) for c = x^(2^k): q[p] = c * (1 << p),
// so that MCT(c)[j][v] = xor over the set bits b of v of q[8j + b].
template <int k>
struct MctBasis {
  uint32_t q[32];
  constexpr MctBasis() : q{} {
    uint32_t c = kOne >> 1;  // x
    for (int i = 0; i < k; i++) c = gf2_mul(c, c);
    for (int p = 0; p < 32; p++) q[p] = gf2_mul(c, 1u << p);
  }
};

// The same for c = x^(-8 nbytes) (the combine tables, TableBlob::comb).
ZCRC_HD constexpr uint32_t gf2_times_xinv_c(uint32_t r) {
  return (r & 0x80000000u) ? (((r ^ kPolyReflected) << 1) | 1u) : (r << 1);
}
template <int nbytes>
struct MctBasisInv {
  uint32_t q[32];
  constexpr MctBasisInv() : q{} {
    uint32_t c = kOne;
    for (int i = 0; i < 8 * nbytes; i++) c = gf2_times_xinv_c(c);
    for (int p = 0; p < 32; p++) q[p] = gf2_mul(c, 1u << p);
  }
};

// Standard reflected byte table T[v] = raw CRC of the single byte v.
inline void build_std_table(uint32_t *table /* 256 */) {
  for (uint32_t v = 0; v < 256; v++) {
    uint32_t r = v;
    for (int b = 0; b < 8; b++) r = gf2_times_x(r);
    table[v] = r;
  }
}

// The inverse byte step: r * x^-8 = (r << 8) ^ W[r >> 24].  The forward
// step is r' = (r >> 8) ^ T[r & 0xFF], and the top bytes of T[0..255] are a
// permutation, so v = r & 0xFF is the entry whose top byte is r' >> 24, and
// r = ((r' ^ T[v]) << 8) | v.  W[T[v] >> 24] = (T[v] << 8) | v.
inline void build_xinv8_table(uint32_t *w /* 256 */) {
  uint32_t t[256];
  build_std_table(t);
  for (uint32_t v = 0; v < 256; v++) w[t[v] >> 24] = (t[v] << 8) | v;
}

// Host-side combine: zlib crc32_combine semantics.
//   crc(A || B) = combine(crc(A), crc(B), |B|)
inline uint32_t gf2_crc_combine(const XPowTable &t, uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
  return gf2_mul(gf2_xpow8(t, len_b), crc_a) ^ crc_b;
}

}  // namespace zcrc
