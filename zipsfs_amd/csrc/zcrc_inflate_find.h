// zcrc_inflate_find.h -- the block-start test of the block-parallel inflate
// (zcrc_inflate_split.hip, inflate_find_kernel): is there a valid dynamic-
// Huffman block header at bit q of a staged window?  Host and device: the
// CPU test tests/test_inflate_find.py runs these same functions over every
// bit position of zlib streams (tools/find_check.hip) and checks them
// against the model's exact header decode (tests/inflate_split_model.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace zcrc {
namespace find {

// 64 bits of the staged window starting at bit q (LSB first)
__host__ __device__ inline uint64_t bits64(const uint32_t *w, uint32_t q) {
  const uint32_t i = q >> 5, s = q & 31u;
  const uint64_t lo = (((uint64_t)w[i + 1] << 32) | w[i]) >> s;
  const uint64_t hi = s ? ((uint64_t)w[i + 2] << (64 - s)) : 0ull;
  return lo | hi;
}

// Quick filter, in two parts, on the 96 bits x0 | x1 << 32 | x2 << 64 that
// start at the candidate position.  head_ok: BTYPE = 2, HLIT <= 29, HDIST
// <= 29 (~22% of the positions of compressed data pass).  cl_ok: the
// HCLEN + 4 code-length code lengths (3 bits each, after the 17 header bits)
// form a complete code -- zlib rejects an incomplete one (~0.4% of those
// pass; tests/test_inflate_find.py).  The finder runs cl_ok only on the
// positions head_ok kept.
__host__ __device__ inline bool head_ok(uint32_t x0) {
  return ((x0 >> 1) & 3u) == 2u && ((x0 >> 3) & 31u) <= 29u && ((x0 >> 8) & 31u) <= 29u;
}
__host__ __device__ inline bool cl_ok(uint32_t x0, uint32_t x1, uint32_t x2) {
  const uint32_t hclen = ((x0 >> 13) & 15u) + 4u;
  uint64_t cl = (uint64_t)(x0 >> 17) | ((uint64_t)x1 << 15) | ((uint64_t)x2 << 47);
  cl &= (1ull << (3 * hclen)) - 1;  // 3 hclen <= 57
  uint32_t kraft = 0;  // units of 2^-7
#pragma unroll
  for (uint32_t i = 0; i < 19; i++) {
    const uint32_t l = (uint32_t)(cl >> (3 * i)) & 7u;
    kraft += (128u >> l) & (0u - (uint32_t)(l != 0));
  }
  return kraft == 128u;
}

// the 96 bits from bit b (< 32) of the words w0..w3
__host__ __device__ inline void window96(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t b, uint32_t &x0,
                                         uint32_t &x1, uint32_t &x2) {
  x0 = (uint32_t)((((uint64_t)w1 << 32) | w0) >> b);
  x1 = (uint32_t)((((uint64_t)w2 << 32) | w1) >> b);
  x2 = (uint32_t)((((uint64_t)w3 << 32) | w2) >> b);
}

// The full dynamic-header check at bit q (lane-parallel: each thread its own
// position): decode the literal/length and distance code lengths with the
// code-length code and apply zlib 1.2.11's acceptance rules (as
// oracle/inflate_port.c dynamic(); the code-length code lengths come in the
// order 16 17 18 0 8 7 9 6 10 5 11 4 12 3 13 2 14 1 15, RFC 1951 3.2.7).
// `avail`: staged bits from q.  sorted:
// this thread's 19-byte scratch for the canonical symbol order.
__host__ __device__ __forceinline__ bool full_ok(const uint32_t *w, uint32_t q, uint32_t avail, uint8_t *sorted) {
  const uint64_t v = bits64(w, q);
  const uint32_t nlen = (uint32_t)((v >> 3) & 31u) + 257u, ndist = (uint32_t)((v >> 8) & 31u) + 1u;
  const uint32_t hclen = (uint32_t)((v >> 13) & 15u) + 4u;
  const uint64_t cl = bits64(w, q + 17);
  uint32_t len_of[19];
#define ZCL(i) ((i) < hclen ? (uint32_t)(cl >> (3 * (i))) & 7u : 0u)
  len_of[16] = ZCL(0);
  len_of[17] = ZCL(1);
  len_of[18] = ZCL(2);
  len_of[0] = ZCL(3);
  len_of[8] = ZCL(4);
  len_of[7] = ZCL(5);
  len_of[9] = ZCL(6);
  len_of[6] = ZCL(7);
  len_of[10] = ZCL(8);
  len_of[5] = ZCL(9);
  len_of[11] = ZCL(10);
  len_of[4] = ZCL(11);
  len_of[12] = ZCL(12);
  len_of[3] = ZCL(13);
  len_of[13] = ZCL(14);
  len_of[2] = ZCL(15);
  len_of[14] = ZCL(16);
  len_of[1] = ZCL(17);
  len_of[15] = ZCL(18);
#undef ZCL
  uint32_t cnt[8];
#pragma unroll
  for (uint32_t L = 0; L < 8; L++) cnt[L] = 0;
  uint32_t k = 0;
#pragma unroll
  for (uint32_t L = 1; L < 8; L++) {
#pragma unroll
    for (uint32_t s = 0; s < 19; s++) {
      if (len_of[s] == L) {
        sorted[k] = (uint8_t)s;
        k++;
        cnt[L]++;
      }
    }
  }
  // canonical code of each length: first code (MSB-first numbering) and
  // the index of its first symbol in `sorted`
  uint32_t first[8], base[8];
  {
    uint32_t code = 0, index = 0;
#pragma unroll
    for (uint32_t L = 1; L < 8; L++) {
      first[L] = code;
      base[L] = index;
      index += cnt[L];
      code = (code + cnt[L]) << 1;
    }
  }
  uint32_t p = q + 17 + 3 * hclen;  // next bit
  const uint32_t total = nlen + ndist, end = q + avail;
  uint32_t idx = 0, prev = 0, kll = 0, kd = 0, mll = 0, md = 0;
  bool eob = false;
  // a register bit buffer: bb holds the bits from p on (nb of them, >= 32
  // at every symbol), refilled one aligned word at a time, so a symbol
  // costs no dependent LDS read (bits64 per symbol did: 3 reads on the chain)
  uint32_t wi = (p >> 5) + 1, nb = 32 - (p & 31u);
  uint64_t bb = w[p >> 5] >> (p & 31u);
  while (idx < total) {
    if (p + 32 > end) return false;  // the header would run past the staged bytes
    if (nb < 32) {
      bb |= (uint64_t)w[wi++] << nb;
      nb += 32;
    }
    const uint32_t b = (uint32_t)bb;
    // branch-free canonical decode: the code's first L bits, MSB first, are
    // rev7 >> (7 - L); the symbol's length is the smallest L whose codes
    // [first, first + cnt) contain them (a prefix code: exactly one, or none
    // for an incomplete code)
    const uint32_t rev7 = __builtin_bitreverse32(b) >> 25;
    uint32_t used = 0, at = 0;
#pragma unroll
    for (uint32_t L = 7; L >= 1; L--) {
      const uint32_t d = (rev7 >> (7 - L)) - first[L];
      const bool hit = d < cnt[L];
      used = hit ? L : used;
      at = hit ? base[L] + d : at;
    }
    const uint32_t sym = used ? sorted[at] : 32u;
    if (sym == 32) return false;
    const uint32_t x = b >> used;
    uint32_t val, rep, extra;
    if (sym < 16) {
      val = sym;
      rep = 1;
      prev = sym;
      extra = 0;
    } else if (sym == 16) {
      if (idx == 0) return false;
      val = prev;
      rep = 3 + (x & 3u);
      extra = 2;
    } else if (sym == 17) {
      val = 0;
      rep = 3 + (x & 7u);
      extra = 3;
      prev = 0;
    } else {
      val = 0;
      rep = 11 + (x & 127u);
      extra = 7;
      prev = 0;
    }
    p += used + extra;  // <= 14 bits of the >= 32 buffered
    bb >>= used + extra;
    nb -= used + extra;
    if (idx + rep > total) return false;
    if (val) {
      // split the run at the literal/length | distance boundary
      const uint32_t in_ll = idx < nlen ? (nlen - idx < rep ? nlen - idx : rep) : 0u;
      kll += in_ll << (15 - val);
      kd += (rep - in_ll) << (15 - val);
      if (in_ll) mll = val > mll ? val : mll;
      if (rep > in_ll) md = val > md ? val : md;
      if (idx <= 256 && 256 < idx + rep) eob = true;
      // over-subscribed already: reject now (garbage positions get here
      // after a few dozen lengths instead of decoding all HLIT + HDIST)
      if (kll > 32768u || kd > 32768u) return false;
    }
    idx += rep;
  }
  if (!eob) return false;
  if (kll > 32768u || (kll < 32768u && mll != 1u)) return false;
  if (kd > 32768u || (kd < 32768u && md > 1u)) return false;
  return true;
}

}  // namespace find
}  // namespace zcrc
