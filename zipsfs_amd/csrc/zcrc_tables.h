// zcrc_tables.h -- host construction of the multiply-by-constant table blob.
#pragma once
#include "zcrc_gf2.h"
#include "zcrc_internal.h"

namespace zcrc {

// braid  = MCT(x^(8*1024))            hot loop: 1 KiB per stream step
// braid256 = MCT(x^(8*256))           small-buffer kernel: 256 B per step
// braid128 = MCT(x^(8*128))           small-buffer kernel, 128-B blocks
// comb   = MCT(x^-32 .. x^-4096)      in-lane and cross-lane combine tree
// tshift = MCT(x^(-8t)), t < 16       16-B alignment padding at a piece end
// xinv8  = r * x^-8 byte table         the small-buffer kernel's last 0-3 padding bytes
// x8grain[j][m] = x^(8 * 65536 * m * 256^j)   split pieces: r * x^(8d), d = whole
//                                       64 KiB grains, in at most four products
inline void build_tables(TableBlob &tb) {
  XPowTable xp;
  build_xpow_table(xp);
  build_mct(gf2_xpow8(xp, 1024), tb.braid);
  build_mct(gf2_xpow8(xp, 256), tb.braid256);
  build_mct(gf2_xpow8(xp, 128), tb.braid128);
  const uint32_t comb_bytes[8] = {4, 8, 16, 32, 64, 128, 256, 512};
  for (int c = 0; c < 8; c++) build_mct(gf2_xinvpow8_small(comb_bytes[c]), tb.comb + c * 1024);
  for (int t = 0; t < 16; t++) build_mct(gf2_xinvpow8_small((uint32_t)t), tb.tshift + t * 1024);
  build_std_table(tb.stdtab);
  build_xinv8_table(tb.xinv8);
  for (int k = 0; k < 64; k++) tb.x8pow[k] = xp.x2k[k + 3];
  for (int j = 0; j < 4; j++) {
    const uint32_t base = xp.x2k[19 + 8 * j];  // x^(2^(19 + 8j)) = x^(8 * 65536 * 256^j)
    uint32_t g = kOne;
    for (int m = 0; m < 256; m++) {
      tb.x8grain[j][m] = g;
      g = gf2_mul(g, base);
    }
  }
}

}  // namespace zcrc
