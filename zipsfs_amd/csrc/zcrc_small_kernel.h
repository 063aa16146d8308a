// zcrc_small_kernel.h -- batched CRC-32 of small whole buffers (<= kSmallMax).
//
// The batch kernel (zcrc_batch_kernel.h) gives every piece a whole wave: 64
// lanes x 16 B per 1 KiB block, then a 6-level fold.  A 1-4 KiB buffer -- the
// typical ZIP entry, SURVEY 8(d) config 4's median is 3,971 B -- leaves that
// wave with one or four blocks in flight between two long dependent phases
// (descriptor, load, fold), so uniform 1 KiB batches ran at 1.1 TB/s and 4 KiB
// at 3.0 (tools/small_probe).  Here a group of G lanes owns one buffer (64/G
// buffers per wave):
//   * blocks are 256 B; lane l of a group reads the C = 16/G consecutive 16-B
//     chunks at 16 C l of every block, so each of its 4C dword streams
//     advances 256 B per block and one braided table, MCT(x^2048)
//     (TableBlob::braid256), serves every stream -- the same conflict-free
//     32x replicated LDS layout as the batch kernel's MCT(x^8192);
//   * a buffer is aligned to its own 16-B-aligned end, and blocks before a
//     shorter buffer's start load nothing (leading zeros are free in the raw
//     domain, as in the batch kernel);
//   * fold: log2(4C) in-lane levels, log2(G) cross-lane levels (combine
//     tables x^-32 .. x^-1024, TableBlob::comb 0..5), then the trailing
//     padding is undone (x^-32/x^-64 tables, then the x^-8 byte table in
//     table 7's unused LDS);
//   * up to kD blocks of loads are in flight before their braid steps, and
//     the next group's descriptor is loaded while the current one runs.
// Persistent: one 1024-thread workgroup per CU, waves walk groups of buffers
// with a grid stride.  tools/quad_probe (profiles/r02/small_kernel/) measured
// 16 lanes: 4 KiB 5.46 TB/s, 8 KiB 5.81, 3000 B 5.34; 8 lanes: 1 KiB 3.63.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "zcrc_batch_kernel.h"

namespace zcrc {

typedef unsigned int small_v4u __attribute__((ext_vector_type(4)));

// Workgroup blk of nblk (the persistent grid, or the batch kernel's
// workgroups that the split plan gave to the small list).
// chunk of the combine area where the x^-8 byte table goes (table 7's)
constexpr uint32_t kXinv8Chunk = 7u * 256u;

// kAblate == 1 (measurement builds, zcrc32_batch_device_read_ceiling): the
// braid steps become one VALU rotate each -- the same loads, no lookups.
// kCoal (G = 8): lane l of a group reads the 16-B chunks at 16 l and 16 l +
// 128 of every 256-B block, so that each load instruction covers 128
// contiguous bytes per buffer (the round-2 layout gave lane l the chunks at
// 32 l and 32 l + 16: every load touched half of each 128-B line of its
// buffer, and a pure read in that layout ran at 6.0 TB/s on 1 KiB buffers
// against 6.8 for 16 lanes, tools/ceiling_probe, profiles/r05/s4).
template <bool kStrided, int G, int kD, int kAblate, bool kCoal>
__device__ __forceinline__ void small_body(const SmallArgs &a, uint32_t *s_lds, uint64_t n, uint32_t blk,
                                           uint32_t nblk) {
  static_assert(G == 8 || G == 16, "lanes per buffer");
  constexpr int C = 16 / G, NS = 4 * C, LOG_NS = NS == 4 ? 2 : 3, LOG_G = G == 8 ? 3 : 4;
  constexpr uint32_t BPW = 64 / G;  // buffers per wave
  const uint32_t tid = threadIdx.x, lane = tid & 63u, g = lane / G, lg = lane % G;
  const uint64_t waves = (uint64_t)nblk * kWaves;
  const uint64_t nq = (n + BPW - 1) / BPW;
  uint64_t q = (uint64_t)blk * kWaves + (tid >> 6);
  if ((uint64_t)blk * kWaves >= nq) return;  // whole workgroup idle: skip the table fill

  // descriptor of list entry k (buffer index, start, length, seed)
  auto desc = [&](uint64_t k, uint64_t &j, uint64_t &p, uint64_t &l, uint32_t &sd) {
    if (kStrided) {
      j = k;
      p = reinterpret_cast<uint64_t>(a.base) + k * a.stride;
      l = a.len;
    } else {
      if (a.sdesc) {  // split plan: one 16-B load, no dependent descriptor loads
        const uint4 d = a.sdesc[k];
        const uint64_t pw = (uint64_t)d.x | ((uint64_t)d.y << 32);
        j = d.z;
        p = pw & 0xFFFFFFFFFFFFull;
        l = pw >> 48;
        sd = d.w;
        return;
      }
      j = k;
      p = reinterpret_cast<uint64_t>(a.ptrs[j]);
      l = a.lens ? a.lens[j] : a.prefix[j + 1] - a.prefix[j];
    }
    sd = a.seeds ? a.seeds[j] : 0u;
  };
  uint64_t nx_j = 0, nx_p = 0, nx_l = 0;
  uint32_t nx_s = 0;
  if (BPW * q + g < n) desc(BPW * q + g, nx_j, nx_p, nx_l, nx_s);

  {  // LDS: braided MCT(x^2048) | combine tables (batch kernel's layout)
    uint4 *dst = reinterpret_cast<uint4 *>(s_lds);
    const uint32_t *b = a.tab->braid256;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t o = 16u * (tid + 1024u * k);
      const uint32_t v = b[(((o >> 16) << 1) | ((o >> 7) & 1u)) * 256u + ((o >> 8) & 255u)];
      dst[tid + 1024u * k] = make_uint4(v, v, v, v);
    }
    // combine tables 0..5 (6 and 7 are not used here); the first 256 words of
    // table 7's area hold the x^-8 byte table for the trailing padding
    const uint4 *cs = reinterpret_cast<const uint4 *>(a.tab->comb);
    uint4 *cd = reinterpret_cast<uint4 *>(s_lds + kLdsCombDword);
    cd[tid] = cs[tid];
    cd[tid + 1024u] = tid >= kXinv8Chunk - 1024u && tid < kXinv8Chunk - 1024u + 64u
                          ? reinterpret_cast<const uint4 *>(a.tab->xinv8)[tid - (kXinv8Chunk - 1024u)]
                          : cs[tid + 1024u];
  }
  __syncthreads();
  const uint32_t lo0 = (lane & 31u) * 4u;
  const uint32_t o0 = lo0, o1 = lo0 + 128u, o2 = lo0 + 65536u, o3 = lo0 + 65536u + 128u;

  for (; q < nq; q += waves) {
    const uint64_t bi = BPW * q + g;
    const bool active = bi < n;
    const uint64_t j = nx_j, pstart = nx_p;
    const uint32_t len = active ? (uint32_t)nx_l : 0u, seed = nx_s;
    if (bi + BPW * waves < n) desc(bi + BPW * waves, nx_j, nx_p, nx_l, nx_s);
    const bool tiny = len < 4u;  // bytewise below (the 4-byte seed injection needs 4 bytes)
    const uint64_t astart = pstart & ~(uint64_t)15;
    const int32_t rs = (int32_t)(pstart & 15u), re = rs + (int32_t)len, span = (re + 15) & ~15;
    const uint32_t inj = ~seed;
    const uint32_t kq = (active && !tiny) ? (uint32_t)(span + 255) >> 8 : 0u;
    const uint32_t kmax = uni32(__reduce_max_sync(0xFFFFFFFFFFFFFFFFull, kq));
    // stream t's register is s[t] ^ q[t] (q: the last step's fourth lookup,
    // taken into the next index by a three-input xor; zcrc_batch_kernel.h
    // piece_raw, ZCRC_STEP2)
    uint32_t s[NS], q[NS];
#pragma unroll
    for (int t = 0; t < NS; t++) s[t] = 0u, q[t] = 0u;
    // chunk c of lane lg: 16 C lg + 16 c (kCoal: 16 lg + 16 G c) in every block
    constexpr int32_t kLaneStep = kCoal ? 16 : 16 * C, kChunkStep = kCoal ? 16 * G : 16;
    int32_t rel0 = kq ? span - 256 * (int32_t)kmax + kLaneStep * (int32_t)lg : -(1 << 30);
    for (uint32_t k = 0; k < kmax; k += kD) {
      small_v4u d[kD][C];
#pragma unroll
      for (int b = 0; b < kD; b++)
#pragma unroll
        for (int c = 0; c < C; c++) {
          const int32_t rel = rel0 + 256 * b + kChunkStep * c;
          d[b][c] = (small_v4u)(0u);
          if (k + b < kmax && rel >= 0)
            d[b][c] = __builtin_nontemporal_load(reinterpret_cast<const small_v4u *>(astart + (uint32_t)rel));
        }
#pragma unroll
      for (int b = 0; b < kD; b++) {
        if (k + b < kmax) {
#pragma unroll
          for (int c = 0; c < C; c++) {
            const int32_t rel = rel0 + 256 * b + kChunkStep * c;
            uint4 w = make_uint4(d[b][c].x, d[b][c].y, d[b][c].z, d[b][c].w);
            if (rel >= 0 && (rel < rs + 4 || rel + 16 > re))
              w = fix_chunk(w, clamp_rel(rs - rel), clamp_rel(re - rel), clamp_rel(rs - rel), inj);
            if (kAblate == 1) {
              s[4 * c + 0] = __builtin_amdgcn_alignbit(s[4 * c + 0] ^ w.x, s[4 * c + 0] ^ w.x, 5);
              s[4 * c + 1] = __builtin_amdgcn_alignbit(s[4 * c + 1] ^ w.y, s[4 * c + 1] ^ w.y, 5);
              s[4 * c + 2] = __builtin_amdgcn_alignbit(s[4 * c + 2] ^ w.z, s[4 * c + 2] ^ w.z, 5);
              s[4 * c + 3] = __builtin_amdgcn_alignbit(s[4 * c + 3] ^ w.w, s[4 * c + 3] ^ w.w, 5);
            } else {
              braid_step2(s_lds, s[4 * c + 0], q[4 * c + 0], w.x, o0, o1, o2, o3);
              braid_step2(s_lds, s[4 * c + 1], q[4 * c + 1], w.y, o0, o1, o2, o3);
              braid_step2(s_lds, s[4 * c + 2], q[4 * c + 2], w.z, o0, o1, o2, o3);
              braid_step2(s_lds, s[4 * c + 3], q[4 * c + 3], w.w, o0, o1, o2, o3);
            }
          }
        }
      }
      rel0 += 256 * kD;
    }
#pragma unroll
    for (int t = 0; t < NS; t++) s[t] ^= q[t];
    uint32_t r;
    if (kCoal && C == 2) {
      // fold, kCoal: a chunk's dwords 4 and 8 B apart (combine tables 0, 1),
      // the lane's two chunks 16 G = 128 B apart (table 5), lanes 16 B apart
      // (tables 2, 3, 4: the table c moves a register back 4 * 2^c bytes)
#pragma unroll
      for (int m = 0; m < NS; m += 2) s[m] ^= comb_apply(s_lds, 0, s[m + 1]);
      s[0] ^= comb_apply(s_lds, 1, s[2]);
      s[4] ^= comb_apply(s_lds, 1, s[6]);
      s[0] ^= comb_apply(s_lds, 5, s[4]);
      r = s[0];
      r ^= row_shl<1>(comb_apply(s_lds, 2, r));
      r ^= row_shl<2>(comb_apply(s_lds, 3, r));
      r ^= row_shl<4>(comb_apply(s_lds, 4, r));
    } else {
      // fold: the lane's dwords sit 4 B apart, lanes 16 C B apart
#pragma unroll
      for (int t = 0; t < LOG_NS; t++)
#pragma unroll
        for (int m = 0; m < NS; m += 2 << t) s[m] ^= comb_apply(s_lds, t, s[m + (1 << t)]);
      // cross-lane levels inside the group (8 or 16 lanes: within a DPP row)
      r = s[0];
      r ^= row_shl<1>(comb_apply(s_lds, LOG_NS + 0, r));
      r ^= row_shl<2>(comb_apply(s_lds, LOG_NS + 1, r));
      r ^= row_shl<4>(comb_apply(s_lds, LOG_NS + 2, r));
      if (LOG_G == 4) r ^= row_shl<8>(comb_apply(s_lds, LOG_NS + 3, r));
    }
    const uint32_t tpad = (uint32_t)(span - re), a4 = tpad >> 2;
    if (a4 & 2u) r = comb_apply(s_lds, 1, r);
    if (a4 & 1u) r = comb_apply(s_lds, 0, r);
    // the last 0-3 bytes: one x^-8 byte-table step each (24 bit steps before:
    // ~100 VALU per buffer group, as much as a 1 KiB buffer's braid steps)
    const uint32_t *xinv8 = s_lds + kLdsCombDword + 4u * kXinv8Chunk;
    for (uint32_t b = 0; b < 3u; b++)
      if (b < (tpad & 3u)) r = (r << 8) ^ xinv8[r >> 24];
    if (active && lg == 0) {
      if (tiny) {
        const uint8_t *bp = reinterpret_cast<const uint8_t *>(pstart);
        r = ~seed;
        for (uint32_t p = 0; p < len; p++) r = (r >> 8) ^ a.tab->stdtab[(r ^ bp[p]) & 0xFFu];
      }
      a.out[j] = ~r;
    }
  }
}

template <bool kStrided, int G, int kD, bool kCoal = false>
__global__ __launch_bounds__(1024) void crc32_small_kernel(SmallArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t s_lds[kLdsBytes / 4];
  small_body<kStrided, G, kD, 0, kCoal>(a, s_lds, a.n, blockIdx.x, gridDim.x);
}

}  // namespace zcrc
