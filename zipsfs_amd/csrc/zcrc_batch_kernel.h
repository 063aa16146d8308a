// zcrc_batch_kernel.h -- the MI355X (gfx950) batched CRC-32 kernel (template).
//
// Replaces the hot loop of ZIPsFS src/cg_crc32.c:37-47 (slice-by-8 table CRC
// over one contiguous RAM buffer, called from fhandle_check_crc32,
// src/ZIPsFS_preloadfileram.c:243) with one persistent launch that checksums
// a whole batch of independent buffers, bit-exact to zlib crc32(seed, ...).
//
// Design (DESIGN.md has the full derivation):
//   * One 1024-thread workgroup per CU (16 waves); the whole 160 KiB LDS holds
//     - a *braided* slice-by-4 table, MCT(x^(8*1024)), replicated 32x so that
//       every lookup of a 32-lane LDS group hits its own bank (conflict-free
//       ds_read_b32 for any data), laid out so that ONE v_perm_b32 turns a
//       data byte into a ready LDS address;
//     - 8 small multiply-by-constant tables for the end-of-piece combine.
//   * Each wave streams 1 KiB blocks: lane l loads 16 B at block + 16 l with
//     one buffer_load_dwordx4 (fully coalesced), 8 blocks in flight.  Lane l
//     runs 4 independent CRC streams (one per dword); every stream advances
//     by exactly 1024 bytes per block, so one table serves all 256 streams:
//         s <- (s xor word) * x^(8*1024)      (4 lookups)
//   * At the end of a piece the 256 stream registers are folded with
//     constant shifts (in-lane x^-32/x^-64, then a 6-level cross-lane tree of
//     x^(-128*2^j)) into one raw register, moved to the piece end with a
//     global-memory MCT (x^(-8t), t = bytes of 16-B alignment padding).
//   * Work split: the concatenated batch (sum of lengths T) is cut into W
//     equal byte ranges, one per wave, with boundaries snapped so that small
//     buffers are never split and split points in large buffers sit at an
//     end-relative 64 KiB grid.  Pieces of a split buffer are moved to the
//     buffer end (x^(8d)) and xor-combined with one atomicXor each.
//   * Bytes outside [piece start, piece end) inside the two boundary 16-B
//     chunks are zeroed in-register; leading padding is free in the raw
//     domain, trailing padding is undone by x^(-8t).  The seed (~crc) is
//     xored into the buffer's first four bytes (zlib chaining semantics).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "zcrc_gf2.h"
#include "zcrc_internal.h"

namespace zcrc {

// ----------------------------------------------------------------- helpers

// kAux: cache-policy bits of the payload loads.  The product streams with
// nt (2): every payload byte is read once, and non-temporal loads lift the
// sustained HBM read rate by ~12% over the default policy on gfx950
// (tools/hbm_probe, tools/crc_variants).
constexpr int kLoadNt = 2;
// per-buffer mode: issue each wave's first 2 kD KiB before its barrier (off:
// measured no faster on 4096 x 64 KiB and 4-6% slower on 16 KiB and 1 KiB
// buffers, because the payload then queues in front of the other waves'
// table and length loads -- tools/crc_ab_fused_np, c2_probe_np,
// profiles/r03/s15-s16; an A/B knob for those tools)
#ifndef ZCRC_PERBUF_PRELOAD
#define ZCRC_PERBUF_PRELOAD 0
#endif
constexpr bool kPerBufPreload = ZCRC_PERBUF_PRELOAD;
// A/B knob (round 6): the plain groups of a piece read in
// the stream-read sweep's issue order -- a group's first 1 KiB block alone,
// a wait for it, then its other kD - 1 blocks -- instead of double-buffered
// groups (kD to 2 kD blocks in flight).  The sweep (zcrc_read_sweep_device)
// issues its loads this way and reads 4-6% faster than every CRC-compatible
// mapping measured in round 5.
#ifndef ZCRC_SWEEP_ORDER
#define ZCRC_SWEEP_ORDER 0
#endif
constexpr bool kSweepOrder = ZCRC_SWEEP_ORDER;

__device__ __forceinline__ uint32_t lds_u32(const uint32_t *lds, uint32_t byte_addr) {
  return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(lds) + byte_addr);
}

// Braided table lookup address for table j (byte j of x):
//   LDS byte address = (j>>1)*65536 + v*256 + (j&1)*128 + (lane&31)*4
// laneoff[j] carries bytes 0 and 2; v_perm drops data byte j into byte 1.
#define ZCRC_SEL(j) (0x0C020400u + ((uint32_t)(j) << 8))

__device__ __forceinline__ uint32_t braid_step(const uint32_t *lds, uint32_t x, uint32_t o0, uint32_t o1,
                                               uint32_t o2, uint32_t o3) {
  const uint32_t a0 = __builtin_amdgcn_perm(x, o0, ZCRC_SEL(0));
  const uint32_t a1 = __builtin_amdgcn_perm(x, o1, ZCRC_SEL(1));
  const uint32_t a2 = __builtin_amdgcn_perm(x, o2, ZCRC_SEL(2));
  const uint32_t a3 = __builtin_amdgcn_perm(x, o3, ZCRC_SEL(3));
  return lds_u32(lds, a0) ^ lds_u32(lds, a1) ^ lds_u32(lds, a2) ^ lds_u32(lds, a3);
}

// The same step on a register kept as two words, r = s ^ q (round 4): the
// index is s ^ q ^ d in one three-input xor, the first three lookups are
// combined by another and the fourth is kept as the new q -- 2 VALU besides
// the 4 address builds, against 4 xors.
__device__ __forceinline__ void braid_step2(const uint32_t *lds, uint32_t &s, uint32_t &q, uint32_t d, uint32_t o0,
                                            uint32_t o1, uint32_t o2, uint32_t o3) {
  const uint32_t x = __builtin_amdgcn_bitop3_b32(s, q, d, 0x96);  // s ^ q ^ d
  const uint32_t t0 = lds_u32(lds, __builtin_amdgcn_perm(x, o0, ZCRC_SEL(0)));
  const uint32_t t1 = lds_u32(lds, __builtin_amdgcn_perm(x, o1, ZCRC_SEL(1)));
  const uint32_t t2 = lds_u32(lds, __builtin_amdgcn_perm(x, o2, ZCRC_SEL(2)));
  q = lds_u32(lds, __builtin_amdgcn_perm(x, o3, ZCRC_SEL(3)));
  s = __builtin_amdgcn_bitop3_b32(t0, t1, t2, 0x96);
}

// The braid entry MCT(x^8192)[j][v] this lane builds for wave `w` of the
// per-buffer mode: j = lane >> 4, v = 4 w + (lane & 3) + 64 ((lane >> 2) & 3),
// as the xor of the compile-time products q[8j + b] over the set bits b of v
// (MctBasis, zcrc_gf2.h).  ~40 VALU on immediates, no memory: the braid then
// needs no load in front of the workgroup's first barrier.  (Selecting among
// elements of a constexpr array compiled to a select of addresses and a load
// from a constant table; MctQ makes every product an immediate.)  tests: the
// per-buffer GPU parity tests read every entry through the hot loop, and
// tests/test_model.py checks the construction against TableBlob::braid.
template <int k, int p>
struct MctQ {
  static constexpr uint32_t value = MctBasis<k>{}.q[p];
};
template <int bit>
__device__ __forceinline__ uint32_t braid_gen_bit(bool j1, bool j2, uint32_t v) {
  const uint32_t q = j2 ? (j1 ? MctQ<13, 24 + bit>::value : MctQ<13, 16 + bit>::value)
                        : (j1 ? MctQ<13, 8 + bit>::value : MctQ<13, bit>::value);
  return ((v >> bit) & 1u) ? q : 0u;
}
__device__ __forceinline__ uint32_t braid_gen_lane(uint32_t lane, uint32_t w) {
  const bool j1 = lane & 16u, j2 = lane & 32u;  // j = lane >> 4
  const uint32_t v = 4u * w + (lane & 3u) + 64u * ((lane >> 2) & 3u);
  return braid_gen_bit<0>(j1, j2, v) ^ braid_gen_bit<1>(j1, j2, v) ^ braid_gen_bit<2>(j1, j2, v) ^
         braid_gen_bit<3>(j1, j2, v) ^ braid_gen_bit<4>(j1, j2, v) ^ braid_gen_bit<5>(j1, j2, v) ^
         braid_gen_bit<6>(j1, j2, v) ^ braid_gen_bit<7>(j1, j2, v);
}

// The combine tables (TableBlob::comb: MCT(x^-32 .. x^-4096)) built in
// registers the same way, for the per-buffer mode (round 4): nothing in
// front of its first barrier then waits on memory.  Chunk t of the combine
// area holds table c = t >> 8 (c = 0..7: x^(-8 * 4 * 2^c)), row j = (t >> 6)
// & 3, entries v = 4 (t & 63) + 0..3; for thread t's two chunks (t and t +
// 1024) c and j are wave-uniform, so every product is an immediate and a
// lane's four entries share the xor over v's bits 2..7 (its lane bits).
template <int kBytes, int p>
struct MctInvQ {
  static constexpr uint32_t value = MctBasisInv<kBytes>{}.q[p];
};
template <int kBytes, int P>
__device__ __forceinline__ uint32_t qsel(uint32_t lane, int bit) {
  return ((lane >> bit) & 1u) ? MctInvQ<kBytes, P>::value : 0u;
}
template <int kBytes, int J>
__device__ __forceinline__ uint4 comb_chunk_gen(uint32_t lane) {
  const uint32_t base = qsel<kBytes, 8 * J + 2>(lane, 0) ^ qsel<kBytes, 8 * J + 3>(lane, 1) ^
                        qsel<kBytes, 8 * J + 4>(lane, 2) ^ qsel<kBytes, 8 * J + 5>(lane, 3) ^
                        qsel<kBytes, 8 * J + 6>(lane, 4) ^ qsel<kBytes, 8 * J + 7>(lane, 5);
  const uint32_t q0 = MctInvQ<kBytes, 8 * J>::value, q1 = MctInvQ<kBytes, 8 * J + 1>::value;
  return make_uint4(base, base ^ q0, base ^ q1, base ^ q0 ^ q1);
}
// chunks w * 64 + lane (tables 0..3) and 1024 + w * 64 + lane (tables 4..7)
// of wave w (wave-uniform)
__device__ __forceinline__ void comb_gen(uint32_t w, uint32_t lane, uint4 &c0, uint4 &c1) {
  switch (w) {
#define ZCRC_COMB_W(W)                                                   \
  case W:                                                                \
    c0 = comb_chunk_gen<(4 << ((W) >> 2)), (W) & 3>(lane);               \
    c1 = comb_chunk_gen<(64 << ((W) >> 2)), (W) & 3>(lane);              \
    break;
    ZCRC_COMB_W(0) ZCRC_COMB_W(1) ZCRC_COMB_W(2) ZCRC_COMB_W(3) ZCRC_COMB_W(4) ZCRC_COMB_W(5) ZCRC_COMB_W(6)
    ZCRC_COMB_W(7) ZCRC_COMB_W(8) ZCRC_COMB_W(9) ZCRC_COMB_W(10) ZCRC_COMB_W(11) ZCRC_COMB_W(12)
    ZCRC_COMB_W(13) ZCRC_COMB_W(14) ZCRC_COMB_W(15)
#undef ZCRC_COMB_W
    default:
      c0 = c1 = make_uint4(0, 0, 0, 0);
  }
}

// Lane i gets lane i + d's value, d < 16, inside its 16-lane row (DPP
// row_shl; lanes past the row end get 0).  The folds below only read it in
// lanes whose source is in the same row, where it equals __shfl_down(x, d) --
// which went through ds_bpermute, an LDS round trip per level.
template <int kD>
__device__ __forceinline__ uint32_t row_shl(uint32_t x) {
  static_assert(kD >= 1 && kD < 16, "row_shl:1..15");
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x100 + kD, 0xF, 0xF, false);
}

// A workgroup barrier that orders LDS alone: it waits for this wave's LDS
// operations (lgkmcnt(0)), not for its outstanding global and buffer loads.
// (__syncthreads() is a workgroup fence on every address space: in the
// per-buffer mode it made every wave wait, at the table barrier, for the
// batch lengths it had loaded for the decision taken after the work --
// loads queued behind the other waves' payload preloads.)
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// r * c for one of the 8 combine constants resident in LDS.
__device__ __forceinline__ uint32_t comb_apply(const uint32_t *lds, int c, uint32_t r) {
  const uint32_t *t = lds + kLdsCombDword + c * 1024;
  return t[r & 0xFFu] ^ t[256 + ((r >> 8) & 0xFFu)] ^ t[512 + ((r >> 16) & 0xFFu)] ^ t[768 + (r >> 24)];
}

// r * x^(-8t), t < 16 (the piece's 16-B alignment padding): the LDS combine
// tables for the 4-byte multiples (x^-32, x^-64), then the exact inverse
// step x^-1 (zcrc_gf2.h) for the remaining 0-3 bytes, on the wave-uniform
// register.  It replaced a global-memory MCT of x^(-8t): four loads that
// cost ~4 us per piece under the stream, 7.6% of a wave's time on config 4
// (tools/crc_variants padding-MCT stamps).
__device__ __forceinline__ uint32_t shift_back(const uint32_t *lds, uint32_t r, uint32_t t) {
  const uint32_t a = t >> 2;  // t < 128: combine tables 0..4 are x^-32 .. x^-512 (4 .. 64 bytes)
  if (a & 16u) r = (uint32_t)__builtin_amdgcn_readfirstlane((int)comb_apply(lds, 4, r));
  if (a & 8u) r = (uint32_t)__builtin_amdgcn_readfirstlane((int)comb_apply(lds, 3, r));
  if (a & 4u) r = (uint32_t)__builtin_amdgcn_readfirstlane((int)comb_apply(lds, 2, r));
  if (a & 2u) r = (uint32_t)__builtin_amdgcn_readfirstlane((int)comb_apply(lds, 1, r));
  if (a & 1u) r = (uint32_t)__builtin_amdgcn_readfirstlane((int)comb_apply(lds, 0, r));
  for (uint32_t i = 0; i < 8u * (t & 3u); i++) r = gf2_times_xinv(r);
  return r;
}

// r * c for a multiply-by-constant table in global memory (L2-resident).
__device__ __forceinline__ uint32_t mct_apply_global(const uint32_t *t, uint32_t r) {
  return t[r & 0xFFu] ^ t[256 + ((r >> 8) & 0xFFu)] ^ t[512 + ((r >> 16) & 0xFFu)] ^ t[768 + (r >> 24)];
}

// a * b for wave-uniform operands, on the scalar unit (bit-serial: 32 steps of
// a few SALU instructions, off the VALU the stream needs)
__device__ __forceinline__ uint32_t gf2_mul_uniform(uint32_t a, uint32_t b) {
  a = (uint32_t)__builtin_amdgcn_readfirstlane((int)a);
  b = (uint32_t)__builtin_amdgcn_readfirstlane((int)b);
  uint32_t p = 0;
#pragma unroll
  for (int i = 0; i < 32; i++) {
    if ((a >> (31 - i)) & 1u) p ^= b;
    b = (b >> 1) ^ ((b & 1u) ? kPolyReflected : 0u);
  }
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)p);
}

// r * x^(8*nbytes) (split pieces: once per piece, r wave-uniform).  A split
// piece ends on a whole 64 KiB grain before the buffer end (kSplitGrain), so
// nbytes = 65536 m and x^(8 nbytes) is at most four products of
// x8grain[j][byte j of m], whose four scalar loads go out together.  (The
// round-1..3 form multiplied by x8pow[k] for every set bit k of nbytes: a
// vector load waited for with vmcnt(0) and ~200 VALU per bit, 4-8 times a
// piece.)  Other lengths take the per-bit path.
__device__ __forceinline__ uint32_t shift_bytes(const TableBlob *tab, uint32_t r, uint64_t nbytes,
                                                bool per_bit = false) {
  if (!per_bit && (nbytes & (kSplitGrain - 1)) == 0 && (nbytes >> 48) == 0) {
    typedef const __attribute__((address_space(4))) uint32_t const_u32;  // scalar loads
    const const_u32 *g = (const const_u32 *)&tab->x8grain[0][0];
    const uint32_t m = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(nbytes >> 16));  // uniform: s_load
    const uint32_t f0 = g[m & 255u], f1 = g[256u + ((m >> 8) & 255u)], f2 = g[512u + ((m >> 16) & 255u)],
                   f3 = g[768u + (m >> 24)];
    r = gf2_mul_uniform(f0, r);
    if (m >> 8) r = gf2_mul_uniform(f1, r);
    if (m >> 16) r = gf2_mul_uniform(f2, r);
    if (m >> 24) r = gf2_mul_uniform(f3, r);
    return r;
  }
  int k = 0;
  while (nbytes) {
    if (nbytes & 1u) r = gf2_mul(tab->x8pow[k], r);
    nbytes >>= 1;
    k++;
  }
  return r;
}

__device__ __forceinline__ uint32_t lowmask_bytes(int k) {
  return k <= 0 ? 0u : (k >= 4 ? 0xFFFFFFFFu : ((1u << (8 * k)) - 1u));
}

// Zero the bytes of a 16-B lane chunk outside [lo, hi) (chunk-relative byte
// offsets) and xor the 4-byte seed injection at chunk offset io.
__device__ __forceinline__ uint4 fix_chunk(uint4 d, int lo, int hi, int io, uint32_t inj) {
  uint32_t w[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint32_t m = lowmask_bytes(hi - 4 * q) & ~lowmask_bytes(lo - 4 * q);
    uint32_t v = w[q] & m;
    const int o = io - 4 * q;
    if (o >= 0 && o < 4) v ^= inj << (8 * o);
    if (o < 0 && o > -4) v ^= inj >> (-8 * o);
    w[q] = v;
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ int clamp_rel(int32_t v) { return v < -64 ? -64 : (v > 64 ? 64 : v); }

// Wave-uniform broadcast (lets hipcc keep descriptors and loop bounds in
// SGPRs; without it every buffer_load gets a waterfall loop -- guide T20).
// (__builtin_amdgcn_readfirstlane returns a signed int: convert through
// uint32_t before widening, never sign-extend into the high half.)
__device__ __forceinline__ uint32_t uni32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return (uint64_t)uni32((uint32_t)v) | ((uint64_t)uni32((uint32_t)(v >> 32)) << 32);
}

// lane k's value of a 64-bit register (k wave-uniform)
__device__ __forceinline__ uint64_t rdlane64(uint64_t v, uint32_t k) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)k) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)k) << 32);
}

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  return x ^ (x >> 16);
}

// ------------------------------------------------------------ batch access

template <bool kStrided>
struct BatchView {
  const BatchArgs &a;
  // fused small batches: the prefix as the workgroup computed it into LDS,
  // read by the prologue's range search (nullptr afterwards: global copy)
  const uint64_t *lpre;
  const uint64_t tot_;
  // the first 64-ary search level over [0, n] (lane l: prefix(min((l+1) step0,
  // n))) is the same for every target: loaded once, with prefix[n], so every
  // search -- the wave's range and each dynamic unit -- starts one dependent
  // round trip later in the tree
  uint64_t l1_;
  __device__ BatchView(const BatchArgs &args, const uint64_t *lds_prefix = nullptr)
      : a(args), lpre(lds_prefix),
        // read once per wave: prefix[n] would otherwise be re-read by every snap
        tot_(kStrided ? args.n * args.len : uni64(lds_prefix ? lds_prefix[args.n] : args.prefix[args.n])) {
    l1_ = 0;
    if (!kStrided && args.n > 62) {
      const uint64_t step = (args.n + 63) / 64, idx = (uint64_t)((threadIdx.x & 63u) + 1) * step;
      l1_ = pre(idx < args.n ? idx : args.n);
    }
  }
  // Window order (round 6, tools/region_probe): for a batch of equal
  // buffers whose static wave ranges are whole runs of wp buffers, logical
  // buffer i < wp * wW is physical buffer (i % wp) * wW + i / wp -- wave w's
  // k-th static buffer is k * wW + w, so at any moment the waves' current
  // buffers form one contiguous window of the batch instead of wW places
  // spread over all of it (the dynamic part, logical i >= wp * wW, is claimed
  // in order and stays as it is).  Pure reads of config 3 in the window
  // order ran 5-8% faster than in the range order on every allocation
  // measured.  Lengths are equal, so the prefix (logical) is unchanged; only
  // pointers, seeds and result indices go through map().  wp = 0: identity.
  uint64_t wp = 0, wW = 0;
  __device__ uint64_t map(uint64_t i) const {
    if (!wp || i >= wp * wW) return i;
    const uint32_t x = (uint32_t)i, q = x / (uint32_t)wp;  // (wp * wW <= n < 2^32 whenever wp != 0)
    return (uint64_t)(x - q * (uint32_t)wp) * wW + q;
  }
  __device__ uint64_t pre(uint64_t i) const { return lpre ? lpre[i] : a.prefix[i]; }
  __device__ uint64_t prefix(uint64_t i) const { return kStrided ? i * a.len : pre(i); }
  __device__ const uint8_t *ptr(uint64_t i) const { return kStrided ? a.base + map(i) * a.stride : a.ptrs[map(i)]; }
  __device__ uint32_t seed(uint64_t i) const { return a.seeds ? a.seeds[map(i)] : 0u; }
  __device__ uint64_t total() const { return tot_; }

  // First i in [0, n] with prefix(i) >= t (prefix(n) = total >= t), plus
  // p_i = prefix(i) and p_im1 = prefix(i-1) (0 for i = 0).  Wave-wide 64-ary
  // search; its last level loads prefix(lo-1 .. lo+62), so the two values the
  // snap needs come from lanes of that level instead of another dependent
  // round trip (each costs ~1-2 us at kernel start: tools/c2_probe timeline).
  // Every lane returns the same values.  (An interpolation window loaded with
  // the first level -- one round trip for equal-size buffers -- measured
  // +4-5% on 4 and 16 KiB batches and nothing on config 2, whose search waits
  // behind the table loads anyway: dropped.)
  __device__ uint64_t lower_bound_ex(uint64_t t, uint64_t &p_i, uint64_t &p_im1) const {
    if (kStrided) {
      uint64_t i;
      if (a.len == 0) i = t == 0 ? 0 : a.n;
      else i = (t + a.len - 1) / a.len < a.n ? (t + a.len - 1) / a.len : a.n;
      p_i = i * a.len;
      p_im1 = i ? (i - 1) * a.len : 0;
      return i;
    }
    const uint32_t lane = threadIdx.x & 63u;
    uint64_t lo = 0, hi = a.n;
    while (hi - lo > 62) {
      const uint64_t step = (hi - lo + 63) / 64;
      uint64_t idx = lo + (uint64_t)(lane + 1) * step;
      if (idx > hi) idx = hi;
      const uint64_t m = __ballot((lo == 0 && hi == a.n ? l1_ : pre(idx)) >= t);
      const uint32_t f = (uint32_t)__builtin_ctzll(m);
      const uint64_t nhi = (lo + (uint64_t)(f + 1) * step) < hi ? (lo + (uint64_t)(f + 1) * step) : hi;
      const uint64_t nlo = f == 0 ? lo : lo + (uint64_t)f * step + 1;
      lo = uni64(nlo);
      hi = uni64(nhi);
    }
    // lane j holds prefix(lo - 1 + j); lanes 1..63 cover lo .. lo + 62 >= hi
    const uint64_t idx = lo + lane - 1;
    const bool in = lo + lane >= 1 && idx <= hi;
    const uint64_t v = pre(in ? idx : hi);
    const uint64_t m = __ballot(in && lane >= 1 && v >= t);
    const uint32_t f = (uint32_t)__builtin_ctzll(m);  // >= 1
    const uint64_t r = uni64(lo - 1 + f);
    p_i = rdlane64(v, f);
    p_im1 = r ? rdlane64(v, f - 1) : 0;
    return r;
  }
  __device__ uint64_t lower_bound(uint64_t t) const {
    uint64_t p, q;
    return lower_bound_ex(t, p, q);
  }

  // Snap a nominal wave boundary t so that buffers shorter than kSplitMin are
  // never split and split points sit at end-relative multiples of kSplitGrain.
  // Monotone non-decreasing in t, so snapped ranges stay ordered.
  // Given i = lower_bound(t), pi = prefix(i), pim1 = prefix(i-1); returns the
  // snapped S and lb = lower_bound(S), first = the first buffer overlapping
  // [S, ...) (lb - 1 when S is strictly inside buffer lb - 1, else lb) --
  // process_range's piece walk starts there, without reading prefix(lb).
  __device__ uint64_t snap_at(uint64_t t, uint64_t i, uint64_t pi, uint64_t pim1, uint64_t &lb,
                              uint64_t &first) const {
    const uint64_t tot = total();
    if (t == 0) return lb = first = 0, 0;
    if (t >= tot) return lb = first = lower_bound(tot), tot;
    lb = first = i;
    if (pi == t) return t;
    const uint64_t b0 = pim1;
    const uint64_t n = pi - b0, p = t - b0;
    if (n < kSplitMin) return pi;  // prefix(i-1) < pi: lower_bound(pi) = i
    const uint64_t q = n - kSplitGrain * ((n - p) / kSplitGrain);
    if (q < kMinPiece) return lb = first = lower_bound(b0), b0;  // empty buffers may precede i-1
    if (q < n) first = i - 1;  // strictly inside buffer i-1 (q == n: its end, = pi)
    return b0 + q;
  }

  // lower_bound_ex of two targets in one 64-ary pass (two independent loads
  // per level instead of two dependent searches).
  __device__ void lower_bound2(uint64_t t0, uint64_t t1, uint64_t &r0, uint64_t &r1, uint64_t &p0, uint64_t &q0,
                               uint64_t &p1, uint64_t &q1) const {
    if (kStrided) {
      r0 = lower_bound_ex(t0, p0, q0);
      r1 = lower_bound_ex(t1, p1, q1);
      return;
    }
    const uint32_t lane = threadIdx.x & 63u;
    uint64_t lo0 = 0, hi0 = a.n, lo1 = 0, hi1 = a.n;
    while (hi0 - lo0 > 62 || hi1 - lo1 > 62) {
      const uint64_t st0 = (hi0 - lo0 + 63) / 64, st1 = (hi1 - lo1 + 63) / 64;
      uint64_t x0 = lo0 + (uint64_t)(lane + 1) * st0, x1 = lo1 + (uint64_t)(lane + 1) * st1;
      if (x0 > hi0) x0 = hi0;
      if (x1 > hi1) x1 = hi1;
      const bool top0 = lo0 == 0 && hi0 == a.n, top1 = lo1 == 0 && hi1 == a.n;
      const uint64_t v0 = top0 ? l1_ : pre(x0), v1 = top1 ? l1_ : pre(x1);
      const uint64_t m0 = __ballot(v0 >= t0), m1 = __ballot(v1 >= t1);
      if (hi0 - lo0 > 62) {
        const uint32_t f = (uint32_t)__builtin_ctzll(m0);
        const uint64_t nh = lo0 + (uint64_t)(f + 1) * st0;
        const uint64_t nl = f == 0 ? lo0 : lo0 + (uint64_t)f * st0 + 1;
        hi0 = uni64(nh < hi0 ? nh : hi0);
        lo0 = uni64(nl);
      }
      if (hi1 - lo1 > 62) {
        const uint32_t f = (uint32_t)__builtin_ctzll(m1);
        const uint64_t nh = lo1 + (uint64_t)(f + 1) * st1;
        const uint64_t nl = f == 0 ? lo1 : lo1 + (uint64_t)f * st1 + 1;
        hi1 = uni64(nh < hi1 ? nh : hi1);
        lo1 = uni64(nl);
      }
    }
    const uint64_t x0 = lo0 + lane - 1, x1 = lo1 + lane - 1;
    const bool in0 = lo0 + lane >= 1 && x0 <= hi0, in1 = lo1 + lane >= 1 && x1 <= hi1;
    const uint64_t v0 = pre(in0 ? x0 : hi0), v1 = pre(in1 ? x1 : hi1);
    const uint64_t m0 = __ballot(in0 && lane >= 1 && v0 >= t0), m1 = __ballot(in1 && lane >= 1 && v1 >= t1);
    const uint32_t f0 = (uint32_t)__builtin_ctzll(m0), f1 = (uint32_t)__builtin_ctzll(m1);
    r0 = uni64(lo0 - 1 + f0);
    r1 = uni64(lo1 - 1 + f1);
    p0 = rdlane64(v0, f0);
    q0 = r0 ? rdlane64(v0, f0 - 1) : 0;
    p1 = rdlane64(v1, f1);
    q1 = r1 ? rdlane64(v1, f1 - 1) : 0;
  }

  // Snapped range [S0, S1) for nominal [t0, t1), the first buffer overlapping
  // it (first0) and lb1 = lower_bound(S1) -- process_range's piece walk --
  // with one dual search.  `last`: S1 = total (the caller's final range).
  __device__ void range(uint64_t t0, uint64_t t1, bool last, uint64_t &S0, uint64_t &S1, uint64_t &first0,
                        uint64_t &lb1) const {
    const uint64_t tot = total();
    const uint64_t c0 = t0 < tot ? t0 : tot, c1 = t1 < tot ? t1 : tot;
    uint64_t i0, i1, p0, q0, p1, q1, lb0, first1;
    lower_bound2(c0, c1, i0, i1, p0, q0, p1, q1);
    S0 = uni64(snap_at(c0, i0, p0, q0, lb0, first0));
    if (last) {
      S1 = tot;
      lb1 = a.n;
    } else {
      S1 = uni64(snap_at(c1, i1, p1, q1, lb1, first1));
    }
    first0 = uni64(first0);
    lb1 = uni64(lb1);
  }
};

// ------------------------------------------------------------ plan scan
// Exclusive prefix helpers for the plan (zcrc_kernels.hip) and the fused plan.

// One DPP step of a 64-bit wave scan: each half moved by the same DPP
// control (lanes without a source, or outside row_mask, read 0).
template <int kCtrl, int kRowMask>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, kCtrl, kRowMask, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), kCtrl, kRowMask, 0xF, false);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// Inclusive wave64 scan in DPP steps (row_shr 1/2/4/8 inside 16-lane rows,
// then row_bcast 15/31 across rows): a few VALU cycles per step.  The
// __shfl_up form went through ds_bpermute, an LDS round trip per step:
// 148 of them and 6.9 us per plan_split_scatter launch (tools/plan_probe).
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v) {
  v += dpp64<0x111, 0xF>(v);  // row_shr:1
  v += dpp64<0x112, 0xF>(v);  // row_shr:2
  v += dpp64<0x114, 0xF>(v);  // row_shr:4
  v += dpp64<0x118, 0xF>(v);  // row_shr:8
  v += dpp64<0x142, 0xA>(v);  // row_bcast:15 -> rows 1, 3
  v += dpp64<0x143, 0xC>(v);  // row_bcast:31 -> rows 2, 3
  return v;
}

__device__ uint64_t block_excl_scan(uint64_t v, uint64_t *s_tmp /* 16 */, uint64_t *total) {
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint64_t inc = wave_incl_scan(v);
  if (lane == 63) s_tmp[wv] = inc;
  __syncthreads();
  uint64_t off = 0, tot = 0;
  for (uint32_t k = 0; k < blockDim.x / 64; k++) {
    const uint64_t s = s_tmp[k];
    if (k < wv) off += s;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return off + inc - v;
}

// (A fused plan -- the first workgroup to run scanned the lengths and the
// others waited on a flag -- was removed in round 1: no workgroup of this
// kernel waits on another one.  DESIGN.md section 4, "Plan".)

// Fused small batches (zcrc32_batch_device, n <= kFusedMaxN): no plan launch
// zeroes out[] first, so the pieces of a split buffer meet in a 64-bit word of
// scratch -- high half: 64 KiB grid cells covered so far, low half: xor of the
// contributions -- updated lock-free with compare-and-swap.  The piece that
// completes the cell count stores the result and returns the word to zero,
// so the scratch is zero again for the next launch (the runtime zero-fills it
// once, when it is allocated).  A retry only follows another piece's update
// of the same word: no piece waits for another one to make progress.
__device__ void split_accumulate(const BatchArgs &a, uint64_t i, uint64_t n, uint64_t lo, uint64_t hi,
                                 uint32_t contrib) {
  // split points sit on the end-relative kSplitGrain grid, so every piece but
  // the first covers whole cells; the first covers the partial cell too
  const uint64_t cells = (n + kSplitGrain - 1) / kSplitGrain;  // <= 2^26 (kMaxLaunchBytes)
  const uint64_t mine = lo == 0 ? (hi + kSplitGrain - 1) / kSplitGrain : (hi - lo) / kSplitGrain;
  unsigned long long *word = reinterpret_cast<unsigned long long *>(a.acc + i);
  unsigned long long expect = 0;
  for (;;) {
    const unsigned long long want = (((expect >> 32) + mine) << 32) | (uint32_t)((uint32_t)expect ^ contrib);
    const unsigned long long got = atomicCAS(word, expect, want);
    if (got == expect) {
      if ((want >> 32) == cells) {
        a.out[i] = (uint32_t)want;
        atomicExch(word, 0ull);
      }
      return;
    }
    expect = got;
  }
}

// ------------------------------------------------------------ the kernel

// kD: 1 KiB blocks per register group (two groups in flight); kAblate == 1
// replaces the table lookups with one VALU op (measurement builds only),
// kAblate == 2 is the round-1..3 step (three xors per dword, A/B builds).
// Process every piece of the byte range [S0, S1) of the concatenated batch
// (S0, S1 snapped; `last_range` also takes the trailing empty buffers).
// Returns the number of pieces.  Wave-uniform; no barriers.
template <uint32_t kD, int kAblate, int kAux, bool kStamp, bool kPre = false, bool kProg = false, int kFold = 0>
__device__ __forceinline__ uint32_t piece_raw(const uint32_t *s_lds, const uint8_t *bptr, uint64_t rel_lo,
                                              uint64_t rel_hi, uint32_t seed, uint32_t lane, uint64_t *t_tail,
                                              const uint4 *pre = nullptr);

// Descriptors of up to 64 pieces of a range walk (kWin), lane k = piece k of
// the window that starts at walk position k0.
struct PieceWindow {
  uint64_t i, b0, b1, p;
  uint32_t s, o;  // o: result index (split plan: oidx[i])
  uint64_t len;   // the caller's length of the buffer (~0: not known), to check b1 - b0 against
};

template <bool kStrided>
__device__ __forceinline__ void load_window(const BatchView<kStrided> &bv, uint64_t i_first, uint64_t npieces,
                                            uint64_t rot, uint64_t k0, uint32_t lane, PieceWindow &w) {
  uint64_t x = k0 + lane + rot;  // rotated position of this lane's piece
  if (x >= npieces) x -= npieces;
  w.i = i_first + (k0 + lane < npieces ? x : 0);
  w.b0 = bv.prefix(w.i);
  w.b1 = bv.prefix(w.i + 1);
  w.p = reinterpret_cast<uint64_t>(bv.ptr(w.i));
  w.s = bv.seed(w.i);
  if (!kStrided && bv.a.oidx) w.o = bv.a.oidx[w.i];
  w.len = !kStrided && bv.a.lens ? bv.a.lens[bv.a.oidx ? w.o : bv.map(w.i)] : ~0ull;
}

// Per-wave rotated visiting order.  Pieces are independent, and the rotation
// de-phases waves whose ranges start on large power-of-two boundaries
// (uniform batches), which otherwise walk the HBM channel interleave in
// lockstep ("partition camping", tools/hbm_probe: up to -13%).
template <bool kRotate>
__device__ __forceinline__ uint64_t walk_rotation(uint32_t salt, uint64_t npieces) {
  return (kRotate && npieces > 1) ? (uint64_t)(hash32(salt) % (uint32_t)npieces) : 0;
}

// kWin: piece descriptors are fetched 64 pieces at a time with one vector
// load per field (lane k: the window's piece k) and read back with
// v_readlane, instead of a dependent scalar round trip per piece.
template <bool kStrided, uint32_t kD, int kAblate, bool kRotate, int kPrio = 0, int kAux = 0, bool kStamp = false,
          bool kFused = false, bool kWin = false>
__device__ __forceinline__ uint64_t process_range(const BatchArgs &args, const BatchView<kStrided> &bv,
                                                  const uint32_t *s_lds, const TableBlob *tab, uint64_t S0,
                                                  uint64_t S1, bool last_wave, uint32_t salt, uint32_t lane,
                                                  bool band, uint64_t first0, uint64_t lb1, uint64_t *t_tail = nullptr,
                                                  bool skip_small = false) {
  // Buffers [i_first, i_end) overlap this wave's range [S0, S1).
  // first0: the first buffer overlapping it, lb1 = lower_bound(S1) (BatchView::range)
  const uint64_t i_first = uni64(first0);
  const uint64_t i_end = last_wave ? args.n : lb1;
  const uint64_t npieces = i_end > i_first ? i_end - i_first : 0;
  // (the window order keeps the waves in step through their buffers: no
  // rotation, which would scatter them again)
  const uint64_t rot = bv.wp ? 0 : walk_rotation<kRotate>(salt, npieces);

  // kPrio: least-progress-first issue priority.  Waves of a CU are otherwise
  // served oldest-first, so with equal byte ranges slot 0-3 finish at ~50% of
  // the kernel and slots 12-15 at 100% (tools/crc_variants stamps).
  const uint64_t range_bytes = S1 > S0 ? S1 - S0 : 1;
  uint64_t done = 0;
  if (kPrio && band) __builtin_amdgcn_s_setprio(3);

  PieceWindow win{0, 0, 0, 0, 0, 0, 0};  // kWin: the current window
  for (uint64_t k = 0; k < npieces; k++) {
    uint64_t i, b0, b1, blen = ~0ull;
    if (kWin && !kStrided) {
      const uint32_t kk = (uint32_t)(k & 63u);
      if (kk == 0) load_window(bv, i_first, npieces, rot, k, lane, win);
      i = rdlane64(win.i, kk);
      b0 = rdlane64(win.b0, kk);
      b1 = rdlane64(win.b1, kk);
      blen = rdlane64(win.len, kk);
    } else {
      i = i_first + k + rot;
      if (i >= i_end) i -= npieces;
      i = uni64(i);
      b0 = uni64(bv.prefix(i)), b1 = uni64(bv.prefix(i + 1));
      if (skip_small) blen = uni64(args.lens[i]);
    }
    // skip_small (the per-buffer mode's fall-back): buffers of at most
    // kPerBufMax bytes were checksummed by their own wave already and count
    // as empty in this prefix
    if (kFused && skip_small && blen <= kPerBufMax) continue;
    const uint64_t n = b1 - b0;
    const uint64_t rel_lo = (S0 > b0 ? S0 - b0 : 0);
    const uint64_t rel_hi = (b1 < S1 || last_wave) ? n : S1 - b0;
    const bool whole = (rel_lo == 0 && rel_hi == n);
    if (kPrio && band) {
      const uint32_t lvl = uni32((uint32_t)((4 * done) / range_bytes));
      if (lvl == 1) __builtin_amdgcn_s_setprio(2);
      else if (lvl == 2) __builtin_amdgcn_s_setprio(1);
      else if (lvl >= 3) __builtin_amdgcn_s_setprio(0);
      done += rel_hi - rel_lo;
    }
    uint32_t seed;
    const uint8_t *bptr;
    // result index: the buffer's (window order: map(i)), or its index before
    // the split plan compacted the batch
    uint64_t oi = bv.map(i);
    if (kWin && !kStrided) {
      seed = (uint32_t)__builtin_amdgcn_readlane((int)win.s, (int)(k & 63u));
      bptr = reinterpret_cast<const uint8_t *>(rdlane64(win.p, (uint32_t)(k & 63u)));
      if (args.oidx) oi = (uint32_t)__builtin_amdgcn_readlane((int)win.o, (int)(k & 63u));
    } else {
      seed = uni32(bv.seed(i));
      bptr = reinterpret_cast<const uint8_t *>(uni64(reinterpret_cast<uint64_t>(bv.ptr(i))));
      if (!kStrided && args.oidx) oi = uni32(args.oidx[i]);
    }

    // A prefix that disagrees with the caller's lengths (corrupted scratch --
    // the round-1/2 fault: an unordered memset zero-filled it under queued
    // launches) must not send the piece walk outside the buffer: the piece is
    // skipped, its result zeroed, and the scratch's fault word set
    // (zcrc32_batch_device_faults).
    if (b1 < b0 || rel_lo > rel_hi || rel_hi > n || (blen != ~0ull && n != blen)) {
      if (lane == 0) {
        args.out[oi] = 0u;
        if (args.fault) atomicOr(args.fault, 1u);
      }
      continue;
    }

    if (n < 4) {  // tiny buffer: bytewise with the standard table (never split)
      uint32_t r = ~seed;
      for (uint32_t p = 0; p < (uint32_t)n; p++) r = (r >> 8) ^ tab->stdtab[(r ^ bptr[p]) & 0xFFu];
      if (lane == 0) args.out[oi] = ~r;
      continue;
    }

    const uint32_t r = piece_raw<kD, kAblate, kAux, kStamp>(s_lds, bptr, rel_lo, rel_hi, seed, lane, t_tail);
    if (whole) {
      if (lane == 0) args.out[oi] = ~r;
    } else {
      const uint64_t d = n - rel_hi;  // bytes after this piece, multiple of kSplitGrain
      uint32_t contrib = d ? shift_bytes(tab, r, d, args.ab_flags & 1u) : (r ^ 0xFFFFFFFFu);
      if (kFused) {
        if (lane == 0) split_accumulate(args, i, n, rel_lo, rel_hi, contrib);
      } else if (lane == 0) {
        atomicXor(args.out + oi, contrib);
      }
    }
  }
  return npieces;
}

// Geometry of a piece: blocks are aligned to the piece's 16-B-aligned end
// aend; block `it` of lane l is the chunk astart + (span - 1024 K) + 1024 it +
// 16 l, addressed through a buffer resource over [astart, aend) (chunks
// before astart read as zeros).
struct PieceGeom {
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t voff0, K, tpad;
  int32_t c0, rs, re;
};

__device__ __forceinline__ PieceGeom piece_geom(const uint8_t *bptr, uint64_t rel_lo, uint64_t rel_hi,
                                                uint32_t lane) {
  PieceGeom g;
  const uint64_t pstart = (uint64_t)bptr + rel_lo;
  const uint64_t pend = (uint64_t)bptr + rel_hi;
  const uint64_t astart = uni64(pstart & ~(uint64_t)15);
  const uint64_t aend = uni64((pend + 15) & ~(uint64_t)15);
  // The block grid ends at the 128-B line after pend, so that no 1 KiB block
  // straddles a line: anchored at aend, a piece of arbitrary length had every
  // block straddle one, fetched by two blocks' loads (config 4 read 1.022x its
  // payload; 1.001x with every length a 1 KiB multiple: DESIGN.md 7b).
  // Chunks in [aend, agrid) are out of the resource range: zeros, no fetch.
  const uint64_t agrid = uni64((pend + 127) & ~(uint64_t)127);
  const uint32_t span = uni32((uint32_t)(aend - astart));  // < 2^31 (kMaxLaunchBytes)
  const uint32_t gspan = uni32((uint32_t)(agrid - astart));
  g.K = uni32((gspan + 1023u) >> 10);
  g.tpad = uni32((uint32_t)(agrid - pend));  // < 128
  // chunk-relative bounds of lane's chunk in block 0, relative to astart; all
  // fit in int32 because span < 2^31
  g.c0 = (int32_t)gspan - 1024 * (int32_t)g.K + 16 * (int32_t)lane;
  g.rs = (int32_t)uni32((uint32_t)(pstart - astart));
  g.re = (int32_t)uni32((uint32_t)(pend - astart));
  g.rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(astart), (short)0, (int)span, 0x00020000);
  g.voff0 = (uint32_t)g.c0;  // negative wraps -> out of range -> zeros
  return g;
}

// The loads of a piece's first two groups (2 kD blocks; blocks past the
// piece read zeros), issued ahead of piece_raw<..., kPre = true> -- e.g.
// before the workgroup's LDS fill and barrier.  Issued unconditionally (an
// empty range when !valid: zeros, no memory access), so that the waits for
// loads issued before them stay counted ones, not vmcnt(0).
template <uint32_t kD, int kAux>
__device__ __forceinline__ void piece_preload(const uint8_t *bptr, uint64_t rel_lo, uint64_t rel_hi, uint32_t lane,
                                              bool valid, uint4 *pre) {
  const PieceGeom g = piece_geom(bptr, rel_lo, rel_hi, lane);
  const __amdgpu_buffer_rsrc_t rsrc = valid ? g.rsrc : __builtin_amdgcn_make_buffer_rsrc(nullptr, (short)0, 0, 0x00020000);
#pragma unroll
  for (uint32_t u = 0; u < 2 * kD; u++) {
    auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, g.voff0 + 1024u * u, 0, kAux);
    pre[u] = make_uint4(v[0], v[1], v[2], v[3]);
  }
}

// One piece, bytes [rel_lo, rel_hi) of the buffer at bptr (at least 4 bytes
// long), as the raw register at the piece end; the seed is injected when the
// piece starts the buffer.  kPre: groups 0 and 1 were loaded by
// piece_preload into pre[0 .. 2 kD).  Wave-uniform; no barriers.
// kProg (per-buffer mode A/B): the wave's priority falls with its progress
// through the piece, 3 in the first quarter of its groups .. 0 in the last,
// so that waves behind issue first and the waves of a CU end together
template <uint32_t kD, int kAblate, int kAux, bool kStamp, bool kPre, bool kProg, int kFold>
__device__ __forceinline__ uint32_t piece_raw(const uint32_t *s_lds, const uint8_t *bptr, uint64_t rel_lo,
                                              uint64_t rel_hi, uint32_t seed, uint32_t lane, uint64_t *t_tail,
                                              const uint4 *pre) {
  // lane constants for the braided lookups
  const uint32_t lo0 = (lane & 31u) * 4u;
  const uint32_t o0 = lo0, o1 = lo0 + 128u, o2 = lo0 + 65536u, o3 = lo0 + 65536u + 128u;
  {
    // ---- one piece: bytes [pstart, pend) of the buffer --------------------
    const PieceGeom geo = piece_geom(bptr, rel_lo, rel_hi, lane);
    const uint32_t K = geo.K, tpad = geo.tpad, voff0 = geo.voff0;
    const int32_t c0 = geo.c0, rs = geo.rs, re = geo.re;
    const __amdgpu_buffer_rsrc_t rsrc = geo.rsrc;
    const uint32_t inj = uni32((rel_lo == 0) ? ~seed : 0u);

    uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    // Round 4: a stream's register is kept as two words, s = s_k ^ q_k
    // (braid_step2): 2 VALU per step besides the 4 v_perm address builds,
    // against 4 xors before -- the hot loop's VALU per two 4 KiB groups went
    // from 264 to 200 instructions.
    uint32_t q0 = 0, q1 = 0, q2 = 0, q3 = 0;
    // Two register groups of kD blocks: one streams in while the other
    // is consumed (no register rotation, no vmcnt(0) at group boundaries).
    uint4 ga[kD], gb[kD];

#define ZCRC_LOADG(G, g)                                                                        \
  {                                                                                             \
    _Pragma("unroll") for (uint32_t u_ = 0; u_ < kD; u_++) {                                \
      auto v_ = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff0 + 1024u * ((g) * kD + u_), \
                                                      0, kAux);                                 \
      G[u_] = make_uint4(v_[0], v_[1], v_[2], v_[3]);                                           \
    }                                                                                           \
  }
#define ZCRC_STEP(x) (kAblate == 1 ? __builtin_amdgcn_alignbit((x), (x), 5) : braid_step(s_lds, (x), o0, o1, o2, o3))
#define ZCRC_STEP2(S, Q, D) braid_step2(s_lds, (S), (Q), (D), o0, o1, o2, o3)
#define ZCRC_CONSUME(d)                \
  if (kAblate == 0) {                  \
    ZCRC_STEP2(s0, q0, (d).x);         \
    ZCRC_STEP2(s1, q1, (d).y);         \
    ZCRC_STEP2(s2, q2, (d).z);         \
    ZCRC_STEP2(s3, q3, (d).w);         \
  } else {                             \
    s0 = ZCRC_STEP(s0 ^ (d).x);        \
    s1 = ZCRC_STEP(s1 ^ (d).y);        \
    s2 = ZCRC_STEP(s2 ^ (d).z);        \
    s3 = ZCRC_STEP(s3 ^ (d).w);        \
  }
  // plain group: every block strictly before block K-1, no fix-up needed
#define ZCRC_PLAIN(G)                                                   \
  {                                                                     \
    _Pragma("unroll") for (uint32_t u_ = 0; u_ < kD; u_++) ZCRC_CONSUME(G[u_]); \
  }
  // edge group: bounds-checked, fix-ups on blocks 0, 1 and K-1
#define ZCRC_EDGE(G, g)                                                                         \
  {                                                                                             \
    _Pragma("unroll") for (uint32_t u_ = 0; u_ < kD; u_++) {                                \
      const uint32_t it_ = (g) * kD + u_;                                                   \
      if (it_ < K) {                                                                            \
        uint4 dd_ = G[u_];                                                                      \
        if (it_ <= 1u || it_ + 1u == K) {                                                       \
          const int32_t c_ = c0 + 1024 * (int32_t)it_;                                          \
          dd_ = fix_chunk(dd_, clamp_rel(rs - c_), clamp_rel(re - c_), clamp_rel(rs - c_), inj); \
        }                                                                                       \
        ZCRC_CONSUME(dd_);                                                                      \
      }                                                                                         \
    }                                                                                           \
  }

    // Groups of kD blocks: group 0 and the last group are "edge" groups
    // (bounds + fix-ups), groups 1..ngroups-2 are plain.  Loop invariant: gb
    // holds group g, loaded; ga is free.
    const uint32_t ngroups = (K + kD - 1) / kD;  // >= 1
    if (kPre) {
#pragma unroll
      for (uint32_t u = 0; u < kD; u++) ga[u] = pre[u], gb[u] = pre[kD + u];
    } else {
      ZCRC_LOADG(ga, 0u);
      if (ngroups > 1) ZCRC_LOADG(gb, 1u);
    }
    ZCRC_EDGE(ga, 0u);
    if (kSweepOrder && !kPre && ngroups > 2) {
      // gb holds group 1 (plain); groups 2 .. ngroups - 2 are loaded one at a
      // time, first block alone; the last group is an edge group
      ZCRC_PLAIN(gb);
      for (uint32_t g = 2; g + 1 < ngroups; g++) {
        {
          auto v_ = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff0 + 1024u * (g * kD), 0, kAux);
          ga[0] = make_uint4(v_[0], v_[1], v_[2], v_[3]);
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the group's first block has landed
        _Pragma("unroll") for (uint32_t u_ = 1; u_ < kD; u_++) {
          auto v_ = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff0 + 1024u * (g * kD + u_), 0, kAux);
          ga[u_] = make_uint4(v_[0], v_[1], v_[2], v_[3]);
        }
        ZCRC_PLAIN(ga);
      }
      ZCRC_LOADG(gb, ngroups - 1);
      ZCRC_EDGE(gb, ngroups - 1);
    } else if (ngroups > 1) {
      const uint32_t nplain = ngroups - 2;
      uint32_t g = 1;
      for (uint32_t pr = 0; pr < nplain / 2; pr++) {
        if (kProg) {  // wave-uniform scalar compares: level = floor(4 pr / npairs)
          const uint32_t q = 4u * pr, np = nplain / 2;
          if (q >= 3u * np) __builtin_amdgcn_s_setprio(0);
          else if (q >= 2u * np) __builtin_amdgcn_s_setprio(1);
          else if (q >= np) __builtin_amdgcn_s_setprio(2);
        }
        ZCRC_LOADG(ga, g + 1);
        ZCRC_PLAIN(gb);
        ZCRC_LOADG(gb, g + 2);
        ZCRC_PLAIN(ga);
        g += 2;
      }
      if (nplain & 1u) {
        ZCRC_LOADG(ga, g + 1);
        ZCRC_PLAIN(gb);
        ZCRC_EDGE(ga, g + 1);
      } else {
        ZCRC_EDGE(gb, g);
      }
    }
#undef ZCRC_LOADG
#undef ZCRC_STEP
#undef ZCRC_STEP2
#undef ZCRC_CONSUME
#undef ZCRC_PLAIN
#undef ZCRC_EDGE

    // ---- fold 256 stream registers into one raw register at `aend` -------
    // stream (lane l, dword q) sits at aend + 16 l + 4 q
    s0 ^= q0, s1 ^= q1, s2 ^= q2, s3 ^= q3;
    if (kFold == 1) return uni32(s0 ^ s1 ^ s2 ^ s3);  // diagnostic (tools/ceiling_probe): no fold
    uint32_t r = (s0 ^ comb_apply(s_lds, 0, s1)) ^ comb_apply(s_lds, 1, s2 ^ comb_apply(s_lds, 0, s3));
    // cross-lane levels x^(-128 * 2^j): j < 4 inside 16-lane rows (DPP);
    // the last two on the four row results, read into scalars.  kFold == 2
    // (A/B): each level's lookups only in the lanes whose result the next
    // level reads (lane 0 of each row ends with the row's fold)
    if (kFold == 2) {
      uint32_t t = 0;
      if ((lane & 1u) == 1u) t = comb_apply(s_lds, 2, r);
      r ^= row_shl<1>(t);
      t = 0;
      if ((lane & 3u) == 2u) t = comb_apply(s_lds, 3, r);
      r ^= row_shl<2>(t);
      t = 0;
      if ((lane & 7u) == 4u) t = comb_apply(s_lds, 4, r);
      r ^= row_shl<4>(t);
      t = 0;
      if ((lane & 15u) == 8u) t = comb_apply(s_lds, 5, r);
      r ^= row_shl<8>(t);
    } else {
      r ^= row_shl<1>(comb_apply(s_lds, 2, r));
      r ^= row_shl<2>(comb_apply(s_lds, 3, r));
      r ^= row_shl<4>(comb_apply(s_lds, 4, r));
      r ^= row_shl<8>(comb_apply(s_lds, 5, r));
    }
    {
      const uint32_t r0 = uni32(r);
      const uint32_t r16 = (uint32_t)__builtin_amdgcn_readlane((int)r, 16);
      const uint32_t r32 = (uint32_t)__builtin_amdgcn_readlane((int)r, 32);
      const uint32_t r48 = (uint32_t)__builtin_amdgcn_readlane((int)r, 48);
      r = uni32(r0 ^ comb_apply(s_lds, 6, r16) ^ comb_apply(s_lds, 7, r32 ^ comb_apply(s_lds, 6, r48)));
    }
    const uint64_t tt0 = kStamp ? __builtin_amdgcn_s_memrealtime() : 0;
    if (tpad) r = shift_back(s_lds, r, tpad);  // -> register at pend
    if (kStamp) r = uni32(r), *t_tail += __builtin_amdgcn_s_memrealtime() - tt0;  // diagnostic: padding MCT
    return r;
  }
}

// zcrc_small_kernel.h (included at the end of this header)
template <bool kStrided, int G, int kD, int kAblate, bool kCoal = false, bool kPipe = false, int kBlk = 256>
__device__ __forceinline__ void small_body(const SmallArgs &a, uint32_t *s_lds, uint64_t n, uint32_t blk,
                                           uint32_t nblk);

// kPB: the per-buffer mode's form (fused only): 4 = round 4 (tables built in
// registers, the decision after the work), 5 = the same with the first
// payload loads issued before the table build, 7 = 5 with the decision's
// lengths loaded behind the preload, decided after the piece, and an
// LDS-only table barrier (lds_barrier), 8 = 5 with the decision taken after
// the piece (lengths loaded first), 9 = 8 with the lengths in four 16-B
// buffer loads per thread, 3 = round 3 (tables and lengths in front of the
// one barrier); 3, 5, 7, 8 and 9 are A/B forms for tools/.
// kPB + 10: priority by progress through the buffer instead of by wave slot
// (piece_raw kProg); kPB + 20: no priorities (A/B forms, tools/c2_probe).
template <bool kStrided, uint32_t kD = kDepth, int kAblate = 0, bool kRotate = true, bool kStamp = false,
          int kPrio = 1, int kAux = kLoadNt, bool kFused = false, bool kWin = kWindowed, int kPB = 4>
__global__ __launch_bounds__(kThreads) void crc32_batch_kernel(BatchArgs args) {
  __shared__ __attribute__((aligned(16))) uint32_t s_lds[kLdsBytes / 4];
  uint32_t grid = gridDim.x;  // the batch's workgroups
  // a small-list workgroup that, its list done, joins the batch's dynamic part
  bool join = false;
  // every buffer equally long (the strided form; the split plan's counts[5]):
  // the window order may apply (BatchView::wp)
  bool equal = kStrided;
  if (!kStrided && !kFused && args.n_dev) {
    // split plan: its counts; when it split, the top n_dev[4] workgroups take
    // the small list (zcrc_small_kernel.h, own LDS table) and the rest the
    // compacted batch -- both in this one launch
    if (uni64(args.n_dev[2])) {
      const uint32_t nsm = (uint32_t)uni64(args.n_dev[4]);
      if (blockIdx.x + nsm >= gridDim.x) {
        SmallArgs sa{};
        sa.ptrs = args.ptrs;
        sa.lens = args.lens;
        sa.sdesc = uni64(args.n_dev[2]) == 2 ? nullptr : args.sdesc;  // direct: the caller's arrays
        sa.seeds = args.seeds;
        sa.out = args.out;
        sa.tab = args.tab;
        const uint64_t ns = uni64(args.n_dev[1]);
        const uint32_t blk = blockIdx.x - (gridDim.x - nsm);
        const uint64_t t_small = kStamp ? __builtin_amdgcn_s_memrealtime() : 0;
        if (uni64(args.n_dev[3]) == 8) small_body<false, 8, 8, kAblate, false, false, 128>(sa, s_lds, ns, blk, nsm);
        else small_body<false, 16, 8, kAblate>(sa, s_lds, ns, blk, nsm);
        if (kStamp && (threadIdx.x & 63u) == 0) {  // diagnostic build: a small-list wave (npieces ~0)
          const uint64_t w = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
          args.stamps[8 * w + 0] = args.stamps[8 * w + 4] = t_small;
          args.stamps[8 * w + 1] = __builtin_amdgcn_s_memrealtime();
          args.stamps[8 * w + 2] = ~0ull;
        }
        // Round 4: with its list done, the workgroup joins the batch's
        // dynamic part -- it loads the batch tables like the others and claims
        // units from the same counter (config 4: the 13 small-list CUs were
        // done at ~1.1 of ~2.0 ms and idled).  ab_flags bit 2
        // (A/B) keeps them out.
        if ((args.ab_flags & 4u) || uni64(args.n_dev[0]) == 0) return;  // uniform per workgroup
        join = true;
        __syncthreads();  // every wave is done with the small body's LDS tables
      }
      grid -= nsm;
      args.ptrs = args.ptrs_split;
      args.seeds = args.seeds_split;
    } else {
      args.oidx = nullptr;
      equal = uni64(args.n_dev[5]) != 0;
    }
    args.n = uni64(args.n_dev[0]);
    if (args.n == 0) return;
  }
  const TableBlob *tab = args.tab;
  const uint64_t t_entry = kStamp ? __builtin_amdgcn_s_memrealtime() : 0;

  // ---- prologue: the table loads are issued first; the plan (fused form)
  // and the wave's range search run while they are in flight; the LDS
  // writes and the barrier come last.  (Fill, then search, measured 4.2 +
  // 3.4 us of a 53 us config-2 launch: tools/crc_variants stamps.)
  // LDS byte o of the braided area holds braid[j][v] with j = 2 * (o >> 16)
  // + ((o >> 7) & 1), v = (o >> 8) & 255 (32 replicas of each entry, 4 B
  // apart).  Thread t writes the 16-B chunks t + 1024 k, so a wave's writes
  // are consecutive (writing one entry's 128 B per lane put every lane on
  // the same banks: 3.6 us of bank conflicts per launch).
  const uint32_t tid = threadIdx.x;
  uint32_t braid_val[8];
  uint4 comb0, comb1;
  auto load_tables = [&]() {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t o = 16u * (tid + 1024u * k);
      braid_val[k] = tab->braid[(((o >> 16) << 1) | ((o >> 7) & 1u)) * 256u + ((o >> 8) & 255u)];
    }
    const uint4 *comb_src = reinterpret_cast<const uint4 *>(tab->comb);
    comb0 = comb_src[tid];
    comb1 = comb_src[tid + 1024u];
  };
  if (!kFused) load_tables();

  // Fused small batch: every workgroup scans the <= kFusedMaxN lengths itself
  // (thread t owns buffers 8t .. 8t+7) while the table loads are in flight,
  // into LDS for its own range search and into the scratch prefix for the
  // piece walk and the unit searches.  Every workgroup writes the same
  // values; each reads only after its own writes and a barrier.
  uint64_t *const lds_pre = reinterpret_cast<uint64_t *>(s_lds);
  bool perbuf_done = false;  // the per-buffer pass ran: the scan and the walk take the long buffers only
  if (kFused) {
    static_assert(kFusedMaxN == 8u * kThreads, "fused scan: 8 lengths per thread");
    static_assert((kFusedMaxN + 1 + 16) * 8 <= kLdsBytes, "fused scan fits in LDS");
    // Per-buffer mode: no more buffers than waves and none longer than
    // kPerBufMax.  The two-launch path would then give every wave at most one
    // range of whole buffers (W = n, no splits); here wave slot s of workgroup
    // g takes buffer s * grid + g whole -- spread over every CU, with no
    // prefix, no range search and no plan.  Every workgroup reads all the
    // lengths, so all of them take the same decision.
    //
    // Round 3: one barrier, and nothing in front of it that waits behind the
    // payload.  At entry each wave issues its share of the decision's
    // lengths, its chunks of the combine tables and its descriptor; it
    // builds its braid entries in registers (braid_gen_lane: no table load);
    // it writes braid, combine tables and its decision flag, and meets the
    // others at the barrier.  The flags need
    // no LDS of their own: wave s's flag is the word of combine entry (c, j,
    // v) = (s >> 2, s & 3, 0), which the same wave writes and which is 0 in
    // every MCT -- so when no flag is set the tables are already right.
    // (Round 2 decided first, behind two extra barriers, with the braid and
    // the lengths loaded after every wave's preload was queued, and the
    // guarded length loads waited for one at a time: the table fill
    // completed 7.7 us after entry, now 3.5 us; tools/c2_probe,
    // profiles/r03/s11, s16.)
    // kPrioMode: 0 by slot, 1 by progress, 2 none; kDP: blocks per register
    // group in the per-buffer path (kPB + 100: 6, + 200: 8; two groups in flight)
    constexpr int kForm = kPB % 10, kPrioMode = (kPB / 10) % 10;
    constexpr uint32_t kDP = (kPB / 100) % 10 == 1 ? 6u : (kPB / 100) % 10 == 2 ? 8u : kD;
    // kPB + 1000 / + 2000 (diagnostics for tools/ceiling_probe, with kAblate
    // only: the results are wrong): no table build / no table build and no
    // decision at the end; + 4000: + 2000 without the table barrier either;
    // + 5000: + 4000 without the fold; kPB + 3000: no decision lengths (the
    // end barriers kept; right only when no buffer exceeds kPerBufMax)
    constexpr int kDiag = kPB / 1000;
    constexpr bool kNoTab = kDiag == 1 || kDiag == 2 || kDiag == 4 || kDiag == 5;
    constexpr bool kNoEnd = kDiag == 2 || kDiag == 4 || kDiag == 5;
    constexpr bool kNoLens = kDiag >= 2 && kDiag != 6, kNoBar = kDiag == 4 || kDiag == 5;
    // kPB + 6000 (A/B): the fold's lane levels masked to the lanes read next
    constexpr int kFoldMode = kDiag == 5 ? 1 : kDiag == 6 ? 2 : 0;
    static_assert(!kNoTab || kAblate, "the table-less diagnostic forms are read-ceiling variants");
    if (kForm >= 4 && args.n <= (uint64_t)grid * kWaves) {
      // Round 4: nothing in front of the payload waits on memory but the
      // wave's own descriptor.  The braid and combine tables are built in
      // registers (braid_gen_lane, comb_gen) and the one barrier in front
      // of the piece waits for ALU work alone; the decision -- is any buffer
      // of the batch longer than kPerBufMax? -- is taken after the work:
      // every wave checksums its own buffer when it is short enough, its
      // lengths arrive while its first payload loads are in flight, and the
      // workgroup compares notes behind two barriers at the end.  When some
      // buffer is longer, the in-kernel scan below runs over the long ones
      // only (the short ones count as empty and are skipped).  Every
      // workgroup reads the same lengths, so all take the same decision.
      const uint32_t lane = tid & 63u, slot = uni32(tid >> 6);
      const uint64_t b = (uint64_t)slot * grid + blockIdx.x;
      const bool wg_busy = blockIdx.x < args.n;  // workgroup-uniform
      uint64_t blen = 0, bp = 0;
      uint32_t bseed = 0;
      if (b < args.n) {
        blen = uni64(args.lens[b]);
        bp = uni64(reinterpret_cast<uint64_t>(args.ptrs[b]));
        bseed = args.seeds ? uni32(args.seeds[b]) : 0u;
      }
      uint64_t L[8];  // the decision's lengths (thread t: buffers t + 1024 j), clamped, unguarded
      auto load_lens = [&]() {
        if (kForm == 9) {
          // form 9: four 16-B buffer loads over [lens, lens + n) (thread t:
          // buffers 2 t + 2048 j and the next), past the end zeros -- no
          // clamped duplicates, half the load instructions
          const __amdgpu_buffer_rsrc_t lr =
              __builtin_amdgcn_make_buffer_rsrc((void *)args.lens, (short)0, (int)(8u * args.n), 0x00020000);
#pragma unroll
          for (uint32_t j = 0; j < 4; j++) {
            auto v = __builtin_amdgcn_raw_buffer_load_b128(lr, 16u * tid + 16384u * j, 0, 0);
            L[2 * j] = (uint64_t)v[0] | ((uint64_t)v[1] << 32);
            L[2 * j + 1] = (uint64_t)v[2] | ((uint64_t)v[3] << 32);
          }
          return;
        }
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) {
          const uint64_t idx = tid + 1024u * j;
          L[j] = args.lens[idx < args.n ? idx : args.n - 1];
        }
      };
      if ((kForm < 7 || kForm >= 8) && !kNoLens) load_lens();
      const bool own = b < args.n && blen <= kPerBufMax;  // wave-uniform
      const uint8_t *bptr = reinterpret_cast<const uint8_t *>(bp);
      uint4 pre[2 * kDP];
      // kPB >= 5: the first payload loads go out as soon as the descriptor is
      // in, ahead of the table build (A/B form)
      if (kForm >= 5) piece_preload<kDP, kAux>(bptr, 0, blen, lane, own && blen >= 4, pre);
      if (kForm == 7 && !kNoLens) {
        // form 7: the decision's lengths behind the preload, so that the
        // first group's wait (vmcnt, counted in issue order) is not a wait for
        // them too
        __builtin_amdgcn_sched_barrier(0);
        load_lens();
      }
      if (wg_busy && !kNoTab) {
        const uint32_t e = braid_gen_lane(lane, slot);
        uint4 *dst = reinterpret_cast<uint4 *>(s_lds);
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) {
          const uint32_t src = (lane >> 4) + 4u * (k & 3u) + 16u * (2u * (k >> 2) + ((lane >> 3) & 1u));
          const uint32_t val = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src * 4u), (int)e);
          dst[tid + 1024u * k] = make_uint4(val, val, val, val);
        }
        uint4 cm0, cm1;
        comb_gen(slot, lane, cm0, cm1);
        uint4 *cdst = reinterpret_cast<uint4 *>(s_lds + kLdsCombDword);
        cdst[tid] = cm0;
        cdst[tid + 1024u] = cm1;
      }
      const uint64_t t_lens = kStamp ? __builtin_amdgcn_s_memrealtime() : 0;  // diagnostic: tables written
      // the tables are in LDS (form 7: an LDS-only barrier, the decision
      // lengths and the preloads may still be in flight)
      if (kNoBar) {
      } else if (kForm == 7) {
        lds_barrier();
      } else {
        __syncthreads();
      }
      const uint64_t t_fill = kStamp ? __builtin_amdgcn_s_memrealtime() : 0;
      if (kForm < 5) piece_preload<kDP, kAux>(bptr, 0, blen, lane, own && blen >= 4, pre);
      // the decision over the lengths L: forms < 7 here, where the compiler
      // hoisted it (and the waits for L) in front of the table barrier; forms
      // 7 and 8 after the wave's piece, when L has long arrived
      auto decide = [&]() -> uint32_t {
        bool big = false;
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) big |= (kForm == 9 || tid + 1024u * j < args.n) & (L[j] > kPerBufMax);
        return __ballot(big) ? 1u : 0u;
      };
      uint32_t any_big = (kForm >= 7 || kNoLens) ? 0u : decide();
      if (own) {
        // younger wave slots issue first (the round-3 per-buffer form below)
        if (kPrioMode == 0) {
          if (slot >= 12) __builtin_amdgcn_s_setprio(3);
          else if (slot >= 8) __builtin_amdgcn_s_setprio(2);
          else if (slot >= 4) __builtin_amdgcn_s_setprio(1);
        } else if (kPrioMode == 1) {
          __builtin_amdgcn_s_setprio(3);
        }
        uint32_t r;
        if (blen < 4) {
          r = ~bseed;
          for (uint32_t p = 0; p < (uint32_t)blen; p++) r = (r >> 8) ^ tab->stdtab[(r ^ bptr[p]) & 0xFFu];
        } else {
          r = piece_raw<kDP, kAblate, kAux, false, true, kPrioMode == 1, kFoldMode>(s_lds, bptr, 0, blen, bseed, lane,
                                                                                 nullptr, pre);
        }
        if (lane == 0) args.out[b] = ~r;
        if (kStamp && lane == 0) {  // diagnostic build (tools/c2_probe): this wave's timeline
          const uint64_t w = (uint64_t)blockIdx.x * kWaves + slot;
          args.stamps[8 * w + 0] = t_fill;
          args.stamps[8 * w + 1] = __builtin_amdgcn_s_memrealtime();
          args.stamps[8 * w + 4] = t_entry;
          args.stamps[8 * w + 5] = t_fill;
          args.stamps[8 * w + 6] = t_lens;
        }
        if (kPrioMode == 1) __builtin_amdgcn_s_setprio(0);
      }
      if (kNoEnd) return;
      if (kForm >= 7 && !kNoLens) any_big = decide();
      __syncthreads();  // every wave is done with the tables: the LDS is free
      if (lane == 0) s_lds[slot] = any_big;
      __syncthreads();
      const uint32_t fw = lane < (uint32_t)kWaves ? s_lds[lane] : 0u;
      if (!__ballot(fw != 0)) return;  // workgroup-uniform, and the same in every workgroup
      __syncthreads();  // every wave has read the flags before the scan overwrites LDS
      perbuf_done = true;
      load_tables();
    } else if (args.n <= (uint64_t)grid * kWaves) {
      const uint32_t lane = tid & 63u, slot = uni32(tid >> 6);
      const uint64_t b = (uint64_t)slot * grid + blockIdx.x;
      const bool wg_busy = blockIdx.x < args.n;  // workgroup-uniform
      // the decision's lengths (thread t: buffers t + 1024 j) with clamped
      // indices and no branch: a guarded load in its own block got its own
      // vmcnt(0), so the eight round trips ran one after another
      bool big = false;
#pragma unroll
      for (uint32_t j = 0; j < 8; j++) {
        const uint64_t idx = tid + 1024u * j;
        const uint64_t L = args.lens[idx < args.n ? idx : args.n - 1];
        big |= (idx < args.n) & (L > kPerBufMax);
      }
      const uint4 *comb_src = reinterpret_cast<const uint4 *>(tab->comb);
      const uint4 cm0 = comb_src[tid], cm1 = comb_src[tid + 1024u];  // unconditional: a guarded copy waited for them
      __builtin_amdgcn_sched_barrier(0);  // issued before the wait for the descriptor below
      uint64_t blen = 0, bp = 0;
      uint32_t bseed = 0;
      if (b < args.n) {
        blen = uni64(args.lens[b]);
        bp = uni64(reinterpret_cast<uint64_t>(args.ptrs[b]));
        bseed = args.seeds ? uni32(args.seeds[b]) : 0u;
      }
      const bool own = b < args.n && blen <= kPerBufMax;  // wave-uniform
      const uint8_t *bptr = reinterpret_cast<const uint8_t *>(bp);
      uint4 pre[2 * kD];
      if (kPerBufPreload) piece_preload<kD, kAux>(bptr, 0, blen, lane, own && blen >= 4, pre);
      if (wg_busy) {
        // braid chunk t + 1024 k holds entry (j, v) = (2 (k >> 2) + ((lane >> 3) & 1),
        // 4 slot + (lane >> 4) + 64 (k & 3)) (the layout above): 64 distinct
        // entries per wave, one built by each lane, exchanged by ds_bpermute
        const uint32_t e = braid_gen_lane(lane, slot);
        uint4 *dst = reinterpret_cast<uint4 *>(s_lds);
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) {
          const uint32_t src = (lane >> 4) + 4u * (k & 3u) + 16u * (2u * (k >> 2) + ((lane >> 3) & 1u));
          const uint32_t val = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src * 4u), (int)e);
          dst[tid + 1024u * k] = make_uint4(val, val, val, val);
        }
      }
      // chunk tid of the combine area is (table tid >> 8, j = (tid >> 6) & 3,
      // v = 4 (tid & 63) .. +3): lane 0 of wave s holds entry (s >> 2, s & 3, 0)
      // (the flag is a second write of that word, after the chunk's, by the
      // same wave: a wave's LDS writes land in order)
      const uint32_t flag = __ballot(big) ? 1u : 0u;
      const uint64_t t_lens = kStamp ? __builtin_amdgcn_s_memrealtime() : 0;  // diagnostic: the lengths are in
      if (wg_busy) {
        uint4 *cdst = reinterpret_cast<uint4 *>(s_lds + kLdsCombDword);
        cdst[tid] = cm0;
        cdst[tid + 1024u] = cm1;
      }
      if (lane == 0) s_lds[kLdsCombDword + 256u * slot] = flag;
      __syncthreads();  // the only barrier of the per-buffer mode
      const uint64_t t_fill = kStamp ? __builtin_amdgcn_s_memrealtime() : 0;
      const uint32_t fw = lane < (uint32_t)kWaves ? s_lds[kLdsCombDword + 256u * lane] : 0u;
      if (!__ballot(fw != 0)) {  // workgroup-uniform: every wave read the same 16 words
        if (b >= args.n || !wg_busy) return;
        // younger wave slots issue first: the SIMDs otherwise serve the
        // oldest waves first and the slots finish in four groups (+0.7% on
        // config 2 against none, -0.4% for the reverse order;
        // profiles/r02/per_buffer/ab_c2_slot_priority.jsonl)
        if (slot >= 12) __builtin_amdgcn_s_setprio(3);
        else if (slot >= 8) __builtin_amdgcn_s_setprio(2);
        else if (slot >= 4) __builtin_amdgcn_s_setprio(1);
        uint32_t r;
        if (blen < 4) {  // bytewise with the standard table
          r = ~bseed;
          for (uint32_t p = 0; p < (uint32_t)blen; p++) r = (r >> 8) ^ tab->stdtab[(r ^ bptr[p]) & 0xFFu];
        } else {
          r = piece_raw<kD, kAblate, kAux, false, kPerBufPreload>(s_lds, bptr, 0, blen, bseed, lane, nullptr, pre);
        }
        if (lane == 0) args.out[b] = ~r;
        if (kStamp && lane == 0) {  // diagnostic build (tools/c2_probe): this wave's timeline
          const uint64_t w = (uint64_t)blockIdx.x * kWaves + slot;
          args.stamps[8 * w + 0] = t_fill;
          args.stamps[8 * w + 1] = __builtin_amdgcn_s_memrealtime();
          args.stamps[8 * w + 4] = t_entry;
          args.stamps[8 * w + 5] = t_fill;
          args.stamps[8 * w + 6] = t_lens;
        }
        return;
      }
      // some buffer is longer than kPerBufMax: the in-kernel scan below
      __syncthreads();  // every wave has read the flags before the scan overwrites LDS
      load_tables();
    } else {
      load_tables();
    }
    uint64_t v[8], sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < 8; k++) {
      const uint64_t idx = 8u * tid + k;
      v[k] = idx < args.n ? args.lens[idx] : 0;
      if (perbuf_done && v[k] <= kPerBufMax) v[k] = 0;
      sum += v[k];
    }
    uint64_t tot;
    uint64_t run = block_excl_scan(sum, lds_pre + kFusedMaxN + 8, &tot);
    uint64_t *gpre = const_cast<uint64_t *>(args.prefix);
#pragma unroll
    for (uint32_t k = 0; k < 8; k++) {
      const uint64_t idx = 8u * tid + k;
      if (idx < args.n) lds_pre[idx] = run, gpre[idx] = run;
      run += v[k];
    }
    if (tid == 0) lds_pre[args.n] = tot, gpre[args.n] = tot;
    __threadfence_block();
    __syncthreads();
  }
  BatchView<kStrided> bv(args, kFused ? lds_pre : nullptr);
  const uint64_t total = bv.total();
  const uint64_t max_waves = (uint64_t)grid * kWaves;
  const uint64_t min_range = args.min_range ? args.min_range : kMinRange;
  uint64_t want = (total + min_range - 1) / min_range;
  // many small buffers: at least a wave per buffer -- per-buffer latency,
  // not bytes, bounds them (4096 x 64 B took 1.8 ms on the 4 waves that
  // 256 KiB asks for by bytes; tools/host_overhead.py)
  if (want < args.n) want = args.n;
  if (want < 1) want = 1;
  const uint64_t W = want < max_waves ? want : max_waves;
  if ((uint64_t)blockIdx.x * kWaves >= W && !join) return;  // whole workgroup idle (uniform: no barrier is skipped)

  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t w = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);

  // Static part: the first Ts = total - Td bytes in W equal snapped ranges,
  // issue priority banded by progress (kPrio).  Dynamic part: the last
  // Td = total >> shift bytes in fixed units claimed from one counter
  // once a wave's static range is done, so the waves that the hardware
  // serves faster (older wave slots, some XCDs: tools/crc_variants stamps)
  // absorb the imbalance.  Units of 128 KiB measured best: larger ones leave
  // stragglers, smaller ones pay per-piece latency.
  const uint64_t unit = args.dyn_unit ? args.dyn_unit : kDynUnit;
  // kDynAuto: half the bytes dynamic for batches of small ragged buffers
  // (per-piece latency varies), a quarter for large buffers (every unit
  // boundary inside a buffer costs a split piece).
  uint32_t shift = args.dyn_shift != kDynAuto ? args.dyn_shift
                   : (args.n && total / args.n < kDynSmallAvg) ? 1u : 2u;
  // A/B (ab_flags bits 4-5, read per call: tools/order_ab.py): 1 -> an eighth
  // dynamic, 2 -> half, 3 -> none
  if (const uint32_t ds = (args.ab_flags >> 4) & 3u) shift = ds == 1 ? 3u : ds == 2 ? 1u : 0u;
  uint64_t Td = (args.ctr && shift) ? (total >> shift) : 0;
  if (Td / W < unit) Td = 0;  // fewer units than waves: static only
  uint64_t Ts = total - Td;
  // (Round 4: the last units halved -- ZCRC_DYN_TAIL, an A/B knob -- ran
  // 0.4-1.5% slower on config 4 and was dropped: DESIGN.md 7d.)
  // Window order (BatchView::wp): equal buffers whose static wave ranges are
  // whole runs of p >= 2 of them (config 3: 48 GiB static over 4,096 waves =
  // 12 buffers of 1 MiB each; config 5's shard: 24).  When the static part
  // is not such a multiple but there is a dynamic part, the static part is
  // cut down to p W whole buffers and the rest joins the dynamic units
  // (which then start on a buffer boundary).  ab_flags bit 3 (A/B): the
  // range order.
  if (equal && !kFused && !(args.ab_flags & 8u) && args.n && args.n < (1ull << 32)) {
    const uint64_t L = kStrided ? args.len : total / args.n;
    if (L && (kStrided || L * args.n == total) && (Td || Ts % (W * L) == 0)) {
      const uint64_t p = Ts / (W * L);
      if (p >= 2 && p * W <= args.n) bv.wp = p, bv.wW = W, Ts = p * W * L, Td = total - Ts;
    }
  }
  const uint64_t units = Td ? (Td + unit - 1) / unit : 0;
  if (join && units <= W) return;  // no claims to join: every unit is pre-assigned (uniform per workgroup)

  // Chunked window order (ab_flags bit 6, A/B): the static part cut into
  // W * wc chunks of ~kWinChunk bytes, wave w taking chunks w, w + W, ...
  // (the byte-level form of BatchView::wp, for any lengths)
  uint64_t wc = 1;
  if ((args.ab_flags & 64u) && !kFused && !join) {
    const uint64_t cb = kWinChunk >> ((args.ab_flags >> 7) & 3u);  // bits 7-8: 1 MiB >> k
    wc = (Ts / W + cb / 2) / cb;
    wc = wc < 1 ? 1 : (wc > 1024 ? 1024 : wc);
    bv.wp = 0;
  }
  const uint64_t C = W * wc;  // chunks; wave w's k-th is chunk k * W + w
  // nominal boundary of chunk j: floor(j * Ts / C), without 128-bit math
  const uint64_t q_tot = Ts / C, r_tot = Ts % C;
  auto nominal = [&](uint64_t j) -> uint64_t { return j >= C ? Ts : q_tot * j + (r_tot * j) / C; };
  uint64_t kc = 0;  // the wave's static chunk
  bool last = (w + 1 == W) && !Td && wc == 1;
  uint64_t S0 = 0, S1 = 0, f0 = 0, lb1 = 0;  // f0: first buffer overlapping [S0, S1)
  if (w < W) bv.range(nominal(w), nominal(w + 1), last, S0, S1, f0, lb1);
  const uint64_t t_search = kStamp ? __builtin_amdgcn_s_memrealtime() : 0;
  if (kFused) {
    __syncthreads();  // every wave's search is done with the LDS prefix
    bv.lpre = nullptr;
  }
  // ---- LDS: braided table x32 replicas + 8 combine tables ---------------
  {
    uint4 *dst = reinterpret_cast<uint4 *>(s_lds);
#pragma unroll
    for (int k = 0; k < 8; k++)
      dst[tid + 1024u * k] = make_uint4(braid_val[k], braid_val[k], braid_val[k], braid_val[k]);
    uint4 *cdst = reinterpret_cast<uint4 *>(s_lds + kLdsCombDword);
    cdst[tid] = comb0;
    cdst[tid + 1024u] = comb1;
  }
  __syncthreads();
  if (w >= W && !join) return;  // no barrier after this point
  bool band = true;


  // diagnostic build: wall-clock stamps (s_memrealtime, 100 MHz) per wave
  const uint64_t t_begin = kStamp ? __builtin_amdgcn_s_memrealtime() : 0;
  uint64_t npieces = 0;
  uint32_t salt = (uint32_t)w;
  // Claims: wave w's first unit is unit w, taken without the counter (all
  // waves reach their first claim within a few microseconds, and 4096
  // atomics on one address in that window serialise: with ~1 unit per wave
  // the dynamic part ran 25% slower than none, tools/crc_variants); later
  // units come from the counter, W + ctr++ (a read of the counter before
  // each atomic, to spare the empty claims at the end, measured 8% slower),
  // prefetched (issued before the
  // current unit is processed, so the atomic's latency hides behind the
  // unit) while more than 2W units remain -- near the end a
  // held-but-unstarted unit would become a straggler.
  // (Round 4: claims spread over 8 counters 256 B apart, a wave's home
  // counter chosen by workgroup, ran 3% slower on config 4: DESIGN.md 7d.)
  uint32_t u = 0, nx = 0;
  bool have_next = false, first_claim = true;
  uint64_t t_tail = 0;                 // diagnostic build: time in the alignment-padding MCTs (unused)
  uint64_t t_static_end = 0, n_dyn = 0;  // ... the static range's end, dynamic units taken,
  uint64_t t_claim = 0, t_usearch = 0;   // time waiting for unprefetched claims, in unit range searches
  for (;;) {
    if (!band && u + 2 * (uint32_t)W < units) {
      if (lane == 0) nx = atomicAdd(args.ctr, 1u);
      have_next = true;
    }
    if (S0 < S1 || last)
      npieces += process_range<kStrided, kD, kAblate, kRotate, kPrio, kAux, kStamp, kFused, kWin>(
          args, bv, s_lds, tab, S0, S1, last, salt, lane, band, f0, lb1, &t_tail, perbuf_done);
    if (band && ++kc < wc) {  // the wave's next static chunk
      const uint64_t j = kc * W + w;
      last = (j + 1 == C) && !Td;
      bv.range(nominal(j), nominal(j + 1), last, S0, S1, f0, lb1);
      continue;
    }
    if (kStamp && first_claim) t_static_end = __builtin_amdgcn_s_memrealtime();
    if (!units) break;
    const uint64_t tc0 = kStamp ? __builtin_amdgcn_s_memrealtime() : 0;
    if (first_claim && !join) {
      u = (uint32_t)w;  // units >= W whenever the dynamic part is on
    } else if (units <= W) {
      break;  // every unit was pre-assigned: no claim (and no atomic) at all
    } else {
      if (!have_next && lane == 0) nx = atomicAdd(args.ctr, 1u);
      u = (uint32_t)W + uni32(nx);
    }
    first_claim = false;
    have_next = false;
    if (kStamp) t_claim += __builtin_amdgcn_s_memrealtime() - tc0;
    if (u >= units) break;
    const uint64_t t0 = Ts + (uint64_t)u * unit;
    last = (u + 1 == units);
    if (kStamp) n_dyn++;
    const uint64_t ts0 = kStamp ? __builtin_amdgcn_s_memrealtime() : 0;
    bv.range(t0, t0 + unit, last, S0, S1, f0, lb1);
    if (kStamp) t_usearch += __builtin_amdgcn_s_memrealtime() - ts0;
    salt = u ^ 0x9E3779B9u;
    if (kPrio && band) __builtin_amdgcn_s_setprio(0);
    band = false;
  }
  if (kFused && units && lane == 0) {
    // the last wave out returns the claim counter to zero for the next launch
    // (no plan kernel resets it); every claim of this launch is complete here
    __threadfence();
    if (atomicAdd(args.done, 1u) + 1u == (uint32_t)W) {
      atomicExch(args.ctr, 0u);
      atomicExch(args.done, 0u);
    }
  }
  if (kStamp && lane == 0) {  // (tools/c2_probe, tools/c4_probe)
    args.stamps[8 * w + 0] = t_begin;
    args.stamps[8 * w + 1] = __builtin_amdgcn_s_memrealtime();
    args.stamps[8 * w + 2] = npieces | (n_dyn << 32) | ((uint64_t)join << 63);
    args.stamps[8 * w + 3] = t_static_end;
    args.stamps[8 * w + 4] = t_entry;
    args.stamps[8 * w + 5] = t_search;
    args.stamps[8 * w + 6] = t_usearch;
    args.stamps[8 * w + 7] = t_claim;
  }
}

}  // namespace zcrc

// the small-buffer body the batch kernel runs for the split plan's small list
#include "zcrc_small_kernel.h"
