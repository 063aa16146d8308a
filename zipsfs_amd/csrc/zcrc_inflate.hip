// zcrc_inflate.hip -- batched raw-DEFLATE decode on MI355X (gfx950).
//
// SURVEY.md 8(f) rank 4.  ZIPsFS inflates a deflated ZIP entry with libzip's
// zip_fread() (src/ZIPsFS.c:2016-2019) inside preloadram_now
// (src/ZIPsFS_preloadfileram.c:286-306) and then CRCs the result (:243).
// libzip inflates with zlib; this file decodes the same format (RFC 1951)
// with zlib 1.2.11's acceptance rules (oracle/inflate_port.c restates them
// and is the checker), so that a whole archive's entries inflate on the GPU
// and go straight into the batched CRC kernel without leaving HBM.
//
// Design:
//   * one 64-lane workgroup per stream; DEFLATE is serial within a stream,
//     so the batch is the parallelism.  ~38 KiB LDS per workgroup -> four
//     streams resident per CU, more waiting in the dispatcher, which also
//     balances ragged stream sizes for free;
//   * LDS holds the 32 KiB window as a ring (every back-reference is an LDS
//     read), a 2^10-entry literal/length LUT and a 2^8-entry distance LUT,
//     plus canonical count/symbol arrays for codes longer than the LUT root;
//   * input: 2 KiB staged in VGPRs (16 B per lane, coalesced 1 KiB loads one
//     block ahead); the wave-uniform bit reader gathers dwords with
//     v_readlane, so decode state lives in SGPRs;
//   * table builds are wave-parallel (ballot counts, ballot-ranked canonical
//     symbol order, every LUT index decoded canonically by its own lane);
//   * matches copy lane-parallel through the ring (i mod dist for
//     overlapping short distances); output leaves the ring in 512-byte
//     lane-parallel flushes.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/zcrc.h"
#include "zcrc_internal.h"

#ifdef ZCRC_INFLATE_TRACE
#define ITRACE(...) do { if (threadIdx.x == 0 && blockIdx.x < 4) printf(__VA_ARGS__); } while (0)
#else
#define ITRACE(...) do { } while (0)
#endif

namespace zcrc {
namespace {

constexpr uint32_t kWin = 32768, kWinMask = kWin - 1;
constexpr uint32_t kLLRoot = 10, kDRoot = 8, kCLRoot = 7;
constexpr uint32_t kFlush = 512;

// LUT entry: [0:4) code length, [4:7) kind, [7:11) extra bits, [11:27) value
enum : uint32_t { K_BAD = 0, K_LIT = 1, K_BASE = 2, K_EOB = 3, K_LONG = 4 };
enum : uint32_t { A_LITLEN = 0, A_DIST = 1, A_CLEN = 2 };

__device__ __forceinline__ uint32_t mk(uint32_t len, uint32_t kind, uint32_t extra, uint32_t val) {
  return len | (kind << 4) | (extra << 7) | (val << 11);
}
__device__ __forceinline__ uint32_t e_len(uint32_t e) { return e & 15u; }
__device__ __forceinline__ uint32_t e_kind(uint32_t e) { return (e >> 4) & 7u; }
__device__ __forceinline__ uint32_t e_extra(uint32_t e) { return (e >> 7) & 15u; }
__device__ __forceinline__ uint32_t e_val(uint32_t e) { return e >> 11; }

__device__ __forceinline__ uint32_t u32u(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane(v); }

// RFC 1951 3.2.5 base/extra tables
__constant__ uint16_t c_len_base[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                        31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t c_len_extra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                        2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t c_dist_base[30] = {1,    2,    3,    4,    5,    7,    9,    13,    17,    25,
                                         33,   49,   65,   97,   129,  193,  257,  385,   513,   769,
                                         1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t c_dist_extra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6,
                                         6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t c_clen_order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

struct Lds {
  uint8_t ring[kWin];
  uint32_t ll[1u << kLLRoot];
  uint32_t dd[1u << kDRoot];  // distance LUT; the code-length LUT while reading a header
  uint16_t llcnt[16], ddcnt[16];
  uint16_t llsym[288], ddsym[32];
  uint16_t offs[16];
  uint8_t lens[336];  // clen code lengths [0,19) | litlen+dist lengths [19, 19+316)
};

__device__ __forceinline__ uint32_t symbol_entry(uint32_t alphabet, uint32_t sym, uint32_t len) {
  if (alphabet == A_LITLEN) {
    if (sym < 256) return mk(len, K_LIT, 0, sym);
    if (sym == 256) return mk(len, K_EOB, 0, 0);
    if (sym < 286) return mk(len, K_BASE, c_len_extra[sym - 257], c_len_base[sym - 257]);
    return mk(len, K_BAD, 0, 0);
  }
  if (alphabet == A_DIST) return sym < 30 ? mk(len, K_BASE, c_dist_extra[sym], c_dist_base[sym]) : mk(len, K_BAD, 0, 0);
  return mk(len, K_LIT, 0, sym);
}

// Build the canonical code for lens[0..n) (RFC 1951 3.2.2) into cnt/sym
// and a 2^root LUT.  Returns false where zlib's inflate_table() rejects the
// set: over-subscribed, or incomplete unless (not CLEN and a single
// length-1 code); an all-zero set is accepted (decoding from it fails).
__device__ bool build_code(Lds &s, const uint8_t *lens, uint32_t n, uint32_t root, uint32_t *lut, uint16_t *cnt,
                           uint16_t *sym, uint32_t alphabet) {
  const uint32_t lane = threadIdx.x;
  // counts per length: ballots over 64-symbol chunks
  uint32_t count[16];
#pragma unroll
  for (int L = 0; L < 16; L++) count[L] = 0;
  for (uint32_t c = 0; c < n; c += 64) {
    const uint32_t sidx = c + lane;
    const uint32_t l = sidx < n ? lens[sidx] : 0u;
#pragma unroll
    for (int L = 1; L < 16; L++) count[L] += (uint32_t)__builtin_popcountll(__ballot(l == (uint32_t)L));
  }
  int left = 1;
  uint32_t max_len = 0;
#pragma unroll
  for (int L = 1; L < 16; L++) {
    left = (left << 1) - (int)count[L];
    if (count[L]) max_len = L;
    if (left < 0) break;
  }
  if (left < 0) return false;
  if (max_len && left > 0 && (alphabet == A_CLEN || max_len != 1)) return false;
  if (lane == 0) {
    uint32_t o = 0;
    cnt[0] = 0;
#pragma unroll
    for (int L = 1; L < 16; L++) {
      cnt[L] = (uint16_t)count[L];
      s.offs[L] = (uint16_t)o;
      o += count[L];
    }
  }
  __syncthreads();
  // canonical symbol order: by (length, symbol); ranks from ballots
  for (uint32_t c = 0; c < n; c += 64) {
    const uint32_t sidx = c + lane;
    const uint32_t l = sidx < n ? lens[sidx] : 0u;
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int L = 1; L < 16; L++) {
      if (!count[L]) continue;
      const uint64_t m = __ballot(l == (uint32_t)L);
      if (!m) continue;
      const uint32_t base = s.offs[L];
      if (l == (uint32_t)L) sym[base + (uint32_t)__builtin_popcountll(m & lt)] = (uint16_t)sidx;
      __syncthreads();
      if (lane == 0) s.offs[L] = (uint16_t)(base + (uint32_t)__builtin_popcountll(m));
      __syncthreads();
    }
  }
  __syncthreads();
  // LUT: lane decodes its own indices canonically (bits LSB-first)
  const uint32_t size = 1u << root;
  for (uint32_t idx = lane; idx < size; idx += 64) {
    int code = 0, first = 0, index = 0;
    uint32_t e = (max_len > root) ? mk(0, K_LONG, 0, 0) : mk(0, K_BAD, 0, 0);
    for (uint32_t L = 1; L <= root; L++) {
      code |= (int)((idx >> (L - 1)) & 1u);
      const int ct = (int)cnt[L];
      if (code - ct < first) {
        e = symbol_entry(alphabet, sym[index + (code - first)], L);
        break;
      }
      index += ct;
      first += ct;
      first <<= 1;
      code <<= 1;
    }
    lut[idx] = e;
  }
  __syncthreads();
  return true;
}

struct Reader {
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t lead;     // src - (src & ~15)
  uint32_t end;      // lead + src_len: bytes at or past it read as zero
  uint64_t src_len;
  uint4 A, B;        // blocks kA, kA+1 (1 KiB each; lane holds 16 B)
  uint32_t kA;
  uint32_t P;        // next byte (relative to the aligned base) to enter bb
  uint64_t bb;       // bit buffer, LSB first
  uint32_t nb;       // valid bits in bb

  __device__ uint4 load_block(uint32_t k) const {
    const uint32_t off = k * 1024u + 16u * threadIdx.x;
    auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0);
    return make_uint4(v[0], v[1], v[2], v[3]);
  }
  __device__ void seek(uint32_t p) {
    P = p;
    bb = 0;
    nb = 0;
    kA = p >> 10;
    A = load_block(kA);
    B = load_block(kA + 1);
  }
  __device__ uint32_t dword_at(uint32_t g) const {
    const bool inA = (g >> 8) == kA;
    const uint32_t c = g & 3u;
    const uint32_t x = inA ? A.x : B.x, y = inA ? A.y : B.y, z = inA ? A.z : B.z, w = inA ? A.w : B.w;
    const uint32_t v = c == 0 ? x : c == 1 ? y : c == 2 ? z : w;
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)((g >> 2) & 63u));
  }
  // top up to >= 32 valid bits
  __device__ void refill() {
    if (nb > 32) return;
    while (P >= (kA + 1) * 1024u) {  // slide the staging window
      A = B;
      kA++;
      B = load_block(kA + 1);
    }
    const uint32_t g = P >> 2;
    const uint32_t lo = dword_at(g), hi = dword_at(g + 1);
    uint32_t w = __builtin_amdgcn_alignbyte(hi, lo, P & 3u);
    if (P + 4u > end) w &= P >= end ? 0u : (1u << (8u * (end - P))) - 1u;
    bb |= (uint64_t)w << nb;
    nb += 32;
    P += 4;
  }
  __device__ uint32_t peek(uint32_t k) const { return (uint32_t)bb & ((1u << k) - 1u); }
  __device__ void drop(uint32_t k) {
    bb >>= k;
    nb -= k;
  }
  __device__ uint32_t bits(uint32_t k) {  // k <= 16
    refill();
    const uint32_t v = peek(k);
    drop(k);
    return v;
  }
  // input bytes consumed (through the last bit used)
  __device__ uint64_t consumed() const { return (uint64_t)P - lead - nb / 8u; }
  __device__ bool overrun() const { return (uint64_t)P > (uint64_t)lead + src_len + 16u; }
};

// canonical decode of a code longer than the LUT root (rare)
__device__ uint32_t decode_slow(Reader &r, const uint16_t *cnt, const uint16_t *sym, uint32_t alphabet) {
  int code = 0, first = 0, index = 0;
  for (uint32_t L = 1; L <= 15; L++) {
    code |= (int)((r.bb >> (L - 1)) & 1u);
    const int ct = cnt[L];
    if (code - ct < first) return symbol_entry(alphabet, sym[index + (code - first)], L);
    index += ct;
    first += ct;
    first <<= 1;
    code <<= 1;
  }
  return mk(0, K_BAD, 0, 0);
}

// A symbol the code cannot accept.  The canonical decoder (the oracle)
// reads the whole code first -- its length, or all 15 bits when no code
// matches -- so those bits count as consumed: past the end of the input the
// kernel's epilogue then reports ZCRC_INFLATE_ERR_INPUT, as the oracle does.
__device__ __forceinline__ int32_t bad_symbol(Reader &r, uint32_t e, int32_t err) {
  r.drop(e_len(e) ? e_len(e) : 15u);
  return err;
}

struct Out {
  uint8_t *dst;
  uint64_t cap;
  uint64_t pos;  // bytes produced
  uint64_t fl;   // bytes flushed to dst
};

__device__ void flush(Lds &s, Out &o, uint64_t upto) {
  const uint32_t lane = threadIdx.x;
  while (o.fl < upto) {
    const uint64_t i = o.fl + lane;
    if (i < upto) o.dst[i] = s.ring[i & kWinMask];
    o.fl = (o.fl + 64 < upto) ? o.fl + 64 : upto;
  }
}

__device__ __forceinline__ void maybe_flush(Lds &s, Out &o) {
  if (o.pos - o.fl >= kFlush) flush(s, o, o.fl + kFlush);
}

// one Huffman-coded block (fixed or dynamic tables already built)
__device__ int32_t codes(Lds &s, Reader &r, Out &o) {
  const uint32_t lane = threadIdx.x;
  for (;;) {
    if (r.overrun()) return ZCRC_INFLATE_ERR_INPUT;
    r.refill();
    uint32_t e = u32u(s.ll[r.peek(kLLRoot)]);
    ITRACE("[%u] sym P=%u nb=%u bb=%llx e=%x kind=%u len=%u val=%u pos=%llu\n", blockIdx.x, r.P, r.nb,
           (unsigned long long)r.bb, e, e_kind(e), e_len(e), e_val(e), (unsigned long long)o.pos);
    if (e_kind(e) == K_LONG) e = u32u(decode_slow(r, s.llcnt, s.llsym, A_LITLEN));
    const uint32_t kind = e_kind(e);
    if (kind == K_LIT) {
      r.drop(e_len(e));
      if (o.pos >= o.cap) return ZCRC_INFLATE_ERR_OUTPUT;
      if (lane == 0) s.ring[o.pos & kWinMask] = (uint8_t)e_val(e);
      o.pos++;
      maybe_flush(s, o);
      continue;
    }
    if (kind == K_EOB) {
      r.drop(e_len(e));
      return ZCRC_INFLATE_OK;
    }
    if (kind != K_BASE || e_len(e) == 0) return bad_symbol(r, e, ZCRC_INFLATE_ERR_SYMBOL);
    r.drop(e_len(e));
    const uint32_t len = e_val(e) + r.peek(e_extra(e));
    r.drop(e_extra(e));
    r.refill();
    uint32_t d = u32u(s.dd[r.peek(kDRoot)]);
    if (e_kind(d) == K_LONG) d = u32u(decode_slow(r, s.ddcnt, s.ddsym, A_DIST));
    if (e_kind(d) != K_BASE || e_len(d) == 0) return bad_symbol(r, d, ZCRC_INFLATE_ERR_SYMBOL);
    r.drop(e_len(d));
    const uint32_t dist = e_val(d) + r.peek(e_extra(d));
    r.drop(e_extra(d));
    if (dist > o.pos) return ZCRC_INFLATE_ERR_DIST;
    if (len > o.cap - o.pos) return ZCRC_INFLATE_ERR_OUTPUT;
    // lane-parallel copy through the ring; every source byte precedes pos
    // (short distances replicate with i mod dist; long ones go 64 at a time)
    const uint32_t p0 = (uint32_t)o.pos;
    for (uint32_t i0 = 0; i0 < len; i0 += 64) {
      const uint32_t i = i0 + lane;
      uint8_t v = 0;
      if (i < len) {
        const uint32_t off = dist < 64 ? i % dist : i;
        v = s.ring[(p0 - dist + off) & kWinMask];
      }
      __builtin_amdgcn_wave_barrier();
      if (i < len) s.ring[(p0 + i) & kWinMask] = v;
      __builtin_amdgcn_wave_barrier();
    }
    o.pos += len;
    maybe_flush(s, o);
  }
}

__device__ int32_t stored(Lds &s, Reader &r, Out &o) {
  const uint32_t lane = threadIdx.x;
  r.drop(r.nb & 7u);  // byte boundary
  r.refill();
  const uint32_t len = r.peek(16);
  r.drop(16);
  r.refill();
  const uint32_t nlen = r.peek(16);
  r.drop(16);
  if (len != (~nlen & 0xFFFFu)) return ZCRC_INFLATE_ERR_STORED_LEN;
  const uint32_t q = r.P - r.nb / 8u;  // next unconsumed byte (aligned-base relative)
  if ((uint64_t)q - r.lead + len > r.src_len) return ZCRC_INFLATE_ERR_INPUT;
  if (len > o.cap - o.pos) return ZCRC_INFLATE_ERR_OUTPUT;
  const uint32_t p0 = (uint32_t)o.pos;
  for (uint32_t i0 = 0; i0 < len; i0 += 64) {
    const uint32_t i = i0 + lane;
    if (i < len) {
      const uint8_t v = __builtin_amdgcn_raw_buffer_load_b8(r.rsrc, q + i, 0, 0);
      s.ring[(p0 + i) & kWinMask] = v;
    }
    __builtin_amdgcn_wave_barrier();
    o.pos = p0 + ((i0 + 64 < len) ? i0 + 64 : len);
    maybe_flush(s, o);
  }
  r.seek(q + len);
  return ZCRC_INFLATE_OK;
}

__device__ int32_t dynamic_tables(Lds &s, Reader &r) {
  const uint32_t lane = threadIdx.x;
  const uint32_t nlen = r.bits(5) + 257, ndist = r.bits(5) + 1, ncode = r.bits(4) + 4;
  if (nlen > 286 || ndist > 30) return ZCRC_INFLATE_ERR_CODES;
  if (lane < 19) s.lens[lane] = 0;
  __syncthreads();
  for (uint32_t k = 0; k < ncode; k++) {
    const uint32_t v = r.bits(3);
    if (lane == 0) s.lens[c_clen_order[k]] = (uint8_t)v;
  }
  __syncthreads();
  // code-length code in the distance slots (max code length 7 = its root)
  if (!build_code(s, s.lens, 19, kCLRoot, s.dd, s.ddcnt, s.ddsym, A_CLEN)) return ZCRC_INFLATE_ERR_CODES;
  uint32_t idx = 0, prev = 0;
  const uint32_t total = nlen + ndist;
  while (idx < total) {
    if (r.overrun()) return ZCRC_INFLATE_ERR_INPUT;
    r.refill();
    const uint32_t e = u32u(s.dd[r.peek(kCLRoot)]);
    if (e_kind(e) != K_LIT || e_len(e) == 0) return bad_symbol(r, e, ZCRC_INFLATE_ERR_CODES);
    r.drop(e_len(e));
    const uint32_t sym = e_val(e);
    uint32_t val, rep;
    if (sym < 16) {
      val = sym;
      rep = 1;
      prev = sym;
    } else if (sym == 16) {
      if (idx == 0) return ZCRC_INFLATE_ERR_CODES;
      val = prev;
      rep = 3 + r.bits(2);
    } else if (sym == 17) {
      val = 0;
      rep = 3 + r.bits(3);
      prev = 0;
    } else {
      val = 0;
      rep = 11 + r.bits(7);
      prev = 0;
    }
    if (idx + rep > total) return ZCRC_INFLATE_ERR_CODES;
    for (uint32_t k = lane; k < rep; k += 64) s.lens[19 + idx + k] = (uint8_t)val;
    idx += rep;
  }
  __syncthreads();
  const uint8_t *ll = s.lens + 19, *dl = s.lens + 19 + nlen;
  if (ll[256] == 0) return ZCRC_INFLATE_ERR_CODES;
  if (!build_code(s, ll, nlen, kLLRoot, s.ll, s.llcnt, s.llsym, A_LITLEN)) return ZCRC_INFLATE_ERR_CODES;
  if (!build_code(s, dl, ndist, kDRoot, s.dd, s.ddcnt, s.ddsym, A_DIST)) return ZCRC_INFLATE_ERR_CODES;
  return ZCRC_INFLATE_OK;
}

__device__ void fixed_tables(Lds &s) {
  const uint32_t lane = threadIdx.x;
  for (uint32_t k = lane; k < 320; k += 64) {
    uint8_t l;
    if (k < 144) l = 8;
    else if (k < 256) l = 9;
    else if (k < 280) l = 7;
    else if (k < 288) l = 8;
    else l = 5;  // 32 distance codes; 30 and 31 decode as invalid
    s.lens[k] = l;
  }
  __syncthreads();
  build_code(s, s.lens, 288, kLLRoot, s.ll, s.llcnt, s.llsym, A_LITLEN);
  build_code(s, s.lens + 288, 32, kDRoot, s.dd, s.ddcnt, s.ddsym, A_DIST);
}

__global__ __launch_bounds__(64) void inflate_kernel(InflateArgs a) {
  __shared__ Lds s;
  const uint64_t i = blockIdx.x;
  if (i >= a.n) return;
  const uint8_t *src = a.src[i];
  const uint64_t src_len = a.src_len[i];
  Out o;
  o.dst = a.dst[i];
  o.cap = a.cap[i];
  o.pos = 0;
  o.fl = 0;
  int32_t st = ZCRC_INFLATE_OK;
  Reader r;
  if (src_len == 0 || src_len > kInflateMaxSrc) {
    st = src_len == 0 ? ZCRC_INFLATE_ERR_INPUT : ZCRC_INFLATE_ERR_TOO_BIG;
  } else {
    const uint64_t base = reinterpret_cast<uint64_t>(src) & ~(uint64_t)15;
    r.lead = (uint32_t)(reinterpret_cast<uint64_t>(src) - base);
    r.src_len = src_len;
    r.end = r.lead + (uint32_t)src_len;
    // The buffer unit range-checks whole dwords (a dword that straddles
    // num_records reads as 0), so the range is rounded up to the 16-byte
    // granule holding the last byte -- same page, never a fault -- and the
    // bytes past `end` are masked in refill().
    r.rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(base), (short)0,
                                               (int)((r.end + 15u) & ~15u), 0x00020000);
    r.seek(r.lead);
    ITRACE("[%u] seek lead=%u A0=%x d0=%x d1=%x\n", blockIdx.x, r.lead, r.A.x, r.dword_at(0), r.dword_at(1));
    uint32_t last = 0;
    do {
      if (r.overrun()) {
        st = ZCRC_INFLATE_ERR_INPUT;
        break;
      }
      ITRACE("[%u] hdr P=%u nb=%u bb=%llx lead=%u srclen=%llu\n", blockIdx.x, r.P, r.nb,
             (unsigned long long)r.bb, r.lead, (unsigned long long)r.src_len);
      last = r.bits(1);
      const uint32_t type = r.bits(2);
      ITRACE("[%u]   last=%u type=%u\n", blockIdx.x, last, type);
      if (type == 0) {
        st = stored(s, r, o);
      } else if (type == 1) {
        fixed_tables(s);
        st = codes(s, r, o);
      } else if (type == 2) {
        st = dynamic_tables(s, r);
        if (st == ZCRC_INFLATE_OK) st = codes(s, r, o);
      } else {
        st = ZCRC_INFLATE_ERR_BLOCK_TYPE;
      }
    } while (!last && st == ZCRC_INFLATE_OK);
    // Bits past the end read as zero.  Whenever the decode used any of them
    // -- whether it then ended cleanly or failed on what they said -- the
    // canonical decoder would have stopped at the first one: input error.
    if (r.consumed() > src_len) st = ZCRC_INFLATE_ERR_INPUT;
  }
  if (st == ZCRC_INFLATE_OK) flush(s, o, o.pos);
  if (threadIdx.x == 0) {
    a.out_len[i] = st == ZCRC_INFLATE_OK ? o.pos : 0;
    a.status[i] = st;
  }
}

}  // namespace

hipError_t launch_inflate(const InflateArgs &args, hipStream_t stream) {
  if (args.n == 0) return hipSuccess;
  hipLaunchKernelGGL(inflate_kernel, dim3((unsigned)args.n), dim3(64), 0, stream, args);
  return hipGetLastError();
}

}  // namespace zcrc
