// zcrc_inflate_impl.h -- the batched inflate kernel, parameterised by the
// LDS window size ZI_WIN.  Included by zcrc_inflate.hip once per variant
// (namespaces w16, w8, w32, and sp: ZI_SPEC = 1, the speculative chunk
// decoder of zcrc_inflate_split.hip); not a standalone header.
//
// ZI_SPEC: output elements are 16-bit -- a byte, or a marker kMarker + w for
// byte w of the unknown 32 KiB history before the chunk (a back-reference
// past the chunk's first output) -- written to the chunk's region of split
// scratch; the decode starts at a candidate bit position and stops at the
// next candidate it reaches (tests/inflate_split_model.py is the spec).
#ifndef ZI_SPEC
#define ZI_SPEC 0
#define ZI_SPEC_DEFAULTED
#endif
namespace {

#if ZI_SPEC
typedef uint16_t elem_t;
#define ZI_DSW "ds_write_b16"
#define ZI_DSR "ds_read_u16"
#define ZI_ESH "1"
#else
typedef uint8_t elem_t;
#define ZI_DSW "ds_write_b8"
#define ZI_DSR "ds_read_u8"
#define ZI_ESH "0"
#endif
constexpr uint32_t kEsh = ZI_SPEC ? 1u : 0u;  // log2(bytes per output element)


// The LDS ring holds the last kWin bytes (ZI_WIN, set by zcrc_inflate.hip).
// DEFLATE distances reach 32 KiB: with a 16 KiB ring the older bytes are
// read back from dst (they are flushed by then), which fits eight streams per
// CU instead of four.
constexpr uint32_t kWin = ZI_WIN, kWinMask = kWin - 1;
constexpr uint32_t kLLRoot = 10, kDRoot = 8, kCLRoot = 7;
constexpr uint32_t kLLRegs = (1u << kLLRoot) / 64, kDRegs = (1u << kDRoot) / 64, kCLRegs = (1u << kCLRoot) / 64;
// bytes decoded ahead of the last flush; pos - fl stays below
// kFlushLag + 1024 + 258, which must be < kWin (copy_match)
constexpr uint32_t kFlushLag = kWin >= 16384 ? 8192 : kWin / 2;
static_assert(kFlushLag + 1024 + 258 < kWin, "flush lag must leave the window's far bytes flushed");

// Register-resident tables are LLVM vectors: a dynamic subscript lowers to
// s_set_gpr_idx + v_mov (no scratch), where a local array would be demoted
// to memory.
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v8u __attribute__((ext_vector_type(8)));
typedef uint32_t v16u __attribute__((ext_vector_type(16)));
template <uint32_t N> struct VecOf;
template <> struct VecOf<2> { typedef v2u T; };
template <> struct VecOf<4> { typedef v4u T; };
template <> struct VecOf<16> { typedef v16u T; };
typedef VecOf<kLLRegs>::T LLTab;
typedef VecOf<kDRegs>::T DTab;
typedef VecOf<kCLRegs>::T CLTab;

// LUT entry: [0:4) code length, [4:7) kind, [7:11) extra bits, [11:27) value;
// literal/length literals also set bit 31 (one sign test in literal_run)
constexpr uint32_t kLitFlag = 0x80000000u;
enum : uint32_t { K_BAD = 0, K_LIT = 1, K_BASE = 2, K_EOB = 3, K_LONG = 4 };
enum : uint32_t { A_LITLEN = 0, A_DIST = 1, A_CLEN = 2 };

__device__ __forceinline__ uint32_t mk(uint32_t len, uint32_t kind, uint32_t extra, uint32_t val) {
  return len | (kind << 4) | (extra << 7) | (val << 11);
}
__device__ __forceinline__ uint32_t e_len(uint32_t e) { return e & 15u; }
__device__ __forceinline__ uint32_t e_kind(uint32_t e) { return (e >> 4) & 7u; }
__device__ __forceinline__ uint32_t e_extra(uint32_t e) { return (e >> 7) & 15u; }
__device__ __forceinline__ uint32_t e_val(uint32_t e) { return e >> 11; }

__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) { return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v); }
// The lane id through a volatile move: values derived from it (lane + 64 r,
// their bit reversals) are then recomputed where they are used instead of
// being hoisted to the kernel entry and kept live across the symbol loop
// (at four waves per SIMD they were 32 spilled VGPRs, reloaded in the copy
// loops).
__device__ __forceinline__ uint32_t lane_id() {
  uint32_t l;
  asm volatile("v_mov_b32 %0, %1" : "=v"(l) : "v"(threadIdx.x));
  return l;
}
__device__ __forceinline__ uint32_t lane_get(uint32_t v, uint32_t lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);
}

// RFC 1951 3.2.5 in closed form: length code k = sym - 257 (k < 28) has
// base 3 + k and no extra bits below 8, else e = (k - 4) / 4 extra bits and
// base ((4 + k % 4) << e) + 3; code 285 is 258.  Distance code d has base
// d + 1 below 4, else e = d / 2 - 1 extra bits and base ((2 + d % 2) << e) + 1.
__device__ __forceinline__ uint32_t symbol_entry(uint32_t alphabet, uint32_t sym, uint32_t len) {
  if (alphabet == A_LITLEN) {
    if (sym < 256) return mk(len, K_LIT, 0, sym) | kLitFlag;  // bit 31: literal (asm sign test)
    if (sym == 256) return mk(len, K_EOB, 0, 0);
    if (sym < 285) {
      const uint32_t k = sym - 257;
      if (k < 8) return mk(len, K_BASE, 0, 3 + k);
      const uint32_t e = (k - 4) >> 2;
      return mk(len, K_BASE, e, ((4u + (k & 3u)) << e) + 3u);
    }
    if (sym == 285) return mk(len, K_BASE, 0, 258);
    return mk(len, K_BAD, 0, 0);  // 286, 287
  }
  if (alphabet == A_DIST) {
    if (sym < 4) return mk(len, K_BASE, 0, sym + 1);
    if (sym < 30) {
      const uint32_t e = (sym >> 1) - 1;
      return mk(len, K_BASE, e, ((2u + (sym & 1u)) << e) + 1u);
    }
    return mk(len, K_BAD, 0, 0);  // 30, 31
  }
  return mk(len, K_LIT, 0, sym);
}

__constant__ uint8_t kClenOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// per-length canonical parameters, for codes longer than the LUT root
struct CodeMeta {
  uint16_t first[16], cnt[16], offs[16];
};

// Lanes that have nothing to write store into `ring[kWin + 4 * lane]` (the
// dummy tail) instead of branching around the store: the hot loop then has
// no divergent branch, so the compiler keeps it unstructurized -- plain
// s_cbranch_scc on SGPR state (with a divergent `if` anywhere inside, the
// whole loop is rewritten into predicate-flag flow: ~90 instructions per
// literal instead of ~30).
constexpr uint32_t kDummy = kWin;
struct Lds {
  elem_t ring[kWin + 256];  // first: the asm takes its LDS address as a constant
  uint16_t llsym[288], ddsym[32], clsym[20];
  CodeMeta llm, ddm;
  uint8_t lens[320];  // litlen lengths [0, nlen), distance lengths [nlen, nlen + ndist)
  uint8_t cllens[20];
#if ZI_SPEC
  // landing targets of a part (zcrc_inflate_split.hip): bit positions of the
  // later parts of its chunk, ascending, and their item indices
  uint64_t tpos[kMaxParts];
  uint32_t titem[kMaxParts];
#endif
};

// Build the canonical code for lens[0..n) (RFC 1951 3.2.2): the VGPR LUT
// (entry idx in lane idx & 63 of lut[idx >> 6]), the canonical symbol order
// sym[], and, when some code is longer than ROOT, the per-length meta in
// LDS.  Returns false where zlib's inflate_table() rejects the set:
// over-subscribed, or incomplete unless (not CLEN and a single length-1
// code); an all-zero set is accepted (decoding from it fails).
//
// Per-length quantities live in lane L (count, offset, first code), so the
// build needs few SGPRs: one uniform pass per length ranks the symbols of
// that length by ballot, lane scans give offsets and first codes, and the
// LUT pass walks the lengths with v_readlane.
template <uint32_t ROOT, uint32_t NREG>
__device__ bool build_code(const uint8_t *lens, uint32_t n, uint16_t *sym, CodeMeta *meta, uint32_t alphabet,
                           typename VecOf<NREG>::T &lut) {
  const uint32_t lane = lane_id();
  const uint32_t nch = (n + 63) >> 6;  // <= 5
  const uint64_t lt = (1ull << lane) - 1ull;
  uint32_t lv[5], rk[5];
#pragma unroll
  for (uint32_t c = 0; c < 5; c++) {
    const uint32_t s = c * 64 + lane;
    lv[c] = (c < nch && s < n) ? lens[s] : 0u;
    rk[c] = 0;
  }
  // count and rank (by symbol) the codes of each length
  uint32_t cntv = 0;
  for (uint32_t L = 1; L < 16; L++) {
    uint32_t run = 0;
#pragma unroll
    for (uint32_t c = 0; c < 5; c++) {
      if (c < nch) {
        const uint64_t m = __ballot(lv[c] == L);
        if (lv[c] == L) rk[c] = run + (uint32_t)__builtin_popcountll(m & lt);
        run += (uint32_t)__builtin_popcountll(m);
      }
    }
    if (lane == L) cntv = run;
  }
  // lane scans over lengths 1..15: offs = sum of counts below, and the
  // Kraft partial sums in units of 2^-15 give the first codes
  const uint32_t kr = (lane >= 1 && lane < 16) ? cntv << (15 - lane) : 0u;
  uint32_t offs_inc = cntv, kr_inc = kr;
#pragma unroll
  for (uint32_t k = 1; k < 16; k <<= 1) {
    const uint32_t a = __shfl_up(offs_inc, k, 64), b = __shfl_up(kr_inc, k, 64);
    if (lane >= k) {
      offs_inc += a;
      kr_inc += b;
    }
  }
  const uint32_t offsv = offs_inc - cntv;
  const uint32_t firstv = (lane < 16) ? (kr_inc - kr) >> (15 - lane) : 0u;
  const uint32_t kraft = lane_get(kr_inc, 15);  // 2^15 = complete
  const uint64_t used = __ballot(cntv != 0 && lane < 16);
  const uint32_t max_len = used ? 63u - (uint32_t)__builtin_clzll(used) : 0u;
  if (kraft > 32768u) return false;  // over-subscribed
  if (max_len && kraft < 32768u && (alphabet == A_CLEN || max_len != 1)) return false;
  if (max_len > ROOT && lane < 16) {
    meta->first[lane] = (uint16_t)firstv;
    meta->cnt[lane] = (uint16_t)cntv;
    meta->offs[lane] = (uint16_t)offsv;
  }
#pragma unroll
  for (uint32_t c = 0; c < 5; c++) {
    if (c < nch) {
      const uint32_t o = (uint32_t)__shfl(offsv, lv[c] & 15u, 64);
      if (lv[c]) sym[o + rk[c]] = (uint16_t)(c * 64 + lane);
    }
  }
  __syncthreads();
  // LUT: lane decodes its own indices canonically
  uint32_t hitL[NREG], hidx[NREG];
#pragma unroll
  for (uint32_t r = 0; r < NREG; r++) hitL[r] = hidx[r] = 0;
  const uint32_t top = max_len < ROOT ? max_len : ROOT;
  for (uint32_t L = 1; L <= top; L++) {
    const uint32_t cL = lane_get(cntv, L);
    if (!cL) continue;
    const uint32_t fL = lane_get(firstv, L), oL = lane_get(offsv, L);
#pragma unroll
    for (uint32_t r = 0; r < NREG; r++) {
      const uint32_t d = (__builtin_bitreverse32(lane + 64u * r) >> (32 - L)) - fL;
      if (d < cL) {
        hitL[r] = L;
        hidx[r] = oL + d;
      }
    }
  }
  const uint32_t miss = (max_len > ROOT) ? mk(0, K_LONG, 0, 0) : mk(0, K_BAD, 0, 0);
#pragma unroll
  for (uint32_t r = 0; r < NREG; r++) lut[r] = hitL[r] ? symbol_entry(alphabet, sym[hidx[r]], hitL[r]) : miss;
  __syncthreads();
  return true;
}

// code longer than the LUT root (rare): canonical decode of the low 15 bits
__device__ __noinline__ uint32_t decode_slow(uint32_t bits15, const CodeMeta *m, const uint16_t *sym, uint32_t root,
                                             uint32_t alphabet) {
  const uint32_t rev = __builtin_bitreverse32(bits15) >> 17;
  for (uint32_t L = root + 1; L <= 15; L++) {
    const uint32_t d = (rev >> (15 - L)) - uni(m->first[L]);
    if (d < uni(m->cnt[L])) return uni(symbol_entry(alphabet, uni(sym[uni(m->offs[L]) + d]), L));
  }
  return mk(0, K_BAD, 0, 0);
}

// Wave-uniform bit reader.  Input is staged in VGPRs as a 4-slot ring of
// 1 KiB blocks (block b in registers 4(b & 3) .. 4(b & 3) + 3; lane l holds
// the 16 B at b * 1024 + 16 l), so dword g is register ((g >> 6) & 12) |
// (g & 3) of lane (g >> 2) & 63: one s_set_gpr_idx move and a v_readlane.
// Blocks kA and kA + 1 are resident, kA + 2 is in flight in `pend` and lands
// in its slot at the next slide, by which time its load has returned.
//
// Refills add 32 bits at a time while at most 32 are buffered.  P advances
// in steps of 4, so P & 3 is fixed between seeks: the dword holding byte P
// is cached in q, and a refill fetches one new dword (g + 1) and funnels
// the pair.  Refills never slide: callers slide first (slide_if_needed),
// which keeps a single site that rewrites the staging registers.
struct Reader {
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t lead;   // src - (src & ~15)
  uint32_t end;    // lead + src_len: bytes at or past it read as zero
  uint32_t limit;  // overrun guard
  v16u st;
  uint4 pend;
  uint32_t kA;
  uint32_t P;    // next byte (relative to the aligned base) to enter bb
  uint32_t q;    // dword P >> 2
  uint32_t sh8;  // 8 * (P & 3)
  uint64_t bb;   // bit buffer, LSB first
  uint32_t nb;   // valid bits in bb

  __device__ uint4 load_block(uint32_t k) const {
    auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, k * 1024u + 16u * threadIdx.x, 0, 0);
    return make_uint4(v[0], v[1], v[2], v[3]);
  }
  __device__ void put_slot(uint32_t slot, uint4 v) {
    switch (slot & 3u) {
      case 0: st.s0 = v.x; st.s1 = v.y; st.s2 = v.z; st.s3 = v.w; break;
      case 1: st.s4 = v.x; st.s5 = v.y; st.s6 = v.z; st.s7 = v.w; break;
      case 2: st.s8 = v.x; st.s9 = v.y; st.sa = v.z; st.sb = v.w; break;
      default: st.sc = v.x; st.sd = v.y; st.se = v.z; st.sf = v.w; break;
    }
  }
  __device__ uint32_t dword_at(uint32_t g) const { return lane_get(st[((g >> 6) & 12u) | (g & 3u)], (g >> 2) & 63u); }
  __device__ void seek(uint32_t p) {
    P = p;
    bb = 0;
    nb = 0;
    kA = p >> 10;
    put_slot(kA, load_block(kA));
    put_slot(kA + 1, load_block(kA + 1));
    pend = load_block(kA + 2);
    q = dword_at(p >> 2);
    sh8 = 8u * (p & 3u);
  }
  // once P has entered block kA + 1: land kA + 2, prefetch kA + 3
  __device__ void slide_if_needed() {
    if ((P >> 10) != kA) {
      put_slot(kA + 2, pend);
      kA++;
      pend = load_block(kA + 2);
    }
  }
  // +32 bits (caller: nb <= 32, slid within the last ~1 KiB); bytes at or
  // past `end` read as zero; false once the input is overrun
  __device__ bool refill() {
    const uint32_t r = dword_at((P >> 2) + 1);
    uint32_t w = (uint32_t)((((uint64_t)r << 32) | q) >> sh8);
    if (P + 4u > end) w &= P >= end ? 0u : (1u << (8u * (end - P))) - 1u;
    bb |= (uint64_t)w << nb;
    nb += 32;
    P += 4;
    q = r;
    return P <= limit;
  }
  // slow paths: slide if due, refill if at most 32 bits are buffered
  __device__ bool ensure() {
    slide_if_needed();
    return nb > 32 || refill();
  }
  __device__ uint32_t peek(uint32_t k) const { return (uint32_t)bb & ((1u << k) - 1u); }
  __device__ void drop(uint32_t k) {
    bb >>= k;
    nb -= k;
  }
  __device__ uint32_t bits(uint32_t k) {  // k <= 16
    ensure();
    const uint32_t v = peek(k);
    drop(k);
    return v;
  }
  // input bytes consumed (through the last bit used)
  __device__ uint64_t consumed() const { return (uint64_t)P - lead - nb / 8u; }
};

// A symbol the code cannot accept.  The canonical decoder (the oracle)
// reads the whole code first -- its length, or all 15 bits when no code
// matches -- so those bits count as consumed: past the end of the input the
// kernel's epilogue then reports ZCRC_INFLATE_ERR_INPUT, as the oracle does.
__device__ __forceinline__ int32_t bad_symbol(Reader &r, uint32_t e, int32_t err) {
  r.drop(e_len(e) ? e_len(e) : 15u);
  return err;
}

// Output: elements [fl, pos) are decoded but still only in the ring.  `room`
// counts the literals/match elements that may be added before something must
// happen: min(cap - pos, kFlushLag - (pos - fl)).  (Elements are bytes, or
// 16-bit values under ZI_SPEC.)
struct Out {
  elem_t *dst;
  uint64_t cap;
  uint64_t pos;  // elements produced
  uint64_t fl;   // elements flushed to dst (a multiple of kFlushStep until the end)
  uint32_t room;
  bool al16;     // dst 16-byte aligned
#if ZI_SPEC
  uint32_t reach;  // furthest back-reference before the chunk's first element
  bool spec;       // the history is unknown (every chunk but the first)
  uint64_t tpos;   // the next landing target (bit position), kSplitNone: none
  uint32_t ti, tn; // its index in Lds::tpos, and the count
  uint32_t landed; // the item landed on (codes() returned kSpecLanded)
#endif
  __device__ void set_room() {
    const uint64_t c = cap - pos;
    const uint32_t f = kFlushLag - (uint32_t)(pos - fl);
    room = c < f ? (uint32_t)c : f;
  }
};

// one element through a buffer resource (bytes, or 16-bit under ZI_SPEC),
// sc1: from L2, never a stale L1 line (reads of flushed output)
__device__ __forceinline__ uint32_t load_elem_sc1(__amdgpu_buffer_rsrc_t r, uint32_t idx) {
  if (kEsh) return __builtin_amdgcn_raw_buffer_load_b16(r, idx << kEsh, 0, 16);
  return __builtin_amdgcn_raw_buffer_load_b8(r, idx, 0, 16);
}
__device__ __forceinline__ void store_elem(uint32_t v, __amdgpu_buffer_rsrc_t r, uint32_t idx) {
  if (kEsh) __builtin_amdgcn_raw_buffer_store_b16((uint16_t)v, r, idx << kEsh, 0, 0);
  else __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, r, idx, 0, 0);
}

// ring [fl, upto) -> dst, 1 KiB per step: one 16-B LDS read and one 16-B
// store per lane when dst is 16-B aligned, else coalesced element steps.
// Stores go through a buffer resource sized to the bytes due, so the
// hardware drops the lanes past `upto` (no divergent branch).
constexpr uint32_t kFlushStep = 1024u >> kEsh;  // elements per 1 KiB step
__device__ __forceinline__ void flush_to(Lds &s, Out &o, uint64_t upto) {
  const uint32_t lane = lane_id();
  while (o.fl < upto) {
    const uint32_t roff = (uint32_t)(o.fl & kWinMask);
    const uint32_t m = (upto - o.fl < kFlushStep) ? (uint32_t)(upto - o.fl) : kFlushStep;
    const __amdgpu_buffer_rsrc_t d =
        __builtin_amdgcn_make_buffer_rsrc(o.dst + o.fl, (short)0, (int)(m << kEsh), 0x00020000);
    if (o.al16 && m == kFlushStep) {
      const uint4 v = *reinterpret_cast<const uint4 *>(&s.ring[roff + (16u >> kEsh) * lane]);
      typedef uint32_t v4w __attribute__((ext_vector_type(4)));
      v4w w;
      w.x = v.x;
      w.y = v.y;
      w.z = v.z;
      w.w = v.w;
      __builtin_amdgcn_raw_buffer_store_b128(w, d, 16u * lane, 0, 0);
    } else {
#pragma unroll
      for (uint32_t k = 0; k < (16u >> kEsh); k++) store_elem(s.ring[roff + 64u * k + lane], d, 64u * k + lane);
    }
    o.fl += m;
  }
  // far matches read flushed elements back with sc1 (L2) loads: let these
  // stores reach L2 first (once per kFlushLag batch)
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
}

// flush one kFlushLag batch when due (pending < kFlushLag + 1024 here, so
// one suffices), then recompute the room.  An `if`, not a `while`: a second
// loop level around flush_to's makes the structurizer treat the whole
// decode state as divergent (VGPRs and select chains instead of SGPRs).
__device__ __forceinline__ void settle(Lds &s, Out &o) {
  if ((uint32_t)(o.pos - o.fl) >= kFlushLag) flush_to(s, o, o.fl + kFlushLag);
  o.set_room();
}

// lane-parallel copy of `len` elements from `dist` back (dist <= pos checked);
// lanes past `len` write to the dummy tail.  Sources older than the ring
// (dist > kWin) are flushed already (pos - fl < kFlushLag + 1024 + 258 <
// kWin) and are read back from dst with sc1 loads, which bypass the CU's
// L1 (a line cached there may predate the flush of its other bytes).
__device__ __forceinline__ void copy_match(Lds &s, const Out &o, uint32_t p0, uint32_t len, uint32_t dist) {
  const uint32_t lane = lane_id();
  const uint32_t src = p0 - dist;
  if (dist > kWin) {
    const __amdgpu_buffer_rsrc_t far =
        __builtin_amdgcn_make_buffer_rsrc(o.dst + (o.pos - dist), (short)0, (int)(len << kEsh), 0x00020000);
    uint32_t v[5];  // len <= 258
#pragma unroll
    for (uint32_t k = 0; k < 5; k++) v[k] = (64u * k < len) ? load_elem_sc1(far, 64u * k + lane) : 0u;
#pragma unroll
    for (uint32_t k = 0; k < 5; k++) {
      const uint32_t i = 64u * k + lane;
      if (64u * k < len) s.ring[i < len ? (p0 + i) & kWinMask : kDummy + 4u * lane] = (elem_t)v[k];
    }
  } else if (dist >= 64u || len <= dist) {
    // every source element precedes the 64-element step that writes it
    for (uint32_t i0 = 0; i0 < len; i0 += 64) {
      const uint32_t i = i0 + lane;
      const elem_t v = s.ring[(src + i) & kWinMask];
      s.ring[i < len ? (p0 + i) & kWinMask : kDummy + 4u * lane] = v;
    }
  } else {
    // short period: element i repeats element i mod dist
    const float rcp = 1.0f / (float)dist;
    for (uint32_t i0 = 0; i0 < len; i0 += 64) {
      const uint32_t i = i0 + lane;
      uint32_t m = i - (uint32_t)((float)i * rcp) * dist;
      m = (int32_t)m < 0 ? m + dist : m;
      m = m >= dist ? m - dist : m;
      const elem_t v = s.ring[(src + m) & kWinMask];
      s.ring[i < len ? (p0 + i) & kWinMask : kDummy + 4u * lane] = v;
    }
  }
}

#if ZI_SPEC
// A back-reference reaching before the chunk's first element (dist > p0,
// dist <= p0 + 32 KiB): element i takes source p0 - dist + (i mod dist) --
// the same element the sequential copy would -- which is either a marker
// (source < 0: byte 32768 + source of the history) or an element produced
// earlier (in the ring, or flushed to dst when older than the ring).  Every
// source precedes the copy, so the 64-lane steps are independent.
__device__ __noinline__ void copy_spec(Lds &s, const Out &o, uint32_t p0, uint32_t len, uint32_t dist) {
  const uint32_t lane = lane_id();
  // Sources below p0 + len - kWin are read back from dst (sc1): they are
  // flushed (pos - fl < kFlushLag + 1024 + 258 < kWin - 258), and their ring
  // slots are the ones this copy's earlier 64-lane steps overwrite (a source
  // p0 + i' - kWin shares slot p0 + i' with element i' when kWin < dist <
  // kWin + len).  Sources at or above it sit in slots no step writes.
  const uint32_t nfar = p0 + len > kWin ? p0 + len - kWin : 0u;
  const __amdgpu_buffer_rsrc_t far = __builtin_amdgcn_make_buffer_rsrc(o.dst, (short)0, (int)(nfar << kEsh), 0x00020000);
  for (uint32_t i0 = 0; i0 < len; i0 += 64) {
    const uint32_t i = i0 + lane;
    const uint32_t m = i % dist;
    const int32_t sidx = (int32_t)p0 - (int32_t)dist + (int32_t)m;
    const uint32_t fv = load_elem_sc1(far, sidx < 0 ? 0x3FFFFFFFu : (uint32_t)sidx);  // out of range: 0
    const uint32_t nv = s.ring[(uint32_t)sidx & kWinMask];
    const uint32_t v = sidx < 0 ? kInflateMarker + (uint32_t)((int32_t)kInflateHist + sidx) : ((uint32_t)sidx < nfar ? fv : nv);
    s.ring[i < len ? (p0 + i) & kWinMask : kDummy + 4u * lane] = (elem_t)v;
  }
}
#endif

// Literal runs, the hot path of poorly compressible data (~93% of the
// symbols of the spectrum payloads), as one hand-scheduled loop, unrolled
// twice: ~20 instructions per literal, one taken branch per two, plus a
// ~24-instruction 32-bit refill every ~3.5 literals (compiled C++ spent ~90
// per literal on predicate flow).  The ring address of the next byte is
// computed while the LUT lookup is in flight; bit 31 of an entry marks a
// literal (one sign test); room is decremented and checked in one step.
// Keeps >= 33 bits buffered, refilling inline; decodes literals while room
// remains; lane 0 writes each byte into the ring, the other lanes into the
// dummy tail (address = pos * sel + dummy, sel = 1 on lane 0 only).
// Returns 0 when the caller must slide or refill first (P entered the next
// block, or the refill would read past `end`), 1 when the next symbol needs
// the general path (non-literal, or no room) -- then >= 33 bits are buffered.
// Fixed registers: bb in s[60:61] (its low word is the LUT index and the
// v_readlane lane select), {q, r} in s[62:63] (funnel-shifted by s_lshr_b64),
// the literal/length LUT in v[40:55] and the input ring in v[60:75], both
// read with s_set_gpr_idx (as the compiler does for a dynamic subscript).
// VGPR temporaries are fixed clobbers (v56..v58), not outputs: an asm with a
// VGPR output counts as a source of divergence and would demote the whole
// decode state to VGPRs.  No hazard needs a wait state: SALU results feed
// SALU, VALU and readlane lane selects; the only VALU->SALU edges are
// v_readlane results.
__device__ __forceinline__ uint32_t literal_run(Reader &r, uint32_t &p, uint32_t &room, const LLTab &ll,
                                                const DTab &dd, uint32_t vsel, uint32_t vdum, uint32_t vdm,
                                                uint32_t vlane, uint32_t ringl, uint32_t &mlen, uint32_t &mdist,
                                                uint32_t rcap = 0xFFFFFFFFu) {
  uint32_t why, t0, t1, t2, t3, t4, t5;
  uint64_t bb = r.bb;
  uint64_t qr = r.q;
  uint32_t nb = r.nb, P = r.P;
  // refills the asm may do on its own: each reads the 4 bytes at P (needs
  // P + 4 <= end) and dword P/4 + 1, resident while P stays in block kA
  const uint32_t kend = P + 4u <= r.end ? (r.end - P) >> 2 : 0u;
  const uint32_t kblk = ((r.kA + 1u) * 1024u - P + 3u) >> 2;
  uint32_t rb = kend < kblk ? kend : kblk;
  rb = uni(rb < rcap ? rb : rcap);  // ZI_SPEC landing targets: never refill past the next one
  asm volatile(
      "L_top_%=:\n\t"
      "s_cmp_le_u32 %[nb], 32\n\t"
      "s_cbranch_scc1 L_ref_%=\n\t"
      "L_have_%=:\n\t"
      "s_bfe_u32 %[t0], s60, 0x40006\n\t"
      "s_set_gpr_idx_on %[t0], gpr_idx(SRC0)\n\t"
      "v_mov_b32 v56, v40\n\t"
      "s_set_gpr_idx_off\n\t"
      "v_and_b32_e64 v58, %[p], %[vwm]\n\t"
      "v_mad_u32_u24 v58, v58, %[vsel], %[vdum]\n\t"
      "v_readlane_b32 %[t1], v56, s60\n\t"
      "s_cmp_gt_i32 %[t1], -1\n\t"
      "s_cbranch_scc1 L_gen_%=\n\t"
      "s_sub_u32 %[room], %[room], 1\n\t"
      "s_cbranch_scc1 L_full_%=\n\t"
      "s_and_b32 %[t0], %[t1], 15\n\t"
      "s_lshr_b64 s[60:61], s[60:61], %[t0]\n\t"
      "s_sub_u32 %[nb], %[nb], %[t0]\n\t"
      "v_lshrrev_b32_e64 v57, 11, %[t1]\n\t"
      ZI_DSW " v58, v57\n\t"
      "s_add_u32 %[p], %[p], 1\n\t"
      "s_cmp_le_u32 %[nb], 32\n\t"
      "s_cbranch_scc1 L_ref_%=\n\t"
      "s_bfe_u32 %[t0], s60, 0x40006\n\t"
      "s_set_gpr_idx_on %[t0], gpr_idx(SRC0)\n\t"
      "v_mov_b32 v56, v40\n\t"
      "s_set_gpr_idx_off\n\t"
      "v_and_b32_e64 v58, %[p], %[vwm]\n\t"
      "v_mad_u32_u24 v58, v58, %[vsel], %[vdum]\n\t"
      "v_readlane_b32 %[t1], v56, s60\n\t"
      "s_cmp_gt_i32 %[t1], -1\n\t"
      "s_cbranch_scc1 L_gen_%=\n\t"
      "s_sub_u32 %[room], %[room], 1\n\t"
      "s_cbranch_scc1 L_full_%=\n\t"
      "s_and_b32 %[t0], %[t1], 15\n\t"
      "s_lshr_b64 s[60:61], s[60:61], %[t0]\n\t"
      "s_sub_u32 %[nb], %[nb], %[t0]\n\t"
      "v_lshrrev_b32_e64 v57, 11, %[t1]\n\t"
      ZI_DSW " v58, v57\n\t"
      "s_add_u32 %[p], %[p], 1\n\t"
      "s_branch L_top_%=\n\t"
      // refill 32 bits: exit (0) if past the end or into the next block
      "L_ref_%=:\n\t"
      "s_sub_u32 %[rb], %[rb], 1\n\t"  // refills left before the end or the next block
      "s_cbranch_scc1 L_zero_%=\n\t"
      "s_lshr_b32 %[t1], %[P], 2\n\t"
      "s_add_u32 %[t1], %[t1], 1\n\t"  // dword g + 1
      "s_bfe_u32 %[t0], %[t1], 0x20008\n\t"  // its block's slot
      "s_and_b32 %[t2], %[t1], 3\n\t"
      "s_lshl2_add_u32 %[t0], %[t0], %[t2]\n\t"  // register 4 * slot + (g + 1) % 4
      "s_lshr_b32 %[t1], %[t1], 2\n\t"
      "s_set_gpr_idx_on %[t0], gpr_idx(SRC0)\n\t"
      "v_mov_b32 v56, v60\n\t"
      "s_set_gpr_idx_off\n\t"
      "v_readlane_b32 s63, v56, %[t1]\n\t"
      "s_lshr_b64 s[64:65], s[62:63], %[sh8]\n\t"
      "s_mov_b32 s65, 0\n\t"
      "s_lshl_b64 s[64:65], s[64:65], %[nb]\n\t"
      "s_or_b64 s[60:61], s[60:61], s[64:65]\n\t"
      "s_mov_b32 s62, s63\n\t"
      "s_add_u32 %[nb], %[nb], 32\n\t"
      "s_add_u32 %[P], %[P], 4\n\t"
      "s_branch L_have_%=\n\t"
      "L_full_%=:\n\t"
      "s_add_u32 %[room], %[room], 1\n\t"
      "L_one_%=:\n\t"
      "s_mov_b32 %[why], 1\n\t"
      "s_branch L_out_%=\n\t"
      // ---- length/distance pair (t1 = literal/length entry, not a literal).
      // Everything is checked before a bit is consumed, except the copy
      // conditions: a pair that decodes but needs the compiled path (far,
      // long, overlapping, no room, or an error) returns 2 with len/dist.
      "L_gen_%=:\n\t"
      "s_bfe_u32 %[t0], %[t1], 0x30004\n\t"
      "s_cmp_lg_u32 %[t0], 2\n\t"
      "s_cbranch_scc1 L_one_%=\n\t"  // EOB, long code, bad symbol
      "s_and_b32 %[t2], %[t1], 15\n\t"  // L
      "s_bfe_u32 %[t3], %[t1], 0x40007\n\t"  // x (length extra bits)
      "s_add_u32 %[t4], %[t2], %[t3]\n\t"
      "s_lshr_b64 s[64:65], s[60:61], %[t4]\n\t"
      "s_bfe_u32 %[t0], s64, 0x20006\n\t"
      "s_set_gpr_idx_on %[t0], gpr_idx(SRC0)\n\t"
      "v_mov_b32 v56, v76\n\t"
      "s_set_gpr_idx_off\n\t"
      "v_readlane_b32 %[t5], v56, s64\n\t"  // distance entry
      "s_bfe_u32 %[t0], %[t5], 0x30004\n\t"
      "s_cmp_lg_u32 %[t0], 2\n\t"
      "s_cbranch_scc1 L_one_%=\n\t"  // long or invalid distance code
      "s_and_b32 %[t0], %[t5], 15\n\t"
      "s_add_u32 %[t4], %[t4], %[t0]\n\t"  // L + x + dL
      "s_bfe_u32 %[t0], %[t5], 0x40007\n\t"  // dx
      "s_add_u32 %[t0], %[t4], %[t0]\n\t"  // c = L + x + dL + dx
      "s_cmp_gt_u32 %[t0], %[nb]\n\t"
      "s_cbranch_scc1 L_one_%=\n\t"  // not all buffered (nb 33..35)
      "s_lshl_b32 %[t3], %[t3], 16\n\t"
      "s_or_b32 %[t3], %[t3], %[t2]\n\t"
      "s_bfe_u32 %[t3], s60, %[t3]\n\t"  // length extra value
      "s_lshr_b32 %[t2], %[t1], 11\n\t"
      "s_add_u32 %[ml], %[t2], %[t3]\n\t"  // len
      "s_bfe_u32 %[t3], %[t5], 0x40007\n\t"
      "s_lshl_b32 %[t3], %[t3], 16\n\t"
      "s_or_b32 %[t3], %[t3], %[t4]\n\t"
      "s_bfe_u64 s[64:65], s[60:61], %[t3]\n\t"  // distance extra value
      "s_lshr_b32 %[t2], %[t5], 11\n\t"
      "s_add_u32 %[md], %[t2], s64\n\t"  // dist
      "s_lshr_b64 s[60:61], s[60:61], %[t0]\n\t"
      "s_sub_u32 %[nb], %[nb], %[t0]\n\t"
      "s_mov_b32 %[why], 2\n\t"
      "s_cmp_gt_u32 %[md], %[p]\n\t"  // too far back (or pos >= 2^32): compiled path
      "s_cbranch_scc1 L_out_%=\n\t"
      "s_cmp_gt_u32 %[md], %[win]\n\t"  // older than the ring
      "s_cbranch_scc1 L_out_%=\n\t"
      "s_cmp_gt_u32 %[ml], 64\n\t"
      "s_cbranch_scc1 L_out_%=\n\t"
      "s_cmp_gt_u32 %[ml], %[room]\n\t"
      "s_cbranch_scc1 L_out_%=\n\t"
      "s_cmp_lt_u32 %[md], %[ml]\n\t"  // overlapping copy
      "s_cbranch_scc1 L_out_%=\n\t"
      // one 64-lane step: ring[p + i] = ring[p - dist + i], i < len
      "s_sub_u32 %[t2], %[p], %[md]\n\t"
      "v_add_u32 v59, %[t2], %[vl]\n\t"
      "v_and_b32 v59, %[wm], v59\n\t"
      "v_lshl_add_u32 v59, v59, " ZI_ESH ", %[rl]\n\t"
      ZI_DSR " v57, v59\n\t"
      "v_add_u32 v58, %[p], %[vl]\n\t"
      "v_and_b32 v58, %[wm], v58\n\t"
      "v_lshl_add_u32 v58, v58, " ZI_ESH ", %[rl]\n\t"
      "v_cmp_gt_u32 vcc, %[ml], %[vl]\n\t"
      "s_nop 1\n\t"
      "v_cndmask_b32 v58, %[vdm], v58, vcc\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      ZI_DSW " v58, v57\n\t"
      "s_add_u32 %[p], %[p], %[ml]\n\t"
      "s_sub_u32 %[room], %[room], %[ml]\n\t"
      "s_branch L_top_%=\n\t"
      "L_zero_%=:\n\t"
      "s_mov_b32 %[why], 0\n\t"
      "L_out_%=:"
      : [nb] "+s"(nb), [room] "+s"(room), [p] "+s"(p), [P] "+s"(P), [rb] "+s"(rb), [why] "=&s"(why), [t0] "=&s"(t0),
        [t1] "=&s"(t1), [t2] "=&s"(t2), [t3] "=&s"(t3), [t4] "=&s"(t4), [t5] "=&s"(t5), [ml] "=&s"(mlen),
        [md] "=&s"(mdist), "+{s[60:61]}"(bb), "+{s[62:63]}"(qr)
      : [vdum] "v"(vdum), [vsel] "v"(vsel), [vdm] "v"(vdm), [vl] "v"(vlane), [vwm] "v"(kWinMask), [rl] "s"(ringl),
        [sh8] "s"(r.sh8), [wm] "i"(kWinMask), [win] "i"(kWin), "{v[40:55]}"(ll),
        "{v[60:75]}"(r.st), "{v[76:79]}"(dd)
      : "memory", "scc", "vcc", "v56", "v57", "v58", "v59", "s64", "s65");
  r.bb = bb;
  r.q = (uint32_t)qr;
  r.nb = nb;
  r.P = P;
  return why;
}

// One Huffman-coded block with the tables in ll / dd.  A single loop with
// one exit: literal runs go through literal_run(), everything else through
// the general path below.
__device__ int32_t codes(Lds &s, Reader &r, Out &o, const LLTab &ll, const DTab &dd) {
  const uint32_t lane = threadIdx.x;
  const uint32_t ring_lds = (uint32_t)reinterpret_cast<uintptr_t>(
      (__attribute__((address_space(3))) uint8_t *)(&s.ring[0]));
  const uint32_t vsel = lane == 0 ? (1u << kEsh) : 0u;
  const uint32_t vdum = ring_lds + (lane == 0 ? 0u : (kDummy + 4u * lane) << kEsh);
  const uint32_t vdm = ring_lds + ((kDummy + 4u * lane) << kEsh);
  int32_t st = ZCRC_INFLATE_OK;
  for (;;) {
    uint32_t len, dist;
    r.slide_if_needed();  // the only slide site of the symbol loop
    if (r.nb <= 32 && !r.refill()) {
      st = ZCRC_INFLATE_ERR_INPUT;
      break;
    }
    uint32_t rcap = 0xFFFFFFFFu;
#if ZI_SPEC
    // landing: at a token boundary equal to the next target the part stops
    // (the later part's decode starts there); a target already passed was
    // not a token boundary (its probe had not synchronised) and is skipped.
    // Within 96 bits of a target the tokens are taken one at a time by the
    // compiled path; before that the asm may refill only up to the target's
    // byte, so it cannot run past it.  (`if`s, not loops: see settle().)
    bool near = false;
    if (o.tpos != kSplitNone) {
      const uint64_t bit = ((uint64_t)(r.P - r.lead) << 3) - r.nb;
      if (o.tpos < bit) {
        o.ti++;
        o.tpos = o.ti < o.tn ? ((uint64_t)uni((uint32_t)(s.tpos[o.ti] >> 32)) << 32) | uni((uint32_t)s.tpos[o.ti])
                             : kSplitNone;
      }
      if (o.tpos == bit) {
        o.landed = uni(s.titem[o.ti]);
        st = kSpecLanded;
        break;
      }
      if (o.tpos != kSplitNone && o.tpos > bit) {
        near = o.tpos - bit < 96u;
        const uint64_t tb = (uint64_t)r.lead + (o.tpos >> 3);  // the target's byte, aligned-base relative
        rcap = tb > r.P ? (uint32_t)((tb - r.P) >> 2) : 0u;
      } else {
        rcap = 0;  // passed targets still ahead in the list: advance first
      }
    }
    if (!near)
#endif
#ifndef ZI_NO_ASM
    {
      // (readfirstlane: the compiler cannot always prove this state
      // uniform, and the asm needs it in SGPRs)
      uint32_t p = uni((uint32_t)o.pos);
      const uint32_t p0 = p;
      r.bb = ((uint64_t)uni((uint32_t)(r.bb >> 32)) << 32) | uni((uint32_t)r.bb);
      r.nb = uni(r.nb);
      r.P = uni(r.P);
      r.q = uni(r.q);
      uint32_t room = uni(o.room), ml = 0, md = 0;
      const uint32_t why = literal_run(r, p, room, ll, dd, vsel, vdum, vdm, lane, ring_lds, ml, md, uni(rcap));
      o.room = room;
      o.pos += p - p0;
      if (!why) continue;
      if (why == 2) {  // a pair decoded in asm: checks and copy below
        len = ml;
        dist = md;
        goto have_pair;
      }
    }
#endif
    {
    const uint32_t ix = (uint32_t)r.bb & ((1u << kLLRoot) - 1u);
    uint32_t e = lane_get(ll[ix >> 6], ix);
    ITRACE("[%u] sym P=%u nb=%u e=%x kind=%u len=%u val=%u pos=%llu\n", blockIdx.x, r.P, r.nb, e, e_kind(e),
           e_len(e), e_val(e), (unsigned long long)o.pos);
    if (__builtin_expect(e_kind(e) == K_LONG, 0)) e = uni(decode_slow(r.peek(15), &s.llm, s.llsym, kLLRoot, A_LITLEN));
    const uint32_t kind = e_kind(e);
    if (kind == K_LIT) {
      r.drop(e_len(e));
      if (__builtin_expect(o.room == 0, 0)) {
        if (o.pos >= o.cap) {
          st = ZCRC_INFLATE_ERR_OUTPUT;
          break;
        }
        settle(s, o);
      }
#ifndef ZI_ABL_NOLIT
      s.ring[lane == 0 ? (uint32_t)o.pos & kWinMask : kDummy + 4u * lane] = (elem_t)e_val(e);
#endif
      o.pos++;
      o.room--;
      continue;
    }
    if (kind == K_EOB) {
      r.drop(e_len(e));
      break;
    }
    if (kind != K_BASE || e_len(e) == 0) {
      st = bad_symbol(r, e, ZCRC_INFLATE_ERR_SYMBOL);
      break;
    }
    r.drop(e_len(e));
    len = e_val(e) + r.peek(e_extra(e));
    r.drop(e_extra(e));
    if (r.nb <= 32 && !r.refill()) {  // <= 8 bytes past the slide check: still resident
      st = ZCRC_INFLATE_ERR_INPUT;
      break;
    }
    const uint32_t jx = (uint32_t)r.bb & ((1u << kDRoot) - 1u);
    uint32_t d = lane_get(dd[jx >> 6], jx);
    if (__builtin_expect(e_kind(d) == K_LONG, 0)) d = uni(decode_slow(r.peek(15), &s.ddm, s.ddsym, kDRoot, A_DIST));
    if (e_kind(d) != K_BASE || e_len(d) == 0) {
      st = bad_symbol(r, d, ZCRC_INFLATE_ERR_SYMBOL);
      break;
    }
    r.drop(e_len(d));
    dist = e_val(d) + r.peek(e_extra(d));
    r.drop(e_extra(d));
    }
  have_pair:
#if ZI_SPEC
    if (dist > o.pos && (!o.spec || dist > o.pos + kInflateHist)) {
#else
    if (dist > o.pos) {
#endif
      st = ZCRC_INFLATE_ERR_DIST;
      break;
    }
    if (__builtin_expect(len > o.room, 0) && len > o.cap - o.pos) {
      st = ZCRC_INFLATE_ERR_OUTPUT;
      break;
    }
#if ZI_SPEC
    if (dist > o.pos) {  // into the unknown history: markers
      const uint32_t back = dist - (uint32_t)o.pos;
      o.reach = back > o.reach ? back : o.reach;
      copy_spec(s, o, (uint32_t)o.pos, len, dist);
    } else {
      copy_match(s, o, (uint32_t)o.pos, len, dist);
    }
#elif !defined(ZI_ABL_NOCOPY)
    copy_match(s, o, (uint32_t)o.pos, len, dist);
#endif
    o.pos += len;
    if (__builtin_expect(len >= o.room, 0)) settle(s, o);  // may overshoot the lag by < 258
    else o.room -= len;
  }
  return st;
}

__device__ int32_t stored(Lds &s, Reader &r, Out &o) {
  const uint32_t lane = lane_id();
  r.drop(r.nb & 7u);  // byte boundary
  const uint32_t len = r.bits(16);
  const uint32_t nlen = r.bits(16);
  if (len != (~nlen & 0xFFFFu)) return ZCRC_INFLATE_ERR_STORED_LEN;
  const uint32_t q = r.P - r.nb / 8u;  // next unconsumed byte (aligned-base relative)
  if ((uint64_t)q - r.lead + len > (uint64_t)(r.end - r.lead)) return ZCRC_INFLATE_ERR_INPUT;
  if (len > o.cap - o.pos) return ZCRC_INFLATE_ERR_OUTPUT;
  // 1 KiB per step: 16 coalesced byte loads per lane, then 16 ring writes
  for (uint32_t i0 = 0; i0 < len; i0 += 1024) {
    uint32_t v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t j = i0 + 64u * k + lane;
      v[k] = __builtin_amdgcn_raw_buffer_load_b8(r.rsrc, q + j, 0, 0);  // lanes past len: discarded below
    }
    const uint32_t p0 = (uint32_t)o.pos;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t j = 64u * k + lane;
      s.ring[i0 + j < len ? (p0 + j) & kWinMask : kDummy + 4u * lane] = (elem_t)v[k];
    }
    o.pos += (len - i0 < 1024u) ? len - i0 : 1024u;
    settle(s, o);
  }
  r.seek(q + len);
  return ZCRC_INFLATE_OK;
}

__device__ int32_t dynamic_tables(Lds &s, Reader &r, LLTab &ll, DTab &dd) {
  const uint32_t lane = lane_id();
  const uint32_t nlen = r.bits(5) + 257, ndist = r.bits(5) + 1, ncode = r.bits(4) + 4;
  if (nlen > 286 || ndist > 30) return ZCRC_INFLATE_ERR_CODES;
  // code-length code lengths: 3 bits each, in kClenOrder order; lane k takes
  // field k from a 30-bit then a 27-bit window
  {
    const uint32_t n1 = ncode < 10 ? ncode : 10;
    r.ensure();
    const uint32_t w1 = r.peek(30);
    r.drop(3 * n1);
    uint32_t w2 = 0;
    if (ncode > 10) {
      r.ensure();
      w2 = r.peek(27);
      r.drop(3 * (ncode - 10));
    }
    if (lane < 19) {
      const uint32_t v = lane < 10 ? (w1 >> (3 * lane)) & 7u : (w2 >> (3 * (lane - 10))) & 7u;
      s.cllens[kClenOrder[lane]] = (uint8_t)(lane < ncode ? v : 0u);
    }
    __syncthreads();
  }
  CLTab cl;
  if (!build_code<kCLRoot, kCLRegs>(s.cllens, 19, s.clsym, nullptr, A_CLEN, cl)) return ZCRC_INFLATE_ERR_CODES;
  uint32_t idx = 0, prev = 0;
  const uint32_t total = nlen + ndist;
  while (idx < total) {
    if (!r.ensure()) return ZCRC_INFLATE_ERR_INPUT;
    const uint32_t ix = r.peek(kCLRoot);
    const uint32_t e = lane_get(cl[ix >> 6], ix & 63u);
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
      rep = 3 + r.peek(2);
      r.drop(2);
    } else if (sym == 17) {
      val = 0;
      rep = 3 + r.peek(3);
      r.drop(3);
      prev = 0;
    } else {
      val = 0;
      rep = 11 + r.peek(7);
      r.drop(7);
      prev = 0;
    }
    if (idx + rep > total) return ZCRC_INFLATE_ERR_CODES;
    for (uint32_t k = lane; k < rep; k += 64) s.lens[idx + k] = (uint8_t)val;
    idx += rep;
  }
  __syncthreads();
  if (s.lens[256] == 0) return ZCRC_INFLATE_ERR_CODES;
  if (!build_code<kLLRoot, kLLRegs>(s.lens, nlen, s.llsym, &s.llm, A_LITLEN, ll)) return ZCRC_INFLATE_ERR_CODES;
  if (!build_code<kDRoot, kDRegs>(s.lens + nlen, ndist, s.ddsym, &s.ddm, A_DIST, dd)) return ZCRC_INFLATE_ERR_CODES;
  return ZCRC_INFLATE_OK;
}

__device__ void fixed_tables(Lds &s, LLTab &ll, DTab &dd) {
  const uint32_t lane = lane_id();
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
  build_code<kLLRoot, kLLRegs>(s.lens, 288, s.llsym, &s.llm, A_LITLEN, ll);
  build_code<kDRoot, kDRegs>(s.lens + 288, 32, s.ddsym, &s.ddm, A_DIST, dd);
}

// ZI_WPE: waves per SIMD the register allocation must allow (LDS decides
// how many streams actually share a CU)
#ifndef ZI_WPE
#define ZI_WPE 1
#define ZI_WPE_DEFAULTED
#endif
#if !ZI_SPEC
__global__ __launch_bounds__(64, ZI_WPE) void inflate_kernel(InflateArgs a) {
  __shared__ __attribute__((aligned(16))) Lds s;
  if (blockIdx.x >= a.n) return;
  const uint64_t i = a.order ? a.order[blockIdx.x] : blockIdx.x;
  if (a.run_if && a.run_if[i] == 0) return;  // the block-parallel decode succeeded (zcrc_inflate_split.hip)
  const uint8_t *src = a.src[i];
  const uint64_t src_len = a.src_len[i];
  Out o;
  o.dst = a.dst[i];
  o.cap = a.cap[i];
  o.pos = 0;
  o.fl = 0;
  o.al16 = (reinterpret_cast<uint64_t>(o.dst) & 15u) == 0;
  o.set_room();
  int32_t st = ZCRC_INFLATE_OK;
  Reader r;
  if (src_len == 0 || src_len > kInflateMaxSrc) {
    st = src_len == 0 ? ZCRC_INFLATE_ERR_INPUT : ZCRC_INFLATE_ERR_TOO_BIG;
  } else {
    const uint64_t base = reinterpret_cast<uint64_t>(src) & ~(uint64_t)15;
    r.lead = (uint32_t)(reinterpret_cast<uint64_t>(src) - base);
    r.end = r.lead + (uint32_t)src_len;
    r.limit = r.end + 16u;
    // The buffer unit range-checks whole dwords (a dword that straddles
    // num_records reads as 0), so the range is rounded up to the 16-byte
    // granule holding the last byte -- same page, never a fault -- and the
    // bytes past `end` are masked in refill().
    r.rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(base), (short)0, (int)((r.end + 15u) & ~15u),
                                               0x00020000);
    r.seek(r.lead);
    LLTab ll;
    DTab dd;
    uint32_t last = 0;
    do {
      if (!r.ensure()) {
        st = ZCRC_INFLATE_ERR_INPUT;
        break;
      }
      last = r.peek(1);
      const uint32_t type = (uint32_t)(r.bb >> 1) & 3u;
      r.drop(3);
      ITRACE("[%u] block last=%u type=%u P=%u nb=%u pos=%llu\n", blockIdx.x, last, type, r.P, r.nb,
             (unsigned long long)o.pos);
      if (type == 0) {
        st = stored(s, r, o);
      } else if (type == 1) {
        fixed_tables(s, ll, dd);
        st = codes(s, r, o, ll, dd);
      } else if (type == 2) {
        st = dynamic_tables(s, r, ll, dd);
        if (st == ZCRC_INFLATE_OK) st = codes(s, r, o, ll, dd);
      } else {
        st = ZCRC_INFLATE_ERR_BLOCK_TYPE;
      }
      st = (int32_t)uni((uint32_t)st);
    } while (!last && st == ZCRC_INFLATE_OK);
    // Bits past the end read as zero.  Whenever the decode used any of them
    // -- whether it then ended cleanly or failed on what they said -- the
    // canonical decoder would have stopped at the first one: input error.
    if (r.consumed() > src_len) st = ZCRC_INFLATE_ERR_INPUT;
  }
  if (st == ZCRC_INFLATE_OK) flush_to(s, o, o.pos);
  if (threadIdx.x == 0) {
    a.out_len[i] = st == ZCRC_INFLATE_OK ? o.pos : 0;
    a.status[i] = st;
  }
}
#else
// The next chunk after k with a candidate (kn = nchunks: none) and its
// candidate (cn = 8 src_len then).
__device__ __forceinline__ void next_candidate(const SpecArgs &a, uint64_t k, uint64_t &kn, uint64_t &cn) {
  kn = k + 1;
  while (kn < a.nchunks && a.cand[kn] == kSplitNone) kn++;
  cn = kn < a.nchunks ? a.cand[kn] : 8 * a.src_len;
}

// Item i's owner: the chunk k <= i / parts with a candidate, whose first
// block the item decodes part j = i - k parts of.  A chunk with a candidate
// borrows the items of the candidate-less chunks after it -- its block spans
// them -- for T = (kn - k) parts parts in all, at most a.max_parts.  false:
// the item has no work.  (Before borrowing, 3 in 4 items of a text stream
// idled: zlib's blocks span ~4 chunks of 8 KiB, profiles/r03/s32.)
__device__ __forceinline__ bool owner(const SpecArgs &a, uint64_t i, uint64_t &k, uint32_t &j, uint32_t &T,
                                      uint64_t &kn, uint64_t &cn) {
  k = i / a.parts;
  while (a.cand[k] == kSplitNone) {
    if (k == 0 || i - (k - 1) * a.parts >= a.max_parts) return false;
    k--;
  }
  j = (uint32_t)(i - k * a.parts);
  next_candidate(a, k, kn, cn);
  const uint64_t t = (kn - k) * a.parts;
  T = (uint32_t)(t < a.max_parts ? t : a.max_parts);
  return j < T;
}

// The usable parts of chunk k's T, one lane each: the probed starts that lie
// strictly after the previous usable one (or the candidate c) and before the
// next candidate -- a probed start is usable when it is above c and above
// every valid start of a lower part (a prefix max over the wave).  Lane t
// gets part t's start in b; the mask has bit t set for a usable part t.
__device__ __forceinline__ uint64_t usable_mask(const SpecArgs &a, uint64_t k, uint32_t T, uint64_t c, uint64_t cn,
                                                uint64_t &b) {
  const uint32_t t = threadIdx.x;
  b = (t > 0 && t < T) ? a.part[k * a.parts + t] : kSplitNone;
  const bool valid = b != kSplitNone && b < cn;
  uint64_t m = valid ? b : 0;  // inclusive prefix max
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint64_t o = __shfl_up(m, d, 64);
    if (t >= d && o > m) m = o;
  }
  uint64_t below = __shfl_up(m, 1, 64);
  if (t == 0) below = 0;
  return __ballot(valid && b > c && b > below);
}

// Reader positioned at bit `bit` of the stream
__device__ __forceinline__ bool reader_at(Reader &r, const SpecArgs &a, uint64_t bit) {
  r.seek(r.lead + (uint32_t)(bit >> 3));
  if (!r.ensure()) return false;
  r.drop((uint32_t)(bit & 7u));
  return true;
}

__device__ __forceinline__ void reader_init(Reader &r, const SpecArgs &a) {
  const uint64_t base = reinterpret_cast<uint64_t>(a.src) & ~(uint64_t)15;
  r.lead = (uint32_t)(reinterpret_cast<uint64_t>(a.src) - base);
  r.end = r.lead + (uint32_t)a.src_len;
  r.limit = r.end + 16u;
  r.rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(base), (short)0, (int)((r.end + 15u) & ~15u),
                                             0x00020000);
}

__device__ __forceinline__ uint64_t reader_bit(const Reader &r) { return ((uint64_t)(r.P - r.lead) << 3) - r.nb; }

// Probe for part j >= 1 of chunk k (tests/inflate_split_model.py probe):
// parse the dynamic header at the chunk's candidate, decode
// a.probe_tokens tokens from the guess c + j (cn - c) / parts without
// output, and record the position after them -- a token boundary once the
// code has resynchronised, which it usually has after a few dozen tokens
// (a later part's landing check is what trusts it).  kSplitNone when the
// guess runs into an end of block or an invalid code first.
__global__ __launch_bounds__(64, ZI_WPE) void inflate_probe_kernel(SpecArgs a) {
  __shared__ __attribute__((aligned(16))) Lds s;
  const uint64_t i = blockIdx.x;
  uint64_t k, kn, cn;
  uint32_t j, T;
  uint64_t out = kSplitNone;
  if (owner(a, i, k, j, T, kn, cn) && j > 0) {
    const uint64_t c = a.cand[k];
    const uint64_t guess = c + (uint64_t)j * ((cn - c) / T);
    Reader r;
    reader_init(r, a);
    LLTab ll;
    DTab dd;
    bool ok = reader_at(r, a, c) && ((r.bb >> 1) & 3u) == 2u;
    if (ok) {
      r.drop(3);
      ok = dynamic_tables(s, r, ll, dd) == ZCRC_INFLATE_OK && guess > reader_bit(r) && reader_at(r, a, guess);
    }
    for (uint32_t t = 0; ok && t < a.probe_tokens; t++) {
      if (!r.ensure()) {
        ok = false;
        break;
      }
      const uint32_t ix = (uint32_t)r.bb & ((1u << kLLRoot) - 1u);
      uint32_t e = lane_get(ll[ix >> 6], ix);
      if (e_kind(e) == K_LONG) e = uni(decode_slow(r.peek(15), &s.llm, s.llsym, kLLRoot, A_LITLEN));
      const uint32_t kind = e_kind(e);
      if (kind == K_LIT && e_len(e)) {
        r.drop(e_len(e));
        continue;
      }
      if (kind != K_BASE || e_len(e) == 0) {
        ok = false;  // end of block, invalid or missing code
        break;
      }
      r.drop(e_len(e) + e_extra(e));
      if (!r.ensure()) {
        ok = false;
        break;
      }
      const uint32_t jx = (uint32_t)r.bb & ((1u << kDRoot) - 1u);
      uint32_t d = lane_get(dd[jx >> 6], jx);
      if (e_kind(d) == K_LONG) d = uni(decode_slow(r.peek(15), &s.ddm, s.ddsym, kDRoot, A_DIST));
      if (e_kind(d) != K_BASE || e_len(d) == 0) {
        ok = false;
        break;
      }
      r.drop(e_len(d) + e_extra(d));
    }
    if (ok && r.consumed() <= a.src_len) out = reader_bit(r);
  }
  if (threadIdx.x == 0) a.part[i] = out;
}

// Speculative decode of item i = (chunk k, part j) of one stream
// (zcrc_inflate_split.hip; tests/inflate_split_model.py part_decode): from
// its start (part 0: the chunk's candidate, chunk 0: bit 0, history known;
// part j: its probed token boundary, with the tables of the block whose
// header is at the candidate) until it lands on a later part's start (per
// token, while in that first block), reaches a block start equal to a later
// candidate, ends the final block, or fails.  Elements go to the item's
// region, which extends over the following items that have no work.
__global__ __launch_bounds__(64, ZI_WPE) void inflate_spec_kernel(SpecArgs a) {
  __shared__ __attribute__((aligned(16))) Lds s;
  const uint64_t i = blockIdx.x;
  SpecRec *rec = a.rec + i;
  uint64_t k = 0, kn = 0, cn = 0, c = 0, start = 0, mask = 0, b = kSplitNone;
  uint32_t j = 0, T = 0, np = 0, me = 0;
  bool work = owner(a, i, k, j, T, kn, cn);
  if (work) {
    c = a.cand[k];
    start = c;
    mask = usable_mask(a, k, T, c, cn, b);
    np = (uint32_t)__popcll(mask);
    if (j > 0) {
      work = (mask >> j) & 1u;
      me = (uint32_t)__popcll(mask & ((1ull << j) - 1u)) + 1u;
      start = a.part[i];
    }
  }
  if (!work) {
    if (threadIdx.x == 0) *rec = SpecRec{0, 0, 0, kSpecSkipped, -1, 0, 0};
    return;
  }
  // (everything below reaches the decode state, whose asm wants SGPRs: made
  // provably uniform)
  k = uni64(k);
  j = uni(j);
  c = uni64(c);
  kn = uni64(kn);
  start = uni64(start);
  np = uni(np);
  me = uni(me);
  // landing targets: the usable parts after this one, ascending
  const uint32_t tn = np - me, t = threadIdx.x;
  if (((mask >> t) & 1u) && t > j) {
    const uint32_t rank = (uint32_t)__popcll(mask & ((1ull << t) - 1u)) - me;
    s.tpos[rank] = b;
    s.titem[rank] = (uint32_t)(k * a.parts + t);
  }
  __syncthreads();
  // Region: the chunk owns the elements of its items and of the items of the
  // candidate-less chunks after it, [k parts, kn parts) x region_elems, split
  // evenly among its usable parts -- a part that steps over a later part's
  // start (unsynchronised probe) and absorbs its range has room for it.
  // (Per-item regions overflowed there: most items have no work, so one
  // item's share was well below a part's output, profiles/r03/s30.)
  const uint64_t span = (kn - k) * a.parts * a.region_elems, nused = np + 1;
  const uint64_t r0 = uni64(k * a.parts * a.region_elems + ((me * span / nused) & ~7ull));
  const uint64_t r1 = uni64(me + 1 == nused ? k * a.parts * a.region_elems + span
                                            : k * a.parts * a.region_elems + (((me + 1) * span / nused) & ~7ull));
  Out o;
  o.dst = a.region + r0;
  o.cap = r1 - r0;
  o.pos = 0;
  o.fl = 0;
  o.al16 = (reinterpret_cast<uint64_t>(o.dst) & 15u) == 0;
  o.reach = 0;
  o.spec = i > 0;
  o.tpos = uni64(tn ? s.tpos[0] : kSplitNone);
  o.ti = 0;
  o.tn = tn;
  o.landed = 0;
  o.set_room();
  int32_t st = ZCRC_INFLATE_OK;
  int32_t link = -1;
  uint32_t last = 0;
  Reader r;
  reader_init(r, a);
  LLTab ll;
  DTab dd;
  // mid: the first round of the loop reads the header at c -- of the block
  // this part starts inside -- and continues that block from `start`, so
  // that one call site of each decode step serves both (second inlined
  // copies of the header decode or the symbol loop did not compile: illegal
  // VGPR to SGPR copies)
  bool mid = j > 0;
  if (!reader_at(r, a, c)) st = ZCRC_INFLATE_ERR_INPUT;
  uint64_t jc = k + 1;  // the next candidate at or past the decode position
  bool first = true;    // part targets live in the chunk's first block only
  while (st == ZCRC_INFLATE_OK && !last) {
    if (!r.ensure()) {
      st = ZCRC_INFLATE_ERR_INPUT;
      break;
    }
    const uint64_t bit = reader_bit(r);
    while (jc < a.nchunks) {
      const uint64_t cj = a.cand[jc];
      if (cj != kSplitNone && cj >= bit) break;
      jc++;
    }
    if (jc < a.nchunks && a.cand[jc] == bit) {
      link = (int32_t)(jc * a.parts);
      break;
    }
    last = r.peek(1);
    const uint32_t type = (uint32_t)(r.bb >> 1) & 3u;
    r.drop(3);
    if (mid && type != 2) {
      st = ZCRC_INFLATE_ERR_CODES;  // (a part's candidate is a dynamic header: the probe read it)
    } else if (type == 0) {
      st = stored(s, r, o);
    } else if (type == 1) {
      fixed_tables(s, ll, dd);
      st = codes(s, r, o, ll, dd);
    } else if (type == 2) {
      st = dynamic_tables(s, r, ll, dd);
      if (mid && st == ZCRC_INFLATE_OK && !reader_at(r, a, start)) st = ZCRC_INFLATE_ERR_INPUT;
      if (st == ZCRC_INFLATE_OK) st = codes(s, r, o, ll, dd);
    } else {
      st = ZCRC_INFLATE_ERR_BLOCK_TYPE;
    }
    st = (int32_t)uni((uint32_t)st);
    if (first) o.tpos = kSplitNone;
    first = false;
    mid = false;
    if (st == kSpecLanded) {
      link = (int32_t)o.landed;
      st = ZCRC_INFLATE_OK;
      break;
    }
  }
  if (st == ZCRC_INFLATE_OK && link < 0 && r.consumed() > a.src_len) st = ZCRC_INFLATE_ERR_INPUT;
  if (st == ZCRC_INFLATE_OK) flush_to(s, o, o.pos);
  if (threadIdx.x == 0) {
    rec->region = r0;
    rec->out_len = o.pos;
    rec->end_bit = reader_bit(r);
    rec->status = st;
    rec->link = link;
    rec->reach = o.reach;
    rec->final_ = (st == ZCRC_INFLATE_OK && link < 0 && last) ? 1u : 0u;
  }
}
#endif

}  // namespace

#if !ZI_SPEC
hipError_t launch(const InflateArgs &args, hipStream_t stream) {
  hipLaunchKernelGGL(inflate_kernel, dim3((unsigned)args.n), dim3(64), 0, stream, args);
  return hipGetLastError();
}
#else
hipError_t launch_spec(const SpecArgs &args, hipStream_t stream) {
  hipLaunchKernelGGL(inflate_spec_kernel, dim3((unsigned)(args.nchunks * args.parts)), dim3(64), 0, stream, args);
  return hipGetLastError();
}
hipError_t launch_probe(const SpecArgs &args, hipStream_t stream) {
  hipLaunchKernelGGL(inflate_probe_kernel, dim3((unsigned)(args.nchunks * args.parts)), dim3(64), 0, stream, args);
  return hipGetLastError();
}
#endif
#ifdef ZI_WPE_DEFAULTED
#undef ZI_WPE
#undef ZI_WPE_DEFAULTED
#endif
#ifdef ZI_SPEC_DEFAULTED
#undef ZI_SPEC
#undef ZI_SPEC_DEFAULTED
#endif
#undef ZI_DSW
#undef ZI_DSR
#undef ZI_ESH
