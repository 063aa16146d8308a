// zcrc_inflate_split.hip -- block-parallel inflate of ONE raw-DEFLATE stream
// on MI355X (gfx950).  SURVEY.md 8(f) rank 4, DESIGN.md section 11b.
//
// ZIPsFS preloads one deflated entry at a time: zip_fread() in 16 MiB calls
// inside preloadram_now (src/ZIPsFS_preloadfileram.c:286-306), libzip
// inflating with zlib, and then the CRC check (:243).  The batched inflate
// (zcrc_inflate.hip) gives each stream one wave, so a single entry decodes at
// one wave's speed.  Here one stream is cut into chunks that decode at once:
//
//   1. inflate_find_kernel: for every chunk of the compressed bytes, the first
//      bit position whose dynamic-Huffman block header is valid by zlib's
//      rules (quick filter on every position, full header check on the ~0.1%
//      that pass it).  A true block start always passes; a false one only
//      costs work.
//   2. sp::inflate_spec_kernel (zcrc_inflate_impl.h, ZI_SPEC): every chunk
//      decodes from its candidate with an unknown history into 16-bit
//      elements (byte or history marker) and stops where it reaches a later
//      candidate (a link) or the final block's end.
//   3. inflate_chain_kernel: follows the links from chunk 0 (a true start, so
//      every chunk it reaches started at a true block boundary), checks the
//      chain (statuses, history reach, capacity) and lays the chunks out.
//   4. inflate_win_*_kernel: the 32 KiB window after each chain chunk, as
//      bytes and references to the previous window, resolved by pointer
//      jumping in log2(chunks) parallel rounds, its tail stored to dst;
//      inflate_body_kernel: all other elements in parallel, from the tails.
//   5. When the chain fails, the serial kernel (one wave) decodes the stream
//      and reports zlib's exact status: launch_inflate with run_if.
//
// The CPU model tests/inflate_split_model.py is the specification; its tests
// and the GPU tests compare the bytes with zlib.decompress.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../../include/zcrc.h"
#include "zcrc_inflate_find.h"
#include "zcrc_internal.h"
#include "zcrc_inflate_internal.h"

namespace zcrc {
namespace {

constexpr uint32_t kFindThreads = 1024;
constexpr uint32_t kFindWin = 16384;     // compressed bytes staged per finder window
constexpr uint32_t kFindLook = 1024;     // + look-ahead: a dynamic header is at most ~563 bytes
constexpr uint32_t kFindWords = (kFindWin + kFindLook) / 4 + 4;
constexpr uint32_t kFindSurv = 1024;     // survivors of the quick filter checked per window

__device__ __forceinline__ uint32_t wuni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t wuni64(uint64_t v) { return ((uint64_t)wuni((uint32_t)(v >> 32)) << 32) | wuni((uint32_t)v); }

// Position of code-length symbol s in the header's order (the inverse of
// 16 17 18 0 8 7 9 6 10 5 11 4 12 3 13 2 14 1 15), 5 bits per symbol
constexpr uint64_t kClenPosLo = 0x520c429d2b6be23ull;  // symbols 0..11
constexpr uint64_t kClenPosHi = 0x820941ccull;         // symbols 12..18

// find::full_ok for one position per WAVE (q wave-uniform): the same
// checks, with the code-length code built by ballots (lane s holds symbol
// s) into a 128-entry lookup table held in two VGPRs, and the length decode
// run on scalar registers -- a table lookup (v_readlane) per symbol instead
// of a per-lane canonical decode.  The lane-per-position form spent ~0.5 us
// per symbol of its longest lane (profiles/r03/s34).  lut: this wave's
// 128 bytes of LDS.
__device__ bool full_ok_wave(const uint32_t *w, uint32_t q, uint32_t avail, uint8_t *lut) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t v = wuni64(find::bits64(w, q));
  const uint32_t nlen = (uint32_t)((v >> 3) & 31u) + 257u, ndist = (uint32_t)((v >> 8) & 31u) + 1u;
  const uint32_t hclen = (uint32_t)((v >> 13) & 15u) + 4u;
  const uint64_t cl = wuni64(find::bits64(w, q + 17));
  const uint32_t pos = lane < 12 ? (uint32_t)(kClenPosLo >> (5 * lane)) & 31u
                                 : (lane < 19 ? (uint32_t)(kClenPosHi >> (5 * (lane - 12))) & 31u : 31u);
  const uint32_t l = pos < hclen ? (uint32_t)(cl >> (3 * pos)) & 7u : 0u;  // lane s: length of symbol s
  // canonical codes (the quick filter made the code complete: 128 entries)
  const uint64_t lt = (1ull << lane) - 1ull;
  uint32_t code = 0, mycode = 0;
#pragma unroll
  for (uint32_t L = 1; L < 8; L++) {
    const uint64_t m = __ballot(l == L);
    if (l == L) mycode = code + (uint32_t)__builtin_popcountll(m & lt);
    code = (code + (uint32_t)__builtin_popcountll(m)) << 1;
  }
  if (l) {  // entries in stream bit order: the reversed code, then any bits
    const uint32_t r = __builtin_bitreverse32(mycode) >> (32 - l);
    for (uint32_t t = 0; t < (1u << (7 - l)); t++) lut[r | (t << l)] = (uint8_t)(lane | (l << 5));
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the wave's LUT writes are done
  __builtin_amdgcn_wave_barrier();
  const uint32_t lut_lo = lut[lane], lut_hi = lut[lane + 64];
  uint32_t p = q + 17 + 3 * hclen;
  const uint32_t total = nlen + ndist, end = q + avail;
  uint32_t idx = 0, prev = 0, kll = 0, kd = 0, mll = 0, md = 0;
  bool eob = false;
  uint32_t wi = (p >> 5) + 1, nb = 32 - (p & 31u);
  uint64_t bb = wuni(w[p >> 5]) >> (p & 31u);
  while (idx < total) {
    if (p + 32 > end) return false;  // the header would run past the staged bytes
    if (nb < 32) {
      bb |= (uint64_t)wuni(w[wi++]) << nb;
      nb += 32;
    }
    const uint32_t x = (uint32_t)bb & 127u;
    const uint32_t e = (uint32_t)__builtin_amdgcn_readlane((int)(x < 64 ? lut_lo : lut_hi), (int)(x & 63u));
    const uint32_t sym = e & 31u, used = e >> 5;
    const uint32_t xb = (uint32_t)(bb >> used);
    uint32_t val, rep, extra;
    if (sym < 16) {
      val = sym;
      rep = 1;
      prev = sym;
      extra = 0;
    } else if (sym == 16) {
      if (idx == 0) return false;
      val = prev;
      rep = 3 + (xb & 3u);
      extra = 2;
    } else if (sym == 17) {
      val = 0;
      rep = 3 + (xb & 7u);
      extra = 3;
      prev = 0;
    } else {
      val = 0;
      rep = 11 + (xb & 127u);
      extra = 7;
      prev = 0;
    }
    p += used + extra;
    bb >>= used + extra;
    nb -= used + extra;
    if (idx + rep > total) return false;
    if (val) {
      const uint32_t in_ll = idx < nlen ? (nlen - idx < rep ? nlen - idx : rep) : 0u;
      kll += in_ll << (15 - val);
      kd += (rep - in_ll) << (15 - val);
      if (in_ll) mll = val > mll ? val : mll;
      if (rep > in_ll) md = val > md ? val : md;
      if (idx <= 256 && 256 < idx + rep) eob = true;
      if (kll > 32768u || kd > 32768u) return false;
    }
    idx += rep;
  }
  if (!eob) return false;
  if (kll > 32768u || (kll < 32768u && mll != 1u)) return false;
  if (kd > 32768u || (kd < 32768u && md > 1u)) return false;
  return true;
}

struct FindArgs {
  const uint8_t *src;
  uint64_t src_len;
  uint64_t chunk;  // compressed bytes per chunk
  uint64_t nchunks;
  uint64_t *cand;
  uint32_t timing;  // measurement builds only (ZCRC_SPLIT_FIND_TIMING): 1 = no full checks, 2 = no quick filter either
};

// One workgroup per chunk k >= 1: the first bit position in [8 k chunk,
// 8 (k+1) chunk) that passes full_ok.  The chunk is staged in windows of
// kFindWin bytes; each thread tests the 32 positions of one staged word at a
// time (a 96-bit funnel of four words per position): the cheap header test
// on all 32 gives a mask, the code-length Kraft sum runs only on its set bits
// (a 512-entry LDS table of triple contributions, read at random addresses, cost more
// than the arithmetic: bank conflicts).  Sub-windows of 4 KiB; the survivors
// of a sub-window get the full check before the next one starts, and the
// search stops at the first sub-window with a true start.
constexpr uint32_t kFindSub = kFindThreads;  // words per sub-window (32 positions each)
__global__ __launch_bounds__(kFindThreads) void inflate_find_kernel(FindArgs a) {
  __shared__ uint32_t w[kFindWords];
  __shared__ uint32_t surv[kFindSurv];
  __shared__ uint8_t lutw[kFindThreads / 64][128];  // each wave's code-length LUT (full_ok_wave)
  // per sub-window parity: its survivor count and best position (double-
  // buffered: a count is reset one sub-window after it was last read)
  __shared__ uint32_t nsurv[2], best[2];
  const uint32_t tid = threadIdx.x;
  const uint64_t k = blockIdx.x;
  if (k == 0) {
    if (tid == 0) a.cand[0] = 0;
    return;
  }
  const uint64_t lo = k * a.chunk;
  const uint64_t hi = lo + a.chunk < a.src_len ? lo + a.chunk : a.src_len;
  uint64_t found = kSplitNone;
  for (uint64_t wlo = lo; wlo < hi && found == kSplitNone; wlo += kFindWin) {
    const uint64_t whi = wlo + kFindWin < hi ? wlo + kFindWin : hi;  // positions [wlo, whi)
    const uint64_t send = whi + kFindLook < a.src_len ? whi + kFindLook : a.src_len;
    const uint32_t nbytes = (uint32_t)(send - wlo);
    // stage [wlo, send) as little-endian words, zeros past the end: aligned
    // dword loads through a buffer resource sized to the bytes there (the
    // range check zeroes the rest), then one funnel shift per word in LDS
    // (a byte load per byte, each under its own bounds branch, was ~2x the
    // whole search on an 8 KiB chunk)
    {
      const uint64_t at = reinterpret_cast<uint64_t>(a.src) + wlo;
      const uint32_t sh = (uint32_t)(at & 3u);
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(at - sh), (short)0, (int)(nbytes + sh), 0x00020000);
      uint32_t v[(kFindWords + kFindThreads - 1) / kFindThreads];
#pragma unroll
      for (uint32_t t = 0; t < (kFindWords + kFindThreads - 1) / kFindThreads; t++)
        v[t] = __builtin_amdgcn_raw_buffer_load_b32(rs, 4u * (tid + kFindThreads * t), 0, 0);
#pragma unroll
      for (uint32_t t = 0; t < (kFindWords + kFindThreads - 1) / kFindThreads; t++)
        if (tid + kFindThreads * t < kFindWords) w[tid + kFindThreads * t] = v[t];
      __syncthreads();
#pragma unroll
      for (uint32_t t = 0; t < (kFindWords + kFindThreads - 1) / kFindThreads; t++) {
        const uint32_t i = tid + kFindThreads * t;
        v[t] = i + 1 < kFindWords ? __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh) : 0u;
      }
      __syncthreads();
#pragma unroll
      for (uint32_t t = 0; t < (kFindWords + kFindThreads - 1) / kFindThreads; t++)
        if (tid + kFindThreads * t < kFindWords) w[tid + kFindThreads * t] = v[t];
    }
    if (tid == 0) nsurv[0] = nsurv[1] = 0, best[0] = best[1] = 0xFFFFFFFFu;
    __syncthreads();  // staged; counters reset
    const uint32_t npos = 8u * (uint32_t)(whi - wlo);
    for (uint32_t sub = 0; sub * 32u * kFindSub < npos; sub++) {
      const uint32_t p = sub & 1u;
      const uint32_t i = sub * kFindSub + tid;  // this thread's word: positions 32 i .. 32 i + 31
      if (32u * i < npos && a.timing < 2) {
        const uint32_t w0 = w[i], w1 = w[i + 1], w2 = w[i + 2], w3 = w[i + 3];
        uint32_t mask = 0;
#pragma unroll
        for (uint32_t b = 0; b < 32; b++) {
          const uint32_t x0 = (uint32_t)((((uint64_t)w1 << 32) | w0) >> b);
          mask |= (uint32_t)find::head_ok(x0) << b;
        }
        if (32u * i + 32u > npos) mask &= (1u << (npos - 32u * i)) - 1u;  // npos is a multiple of 8
        while (mask) {
          const uint32_t b = (uint32_t)__builtin_ctz(mask);
          mask &= mask - 1u;
          uint32_t x0, x1, x2;
          find::window96(w0, w1, w2, w3, b, x0, x1, x2);
          if (find::cl_ok(x0, x1, x2)) {
            const uint32_t j = atomicAdd(&nsurv[p], 1u);
            if (j < kFindSurv) surv[j] = 32u * i + b;
          }
        }
      }
      __syncthreads();  // every thread has also read the other parity's counters of the last sub-window
      if (tid == 0) nsurv[p ^ 1u] = 0, best[p ^ 1u] = 0xFFFFFFFFu;
      const uint32_t ns = nsurv[p] < kFindSurv ? nsurv[p] : kFindSurv;  // more: the rest go unchecked (parallelism lost, never correctness)
      // one survivor per wave at a time (the CPU test checks find::full_ok,
      // which full_ok_wave restates; the GPU test checks the chain finds
      // every block start)
      const uint32_t wv = tid >> 6;
      for (uint32_t j = wv; j < ns && !a.timing; j += kFindThreads / 64) {
        const uint32_t q = wuni(surv[j]);
        if (full_ok_wave(w, q, 8u * nbytes - q, lutw[wv]) && (tid & 63u) == 0) atomicMin(&best[p], q);
      }
      __syncthreads();
      const uint32_t bq = best[p];  // workgroup-uniform
      if (bq != 0xFFFFFFFFu) {
        found = 8 * wlo + bq;
        break;
      }
    }
    __syncthreads();  // before the next window overwrites w
  }
  if (tid == 0) a.cand[k] = found;
}

struct ChainArgs {
  const SpecRec *rec;
  uint64_t nchunks;
  uint64_t cap;
  uint32_t *chain;     // chain chunks in order; chain[nchunks] = their count
  uint64_t *off;       // output offset of chunk k (valid on the chain)
  uint32_t *run_serial;
  uint64_t *out_len;   // the caller's (1 stream)
  int32_t *status;
  // the serial fall-back's one-stream argument arrays
  const uint8_t **fb_src;
  uint64_t *fb_src_len;
  uint8_t **fb_dst;
  uint64_t *fb_cap;
  const uint8_t *src;
  uint64_t src_len;
  uint8_t *dst;
};

constexpr uint32_t kChainLds = 16384;  // chunks whose links are staged in LDS (the host keeps nchunks <= this)

// Follow the links from chunk 0 (LDS walk by one thread), then give every
// chain chunk its output offset (block scan in index order: links only go
// forward).  Failure -> run_serial = 1.
__global__ __launch_bounds__(1024) void inflate_chain_kernel(ChainArgs a) {
  __shared__ uint32_t nxt[kChainLds];
  __shared__ uint64_t part[16];
  __shared__ uint32_t ok_s;
  const uint32_t tid = threadIdx.x;
  const uint32_t n = (uint32_t)a.nchunks;
  // successor: the next chunk, kFinal, or kFail (an error, or neither linked
  // nor final); kOn marks the chain
  constexpr uint32_t kFinal = 0xFFFFFEu, kFail = 0xFFFFFFu, kOn = 0x80000000u;
  for (uint32_t k = tid; k < n; k += 1024) {
    const SpecRec r = a.rec[k];
    uint32_t s = kFail;
    if (r.status == ZCRC_INFLATE_OK) s = r.final_ ? kFinal : (r.link > (int32_t)k ? (uint32_t)r.link : kFail);
    nxt[k] = s;
  }
  if (tid == 0) {
    *a.fb_src = a.src;
    *a.fb_src_len = a.src_len;
    *a.fb_dst = a.dst;
    *a.fb_cap = a.cap;
  }
  __syncthreads();
  if (tid == 0) {
    // mark the chain: on-chain chunks get bit 30 set in their entry
    uint32_t k = 0;
    bool ok = true;
    for (;;) {  // links only go forward: this ends
      const uint32_t s = nxt[k];
      nxt[k] = s | kOn;
      if (s == kFinal) break;
      if (s == kFail) {
        ok = false;
        break;
      }
      k = s;
    }
    ok_s = ok;
  }
  __syncthreads();
  if (!ok_s) {
    if (tid == 0) {
      *a.run_serial = 1;
      a.chain[a.nchunks] = 0;
    }
    return;
  }
  // exclusive scan of out_len over the chain, in index order; then checks
  const uint32_t per = (n + 1023) / 1024;
  const uint32_t k0 = tid * per, k1 = k0 + per < n ? k0 + per : n;
  uint64_t sum = 0;
  for (uint32_t k = k0; k < k1; k++)
    if (nxt[k] & kOn) sum += a.rec[k].out_len;
  // block scan of the per-thread sums (wave scan, then wave totals)
  const uint32_t lane = tid & 63u, wv = tid >> 6;
  uint64_t inc = sum;
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint64_t t = __shfl_up(inc, d, 64);
    if (lane >= d) inc += t;
  }
  if (lane == 63) part[wv] = inc;
  __syncthreads();
  uint64_t base = 0, tot = 0;
  for (uint32_t i = 0; i < 16; i++) {
    if (i < wv) base += part[i];
    tot += part[i];
  }
  uint64_t run = base + inc - sum;
  bool good = true;
  for (uint32_t k = k0; k < k1; k++) {
    if (nxt[k] & kOn) {
      const SpecRec r = a.rec[k];
      if (r.reach > run) good = false;  // a back-reference before the stream start
      a.off[k] = run;
      run += r.out_len;
    }
  }
  if (!good) ok_s = 0;  // benign race: every writer writes 0
  __syncthreads();
  if (tid == 0) {
    const bool fine = ok_s && tot <= a.cap;
    *a.run_serial = fine ? 0u : 1u;
    if (fine) {
      *a.out_len = tot;
      *a.status = ZCRC_INFLATE_OK;
    }
    // chain list in order (only read when fine)
    uint32_t m = 0;
    for (uint32_t k = 0; k < n; k++)
      if (nxt[k] & kOn) a.chain[m++] = k;
    a.chain[a.nchunks] = fine ? m : 0u;
  }
}

struct ResolveArgs {
  const uint16_t *region;
  uint64_t region_elems;
  const SpecRec *rec;
  const uint32_t *chain;  // chain[nchunks] = count (0: the serial decode runs instead)
  const uint64_t *off;
  uint64_t nchunks;
  uint8_t *dst;
};

// element -> byte: a marker is byte (v - kInflateMarker) of the kInflateHist
// bytes before the chunk at output offset `off`.
__device__ __forceinline__ uint8_t resolve_dst(uint32_t v, const uint8_t *dst, uint64_t off) {
  return v < kInflateMarker ? (uint8_t)v : dst[off - kInflateHist + (v - kInflateMarker)];
}

// The 32 KiB windows: W_m = the last 32 KiB of output through the end of
// chain chunk m, one 32-bit entry per byte -- the byte (kWinByte | value) or
// a reference (c << 15 | p) to byte p of W_c.  Built from the chunk's last
// 32 Ki elements (a marker w of chunk m refers to byte w of W_{m-1}; when the
// chunk is shorter than 32 KiB the window's front refers to W_{m-1} shifted),
// then resolved by pointer jumping: each round replaces a reference by what
// it points at, so after round r every remaining reference reaches 2^r
// chunks back, and ceil(log2 chunks) rounds leave bytes only (W_0 has no
// reference).  Each round is one parallel pass -- the chain's one
// sequential dependency costs log2(chunks) launches, not a step per chunk
// (the first form, an LDS ring walked chunk by chunk, took 3-7 us per chunk:
// 6.8 ms on a 64 MiB entry).
constexpr uint32_t kWinByte = 0x80000000u;
struct WinArgs {
  const uint16_t *region;
  uint64_t region_elems;
  const SpecRec *rec;
  const uint32_t *chain;  // chain[nchunks] = count (0: the serial decode runs instead)
  const uint64_t *off;
  uint64_t nchunks;
  const uint32_t *win_in;  // jump: the previous round's windows
  uint32_t *win;           // nchunks x kInflateHist entries, by chain position
  uint8_t *dst;
};

// grid: (kInflateHist / 1024, nchunks); block (x, m) builds entries
// [1024 x, 1024 x + 1024) of W_m
__global__ __launch_bounds__(1024) void inflate_win_build_kernel(WinArgs a) {
  const uint32_t m = blockIdx.y;
  if (m >= a.chain[a.nchunks]) return;
  const uint32_t k = a.chain[m];
  const uint64_t len = a.rec[k].out_len;
  const uint32_t n = len < kInflateHist ? (uint32_t)len : kInflateHist;
  const uint32_t i = blockIdx.x * 1024u + threadIdx.x;
  uint32_t v;
  if (i >= kInflateHist - n) {
    const uint32_t e = a.region[a.rec[k].region + (len - kInflateHist + i)];
    v = e < kInflateMarker ? (kWinByte | e) : (m ? ((m - 1) << 15) | (e - kInflateMarker) : kWinByte);
  } else {
    v = m ? ((m - 1) << 15) | (i + n) : kWinByte;  // W_0's front: before the stream, never referenced
  }
  a.win[(uint64_t)m * kInflateHist + i] = v;
}

__global__ __launch_bounds__(1024) void inflate_win_jump_kernel(WinArgs a) {
  const uint32_t m = blockIdx.y;
  if (m >= a.chain[a.nchunks]) return;
  const uint64_t at = (uint64_t)m * kInflateHist + blockIdx.x * 1024u + threadIdx.x;
  uint32_t v = a.win_in[at];
  if (!(v & kWinByte)) v = a.win_in[(uint64_t)(v >> 15) * kInflateHist + (v & (kInflateHist - 1))];
  a.win[at] = v;
}

// each chunk's last (up to) 32 KiB of output, from its resolved window
__global__ __launch_bounds__(1024) void inflate_win_store_kernel(WinArgs a) {
  const uint32_t m = blockIdx.y;
  if (m >= a.chain[a.nchunks]) return;
  const uint32_t k = a.chain[m];
  const uint64_t len = a.rec[k].out_len;
  const uint32_t n = len < kInflateHist ? (uint32_t)len : kInflateHist;
  const uint32_t i = blockIdx.x * 1024u + threadIdx.x;
  if (i >= kInflateHist - n) a.dst[a.off[k] + len - kInflateHist + i] = (uint8_t)a.win[(uint64_t)m * kInflateHist + i];
}

// Every chain chunk's elements before its last 32 KiB: markers from the
// resolved tails in dst (written by the previous launch).
__global__ __launch_bounds__(256) void inflate_body_kernel(ResolveArgs a) {
  const uint32_t m_end = a.chain[a.nchunks];
  constexpr uint32_t kTile = 256 * 16;
  for (uint32_t m = blockIdx.y; m < m_end; m += gridDim.y) {
    const uint32_t k = a.chain[m];
    const uint64_t len = a.rec[k].out_len, off = a.off[k];
    const uint64_t body = len > kInflateHist ? len - kInflateHist : 0;
    const uint16_t *el = a.region + a.rec[k].region;
    for (uint64_t t = (uint64_t)blockIdx.x * kTile; t < body; t += (uint64_t)gridDim.x * kTile) {
#pragma unroll
      for (uint32_t j = 0; j < 16; j++) {
        const uint64_t e = t + threadIdx.x + 256u * j;
        if (e < body) a.dst[off + e] = resolve_dst(el[e], a.dst, off);
      }
    }
  }
}

}  // namespace

// Default: chunks of kInflateSplitChunk, or larger so that the chunks just
// fill the speculative decoder's resident workgroups -- more chunks than
// that only queue (the decode time stays ~src_len / (resident x rate)) and
// add pointer-jumping rounds.  The 32 Ki-history decoder (two per CU, no
// reads of old output back from HBM) while its residents suffice, else the
// 16 Ki ring (four per CU).  ZCRC_SPLIT_RING=16|32 forces one (measurement).
InflateSplitShape inflate_split_shape(uint64_t src_len, uint64_t cap, uint64_t want, int num_cus) {
  const char *fr = getenv("ZCRC_SPLIT_RING");  // (read per call: tests set it)
  const int force = fr ? atoi(fr) : 0;
  const uint64_t cus = (uint64_t)(num_cus > 0 ? num_cus : 1);
  InflateSplitShape sh;
  // text-like streams (ratio >= 2.5) reach back far more often: the whole
  // history in LDS pays even at half the residents (64 MiB of text: 7.7
  // against 9.4 ms; spectrum-like at 1.25: 13.2 against 10.2 ms,
  // profiles/r03/s29/bench_ring*.jsonl)
  sh.wide = force ? force == 32
                  : ((src_len + kInflateSplitChunk - 1) / kInflateSplitChunk <= kSpecPerCuWide * cus ||
                     cap >= src_len / 2 * 5);
  uint64_t c = want;
  if (!c) {
    const uint64_t resident = (sh.wide ? kSpecPerCuWide : kSpecPerCu) * cus;
    c = (src_len + resident - 1) / resident;
    if (c < kInflateSplitChunk) c = kInflateSplitChunk;
  }
  const uint64_t need = (src_len + kChainLds - 1) / kChainLds;  // at most kChainLds chunks
  sh.chunk = c < need ? need : c;
  // parts: for small streams (at most a quarter as many chunks as resident
  // decoders), cut each chunk's first block into parts (items), up to
  // kMaxParts; items stay <= kChainLds.  Typically half the chunks or fewer
  // find a block start (zlib's blocks span 2-4 chunks of 8 KiB), so 2 x
  // resident / chunks parts fill the decoders.  Above that the probes'
  // header parses and the pointer-jumping rounds over twice the items cost
  // more than the shorter decodes save (16 MiB spectrum 5.6 against 3.8 ms,
  // 64 MiB text 9.3 against 6.4 ms: profiles/r03/s38 against s35).
  const uint64_t nch = src_len ? (src_len + sh.chunk - 1) / sh.chunk : 1;
  const uint64_t resident = (sh.wide ? kSpecPerCuWide : kSpecPerCu) * cus;
  uint64_t parts = 4 * nch <= resident ? 2 * resident / nch : 1;
  const char *fp = getenv("ZCRC_SPLIT_PARTS");  // (read per call: tests set it)
  const int force_parts = fp ? atoi(fp) : 0;
  if (force_parts > 0) parts = (uint64_t)force_parts;
  if (parts > kMaxChunkParts) parts = kMaxChunkParts;
  if (parts < 1) parts = 1;
  while (parts > 1 && nch * parts > kChainLds) parts--;
  sh.parts = (uint32_t)parts;
  return sh;
}

// item regions: 3 x the average share + kInflateSplitSlack each; a chunk
// with a candidate owns its items' and the following candidate-less chunks'
// regions and splits them among its parts (inflate_spec_kernel)
static uint64_t region_elems(uint64_t cap, uint64_t nitems) {
  return ((3 * cap) / nitems + kInflateSplitSlack + 7) & ~7ull;
}

uint64_t inflate_split_scratch_bytes(uint64_t src_len, uint64_t cap, InflateSplitShape shape) {
  const uint64_t nch = src_len ? (src_len + shape.chunk - 1) / shape.chunk : 1;
  const uint64_t nit = nch * shape.parts;
  return 256 + nch * 8 + nit * (8 + sizeof(SpecRec) + 4 + 8) + 8 + 64 + nit * region_elems(cap, nit) * 2 +
         2 * 4ull * kInflateHist * nit + 64 * 14;
}

// One stream: find, speculative decode, chain, resolve, serial fall-back.
hipError_t launch_inflate_split(const uint8_t *src, uint64_t src_len, uint8_t *dst, uint64_t cap,
                                uint64_t *out_len, int32_t *status, InflateSplitShape shape, void *scratch,
                                int num_cus, hipStream_t stream) {
  const uint64_t chunk = shape.chunk;
  const uint64_t nch = src_len ? (src_len + chunk - 1) / chunk : 1;
  const uint64_t nit = nch * shape.parts;  // items: (chunk, part)
  const uint64_t relems = region_elems(cap, nit);
  uint8_t *p = static_cast<uint8_t *>(scratch);
  auto take = [&](uint64_t bytes) {
    uint8_t *r = p;
    p += (bytes + 63) & ~63ull;
    return r;
  };
  uint32_t *run_serial = reinterpret_cast<uint32_t *>(take(64));
  const uint8_t **fb_src = reinterpret_cast<const uint8_t **>(take(8));
  uint64_t *fb_src_len = reinterpret_cast<uint64_t *>(take(8));
  uint8_t **fb_dst = reinterpret_cast<uint8_t **>(take(8));
  uint64_t *fb_cap = reinterpret_cast<uint64_t *>(take(8));
  uint64_t *cand = reinterpret_cast<uint64_t *>(take(8 * nch));
  uint64_t *part = reinterpret_cast<uint64_t *>(take(8 * nit));
  SpecRec *rec = reinterpret_cast<SpecRec *>(take(sizeof(SpecRec) * nit));
  uint32_t *chain = reinterpret_cast<uint32_t *>(take(4 * (nit + 1)));
  uint64_t *off = reinterpret_cast<uint64_t *>(take(8 * nit));
  uint16_t *region = reinterpret_cast<uint16_t *>(take(2 * nit * relems));
  uint32_t *win[2] = {reinterpret_cast<uint32_t *>(take(4ull * kInflateHist * nit)),
                      reinterpret_cast<uint32_t *>(take(4ull * kInflateHist * nit))};

  const char *ft = getenv("ZCRC_SPLIT_FIND_TIMING");  // measurement only: candidates are then none
  FindArgs fa{src, src_len, chunk, nch, cand, ft ? (uint32_t)atoi(ft) : 0u};
  hipLaunchKernelGGL(inflate_find_kernel, dim3((unsigned)nch), dim3(kFindThreads), 0, stream, fa);
  const char *pt = getenv("ZCRC_SPLIT_PROBE");  // test knob: tokens per probe (a few: unsynchronised part starts)
  // test knob: ZCRC_SPLIT_BORROW=0 keeps each chunk to its own items
  const char *bw = getenv("ZCRC_SPLIT_BORROW");
  SpecArgs sa{src, src_len, cand, rec, region, relems, nch, part, shape.parts,
              pt && atoi(pt) > 0 ? (uint32_t)atoi(pt) : kInflateProbeTokens,
              bw && atoi(bw) == 0 ? shape.parts : kMaxParts};
  hipError_t e = hipSuccess;
  if (sa.max_parts > 1) e = launch_inflate_probe(sa, stream);
  if (e == hipSuccess) e = launch_inflate_spec(sa, shape.wide, stream);
  if (e != hipSuccess) return e;
  ChainArgs ca{rec, nit, cap, chain, off, run_serial, out_len, status, fb_src, fb_src_len, fb_dst, fb_cap,
               src, src_len, dst};
  hipLaunchKernelGGL(inflate_chain_kernel, dim3(1), dim3(1024), 0, stream, ca);
  // windows: build, ceil(log2 nch) pointer-jumping rounds, store the tails
  uint32_t rounds = 0;
  while ((1ull << rounds) < nit) rounds++;
  WinArgs wa{region, relems, rec, chain, off, nit, nullptr, win[0], dst};
  const dim3 wgrid(kInflateHist / 1024, (unsigned)nit);
  hipLaunchKernelGGL(inflate_win_build_kernel, wgrid, dim3(1024), 0, stream, wa);
  for (uint32_t r = 0; r < rounds; r++) {
    wa.win_in = win[r & 1];
    wa.win = win[(r + 1) & 1];
    hipLaunchKernelGGL(inflate_win_jump_kernel, wgrid, dim3(1024), 0, stream, wa);
  }
  hipLaunchKernelGGL(inflate_win_store_kernel, wgrid, dim3(1024), 0, stream, wa);
  ResolveArgs ra{region, relems, rec, chain, off, nit, dst};
  const unsigned gy = (unsigned)(nit < 4096 ? nit : 4096);
  const unsigned gx = (unsigned)((4u * (unsigned)num_cus + gy - 1) / gy) + 1u;
  hipLaunchKernelGGL(inflate_body_kernel, dim3(gx, gy), dim3(256), 0, stream, ra);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  // the serial decode, run only when the chain failed
  InflateArgs ia{};
  ia.src = fb_src;
  ia.src_len = fb_src_len;
  ia.dst = fb_dst;
  ia.cap = fb_cap;
  ia.out_len = out_len;
  ia.status = status;
  ia.n = 1;
  ia.run_if = run_serial;
  e = launch_inflate(ia, num_cus, stream, nullptr);
  if (e == hipSuccess && getenv("ZCRC_SPLIT_TRACE")) {  // diagnostics: why a chain did (not) form
    std::vector<uint64_t> hc(nch), hp(nit);
    std::vector<SpecRec> hr(nit);
    std::vector<uint32_t> hch(nit + 1), hrs(1);
    e = hipStreamSynchronize(stream);
    if (e == hipSuccess) e = hipMemcpy(hc.data(), cand, 8 * nch, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(hp.data(), part, 8 * nit, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(hr.data(), rec, sizeof(SpecRec) * nit, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(hch.data(), chain, 4 * (nit + 1), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(hrs.data(), run_serial, 4, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return e;
    fprintf(stderr, "[split] src %llu cap %llu chunk %llu chunks %llu parts %u items %llu wide %d region %llu elems; "
            "chain %u serial %u\n", (unsigned long long)src_len, (unsigned long long)cap, (unsigned long long)chunk,
            (unsigned long long)nch, shape.parts, (unsigned long long)nit, (int)shape.wide,
            (unsigned long long)relems, hch[nit], hrs[0]);
    for (uint64_t i = 0; i < nit; i++) {
      const SpecRec &r = hr[i];
      if (r.status == kSpecSkipped) continue;
      fprintf(stderr, "[split]   item %llu (chunk %llu part %llu) cand %lld part %lld: status %d link %d out %llu "
              "reach %u final %u end_bit %llu\n", (unsigned long long)i, (unsigned long long)(i / shape.parts),
              (unsigned long long)(i % shape.parts), (long long)hc[i / shape.parts], (long long)hp[i], r.status,
              r.link, (unsigned long long)r.out_len, r.reach, r.final_, (unsigned long long)r.end_bit);
    }
  }
  return e;
}

}  // namespace zcrc
