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
//   * one 64-lane workgroup per stream: DEFLATE is serial within a stream,
//     so the batch is the parallelism.  All decode state is wave-uniform and
//     lives in SGPRs; a single wave per SIMD issues one instruction every
//     ~4 cycles, so the figure of merit is instructions per symbol;
//   * Huffman lookup tables live in VGPRs, not LDS: entry idx of a 2^R table
//     sits in lane idx & 63 of register idx >> 6, so a lookup is
//     s_set_gpr_idx (dynamic register) + v_readlane -- no LDS round trip on
//     the symbol chain.  Literal/length root 10 (16 VGPRs), distance root 8
//     (4 VGPRs), code-length root 7 (2 VGPRs); longer codes take a canonical
//     slow path with per-length (first, count, offset) kept in LDS;
//   * LDS holds the window as a ring (back-references are lane-parallel LDS
//     copies; older bytes are read back from dst) and the canonical symbol
//     order the table builds need.  Three instantiations by batch size:
//     32 KiB ring at 4 streams per CU, 16 KiB at 8, 8 KiB at 16;
//   * input: three 1 KiB blocks staged in VGPRs (16 B per lane, coalesced
//     buffer loads issued one block ahead of use); the bit reader gathers
//     dwords with v_readlane;
//   * output leaves the ring in batches of 16-B stores (8 KiB; 4 KiB for the
//     8 KiB ring), lagging the decode by less than the ring size;
//   * table builds are wave-parallel: ballot counts, ballot-ranked
//     canonical order, every lane decodes its own LUT indices.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/zcrc.h"
#include "zcrc_internal.h"
#include "zcrc_inflate_internal.h"

#ifdef ZCRC_INFLATE_TRACE
#define ITRACE(...) do { if (threadIdx.x == 0 && blockIdx.x < 4) printf(__VA_ARGS__); } while (0)
#else
#define ITRACE(...) do { } while (0)
#endif

namespace zcrc {
namespace w16 {  // 16 KiB ring: eight streams per CU, far matches read back from dst
#define ZI_WIN 16384u
#include "zcrc_inflate_impl.h"
#undef ZI_WIN
}  // namespace w16
namespace w8 {  // 8 KiB ring, sixteen streams per CU (four waves per SIMD)
#define ZI_WIN 8192u
#ifndef ZI_W8_WPE
#define ZI_W8_WPE 4
#endif
#define ZI_WPE ZI_W8_WPE
#include "zcrc_inflate_impl.h"
#undef ZI_WPE
#undef ZI_WIN
}  // namespace w8
namespace w32 {  // the whole 32 KiB window in LDS: four streams per CU
#define ZI_WIN 32768u
#include "zcrc_inflate_impl.h"
#undef ZI_WIN
}  // namespace w32
// speculative chunk decode (16-bit elements, zcrc_inflate_split.hip): the
// whole 32 Ki-element history in LDS (two streams per CU, no reads of older
// output back from HBM -- on text ~13% of the matches reach past 16 Ki), or
// a 16 Ki-element ring at four per CU for streams with more chunks than
// that many resident decoders
namespace sp32 {
#define ZI_WIN 32768u
#define ZI_SPEC 1
#include "zcrc_inflate_impl.h"
#undef ZI_SPEC
#undef ZI_WIN
}  // namespace sp32
namespace sp16 {
#define ZI_WIN 16384u
#define ZI_SPEC 1
#include "zcrc_inflate_impl.h"
#undef ZI_SPEC
#undef ZI_WIN
}  // namespace sp16

hipError_t launch_inflate_spec(const SpecArgs &args, bool wide, hipStream_t stream) {
  return wide ? sp32::launch_spec(args, stream) : sp16::launch_spec(args, stream);
}
hipError_t launch_inflate_probe(const SpecArgs &args, hipStream_t stream) { return sp16::launch_probe(args, stream); }

// Longest-first dispatch.  Workgroups start in index order, so when a batch
// has more streams than can be resident, a slow stream that happens to sit
// at the end of the batch starts last and finishes alone.  Decode time
// tracks the compressed size, so one workgroup counting-sorts the streams
// by quarter-octave of src_len, largest first (order within a bucket is
// arbitrary; every stream's result is its own).
__global__ __launch_bounds__(1024) void inflate_order_kernel(const uint64_t *src_len, uint64_t n, uint32_t *order) {
  constexpr int kBuckets = 4 * 40;  // quarter octaves up to 2^40
  __shared__ uint32_t cnt[kBuckets];
  for (int b = threadIdx.x; b < kBuckets; b += blockDim.x) cnt[b] = 0;
  __syncthreads();
  auto bucket = [&](uint64_t len) -> int {  // descending: bucket 0 holds the largest
    if (len < 2) return kBuckets - 1;
    const int lg = 63 - __builtin_clzll(len);
    const int q = lg >= 2 ? (int)((len >> (lg - 2)) & 3u) : 0;
    const int k = 4 * (lg < 39 ? lg : 39) + q;
    return kBuckets - 1 - k;
  };
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(&cnt[bucket(src_len[i])], 1u);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t run = 0;
    for (int b = 0; b < kBuckets; b++) {
      const uint32_t c = cnt[b];
      cnt[b] = run;
      run += c;
    }
  }
  __syncthreads();
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) order[atomicAdd(&cnt[bucket(src_len[i])], 1u)] = (uint32_t)i;
}

// Up to four streams per CU all fit at once with the full window (no reads
// back from dst: text-like streams decode ~20% faster); up to eight take
// the 16 KiB ring (profiles/r01/v8); larger batches take the 8 KiB ring at
// sixteen streams per CU -- more waves to hide the scalar dependency chains:
// binary-like streams +32%, text-like -4% from the extra reads back from
// dst (profiles/r01/v9) -- and are dispatched longest-first.
hipError_t launch_inflate(const InflateArgs &args, int num_cus, hipStream_t stream, uint32_t *order_scratch) {
  if (args.n == 0) return hipSuccess;
  if (args.n <= 4ull * (uint64_t)num_cus) return w32::launch(args, stream);
  InflateArgs a = args;
  if (order_scratch && args.n > 8ull * (uint64_t)num_cus && args.n <= 0xFFFFFFFFull) {  // queued streams
    hipLaunchKernelGGL(inflate_order_kernel, dim3(1), dim3(1024), 0, stream, args.src_len, args.n, order_scratch);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    a.order = order_scratch;
  }
  if (args.n > 8ull * (uint64_t)num_cus) return w8::launch(a, stream);
  return w16::launch(a, stream);
}

}  // namespace zcrc
