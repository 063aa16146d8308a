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
//   * LDS (~34 KiB, four streams per CU) holds the 32 KiB window as a ring
//     (back-references are lane-parallel LDS copies) and the canonical symbol
//     order the table builds need;
//   * input: three 1 KiB blocks staged in VGPRs (16 B per lane, coalesced
//     buffer loads issued one block ahead of use); the bit reader gathers
//     dwords with v_readlane;
//   * output leaves the ring in 8 KiB batches of 16-B stores, lagging the
//     decode (a byte is overwritten only 32 KiB later);
//   * table builds are wave-parallel: ballot counts, ballot-ranked
//     canonical order, every lane decodes its own LUT indices.
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
namespace w16 {  // 16 KiB ring: eight streams per CU, far matches read back from dst
#define ZI_WIN 16384u
#include "zcrc_inflate_impl.h"
#undef ZI_WIN
}  // namespace w16
namespace w32 {  // the whole 32 KiB window in LDS: four streams per CU
#define ZI_WIN 32768u
#include "zcrc_inflate_impl.h"
#undef ZI_WIN
}  // namespace w32

// Up to four streams per CU all fit at once with the full window (no reads
// back from dst: text-like streams decode ~20% faster); larger batches take
// the 16 KiB ring and twice the streams per CU (profiles/r01/v8).
hipError_t launch_inflate(const InflateArgs &args, int num_cus, hipStream_t stream) {
  if (args.n == 0) return hipSuccess;
  if (args.n <= 4ull * (uint64_t)num_cus) return w32::launch(args, stream);
  return w16::launch(args, stream);
}

}  // namespace zcrc
