// zcrc_inflate_internal.h -- inflate launch interfaces (not public ABI).
// Kept apart from zcrc_internal.h so that inflate edits leave the CRC
// kernels' source hash (zipsfs_amd/crc32.py kernel_source_hash) unchanged.
#pragma once
#include "zcrc_internal.h"

namespace zcrc {

// batched raw-DEFLATE decode (zcrc_inflate.hip): device arrays of n
struct InflateArgs {
  const uint8_t *const *src;
  const uint64_t *src_len;
  uint8_t *const *dst;
  const uint64_t *cap;
  uint64_t *out_len;
  int32_t *status;
  uint64_t n;
  // optional dispatch order (workgroup b decodes stream order[b]); nullptr:
  // stream b.  launch_inflate fills it longest-first when streams queue.
  const uint32_t *order;
  // optional: stream i is decoded only when run_if[i] != 0 (the serial
  // fall-back of the block-parallel decode, zcrc_inflate_split.hip)
  const uint32_t *run_if;
};
// Block-parallel (speculative) inflate of one stream (zcrc_inflate_split.hip;
// the spec is tests/inflate_split_model.py).  Chunk k's decode writes 16-bit
// elements: a byte, or kInflateMarker + w = byte w of the kInflateHist bytes
// before the chunk's first element.
constexpr uint32_t kInflateMarker = 0x8000u;
constexpr uint32_t kInflateHist = 32768u;
constexpr uint64_t kSplitNone = ~0ull;  // no candidate block start in the chunk
constexpr int32_t kSpecSkipped = -1;    // SpecRec::status of an item without work
constexpr int32_t kSpecLanded = 100;    // codes(): stopped on a later part's start (internal)
constexpr uint32_t kMaxParts = 64;      // parts of one block: one lane each (a chunk's first block cut into parts)
constexpr uint32_t kMaxChunkParts = 16; // items per chunk
struct SpecRec {
  uint64_t region;   // element offset of the item's output in the region array
  uint64_t out_len;  // elements produced
  uint64_t end_bit;  // bit position where the decode stopped
  int32_t status;    // ZCRC_INFLATE_*, or kSpecSkipped
  int32_t link;      // the chunk whose candidate it stopped at, -1: none
  uint32_t reach;    // furthest back-reference before its first element (bytes)
  uint32_t final_;   // 1: it decoded the final block
};
struct SpecArgs {
  const uint8_t *src;
  uint64_t src_len;
  const uint64_t *cand;  // per chunk: candidate bit position, or kSplitNone
  SpecRec *rec;          // per item (chunk k, part j) = item k * parts + j
  uint16_t *region;      // item outputs (SpecRec::region); chunk k with a candidate owns
  uint64_t region_elems; // [k parts, k' parts) x region_elems up to the next such chunk k', split among its parts
  uint64_t nchunks;
  uint64_t *part;        // per item: the probed start of part j >= 1 (kSplitNone: none)
  uint32_t parts;        // items per chunk (<= kMaxChunkParts)
  uint32_t probe_tokens;
  uint32_t max_parts;    // parts of one chunk's first block, its own items and those it borrows (<= kMaxParts)
};
constexpr uint64_t kInflateMaxSrc = 0xF0000000ull;  // 32-bit buffer range and block arithmetic
// order_scratch: >= 4 * n bytes of device memory for the dispatch order
// (used when the batch exceeds the streams resident at once; may be null)
hipError_t launch_inflate(const InflateArgs &args, int num_cus, hipStream_t stream, uint32_t *order_scratch);
// wide: the 32 Ki-element-history decoder (kSpecPerCuWide per CU), else the
// 16 Ki-element ring (kSpecPerCu per CU)
hipError_t launch_inflate_spec(const SpecArgs &args, bool wide, hipStream_t stream);
hipError_t launch_inflate_probe(const SpecArgs &args, hipStream_t stream);
constexpr uint64_t kInflateSplitChunk = 8192;   // compressed bytes per chunk (at least; at most 16,384 chunks)
constexpr uint64_t kInflateSplitSlack = 16384;  // elements added to each chunk's region
constexpr uint64_t kInflateSplitMinSrc = 65536; // smaller streams decode serially
// chunk size for a stream (want = 0: the default), the scratch the split
// decode of one stream needs, and the launch chain (zcrc_inflate_split.hip)
struct InflateSplitShape {
  uint64_t chunk;  // compressed bytes per chunk
  bool wide;       // the 32 Ki-element-history decoder
  uint32_t parts;  // items per chunk
};
InflateSplitShape inflate_split_shape(uint64_t src_len, uint64_t cap, uint64_t want, int num_cus);
constexpr uint32_t kSpecPerCu = 4;      // sp16::inflate_spec_kernel workgroups per CU (34.5 KB of LDS each)
constexpr uint32_t kSpecPerCuWide = 2;  // sp32:: (67 KB each)
uint64_t inflate_split_scratch_bytes(uint64_t src_len, uint64_t cap, InflateSplitShape shape);
constexpr uint32_t kInflateProbeTokens = 64;  // tokens a part's probe decodes past its guess
hipError_t launch_inflate_split(const uint8_t *src, uint64_t src_len, uint8_t *dst, uint64_t cap,
                                uint64_t *out_len, int32_t *status, InflateSplitShape shape, void *scratch,
                                int num_cus, hipStream_t stream);
// purposes of the runtime's per-stream scratch cache (zcrc_runtime.hip)
enum ScratchUse { kScratchBatch = 0, kScratchInflateOrder = 1, kScratchFused = 2, kScratchInflateSplit = 3, kScratchStridedCtr = 4 };


}  // namespace zcrc
