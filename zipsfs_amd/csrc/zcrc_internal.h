// zcrc_internal.h -- shared constants and launch interfaces (not public ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace zcrc {

constexpr int kWaves = 16;                     // waves per workgroup (one WG per CU)
constexpr int kThreads = kWaves * 64;          // 1024
// 1 KiB blocks per register group (two groups in flight per wave).  Round 5:
// 2 instead of 4 -- same box, three interleaved pairs of bench runs per
// config: config 3 10.17 -> 10.05 ms, config 4 2.000 -> 1.983, config 2 48.4
// -> 47.9 us (profiles/r05/depth_ab/); a plain sweep of the same region reads
// fastest with few loads in flight per wave (profiles/r05/read_patterns/)
#ifndef ZCRC_DEPTH
#define ZCRC_DEPTH 2
#endif
constexpr uint32_t kDepth = ZCRC_DEPTH;
constexpr uint64_t kMinRange = 64ull << 10;    // default minimum bytes per wave range
constexpr uint64_t kSplitGrain = 64ull << 10;  // split points: end-relative multiples
constexpr uint64_t kSplitMin = 2 * kSplitGrain;  // buffers below this are never split
constexpr uint64_t kMinPiece = 4096;           // no split piece shorter than this
constexpr uint64_t kDynUnit = 128ull << 10;    // dynamic-half unit (nominal bytes)
constexpr uint32_t kDynAuto = 0xFF;            // dyn_shift: choose by mean buffer size
constexpr uint32_t kDynShift = kDynAuto;       // dynamic part = total >> shift
constexpr uint64_t kDynSmallAvg = 512ull << 10;  // mean below: half dynamic, else a quarter
constexpr size_t kCtrBytes = 256;              // work counter, own cache lines
constexpr uint32_t kLdsBytes = 163840;         // all 160 KiB of the CU's LDS
constexpr uint32_t kLdsCombDword = 32768;      // combine tables start at 128 KiB
constexpr uint32_t kPlanPerThread = 8;
constexpr bool kWindowed = true;       // piece descriptors fetched 64 at a time
constexpr uint64_t kFusedMaxN = 8192;  // one-launch small batches: the kernel scans the lengths itself
constexpr uint64_t kPerBufMax = kMinRange;  // one-launch batches of buffers up to this: one wave per buffer
// the per-buffer mode's form in the product (crc32_batch_kernel's kPB): 15 =
// the first payload loads ahead of the table build, priority by progress
// (round 4: 45.7-46.3 us against 46.6-47.1 for 4 on config 2, two boxes;
// tools/c2_probe, profiles/r04/s7, s8)
constexpr int kPerBufForm = 15;
constexpr uint64_t kPlanTile = 1024 * kPlanPerThread;
// one launch covers at most this many bytes (keeps every piece < 2 GiB)
constexpr uint64_t kMaxLaunchBytes = 1ull << 42;

// Multiply-by-constant tables, uploaded once per device (~110 KiB).
struct TableBlob {
  uint32_t braid[4 * 256];       // MCT(x^(8*1024)): the hot-loop table
  uint32_t comb[8 * 4 * 256];    // x^-32, x^-64, x^-128 .. x^-4096 (combine tree)
  uint32_t tshift[16 * 4 * 256]; // x^(-8t), t = 0..15 (16-B alignment padding)
  uint32_t stdtab[256];          // standard byte table (buffers < 4 bytes)
  uint32_t x8pow[64];            // x^(8 * 2^k)
  uint32_t braid256[4 * 256];    // MCT(x^(8*256)): the small-buffer kernel's table
  uint32_t xinv8[256];           // r * x^-8 = (r << 8) ^ xinv8[r >> 24] (one zero byte taken off)
  uint32_t x8grain[4][256];      // x^(8 * 65536 * m * 256^j): a split piece's shift by whole 64 KiB grains
  uint32_t braid128[4 * 256];    // MCT(x^(8*128)): the small-buffer kernel's table for 128-B blocks
};

struct BatchArgs {
  // general form: device array of device pointers + exclusive prefix of lens
  const uint8_t *const *ptrs;
  const uint64_t *prefix;  // n+1 entries
  // strided form: buffer i = base + i*stride, length len
  const uint8_t *base;
  uint64_t stride;
  uint64_t len;
  const uint32_t *seeds;  // nullable: all-zero seeds (fresh CRC)
  uint32_t *out;
  uint64_t n;
  const TableBlob *tab;
  uint64_t min_range;  // bytes per wave at least (0 = kMinRange)
  uint64_t *stamps;    // diagnostic builds only (kStamp): 8 words per wave
  // dynamic part: the last total >> dyn_shift bytes are handed out in units
  // of dyn_unit bytes (0 = kDynUnit) through *ctr, which must be zero at
  // launch; ctr == nullptr or dyn_shift == 0 -> purely static partition
  uint32_t *ctr;
  uint32_t dyn_shift;
  uint64_t dyn_unit;
  uint32_t ab_flags;  // A/B knobs (0 in the product; ZCRC_AB_FLAGS): bit 0 = split shifts bit by bit (rounds
                      // 1-3), bit 2 = the split plan's small-list workgroups do not join the dynamic part,
                      // bit 3 = no window order for equal buffers (BatchView::wp: the round-5 range order),
                      // bits 4-5 = the dynamic share (1: an eighth, 2: half, 3: none; 0: as configured),
                      // bit 6 = chunked window order (the static part in W x ~kWinChunk chunks, round-robin),
                      // bits 7-8 = its chunk kWinChunk >> k
  // fused small batches (kFusedMaxN): lengths to scan in-kernel (the scan is
  // written to `prefix`), split-piece accumulators (n words) and the
  // finished-wave counter; acc, *ctr and *done are zero at launch and left
  // zero by the kernel
  const uint64_t *lens;
  uint64_t *acc;
  uint32_t *done;
  // split plan (launch_plan_split): n_dev[0] is the batch's count (n is only
  // an upper bound; nullptr -> n).  When the plan split the batch
  // (n_dev[2] != 0) the kernel reads ptrs_split/seeds_split and writes buffer
  // i's result to out[oidx[i]]; otherwise ptrs/seeds and out[i].
  const uint64_t *n_dev;
  const uint32_t *oidx;
  const uint8_t *const *ptrs_split;
  const uint32_t *seeds_split;
  const uint4 *sdesc;    // the split plan's small list: SmallArgs::sdesc
  uint32_t *fault;       // nullable: set to nonzero when a piece's prefix bounds are inconsistent
};
constexpr size_t kFaultByte = 192;  // the fault word's offset in a scratch's counter area (kCtrBytes)

// Small-buffer kernel (zcrc_small_kernel.h): whole buffers of at most
// kSmallMax bytes, 8 or 16 lanes per buffer.  General form: entry k of the
// list is buffer j = k with ptrs[j], length lens[j] (or prefix[j+1] -
// prefix[j] when lens is null), seeds[j], out[j] -- or, with sdesc, the
// pointer, length, index j and seed of sdesc[k]; the count is n.  Strided
// form: buffer k = base + k*stride of length len.  The split plan's small
// list (sdesc) runs inside the batch kernel's launch (crc32_batch_kernel,
// BatchArgs::sdesc).
constexpr uint64_t kSmallMax = 8192;
struct SmallArgs {
  const uint8_t *const *ptrs;
  const uint64_t *lens;
  const uint64_t *prefix;
  const uint4 *sdesc;  // split plan: entry k = {pointer | length << 48 (2 words), buffer index, seed}
  const uint8_t *base;
  uint64_t stride;
  uint64_t len;
  const uint32_t *seeds;
  uint32_t *out;
  uint64_t n;
  const uint64_t *n_dev;
  const TableBlob *tab;
};
// lanes: 16 or 8 lanes per buffer (8 pays below ~2 KiB: more buffers in flight)
hipError_t launch_small(const SmallArgs &args, bool strided, int lanes, int num_cus, hipStream_t stream,
                        hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr);
const char *small_kernel_name(int lanes);

// t0/t1: optional events stamped with the kernel's own start and end
// ablate: the read-ceiling variant (table lookups replaced by one VALU op; no CRCs)
hipError_t launch_batch(const BatchArgs &args, bool strided, int num_cus, hipStream_t stream,
                        hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr, bool fused = false, bool ablate = false);
// measurement only: the plain stream read of [d_base, d_base + bytes) (zcrc_read_sweep_device)
hipError_t launch_read_sweep(const void *d_base, uint64_t bytes, uint32_t *d_sink, int num_cus, hipStream_t stream);
inline uint64_t plan_tiles(uint64_t n) { return n == 0 ? 1 : (n + kPlanTile - 1) / kPlanTile; }
const char *product_kernel_name();
const char *fused_kernel_name();
hipError_t launch_plan(const uint64_t *d_lens, uint64_t n, uint64_t *d_prefix, uint64_t *d_tile_sum,
                       uint32_t *d_out, uint32_t *d_ctr, hipStream_t stream);

// Split plan (device batches of more than kFusedMaxN buffers).  When buffers
// of at most kSmallMax bytes are worth at least two of the batch kernel's
// workgroups (zcrc_kernels.hip), they are listed for the small-buffer kernel (sdesc, count counts[1]) and the
// others compacted -- those below kBigMin first, then the others, each in index
// order -- into a batch for the batch kernel (ptrs_c,
// seeds_c, prefix_c, original index oidx, count counts[0]); counts[2] = 1.
// Otherwise prefix_c is the plain prefix of all n buffers, counts = {n, 0,
// 0}.  out[] of the batch kernel's buffers is zeroed.  force: split whenever
// there is a small buffer.  A split batch runs in one batch-kernel launch:
// counts[4] of its `grid` workgroups take the small list.  Scratch layout:
// SplitScratch (zcrc_runtime.hip).
struct SplitPlan {
  const uint8_t *const *ptrs;
  const uint64_t *lens;
  const uint32_t *seeds;  // nullable
  uint64_t n;
  uint64_t *tile_sum;     // kTileWords per tile: medium, big, small bytes, medium | big << 32 counts, small count,
                          // small lengths' sum of squares, buffers whose length differs from lens[0]
  uint64_t *tile_pre;     // kTileWords x (tiles + 1): exclusive tile prefixes + totals (above kPlanDirectTiles)
  uint64_t *prefix_c;     // n + 1
  const uint8_t **ptrs_c;
  uint32_t *seeds_c;      // written when seeds != nullptr
  uint32_t *oidx, *out;
  uint4 *sdesc;           // the small list, one 16-B descriptor per entry (SmallArgs::sdesc)
  uint64_t *counts;       // [0] n_large, [1] n_small, [2] split (1; 2: direct, the small body walks ptrs/lens in
                          // index order), [3] small lanes per buffer, [4] small workgroups, [5] every length
                          // equal (unsplit batches only: the batch kernel's window order, BatchView::wp)
  uint32_t grid;          // the batch kernel's workgroups
  uint32_t small_cost;    // CU time of a small-list byte, in quarters of a batch-kernel byte
  uint32_t force;
  uint32_t *ctr;          // the batch kernel's work counter (zeroed)
  uint64_t big_min;       // on a split, buffers of at least this go after the others (kBigMin)
  uint32_t direct_ok;     // a batch of about equal small buffers may skip the lists (mode 2)
  uint64_t *stamps;       // diagnostics (tools/plan_probe): 8 s_memrealtime stamps per scatter workgroup, or null
};
hipError_t launch_plan_split(const SplitPlan &p, hipStream_t stream);
constexpr uint32_t kSizeClasses = kSmallMax / 256 + 1;  // small list order: 256-B block count
constexpr uint32_t kTileWords = 7;
constexpr uint64_t kWinChunk = 1ull << 20;  // chunked window order (ab_flags bit 6): static chunk size
constexpr uint64_t kBigMin = 1ull << 20;  // split plan: buffers of at least this go last in the batch kernel's order
constexpr uint64_t kPlanDirectTiles = 512;  // up to this many tiles each scatter workgroup sums the tile words itself
// split plan tiles: 1024 x per buffers per plan_split_count / plan_split_scatter
// workgroup, per the smallest of 1, 2, 4, 8 that keeps the tiles within
// kSplitMaxTiles (round 4: config 4's 100k buffers in 98 tiles of 1024 --
// 11.2 us per plan -- instead of 13 of 8192 -- 24.2 us; 1M buffers 20.9 us
// at per 4, 44.6 at per 1, whose 977 tiles go through plan_split_tiles;
// tools/plan_probe, profiles/r04/s6).  The small list is ordered by size
// class tile by tile.
constexpr uint64_t kSplitMaxTiles = 256;
inline uint32_t split_per_thread(uint64_t n) {
  uint32_t per = 1;
  while (per < 8 && (n + 1024ull * per - 1) / (1024ull * per) > kSplitMaxTiles) per *= 2;
  return per;
}
inline uint64_t split_tiles(uint64_t n) {
  const uint64_t t = 1024ull * split_per_thread(n);
  return n == 0 ? 1 : (n + t - 1) / t;
}
constexpr uint32_t kSmallCostDefault = 14;  // 3.5 batch-kernel bytes (zcrc_kernels.hip, plan_split_scatter)

}  // namespace zcrc

namespace zcrc {
// record an error for zcrc_last_error() (this thread) and return `code`
int set_error(int code, const char *msg);

// libzcrc's host CRC-32 (zcrc_host.cpp): zlib crc32(crc, data, n) on the CPU,
// used only by the drop-in zcrc32() (include/zcrc.h, "Drop-in contract")
uint32_t host_crc32(const void *data, size_t n, uint32_t crc);
bool host_crc32_uses_clmul();

hipError_t launch_fill_synthetic(const uint64_t *d_ptrs, const uint64_t *d_lens, uint64_t n, uint64_t index0,
                                 uint64_t index_step, uint64_t seed, hipStream_t stream);
}  // namespace zcrc
