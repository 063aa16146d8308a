/*
 * zcrc.h -- C ABI of libzcrc, the MI355X batched CRC-32 engine for ZIPsFS.
 *
 * Drop-in boundary.  ZIPsFS computes the CRC of a fully preloaded ZIP entry
 * with the *static* function
 *     static uint32_t cg_crc32(const void *data, size_t n_bytes, uint32_t crc,
 *                              pthread_mutex_t *mutex);          src/cg_crc32.c:26
 * textually included by src/ZIPsFS_preloadfileram.c:11 and called once, in
 * fhandle_check_crc32 (src/ZIPsFS_preloadfileram.c:243).  The replacement
 * zipsfs_amd/cg_crc32.c keeps that exact static signature and include guard
 * and forwards to zcrc32() below (INTEGRATION.md shows the one-line build
 * change).  Everything else here is new surface with no reference caller:
 * batched host- and device-resident entry points and the GF(2) combine.
 *
 * Semantics of every CRC entry point: zlib crc32(crc, data, n) -- CRC-32/
 * ISO-HDLC, reflected poly 0xEDB88320, pre/post inverted, `crc` is the value
 * of a previous call (0 for a fresh CRC) -- bit-exact to src/cg_crc32.c.
 *
 * Errors.  The reference has no error path (src/cg_crc32.c always returns).
 * Every batched and device-resident entry point computes on the GPU only;
 * functions returning int return 0 on success and a negative code on
 * failure (zcrc_last_error() gives the text), never a CPU answer.  The one
 * exception is the drop-in zcrc32(), which like cg_crc32 cannot fail: see
 * "Drop-in contract" below.
 *
 * Threading: all functions are thread-safe; device initialisation happens
 * once per process (pthread_once semantics).  Host-pointer functions are
 * synchronous.  Device-pointer functions are asynchronous on `stream`
 * (a hipStream_t passed as void*, NULL = default stream).
 */
#ifndef ZCRC_H
#define ZCRC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZCRC_OK 0
#define ZCRC_ERR_HIP (-1)      /* HIP runtime error (no device, launch, copy) */
#define ZCRC_ERR_ARG (-2)      /* invalid argument                              */
#define ZCRC_ERR_TOO_BIG (-3)  /* one launch limited to 4 TiB of payload        */

/* Replaces cg_crc32(data, n_bytes, crc, mutex), src/cg_crc32.c:26.
 * `data` is host memory, borrowed for the call.
 *
 * Drop-in contract: zcrc32 never fails and never aborts -- the
 * caller holds mutex_fhandle (src/ZIPsFS_preloadfileram.c:309-321).  Entries
 * of at least zcrc32_set_gpu_min_bytes() bytes (env ZCRC_GPU_MIN_BYTES; the
 * default is the measured host/GPU crossover) are checksummed
 * on the GPU; smaller ones, calls that find every staging slot busy (the
 * drop-in never waits for nor creates staging: the caller holds the lock;
 * see zcrc32_prewarm), and any call
 * whose GPU attempt fails (no device, HIP error) are answered by libzcrc's
 * own host CRC-32 (PCLMUL folding, zcrc_host.cpp).  The first fallback is
 * reported on stderr; all are counted by zcrc32_dropin_stats. */
uint32_t zcrc32(const void *data, size_t n_bytes, uint32_t crc);
/* Sets the drop-in's GPU threshold (bytes); returns the previous value. */
size_t zcrc32_set_gpu_min_bytes(size_t min_bytes);
/* Drop-in calls so far: answered on the GPU / on the host below the
 * threshold / on the host after a GPU failure.  Any pointer may be NULL. */
void zcrc32_dropin_stats(uint64_t *gpu_calls, uint64_t *host_calls, uint64_t *fallback_calls);

/* The GPU path of zcrc32 alone: reports failure instead of answering from
 * the host (ZCRC_ERR_*), whatever the size. */
int zcrc32_checked(const void *data, size_t n_bytes, uint32_t crc, uint32_t *out_crc);

/* Host-resident batch: out[i] = crc32(seeds ? seeds[i] : 0, ptrs[i], lens[i]).
 * Buffers are staged through pinned memory and checksummed on the GPU in
 * as few launches as fit the staging area.  flags: reserved, pass 0.
 * Staging: a process-wide pool of 16 MiB pinned + 16 MiB HBM slots, at most
 * ZCRC_STAGING_MIB (env, default 256) of each per device.  A call leases one
 * slot (waiting while none is free, at most 10 s: then ZCRC_ERR_HIP) plus a
 * second if one is free, and returns them before it returns; streams hold
 * theirs from the first update() to final(). */
int zcrc32_batch(const void *const *ptrs, const size_t *lens, const uint32_t *seeds_or_null,
                 uint32_t *out, size_t n, unsigned flags);

/* Device-resident batch.  d_ptrs: device array of n device pointers;
 * d_lens: device array of n byte counts; d_seeds_or_null: device array or
 * NULL; d_out: device array of n results.  Asynchronous on `stream`; its
 * scratch (work counter, length prefix, plan tile sums: 256 + 8*(n+1) +
 * 8*ceil(n/8192) bytes; above 8192 buffers the split plan's layout instead,
 * 16*n + (320 + 24*n + 112*T rounded up to 16) bytes with T = ceil(n/(1024*p))
 * tiles, p the smallest of 1, 2, 4, 8 for which T <= 256) is a grow-only
 * buffer from a cache, leased per call and never shared between streams
 * (keyed by handle and, where the runtime has it, hipStreamGetId: a recycled
 * handle gets fresh scratch), so streams may be created and destroyed
 * freely; idle entries above ZCRC_SCRATCH_CACHE_MIB (default 2048) per
 * device are freed by a library thread, after a device synchronize and 2 s
 * idle, never on the caller's call (calls under graph capture take
 * stream-ordered allocations instead; a process that captures graphs in
 * global mode while streams come and go should raise the budget or call
 * zcrc_release_cached outside capture, since that synchronize is
 * device-wide: measured, ~30 trims invalidated 8 of ~790 global-mode captures
 * held open next to them, with or without the library thread in relaxed
 * capture mode; without trims none).  To read the results of work queued on a stream that is then
 * destroyed, wait on an event recorded before the destroy: on ROCm 7.2 a
 * plain-HIP reproducer read the last kernel's store of a destroyed stream
 * after hipStreamDestroy and hipDeviceSynchronize had returned, and found it
 * there 200 ms later (5 reads in 1,400).  Above 8192
 * buffers the plan may
 * split the batch on the device: when buffers of at most 8 KiB are worth at
 * least two of the CRC kernel's workgroups, some workgroups of the same
 * launch run the small-buffer body on them (ZCRC_SMALL=0 in the environment:
 * never; =2: whenever there is one). */
int zcrc32_batch_device(const void *const *d_ptrs, const uint64_t *d_lens,
                        const uint32_t *d_seeds_or_null, uint32_t *d_out, size_t n, void *stream);

/* Same, with a bound the caller knows for every length (max_len >= every
 * d_lens[i]; 0 = unknown) -- ZIPsFS knows its entries' sizes from the
 * central directory.  With max_len <= 8192 and more than 8192 buffers the
 * batch runs in ONE small-buffer kernel launch over the caller's arrays
 * (8 lanes per buffer up to 2 KiB, else 16), without the split plan's scans
 * and scratch; otherwise exactly zcrc32_batch_device.  Results never depend
 * on max_len: a longer buffer is still checksummed right, only slower.  Best
 * for batches of about equal lengths (each wave takes 4 or 8 buffers in
 * index order). */
int zcrc32_batch_device_maxlen(const void *const *d_ptrs, const uint64_t *d_lens,
                               const uint32_t *d_seeds_or_null, uint32_t *d_out, size_t n, uint64_t max_len,
                               void *stream);

/* Same, with caller-owned scratch (graph-capturable: no allocation inside).
 * Needs zcrc32_batch_device_scratch_bytes(n) bytes of device memory,
 * 256-byte aligned for best performance.  One scratch per in-flight call. */
size_t zcrc32_batch_device_scratch_bytes(size_t n);
int zcrc32_batch_device_ws(const void *const *d_ptrs, const uint64_t *d_lens,
                           const uint32_t *d_seeds_or_null, uint32_t *d_out, size_t n,
                           void *d_scratch, size_t scratch_bytes, void *stream);

/* Integrity check of the last zcrc32_batch_device / _ws launch on a scratch
 * (d_scratch, or NULL for the cached scratch of the most recently finished
 * zcrc32_batch_device call on `stream` -- scratch never changes streams; with
 * two calls on one stream in flight at once it may be either's, and with
 * none idle *faults is 0): synchronizes `stream`
 * and sets *faults nonzero when the CRC kernel found inconsistent length-
 * prefix bounds in the scratch (a corrupted scratch -- e.g. written by
 * another stream -- makes the kernel skip those buffers, with result 0,
 * instead of reading outside them).  Batches of at most 16 x CUs buffers use
 * no prefix and report 0. */
int zcrc32_batch_device_faults(const void *d_scratch_or_null, void *stream, uint32_t *faults);

/* Device-resident batch of equal-size chunks: buffer i = d_base + i*stride,
 * each `len` bytes (fixed-size cache chunks).  One launch per 4 TiB, plus a
 * memset of d_out when chunks may be split across waves and, for batches of
 * >= 1 GiB, a 256-byte stream-ordered allocation for the work counter. */
int zcrc32_batch_device_strided(const void *d_base, uint64_t stride, uint64_t len, size_t n,
                                const uint32_t *d_seeds_or_null, uint32_t *d_out, void *stream);

/* Batched raw-DEFLATE decode on the GPU.  ZIP method 8
 * entries are what libzip/zlib inflate under zip_fread() in preloadram_now
 * (src/ZIPsFS.c:2016-2019, src/ZIPsFS_preloadfileram.c:286-306); the format
 * is RFC 1951 and streams are accepted exactly when zlib 1.2.11 accepts them.
 * All pointers are device arrays of n entries: d_src/d_src_len the
 * compressed streams (< 3.75 GiB each), d_dst/d_cap the output buffers,
 * d_out_len the bytes produced (0 unless ok), d_status a ZCRC_INFLATE_* per
 * stream.  One workgroup per stream; asynchronous on `stream`.  Returns
 * ZCRC_OK when the launch was queued (per-stream results are in d_status). */
#define ZCRC_INFLATE_OK 0
#define ZCRC_INFLATE_ERR_BLOCK_TYPE 1  /* block type 3                             */
#define ZCRC_INFLATE_ERR_STORED_LEN 2  /* stored block LEN != ~NLEN                 */
#define ZCRC_INFLATE_ERR_CODES 3       /* invalid dynamic header / code lengths     */
#define ZCRC_INFLATE_ERR_SYMBOL 4      /* invalid literal/length or distance code   */
#define ZCRC_INFLATE_ERR_DIST 5        /* distance too far back                     */
#define ZCRC_INFLATE_ERR_OUTPUT 6      /* output larger than d_cap                  */
#define ZCRC_INFLATE_ERR_INPUT 7       /* input ends before the final block         */
#define ZCRC_INFLATE_ERR_TOO_BIG 8     /* compressed stream of 3.75 GiB or more     */
int zcrc_inflate_batch_device(const void *const *d_src, const uint64_t *d_src_len, void *const *d_dst,
                              const uint64_t *d_cap, uint64_t *d_out_len, int32_t *d_status, size_t n,
                              void *stream);
/* ONE raw-DEFLATE stream in device memory, decoded by many waves at once
 * (block-parallel, speculative: DESIGN.md section 11b).  ZIPsFS preloads one
 * deflated entry at a time (zip_fread() in preloadram_now,
 * src/ZIPsFS_preloadfileram.c:286-306), which the batch call above would
 * decode on a single wave.  The compressed bytes are cut into chunks of
 * chunk_bytes (0: 8 KiB, grown to fill the resident decoders and so that
 * there are at most 16,384); each chunk
 * decodes from the first valid block header in it with an unknown history,
 * the chunks reachable from the stream's start are stitched together, and
 * when that fails (corrupt data, a chunk's output far above the average
 * ratio) the stream is decoded serially, with zlib's status.  Same results
 * as zcrc_inflate_batch_device for one stream (*d_out_len, *d_status).
 * Scratch: about 6 x cap bytes of HBM plus ~288 KiB per decode item (two
 * 128 KiB history windows and slack; items = chunks x parts, at most 16,384),
 * kept per HIP stream.  Not graph-capturable (ZCRC_ERR_ARG under capture).
 * Asynchronous. */
int zcrc_inflate_device(const void *d_src, uint64_t src_len, void *d_dst, uint64_t cap, uint64_t *d_out_len,
                        int32_t *d_status, uint64_t chunk_bytes, void *stream);
/* Same for host memory, plus the CRC-32 of every output: the preload of a
 * deflated entry (raw stream via libzip ZIP_FL_COMPRESSED) inflated and
 * checksummed in one call.  Streams are packed into pinned staging, inflated
 * and checksummed on the GPU and copied back; synchronous.  out_len[i] = 0 and
 * crc_or_null[i] = 0 unless status[i] == ZCRC_INFLATE_OK.  flags: pass 0.
 * The calling thread keeps its device buffer (inputs | outputs | descriptors)
 * for its next call when it is at most 1 GiB, as zcrc_zip_verify_host keeps
 * its image and arena buffers (at most 1 GiB each); larger ones are freed on
 * return. */
int zcrc_inflate_batch(const void *const *src, const size_t *src_len, void *const *dst, const size_t *cap,
                       size_t *out_len, int32_t *status, uint32_t *crc_or_null, size_t n, unsigned flags);

/* Streaming / incremental CRC.  ZIPsFS fills a preload
 * buffer in <= 16 MiB zip_fread() chunks (src/ZIPsFS_preloadfileram.c:286-306)
 * and only then CRCs the whole entry under mutex_fhandle (:309-321).  A
 * stream checksums each chunk as it lands: update() enqueues the chunk's H2D
 * copy and kernel on the stream's own HIP stream (the running CRC stays on
 * the device), so the GPU work overlaps the next inflate; final() waits and
 * returns crc32(seed, all bytes so far).  One thread at a time per stream;
 * streams are independent.
 *
 * zcrc32_stream_open_registered(seed, segment, bytes) also page-locks the
 * caller's preload segment (ZIPsFS: the entry's textbuffer segment,
 * src/cg_textbuffer.c:103-106) until close(): the kernels read chunks inside
 * it over PCIe straight from it, and update() returns at once, without
 * copying (the update that completes the segment waits for its kernels, so
 * that final() -- under the caller's lock -- has nothing left to wait for).
 * The segment must stay mapped, and its updated bytes unchanged, until
 * close().  If the segment cannot be registered the stream works as an
 * unregistered one.  Without registration update() copies each piece into a
 * pinned staging slot, which the kernel reads over PCIe (never waiting for a
 * slot: with every slot of the pool leased, the HIP runtime copies from the
 * pageable source into HBM itself).  Errors are sticky: after a
 * failed update() every later update() and final() return that error until
 * the stream is closed; a partial CRC is never returned. */
typedef struct zcrc32_stream zcrc32_stream;
zcrc32_stream *zcrc32_stream_open(uint32_t seed);            /* NULL on failure */
zcrc32_stream *zcrc32_stream_open_registered(uint32_t seed, const void *segment, size_t segment_bytes);
int zcrc32_stream_update(zcrc32_stream *s, const void *data, size_t n_bytes);
int zcrc32_stream_final(zcrc32_stream *s, uint32_t *crc);      /* stream stays usable */
void zcrc32_stream_close(zcrc32_stream *s);
/* How the stream's 4 MiB pieces went to the GPU: read from the registered
 * segment / copied through pinned staging / runtime-staged pageable copy (no
 * slot was free).  Every piece is checksummed on the GPU. */
int zcrc32_stream_stats(const zcrc32_stream *s, uint64_t *registered_pieces, uint64_t *staged_pieces,
                        uint64_t *pageable_pieces);

/* Device initialisation plus up to `staging_slots` pinned staging slots per
 * logical device of the set (zcrc_device_set), created now and exercised by two staged calls (~20 ms once; the HIP
 * runtime's first few SDMA copies of a process can block their caller for
 * milliseconds) -- call it at startup (ZIPsFS: before the preload threads),
 * outside any lock.  The drop-in never creates a slot itself (it runs under
 * mutex_fhandle): a call that finds none free answers from the host CRC and
 * a background thread creates one for the next call. */
int zcrc32_prewarm(size_t staging_slots);

/* Batched ZIP verification.  ZIPsFS takes each
 * entry's expected CRC from the central directory (libzip zip_stat, st.crc:
 * src/ZIPsFS.c:998; exposed as <entry>@ARCHIVECRC32.TXT,
 * src/ZIPsFS_special_file.c:155-163) and checks it after a full preload.
 * zcrc_zip_scan parses the central directory of an archive image (ZIP64
 * included) on the host; zcrc_zip_verify_* checksum the data of every
 * stored (method 0) entry in ONE batched GPU launch, inflate every deflated
 * (method 8) entry on the GPU (one launch per <= 16 GiB of output) and
 * checksum the outputs in one more, and compare.  Encrypted entries and
 * other methods are reported as UNVERIFIED. */
#define ZCRC_ZIP_OK 1
#define ZCRC_ZIP_MISMATCH 0             /* CRC-32 or uncompressed size differs        */
#define ZCRC_ZIP_UNVERIFIED (-1)        /* encrypted or other method: not checked     */
#define ZCRC_ZIP_BAD (-2)               /* local header or data range outside archive */
#define ZCRC_ZIP_INFLATE_ERROR (-3)     /* deflate stream invalid (see inflate_status) */
typedef struct zcrc_zip_entry {
  uint64_t data_offset;  /* first byte of the entry's stored data in the archive */
  uint64_t comp_size;    /* bytes of entry data in the archive */
  uint64_t uncomp_size;
  uint64_t name_offset;  /* file name (central directory copy) in the archive */
  uint32_t name_len;
  uint32_t crc_expected; /* central directory CRC-32 */
  uint32_t crc_computed; /* set by zcrc_zip_verify_* (stored and deflated entries) */
  uint16_t method;       /* 0 stored, 8 deflate, ... */
  uint16_t flags;        /* general purpose bit flags */
  int32_t status;        /* ZCRC_ZIP_* */
  int32_t inflate_status; /* ZCRC_INFLATE_* for deflated entries, else 0 */
} zcrc_zip_entry;

/* Parse the central directory.  entries may be NULL to count; *n_entries
 * receives the number of entries (even when it exceeds `capacity`). */
int zcrc_zip_scan(const void *archive, size_t archive_len, zcrc_zip_entry *entries, size_t capacity,
                  size_t *n_entries);
/* Verify with the archive image in host memory (staged to HBM once). */
int zcrc_zip_verify_host(const void *archive, size_t archive_len, zcrc_zip_entry *entries, size_t n);
/* Verify with the archive image resident in device memory (d_archive);
 * synchronous on `stream`. */
int zcrc_zip_verify_device(const void *d_archive, size_t archive_len, zcrc_zip_entry *entries, size_t n,
                           void *stream);

/* Stored-entry extraction: what zip_fread() delivers for
 * a method-0 entry in preloadram_now (src/ZIPsFS_preloadfileram.c:286-288),
 * plus the check fhandle_check_crc32 makes on it (:237-250), for a batch.
 * For every entries[i] (from zcrc_zip_scan) that is stored, unencrypted, in
 * range and fits dst[i] (cap[i] >= comp_size; dst[i] may be NULL for an
 * empty entry), the entry's bytes are copied
 * into dst[i] and the CRC-32 of the copy is compared with the central
 * directory's: status ZCRC_ZIP_OK or ZCRC_ZIP_MISMATCH, crc_computed set.
 * Other entries are not copied and come back ZCRC_ZIP_UNVERIFIED (BAD stays
 * BAD).  _device: d_archive and d_dst[i] are device memory (d_dst itself is a
 * host array); one batched copy launch and one batched CRC launch on
 * `stream`, synchronous.  _host: host memory; the copy is a host memcpy and
 * the CRCs one zcrc32_batch call over the copies. */
int zcrc_zip_extract_stored_device(const void *d_archive, size_t archive_len, zcrc_zip_entry *entries,
                                   void *const *d_dst, const size_t *cap, size_t n, void *stream);
int zcrc_zip_extract_stored_host(const void *archive, size_t archive_len, zcrc_zip_entry *entries,
                                 void *const *dst, const size_t *cap, size_t n);

/* GF(2) algebra (pure integer math, no data access):
 * crc32(A||B) == zcrc32_combine(crc32(A), crc32(B), |B|)   (zlib semantics). */
uint32_t zcrc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);

/* Synthetic payload (bench/test data, not a CRC path): fills device buffer
 * d_ptrs[i] (d_lens[i] bytes) with the counter-based payload of SURVEY.md
 * 8(d) for payload index index0 + i*index_step:
 *   word j = splitmix64(seed ^ (index << 32 | j)), little-endian. */
int zcrc_fill_synthetic(const uint64_t *d_ptrs, const uint64_t *d_lens, size_t n, uint64_t index0,
                        uint64_t index_step, uint64_t seed, void *stream);

/* Memory the library keeps between calls: the calling thread's device
 * buffers of zcrc_inflate_batch and the ZIP entry points (kept up to 1 GiB
 * each per purpose, at most ZCRC_TL_CACHE_MIB -- default 8192 -- per device
 * over all threads), and every device's idle cached scratch of the
 * device-pointer calls.  zcrc_release_cached frees them (the pinned staging
 * pool stays); *freed_bytes (may be NULL) = device bytes freed.
 * zcrc_cache_info reports device `dev`'s cached scratch entries and bytes and
 * the thread-local bytes kept there by all threads. */
int zcrc_release_cached(uint64_t *freed_bytes);
int zcrc_cache_info(int dev, uint64_t *scratch_entries, uint64_t *scratch_bytes, uint64_t *thread_local_bytes);

/* Measurement only: the same launches as zcrc32_batch_device (same plan,
 * same workgroups, same loads, same fold) with every table lookup of the
 * hot loop replaced by one VALU rotate -- the same-shape read ceiling the
 * CRC rate is judged against (bench.py roofline.read_ceiling).  d_out does
 * NOT receive CRCs. */
int zcrc32_batch_device_read_ceiling(const void *const *d_ptrs, const uint64_t *d_lens, uint32_t *d_out, size_t n,
                                     void *stream);
/* Measurement only: the chip's stream-read peak over the same bytes -- one
 * plain grid-stride read of the contiguous device region [d_base, d_base +
 * bytes) (16-byte aligned; a final < 16 B is not read), non-temporal 16-B
 * loads, no CRC and no per-buffer structure (bench.py
 * roofline.stream_read_gbs).  d_sink: device memory of at least 4096 bytes,
 * written only in a case that does not matter (it keeps the loads alive).
 * Asynchronous on `stream`. */
int zcrc_read_sweep_device(const void *d_base, uint64_t bytes, uint32_t *d_sink, void *stream);

/* Diagnostics / measurement. */
/* Host staging pool: pinned bytes allocated (all devices), slots leased now,
 * most slots ever leased at once, and the per-device slot budget. */
int zcrc_staging_info(uint64_t *pinned_bytes, uint64_t *slots_in_use, uint64_t *slots_peak, uint64_t *slots_budget);
const char *zcrc_last_error(void);
const char *zcrc_version(void);
/* The batched CRC kernel the device entry points launch, as rocprofv3 names it. */
const char *zcrc_kernel_name(void);
/* The batched CRC kernel zcrc32_batch_device launches for a batch of n
 * buffers: the one-launch form for n <= 16 x CUs (ZCRC_FUSED), else the
 * two-launch form above. */
const char *zcrc_kernel_name_for(size_t n);
/* The small-buffer kernel the general-form device entry points launch. */
const char *zcrc_small_kernel_name(void);
int zcrc_device_info(int *num_cus, int *arch_major, int *arch_minor);
/* The device set the host-memory entry points spread over (zcrc32,
 * zcrc32_checked, zcrc32_batch, zcrc32_stream_open*, zcrc_inflate_batch,
 * zcrc_zip_verify_host): env ZCRC_DEVICES (read once; comma-separated HIP
 * device indices, repeats allowed), default every visible gfx950.  A host
 * call of T bytes runs on min(devices, T / ZCRC_SHARD_MIN_BYTES) of them
 * (default 8 MiB per device; at least 1, the least loaded): buffers are cut
 * into byte-balanced shards, one per device, and a buffer cut at a shard
 * boundary is reassembled with the GF(2) combine.  A stream lives on the
 * least loaded device when opened.  Device-pointer entry points use the
 * caller's current device.  Writes up to `capacity` indices; *n = set size. */
int zcrc_device_set(int *devices, size_t capacity, size_t *n);
/* The shard plan of a host batch (no device needed): with lens[0..n) cut
 * into `shards` byte-balanced shards, buffer i starts in shard first[i] and
 * has pieces[i] pieces (its later pieces open the following shards);
 * shard_bytes[g] = bytes of shard g.  Any output may be NULL. */
int zcrc_shard_plan(const size_t *lens, size_t n, size_t shards, uint32_t *first, uint32_t *pieces,
                    uint64_t *shard_bytes);
/* When enabled, each device launch of the CRC kernels is timed by
 * timestamps of its own dispatch packet; zcrc_profile_read returns the
 * summed milliseconds and launch count of the batch kernel since the last
 * reset, zcrc_profile_read_kind the same for kind 0 (batch kernel) or 1
 * (small-buffer kernel, zcrc_small_kernel_name()). */
void zcrc_profile_enable(int on);
int zcrc_profile_read(double *total_ms, int *launches);
int zcrc_profile_read_kind(int kind, double *total_ms, int *launches);
void zcrc_profile_reset(void);

#ifdef __cplusplus
}
#endif
#endif /* ZCRC_H */
