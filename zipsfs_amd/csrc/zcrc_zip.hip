// zcrc_zip.hip -- ZIP central-directory scan + batched GPU verification.
//
// The reference gets each entry's expected CRC through libzip (zip_stat,
// st.crc: src/ZIPsFS.c:985-1001) and verifies it only after a full preload
// (src/ZIPsFS_preloadfileram.c:237-250).  Here a whole archive is checked at
// once: the host walks the central directory (APPNOTE 4.3.12/4.3.14/4.3.16,
// ZIP64 4.5.3) and the data of every stored entry -- a plain byte range of the
// archive -- is checksummed by one zcrc32_batch* launch.  Deflated entries
// (method 8, the zip_fread()/zlib path of src/ZIPsFS.c:2016-2019) are
// inflated on the GPU into an HBM arena (zcrc_inflate_batch_device) and the
// outputs checksummed by the same batched CRC kernel.  The scan is bounds
// checked against the image; it never reads outside [archive, archive+len).
//
// Stored-entry extraction replaces the zip_fread() of a
// method-0 entry in preloadram_now (src/ZIPsFS_preloadfileram.c:286-288,
// src/ZIPsFS.c:2014-2019) and the CRC that follows it (:243): the entry's
// bytes are copied into the caller's buffer and the CRC of the copy -- the
// bytes fhandle_check_crc32 would check -- is compared with the central
// directory's, for a whole batch of entries in one copy launch and one CRC
// launch.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/zcrc.h"
#include "zcrc_internal.h"
#include "zcrc_inflate_internal.h"
#include "zcrc_runtime.h"

namespace {

inline uint16_t rd16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }
inline uint32_t rd32(const uint8_t *p) { return (uint32_t)rd16(p) | ((uint32_t)rd16(p + 2) << 16); }
inline uint64_t rd64(const uint8_t *p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }

constexpr uint32_t kSigEocd = 0x06054b50u, kSigZ64Loc = 0x07064b50u, kSigZ64Eocd = 0x06064b50u;
constexpr uint32_t kSigCentral = 0x02014b50u, kSigLocal = 0x04034b50u;

int zfail(const char *msg) { return zcrc::set_error(ZCRC_ERR_ARG, msg); }

// Locate the central directory: (offset, size, entries).
int find_cd(const uint8_t *a, uint64_t len, uint64_t *cd_off, uint64_t *cd_size, uint64_t *count) {
  if (len < 22) return zfail("archive shorter than an end-of-central-directory record");
  const uint64_t lo = len > 22 + 65535 ? len - 22 - 65535 : 0;
  uint64_t e = len - 22;
  for (;; e--) {
    if (rd32(a + e) == kSigEocd && e + 22 + rd16(a + e + 20) <= len) break;
    if (e == lo) return zfail("end-of-central-directory record not found");
  }
  uint64_t n = rd16(a + e + 10), size = rd32(a + e + 12), off = rd32(a + e + 16);
  if (e >= 20 && rd32(a + e - 20) == kSigZ64Loc) {  // ZIP64 locator directly before the EOCD
    const uint64_t z = rd64(a + e - 20 + 8);
    if (len < 56 || z > len - 56 || rd32(a + z) != kSigZ64Eocd)
      return zfail("bad ZIP64 end-of-central-directory record");
    n = rd64(a + z + 32);
    size = rd64(a + z + 40);
    off = rd64(a + z + 48);
  }
  if (off > len || size > len - off) return zfail("central directory outside the archive");
  *cd_off = off;
  *cd_size = size;
  *count = n;
  return ZCRC_OK;
}

}  // namespace

extern "C" int zcrc_zip_scan(const void *archive, size_t archive_len, zcrc_zip_entry *entries, size_t capacity,
                             size_t *n_entries) {
  if (!archive || !n_entries) return zfail("null argument");
  const uint8_t *a = static_cast<const uint8_t *>(archive);
  const uint64_t len = archive_len;
  uint64_t cd_off, cd_size, count;
  int rc = find_cd(a, len, &cd_off, &cd_size, &count);
  if (rc) return rc;
  uint64_t p = cd_off;
  const uint64_t end = cd_off + cd_size;
  size_t k = 0;
  for (uint64_t i = 0; i < count; i++, k++) {
    if (p + 46 > end || rd32(a + p) != kSigCentral) return zfail("bad central directory header");
    const uint8_t *h = a + p;
    const uint16_t flags = rd16(h + 8), method = rd16(h + 10);
    const uint32_t crc = rd32(h + 16);
    uint64_t csize = rd32(h + 20), usize = rd32(h + 24);
    const uint16_t nlen = rd16(h + 28), xlen = rd16(h + 30), clen = rd16(h + 32);
    uint64_t lho = rd32(h + 42);
    if (p + 46 + (uint64_t)nlen + xlen + clen > end) return zfail("central directory entry overruns");
    // ZIP64 extended information: only the fields saturated in the header, in order
    const uint8_t *x = h + 46 + nlen, *xe = x + xlen;
    while (x + 4 <= xe) {
      const uint16_t id = rd16(x), sz = rd16(x + 2);
      if (x + 4 + sz > xe) break;
      if (id == 0x0001) {
        const uint8_t *f = x + 4, *fe = x + 4 + sz;
        if (usize == 0xFFFFFFFFu && f + 8 <= fe) usize = rd64(f), f += 8;
        if (csize == 0xFFFFFFFFu && f + 8 <= fe) csize = rd64(f), f += 8;
        if (lho == 0xFFFFFFFFu && f + 8 <= fe) lho = rd64(f), f += 8;
      }
      x += 4 + sz;
    }
    if (entries && k < capacity) {
      zcrc_zip_entry &E = entries[k];
      memset(&E, 0, sizeof(E));
      E.comp_size = csize;
      E.uncomp_size = usize;
      E.crc_expected = crc;
      E.method = method;
      E.flags = flags;
      E.name_offset = p + 46;
      E.name_len = nlen;
      E.status = ZCRC_ZIP_UNVERIFIED;
      // local header -> data offset
      if (len < 30 || lho > len - 30 || rd32(a + lho) != kSigLocal) {  // lho may be any 64-bit value
        E.status = ZCRC_ZIP_BAD;
      } else {
        const uint64_t d = lho + 30 + rd16(a + lho + 26) + rd16(a + lho + 28);
        if (d > len || csize > len - d) E.status = ZCRC_ZIP_BAD;
        E.data_offset = d;
      }
    }
    p += 46 + (uint64_t)nlen + xlen + clen;
  }
  *n_entries = k;
  return ZCRC_OK;
}

namespace {

// stored, unencrypted, in range, consistent sizes
bool verifiable(const zcrc_zip_entry &E) {
  return E.status != ZCRC_ZIP_BAD && E.method == 0 && !(E.flags & 1u) && E.comp_size == E.uncomp_size;
}
// deflated, unencrypted, in range
bool deflatable(const zcrc_zip_entry &E) { return E.status != ZCRC_ZIP_BAD && E.method == 8 && !(E.flags & 1u); }

constexpr uint64_t kArenaBytes = 16ull << 30;  // inflate output per chunk

// Output room for a deflated entry.  DEFLATE expands at most 1032:1 (a
// 258-byte match in two 1-bit codes), so a stream whose output would exceed
// 1032 * comp_size + 64 bytes does not exist: capping the room there never
// changes a verdict (a larger claimed size cannot be produced and is a
// mismatch), and it keeps a crafted ZIP64 size (up to 2^64) from sizing the
// arena.  Entries whose room exceeds one arena are left UNVERIFIED.
uint64_t inflate_room(const zcrc_zip_entry &E) {
  const uint64_t bound = E.comp_size > (UINT64_MAX - 64) / 1032 ? UINT64_MAX : 1032 * E.comp_size + 64;
  return E.uncomp_size < bound ? E.uncomp_size : bound;
}

void finish(zcrc_zip_entry *entries, const std::vector<size_t> &idx, const std::vector<uint32_t> &crc) {
  for (size_t j = 0; j < idx.size(); j++) {
    zcrc_zip_entry &E = entries[idx[j]];
    E.crc_computed = crc[j];
    E.status = crc[j] == E.crc_expected ? ZCRC_ZIP_OK : ZCRC_ZIP_MISMATCH;
  }
}

// Deflated entries idx[a, b): one inflate launch into an arena, one CRC launch
// over the outputs (lengths = the central directory's uncompressed sizes; an
// entry whose inflate fails or yields another size is not a match anyway).
int verify_deflated_chunk(const uint8_t *d_archive, zcrc_zip_entry *entries, const std::vector<size_t> &idx,
                          size_t a, size_t b, hipStream_t st) {
  const size_t m = b - a;
  std::vector<uint64_t> h(4 * m);  // src | src_len | dst | cap
  uint64_t arena_bytes = 0;
  for (size_t j = 0; j < m; j++) {
    const zcrc_zip_entry &E = entries[idx[a + j]];
    h[j] = reinterpret_cast<uint64_t>(d_archive) + E.data_offset;
    h[m + j] = E.comp_size;
    h[2 * m + j] = arena_bytes;
    h[3 * m + j] = inflate_room(E);  // <= kArenaBytes: the chunking below guarantees it
    arena_bytes += h[3 * m + j];
  }
  // thread-local device buffers (zcrc_runtime.h; this call synchronizes before it returns)
  void *d_arena = nullptr, *d_desc = nullptr;
  if (zcrc::tl_device_buffer(zcrc::kTlZipArena, arena_bytes + 16, &d_arena)) return zfail("inflate arena allocation failed");
  if (zcrc::tl_device_buffer(zcrc::kTlZipDesc, 8 * 5 * m + 8 * m, &d_desc)) return zfail("inflate descriptor allocation failed");
  zcrc::SyncOnExit guard(st, zcrc::kTlZipArena);  // (disarmed after the synchronize below)
  for (size_t j = 0; j < m; j++) h[2 * m + j] += reinterpret_cast<uint64_t>(d_arena);
  uint64_t *dd = static_cast<uint64_t *>(d_desc);
  uint64_t *d_src = dd, *d_srclen = dd + m, *d_dst = dd + 2 * m, *d_cap = dd + 3 * m, *d_olen = dd + 4 * m;
  int32_t *d_status = reinterpret_cast<int32_t *>(dd + 5 * m);
  uint32_t *d_crc = reinterpret_cast<uint32_t *>(d_status + m);
  std::vector<uint64_t> olen(m);
  std::vector<int32_t> status(m);
  std::vector<uint32_t> crc(m);
  int rc = ZCRC_OK;
  if (hipMemcpyAsync(dd, h.data(), 8 * 4 * m, hipMemcpyHostToDevice, st) != hipSuccess)
    rc = zfail("descriptor upload failed");
  if (!rc)
    rc = zcrc_inflate_batch_device(reinterpret_cast<const void *const *>(d_src), d_srclen,
                                   reinterpret_cast<void *const *>(d_dst), d_cap, d_olen, d_status, m, st);
  // CRC of what each inflate produced (0 bytes unless it succeeded)
  if (!rc) rc = zcrc32_batch_device(reinterpret_cast<const void *const *>(d_dst), d_olen, nullptr, d_crc, m, st);
  if (!rc && (hipMemcpyAsync(olen.data(), d_olen, 8 * m, hipMemcpyDeviceToHost, st) != hipSuccess ||
              hipMemcpyAsync(status.data(), d_status, 4 * m, hipMemcpyDeviceToHost, st) != hipSuccess ||
              hipMemcpyAsync(crc.data(), d_crc, 4 * m, hipMemcpyDeviceToHost, st) != hipSuccess))
    rc = zfail("result download failed");
  if (hipStreamSynchronize(st) != hipSuccess) {
    if (!rc) rc = zfail("stream synchronize failed");
    zcrc::tl_device_drop(zcrc::kTlZipArena);
    zcrc::tl_device_drop(zcrc::kTlZipDesc);
  }
  guard.armed = false;
  int trc = zcrc::tl_device_trim(zcrc::kTlZipArena, 1ull << 30);  // arenas above 1 GiB are not kept
  const int trd = zcrc::tl_device_trim(zcrc::kTlZipDesc, 1ull << 30);
  if (!trc) trc = trd;
  if (rc) return rc;
  if (trc) return trc;
  for (size_t j = 0; j < m; j++) {
    zcrc_zip_entry &E = entries[idx[a + j]];
    E.inflate_status = status[j];
    if (status[j] != ZCRC_INFLATE_OK) {
      E.status = ZCRC_ZIP_INFLATE_ERROR;
      continue;
    }
    E.crc_computed = crc[j];
    E.status = (olen[j] == E.uncomp_size && crc[j] == E.crc_expected) ? ZCRC_ZIP_OK : ZCRC_ZIP_MISMATCH;
  }
  return ZCRC_OK;
}

// ---------------------------------------------------------- stored entries

// Batched byte-range copy, any alignment.  Range j: len[j] bytes from src[j]
// to dst[j], cut into tiles of kCopyTileChunks destination-aligned 16-B
// chunks; workgroup b copies tile b (tile_range[b] = j, tile_first[b] = first
// chunk).  Interior chunks are one 16-B store whose bytes come from five
// aligned source dwords funnelled by v_alignbyte; a chunk whose five dwords
// do not all lie inside the source range (the range's edges -- a buffer load
// returns zero for a whole dword that straddles the range end) goes
// bytewise, like the partial destination chunks at both ends.
constexpr uint32_t kCopyThreads = 256, kCopyTileChunks = 4096;  // 64 KiB per tile

__global__ __launch_bounds__(kCopyThreads) void copy_ranges_kernel(const uint64_t *src, const uint64_t *dst,
                                                                   const uint64_t *len, const uint32_t *tile_range,
                                                                   const uint64_t *tile_first) {
  const uint32_t j = tile_range[blockIdx.x];
  const uint64_t s = src[j], d = dst[j], n = len[j];
  const uint64_t d_al = d & ~(uint64_t)15, d_end = d + n;
  const uint64_t nchunks = (((d_end + 15) & ~(uint64_t)15) - d_al) >> 4;
  const uint64_t c0 = tile_first[blockIdx.x];
  const uint64_t c1 = c0 + kCopyTileChunks < nchunks ? c0 + kCopyTileChunks : nchunks;
  // source window of this tile: [w0, w1), dword aligned at w0
  const uint64_t first_a = d_al + 16 * c0 > d ? d_al + 16 * c0 : d;
  const uint64_t w0 = (s + (first_a - d)) & ~(uint64_t)3;
  const uint64_t w1 = s + ((d_al + 16 * c1 < d_end ? d_al + 16 * c1 : d_end) - d);
  __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(w0), (short)0, (int)(w1 - w0), 0x00020000);
  for (uint64_t c = c0 + threadIdx.x; c < c1; c += kCopyThreads) {
    const uint64_t a = d_al + 16 * c;  // destination chunk
    const uint64_t sa = s + (a - d);   // its source (>= w0 when a >= d)
    if (a >= d && a + 16 <= d_end && (sa & ~(uint64_t)3) + 20 <= w1) {
      const uint32_t q = (uint32_t)((sa & ~(uint64_t)3) - w0), sh = (uint32_t)(sa & 3);
      uint32_t w[5];
#pragma unroll
      for (int k = 0; k < 5; k++) w[k] = __builtin_amdgcn_raw_buffer_load_b32(rs, q + 4u * k, 0, 0);
      uint4 v;
      v.x = __builtin_amdgcn_alignbyte(w[1], w[0], sh);
      v.y = __builtin_amdgcn_alignbyte(w[2], w[1], sh);
      v.z = __builtin_amdgcn_alignbyte(w[3], w[2], sh);
      v.w = __builtin_amdgcn_alignbyte(w[4], w[3], sh);
      *reinterpret_cast<uint4 *>(a) = v;
    } else {
      for (uint32_t b = 0; b < 16; b++)
        if (a + b >= d && a + b < d_end)
          *reinterpret_cast<uint8_t *>(a + b) = *reinterpret_cast<const uint8_t *>(s + (a + b - d));
    }
  }
}

// Entries eligible for extraction: stored, unencrypted, consistent sizes, in
// range, and a destination of at least comp_size bytes (none needed for an
// empty entry).
bool extractable(const zcrc_zip_entry &E, size_t archive_len, const void *dst, size_t cap) {
  return verifiable(E) && (dst || !E.comp_size) && cap >= E.comp_size && E.data_offset <= archive_len &&
         E.comp_size <= archive_len - E.data_offset;
}

}  // namespace

extern "C" int zcrc_zip_extract_stored_device(const void *d_archive, size_t archive_len, zcrc_zip_entry *entries,
                                              void *const *d_dst, const size_t *cap, size_t n, void *stream) {
  if (!d_archive || (n && (!entries || !d_dst || !cap))) return zfail("null argument");
  hipStream_t st = static_cast<hipStream_t>(stream);
  std::vector<size_t> idx;
  std::vector<uint64_t> hs, hd, hl;  // src | dst | len
  std::vector<uint32_t> t_range;
  std::vector<uint64_t> t_first;
  for (size_t i = 0; i < n; i++) {
    zcrc_zip_entry &E = entries[i];
    if (E.status == ZCRC_ZIP_BAD) continue;
    E.status = ZCRC_ZIP_UNVERIFIED;
    E.crc_computed = 0;
    if (!extractable(E, archive_len, d_dst[i], cap[i])) continue;
    const uint64_t d = reinterpret_cast<uint64_t>(d_dst[i]);
    const uint64_t nchunks = E.comp_size ? (((d + E.comp_size + 15) & ~(uint64_t)15) - (d & ~(uint64_t)15)) >> 4 : 0;
    for (uint64_t c = 0; c < nchunks; c += kCopyTileChunks) {
      t_range.push_back((uint32_t)idx.size());
      t_first.push_back(c);
    }
    idx.push_back(i);
    hs.push_back(reinterpret_cast<uint64_t>(d_archive) + E.data_offset);
    hd.push_back(d);
    hl.push_back(E.comp_size);
  }
  const size_t m = idx.size(), tiles = t_range.size();
  if (!m) return ZCRC_OK;
  if (m > 0xFFFFFFFFu || tiles > 0x7FFFFFFFu) return zfail("too many entries for one extraction");
  void *dv = nullptr;
  const size_t bytes = 8 * 3 * m + 4 * m + 8 * tiles + 4 * tiles;
  if (zcrc::tl_device_buffer(zcrc::kTlZipCopy, bytes, &dv)) return zfail("descriptor allocation failed");
  uint64_t *d_src = static_cast<uint64_t *>(dv), *d_dstp = d_src + m, *d_len = d_dstp + m;
  uint64_t *d_tfirst = d_len + m;
  uint32_t *d_crc = reinterpret_cast<uint32_t *>(d_tfirst + tiles), *d_trange = d_crc + m;
  std::vector<uint32_t> crc(m);
  int rc = ZCRC_OK;
  if (hipMemcpyAsync(d_src, hs.data(), 8 * m, hipMemcpyHostToDevice, st) != hipSuccess ||
      hipMemcpyAsync(d_dstp, hd.data(), 8 * m, hipMemcpyHostToDevice, st) != hipSuccess ||
      hipMemcpyAsync(d_len, hl.data(), 8 * m, hipMemcpyHostToDevice, st) != hipSuccess ||
      (tiles && (hipMemcpyAsync(d_tfirst, t_first.data(), 8 * tiles, hipMemcpyHostToDevice, st) != hipSuccess ||
                 hipMemcpyAsync(d_trange, t_range.data(), 4 * tiles, hipMemcpyHostToDevice, st) != hipSuccess)))
    rc = zfail("descriptor upload failed");
  if (!rc && tiles) {
    hipLaunchKernelGGL(copy_ranges_kernel, dim3((unsigned)tiles), dim3(kCopyThreads), 0, st, d_src, d_dstp, d_len,
                       d_trange, d_tfirst);
    if (hipGetLastError() != hipSuccess) rc = zfail("copy launch failed");
  }
  // the CRC of the copies, as fhandle_check_crc32 checks the preload buffer
  if (!rc) rc = zcrc32_batch_device(reinterpret_cast<const void *const *>(d_dstp), d_len, nullptr, d_crc, m, stream);
  if (!rc && hipMemcpyAsync(crc.data(), d_crc, 4 * m, hipMemcpyDeviceToHost, st) != hipSuccess)
    rc = zfail("result download failed");
  if (hipStreamSynchronize(st) != hipSuccess) {
    if (!rc) rc = zfail("stream synchronize failed");
    zcrc::tl_device_drop(zcrc::kTlZipCopy);
  }
  const int trc = zcrc::tl_device_trim(zcrc::kTlZipCopy, 1ull << 30);
  if (rc) return rc;
  if (trc) return trc;
  finish(entries, idx, crc);
  return ZCRC_OK;
}

extern "C" int zcrc_zip_extract_stored_host(const void *archive, size_t archive_len, zcrc_zip_entry *entries,
                                            void *const *dst, const size_t *cap, size_t n) {
  if (!archive || (n && (!entries || !dst || !cap))) return zfail("null argument");
  const uint8_t *a = static_cast<const uint8_t *>(archive);
  std::vector<size_t> idx;
  std::vector<const void *> ptrs;
  std::vector<size_t> lens;
  for (size_t i = 0; i < n; i++) {
    zcrc_zip_entry &E = entries[i];
    if (E.status == ZCRC_ZIP_BAD) continue;
    E.status = ZCRC_ZIP_UNVERIFIED;
    E.crc_computed = 0;
    if (!extractable(E, archive_len, dst[i], cap[i])) continue;
    if (E.comp_size) memcpy(dst[i], a + E.data_offset, E.comp_size);  // what zip_fread delivers for a stored entry
    idx.push_back(i);
    ptrs.push_back(dst[i]);
    lens.push_back(E.comp_size);
  }
  if (idx.empty()) return ZCRC_OK;
  std::vector<uint32_t> crc(idx.size());
  const int rc = zcrc32_batch(ptrs.data(), lens.data(), nullptr, crc.data(), idx.size(), 0);
  if (rc) return rc;
  finish(entries, idx, crc);
  return ZCRC_OK;
}

extern "C" int zcrc_zip_verify_device(const void *d_archive, size_t archive_len, zcrc_zip_entry *entries, size_t n,
                                      void *stream) {
  if (!d_archive || (n && !entries)) return zfail("null argument");
  hipStream_t st = static_cast<hipStream_t>(stream);
  std::vector<size_t> idx, didx;
  std::vector<uint64_t> hp, hl;
  for (size_t i = 0; i < n; i++) {
    zcrc_zip_entry &E = entries[i];
    if (E.status == ZCRC_ZIP_BAD) continue;
    E.status = ZCRC_ZIP_UNVERIFIED;  // until checked below
    if (E.data_offset > archive_len || E.comp_size > archive_len - E.data_offset) continue;
    if (verifiable(E)) {
      idx.push_back(i);
      hp.push_back(reinterpret_cast<uint64_t>(d_archive) + E.data_offset);
      hl.push_back(E.comp_size);
    } else if (deflatable(E) && inflate_room(E) <= kArenaBytes) {
      didx.push_back(i);
    }
  }
  std::vector<uint32_t> crc(idx.size());
  if (!idx.empty()) {
    const size_t m = idx.size();
    void *d = nullptr;
    if (zcrc::tl_device_buffer(zcrc::kTlZipDesc, m * 20, &d)) return zfail("descriptor allocation failed");
    uint64_t *dp = static_cast<uint64_t *>(d), *dl = dp + m;
    uint32_t *dout = reinterpret_cast<uint32_t *>(dl + m);
    int rc = ZCRC_OK;
    if (hipMemcpyAsync(dp, hp.data(), 8 * m, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(dl, hl.data(), 8 * m, hipMemcpyHostToDevice, st) != hipSuccess)
      rc = zfail("descriptor upload failed");
    if (!rc) rc = zcrc32_batch_device(reinterpret_cast<const void *const *>(dp), dl, nullptr, dout, m, stream);
    if (!rc && hipMemcpyAsync(crc.data(), dout, 4 * m, hipMemcpyDeviceToHost, st) != hipSuccess)
      rc = zfail("result download failed");
    if (hipStreamSynchronize(st) != hipSuccess) {
      if (!rc) rc = zfail("stream synchronize failed");
      zcrc::tl_device_drop(zcrc::kTlZipDesc);
    }
    const int trc = zcrc::tl_device_trim(zcrc::kTlZipDesc, 1ull << 30);
    if (rc) return rc;
    if (trc) return trc;
  }
  finish(entries, idx, crc);
  // deflated entries in chunks of <= kArenaBytes of output
  for (size_t a = 0; a < didx.size();) {
    size_t b = a;
    uint64_t bytes = 0;
    while (b < didx.size() && (b == a || bytes + inflate_room(entries[didx[b]]) <= kArenaBytes))
      bytes += inflate_room(entries[didx[b++]]);  // each <= kArenaBytes: no wrap
    const int rc = verify_deflated_chunk(static_cast<const uint8_t *>(d_archive), entries, didx, a, b, st);
    if (rc) return rc;
    a = b;
  }
  return ZCRC_OK;
}

namespace {

// One device's share of zcrc_zip_verify_host: the sub-image [lo, hi) holding
// the data of entries idx[a, b) is staged into HBM once and verified there
// (offsets rebased to the sub-image).
int verify_host_run(const uint8_t *archive, zcrc_zip_entry *entries, const std::vector<size_t> &idx, size_t a,
                    size_t b) {
  if (a == b) return ZCRC_OK;
  uint64_t lo = UINT64_MAX, hi = 0;
  for (size_t k = a; k < b; k++) {
    const zcrc_zip_entry &E = entries[idx[k]];
    lo = std::min<uint64_t>(lo, E.data_offset);
    hi = std::max<uint64_t>(hi, E.data_offset + E.comp_size);
  }
  std::vector<zcrc_zip_entry> local(b - a);
  for (size_t k = a; k < b; k++) {
    local[k - a] = entries[idx[k]];
    local[k - a].data_offset -= lo;
  }
  const uint64_t len = hi - lo;
  const int rc = zcrc::with_lease_stream([&](hipStream_t st) {
    void *d = nullptr;
    if (zcrc::tl_device_buffer(zcrc::kTlZipImage, len ? len : 1, &d)) return zfail("archive allocation failed");
    zcrc::SyncOnExit guard(st, zcrc::kTlZipImage);
    if (len && hipMemcpyAsync(d, archive + lo, len, hipMemcpyHostToDevice, st) != hipSuccess)
      return zfail("archive upload failed");
    int r = zcrc_zip_verify_device(d, len, local.data(), local.size(), st);
    if (hipStreamSynchronize(st) != hipSuccess) {
      if (!r) r = zfail("stream synchronize failed");
      zcrc::tl_device_drop(zcrc::kTlZipImage);
    }
    guard.armed = false;
    const int trc = zcrc::tl_device_trim(zcrc::kTlZipImage, 1ull << 30);
    return r ? r : trc;
  });
  if (rc) return rc;
  for (size_t k = a; k < b; k++) {
    zcrc_zip_entry &E = entries[idx[k]];
    E.status = local[k - a].status;
    E.crc_computed = local[k - a].crc_computed;
    E.inflate_status = local[k - a].inflate_status;
  }
  return ZCRC_OK;
}

}  // namespace

// Over the device set (zcrc_runtime.h): the entries, in archive order, are cut
// into runs of about equal data bytes, one per device, and each device
// stages only its run's part of the image -- a ZIP's entry data is laid out
// in order, so the parts barely overlap and the image crosses PCIe about once
// in all.
extern "C" int zcrc_zip_verify_host(const void *archive, size_t archive_len, zcrc_zip_entry *entries, size_t n) {
  if (!archive || (n && !entries)) return zfail("null argument");
  std::vector<size_t> idx;
  uint64_t total = 0;
  for (size_t i = 0; i < n; i++) {
    zcrc_zip_entry &E = entries[i];
    if (E.status == ZCRC_ZIP_BAD) continue;
    if (E.data_offset > archive_len || E.comp_size > archive_len - E.data_offset) {
      E.status = ZCRC_ZIP_UNVERIFIED;  // as zcrc_zip_verify_device leaves it
      continue;
    }
    idx.push_back(i);
    total += E.comp_size;
  }
  std::stable_sort(idx.begin(), idx.end(),
                   [&](size_t x, size_t y) { return entries[x].data_offset < entries[y].data_offset; });
  const size_t shards = std::max<size_t>(1, std::min(idx.size(), zcrc::host_shards(total)));
  std::vector<size_t> cut(shards + 1, idx.size());
  cut[0] = 0;
  uint64_t acc = 0;
  for (size_t g = 1, k = 0; g < shards; g++) {
    const uint64_t want = (uint64_t)((unsigned __int128)total * g / shards);
    while (k < idx.size() && acc < want) acc += entries[idx[k++]].comp_size;
    cut[g] = k;
  }
  const uint8_t *a = static_cast<const uint8_t *>(archive);
  return zcrc::run_sharded(shards, [&](size_t g) { return verify_host_run(a, entries, idx, cut[g], cut[g + 1]); });
}
