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
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../include/zcrc.h"
#include "zcrc_internal.h"

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
  void *d_arena = nullptr, *d_desc = nullptr;
  if (hipMallocAsync(&d_arena, arena_bytes + 16, st) != hipSuccess) return zfail("inflate arena allocation failed");
  if (hipMallocAsync(&d_desc, 8 * 5 * m + 8 * m, st) != hipSuccess) {
    (void)hipFreeAsync(d_arena, st);
    return zfail("inflate descriptor allocation failed");
  }
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
  (void)hipFreeAsync(d_desc, st);
  (void)hipFreeAsync(d_arena, st);
  if (!rc && hipStreamSynchronize(st) != hipSuccess) rc = zfail("stream synchronize failed");
  if (rc) return rc;
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

}  // namespace

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
    if (hipMallocAsync(&d, m * 20, st) != hipSuccess) return zfail("hipMallocAsync failed");
    uint64_t *dp = static_cast<uint64_t *>(d), *dl = dp + m;
    uint32_t *dout = reinterpret_cast<uint32_t *>(dl + m);
    int rc = ZCRC_OK;
    if (hipMemcpyAsync(dp, hp.data(), 8 * m, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(dl, hl.data(), 8 * m, hipMemcpyHostToDevice, st) != hipSuccess)
      rc = zfail("descriptor upload failed");
    if (!rc) rc = zcrc32_batch_device(reinterpret_cast<const void *const *>(dp), dl, nullptr, dout, m, stream);
    if (!rc && hipMemcpyAsync(crc.data(), dout, 4 * m, hipMemcpyDeviceToHost, st) != hipSuccess)
      rc = zfail("result download failed");
    (void)hipFreeAsync(d, st);
    if (!rc && hipStreamSynchronize(st) != hipSuccess) rc = zfail("stream synchronize failed");
    if (rc) return rc;
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

extern "C" int zcrc_zip_verify_host(const void *archive, size_t archive_len, zcrc_zip_entry *entries, size_t n) {
  if (!archive || (n && !entries)) return zfail("null argument");
  // stage the image once and verify it where the GPU reads it
  hipStream_t st = nullptr;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return zfail("stream create failed");
  void *d = nullptr;
  int rc = ZCRC_OK;
  if (hipMallocAsync(&d, archive_len ? archive_len : 1, st) != hipSuccess) rc = zfail("archive allocation failed");
  if (!rc && archive_len && hipMemcpyAsync(d, archive, archive_len, hipMemcpyHostToDevice, st) != hipSuccess)
    rc = zfail("archive upload failed");
  if (!rc) rc = zcrc_zip_verify_device(d, archive_len, entries, n, st);
  if (d) (void)hipFreeAsync(d, st);
  (void)hipStreamSynchronize(st);
  (void)hipStreamDestroy(st);
  return rc;
}
