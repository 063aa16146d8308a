// zcrc_zip.hip -- ZIP central-directory scan + batched GPU verification.
//
// The reference gets each entry's expected CRC through libzip (zip_stat,
// st.crc: src/ZIPsFS.c:985-1001) and verifies it only after a full preload
// (src/ZIPsFS_preloadfileram.c:237-250).  Here a whole archive is checked at
// once: the host walks the central directory (APPNOTE 4.3.12/4.3.14/4.3.16,
// ZIP64 4.5.3) and the data of every stored entry -- a plain byte range of the
// archive -- is checksummed by one zcrc32_batch* launch.  The scan is bounds
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
    if (z + 56 > len || rd32(a + z) != kSigZ64Eocd) return zfail("bad ZIP64 end-of-central-directory record");
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
      if (lho + 30 > len || rd32(a + lho) != kSigLocal) {
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

void finish(zcrc_zip_entry *entries, size_t n, const std::vector<size_t> &idx, const std::vector<uint32_t> &crc) {
  for (size_t j = 0; j < idx.size(); j++) {
    zcrc_zip_entry &E = entries[idx[j]];
    E.crc_computed = crc[j];
    E.status = crc[j] == E.crc_expected ? ZCRC_ZIP_OK : ZCRC_ZIP_MISMATCH;
  }
  for (size_t i = 0; i < n; i++)
    if (!verifiable(entries[i]) && entries[i].status != ZCRC_ZIP_BAD) entries[i].status = ZCRC_ZIP_UNVERIFIED;
}

}  // namespace

extern "C" int zcrc_zip_verify_host(const void *archive, size_t archive_len, zcrc_zip_entry *entries, size_t n) {
  if (!archive || (n && !entries)) return zfail("null argument");
  const uint8_t *a = static_cast<const uint8_t *>(archive);
  std::vector<size_t> idx;
  std::vector<const void *> ptrs;
  std::vector<size_t> lens;
  for (size_t i = 0; i < n; i++)
    if (verifiable(entries[i]) && entries[i].data_offset + entries[i].comp_size <= archive_len) {
      idx.push_back(i);
      ptrs.push_back(a + entries[i].data_offset);
      lens.push_back(entries[i].comp_size);
    }
  std::vector<uint32_t> crc(idx.size());
  if (!idx.empty()) {
    const int rc = zcrc32_batch(ptrs.data(), lens.data(), nullptr, crc.data(), idx.size(), 0);
    if (rc) return rc;
  }
  finish(entries, n, idx, crc);
  return ZCRC_OK;
}

extern "C" int zcrc_zip_verify_device(const void *d_archive, size_t archive_len, zcrc_zip_entry *entries, size_t n,
                                      void *stream) {
  if (!d_archive || (n && !entries)) return zfail("null argument");
  hipStream_t st = static_cast<hipStream_t>(stream);
  std::vector<size_t> idx;
  std::vector<uint64_t> hp, hl;
  for (size_t i = 0; i < n; i++)
    if (verifiable(entries[i]) && entries[i].data_offset + entries[i].comp_size <= archive_len) {
      idx.push_back(i);
      hp.push_back(reinterpret_cast<uint64_t>(d_archive) + entries[i].data_offset);
      hl.push_back(entries[i].comp_size);
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
  finish(entries, n, idx, crc);
  return ZCRC_OK;
}
