/*
 * oracle/crc32_port.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of ZIPsFS's CRC-32 hot path (reference: src/cg_crc32.c).
 * It is the *checker* for the MI355X engine and the timed CPU baseline in
 * bench.py ("kind": "port").  Nothing in zipsfs_amd/ links, loads or calls
 * this file: the product path is HIP-only and fails loudly without its .so.
 *
 * Parity pinning: every function here is checked (tests/test_oracle.py)
 * against golden vectors produced by the reference source itself, compiled
 * from /root/reference/src/cg_crc32.c by oracle/Makefile into oracle/_ref/
 * (see tests/golden/gen_golden.py), against the reference test-suite KAT
 * `seq 1000` -> 8DC4565D (testing/testfiles/ZIPsFS_testfiles_preload.sh:30,32,53),
 * the CRC-32/ISO-HDLC check value "123456789" -> CBF43926, and zlib.crc32.
 *
 * What is restated (not copied):
 *   - the byte table in the reference's *complemented* register domain
 *     (src/cg_crc32.c:10-13): entry i is the reflected CRC step of i with
 *     the feedback polarity inverted, then xor 0xFF000000;
 *   - the 8 word tables for slicing-by-8 over little-endian uint64 words,
 *     with the affine correction for lanes k>=1 (src/cg_crc32.c:14-24);
 *   - the main loop a = crc ^ word; crc = xor of 8 lane lookups
 *     (src/cg_crc32.c:37-46) and the bytewise tail (src/cg_crc32.c:47);
 *   - zlib crc32(seed, data, n) chaining semantics, which the reference's
 *     complemented-domain state reproduces exactly.
 * Unaligned input is allowed, as in the reference (src/cg_crc32.c:27).
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <pthread.h>

#define ORACLE_POLY_REFLECTED 0xEDB88320u

/* ------------------------------------------------------------------ tables */

/* Byte table in the complemented domain (src/cg_crc32.c:10-13).
 * Instead of running the inverted-feedback loop we use the identity proved
 * in SURVEY.md section 0:  C[i] = T_std[i ^ 0xFF] ^ 0xFF000000, where T_std
 * is the ordinary reflected table.  tests/test_oracle.py checks all 256
 * entries against the literal loop form as well. */
static uint32_t std_byte_step(uint32_t r) {
  for (int b = 0; b < 8; b++) r = (r >> 1) ^ (ORACLE_POLY_REFLECTED & (0u - (r & 1u)));
  return r;
}

static uint32_t comp_table[256];      /* complemented-domain byte table      */
static uint32_t comp_slice[8][256];   /* slicing-by-8, lane k = byte k of u64 */
static pthread_once_t tables_once = PTHREAD_ONCE_INIT;

static void build_tables(void) {
  for (uint32_t i = 0; i < 256; i++) comp_table[i] = std_byte_step(i ^ 0xFFu) ^ 0xFF000000u;
  /* Lane k of an 8-byte word: run the complemented byte step over the 8
   * bytes of a word that is zero except for byte k == i.  Lanes k>=1 carry
   * an extra affine term (the complement fed through k zero bytes) that the
   * reference cancels by xoring lane 0's entry for i == 0
   * (src/cg_crc32.c:21).  We cancel it the same way. */
  for (int k = 0; k < 8; k++) {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t w = 0;
      for (int j = 0; j < 8; j++) {
        const uint32_t in = (j == k) ? (w ^ i) : w;
        w = comp_table[in & 0xFFu] ^ (w >> 8);
      }
      comp_slice[k][i] = w ^ (k ? comp_slice[0][0] : 0u);
    }
  }
}

/* ------------------------------------------------------------ the CRC-32 */

/* oracle_cg_crc32: same contract as static cg_crc32() in
 * src/cg_crc32.c:26 (minus the mutex, which only guards lazy table init). */
uint32_t oracle_cg_crc32(const void *data, size_t n, uint32_t crc) {
  pthread_once(&tables_once, build_tables);
  const unsigned char *p = (const unsigned char *)data;
  const size_t nwords = n / 8;
  for (size_t i = 0; i < nwords; i++) {
    uint64_t word;
    memcpy(&word, p + 8 * i, 8); /* unaligned little-endian load (:38) */
    const uint64_t a = (uint64_t)crc ^ word;
    crc = comp_slice[0][(uint8_t)(a)]       ^ comp_slice[1][(uint8_t)(a >> 8)] ^
          comp_slice[2][(uint8_t)(a >> 16)] ^ comp_slice[3][(uint8_t)(a >> 24)] ^
          comp_slice[4][(uint8_t)(a >> 32)] ^ comp_slice[5][(uint8_t)(a >> 40)] ^
          comp_slice[6][(uint8_t)(a >> 48)] ^ comp_slice[7][(uint8_t)(a >> 56)];
  }
  for (size_t i = nwords * 8; i < n; i++) crc = comp_table[(uint8_t)crc ^ p[i]] ^ (crc >> 8);
  return crc;
}

/* The literal inverted-feedback loop of src/cg_crc32.c:10-13, kept only so
 * the test-suite can check the table identity entry by entry. */
uint32_t oracle_comp_table_literal(uint32_t r) {
  for (int j = 0; j < 8; j++) r = ((r & 1u) ? 0u : ORACLE_POLY_REFLECTED) ^ (r >> 1);
  return r ^ 0xFF000000u;
}
uint32_t oracle_comp_table_entry(uint32_t i) {
  pthread_once(&tables_once, build_tables);
  return comp_table[i & 0xFFu];
}

/* Plain bit-serial zlib-style CRC (no tables): a second, independent CPU
 * formulation used only as a cross-check inside the tests. */
uint32_t oracle_crc32_bitwise(const void *data, size_t n, uint32_t crc) {
  const unsigned char *p = (const unsigned char *)data;
  uint32_t r = ~crc;
  for (size_t i = 0; i < n; i++) {
    r ^= p[i];
    for (int b = 0; b < 8; b++) r = (r >> 1) ^ (ORACLE_POLY_REFLECTED & (0u - (r & 1u)));
  }
  return ~r;
}

/* ------------------------------------------------------- payload generator */
/* counter-based splitmix64 payload, so that the GPU
 * can regenerate any buffer without host traffic and the CPU can regenerate
 * the same bytes to check it. */
static inline uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

uint64_t oracle_mix64(uint64_t z) { return mix64(z); }

/* Bytes [0,len) of synthetic buffer `index`: word j = mix64(seed ^ (index<<32 | j)). */
void oracle_fill_payload(uint8_t *dst, uint64_t len, uint64_t index, uint64_t seed) {
  const uint64_t nfull = len / 8;
  for (uint64_t j = 0; j < nfull; j++) {
    const uint64_t w = mix64(seed ^ ((index << 32) + j));
    memcpy(dst + 8 * j, &w, 8);
  }
  if (len % 8) {
    const uint64_t w = mix64(seed ^ ((index << 32) + nfull));
    memcpy(dst + 8 * nfull, &w, (size_t)(len % 8));
  }
}

/* Config-4 bounded power-law sizes. */
uint64_t oracle_zipf_len(uint64_t i) {
  const uint64_t h = mix64(0x5A1F5EEDull ^ ((i + 1) * 0xD1B54A32D192ED03ull));
  const double u = (double)(h >> 11) * (1.0 / 9007199254740992.0);
  const double t = 1.0 - u * 127.0 / 128.0;
  double len = 1024.0 / (t * t);
  if (len < 1024.0) len = 1024.0;
  if (len > 16777216.0) len = 16777216.0;
  return (uint64_t)len; /* floor: len >= 1024 > 0 */
}

/* CRC of synthetic buffer `index` without materialising it (streams 64 KiB
 * pieces through the restatement, chaining the seed). */
uint32_t oracle_crc_payload(uint64_t len, uint64_t index, uint64_t seed, uint32_t crc) {
  uint8_t chunk[65536];
  uint64_t done = 0;
  while (done < len) {
    const uint64_t take = (len - done) < sizeof(chunk) ? (len - done) : sizeof(chunk);
    /* word-aligned pieces: done is a multiple of 65536, so word indices line up */
    const uint64_t w0 = done / 8;
    const uint64_t nw = (take + 7) / 8;
    for (uint64_t j = 0; j < nw; j++) {
      const uint64_t w = mix64(seed ^ ((index << 32) + w0 + j));
      const uint64_t off = 8 * j;
      const uint64_t cnt = (take - off) < 8 ? (take - off) : 8;
      memcpy(chunk + off, &w, (size_t)cnt);
    }
    crc = oracle_cg_crc32(chunk, (size_t)take, crc);
    done += take;
  }
  return crc;
}

/* ---------------------------------------------------- batched CPU baseline */
/* Round-robin buffer ownership over a pthread pool, as in BASELINE.md
 * ("nproc threads, pthread pool, round-robin buffer ownership"). */
typedef uint32_t (*crc_fn_t)(const void *, size_t, uint32_t);
typedef struct {
  const uint8_t *const *ptrs; const uint64_t *lens; const uint32_t *seeds;
  uint32_t *out; uint64_t n; int tid, nthreads; crc_fn_t fn;
} batch_job_t;

static void *batch_worker(void *arg) {
  batch_job_t *j = (batch_job_t *)arg;
  for (uint64_t i = (uint64_t)j->tid; i < j->n; i += (uint64_t)j->nthreads)
    j->out[i] = j->fn(j->ptrs[i], (size_t)j->lens[i], j->seeds ? j->seeds[i] : 0u);
  return NULL;
}

static int run_batch(crc_fn_t fn, const uint8_t *const *ptrs, const uint64_t *lens,
                     const uint32_t *seeds, uint32_t *out, uint64_t n, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 1024) nthreads = 1024;
  pthread_t th[1024];
  batch_job_t jobs[1024];
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (batch_job_t){ptrs, lens, seeds, out, n, t, nthreads, fn};
    if (t && pthread_create(&th[t], NULL, batch_worker, &jobs[t]) != 0) return -1;
  }
  batch_worker(&jobs[0]);
  for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
  return 0;
}

/* Payload of buffers i (index idx[i]) written by the thread that will own
 * them in run_batch (round-robin): first touch places each page on the
 * NUMA node of the core that later checksums it (bench.py cpu_baseline). */
typedef struct {
  uint8_t *const *ptrs; const uint64_t *lens, *idx; uint64_t seed, n; int tid, nthreads;
} fill_job_t;

static void *fill_worker(void *arg) {
  fill_job_t *j = (fill_job_t *)arg;
  for (uint64_t i = (uint64_t)j->tid; i < j->n; i += (uint64_t)j->nthreads)
    oracle_fill_payload(j->ptrs[i], j->lens[i], j->idx[i], j->seed);
  return NULL;
}

int oracle_fill_payload_batch(uint8_t *const *ptrs, const uint64_t *lens, const uint64_t *idx, uint64_t seed,
                              uint64_t n, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 1024) nthreads = 1024;
  pthread_t th[1024];
  fill_job_t jobs[1024];
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (fill_job_t){ptrs, lens, idx, seed, n, t, nthreads};
    if (t && pthread_create(&th[t], NULL, fill_worker, &jobs[t]) != 0) return -1;
  }
  fill_worker(&jobs[0]);
  for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
  return 0;
}

int oracle_crc32_batch(const uint8_t *const *ptrs, const uint64_t *lens, const uint32_t *seeds,
                       uint32_t *out, uint64_t n, int nthreads) {
  pthread_once(&tables_once, build_tables);
  return run_batch(oracle_cg_crc32, ptrs, lens, seeds, out, n, nthreads);
}

/* Same pool driving any crc function with the cg_crc32-minus-mutex shape,
 * e.g. the reference build in oracle/_ref/ (bench.py cpu_baseline). */
int oracle_crc32_batch_fn(void *fn, const uint8_t *const *ptrs, const uint64_t *lens,
                          const uint32_t *seeds, uint32_t *out, uint64_t n, int nthreads) {
  pthread_once(&tables_once, build_tables);
  return run_batch((crc_fn_t)fn, ptrs, lens, seeds, out, n, nthreads);
}
