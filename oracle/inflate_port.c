/*
 * oracle/inflate_port.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of raw DEFLATE decoding (RFC 1951) with the acceptance
 * rules of zlib 1.2.11, the checker for libzcrc's GPU inflate (SURVEY.md
 * section 8(f) rank 4).  Nothing in zipsfs_amd/ links or calls this file.
 *
 * Where the algorithm lives: ZIPsFS reads deflated entries with libzip's
 * zip_fread() (src/ZIPsFS.c:2016-2019 my_zip_fread, called by
 * preloadram_now src/ZIPsFS_preloadfileram.c:286-306), and libzip inflates
 * with zlib.  Both are third-party and absent from the reference tree; the
 * image pins zlib 1.2.11 (Python zlib.ZLIB_RUNTIME_VERSION, /usr/lib libz).
 * This file restates the published format (RFC 1951 sections 3.2.3-3.2.7)
 * and zlib's validity rules (the ones its inflate_table()/inflate() enforce):
 *   - block type 3 is an error; stored LEN must equal ~NLEN;
 *   - dynamic headers: HLIT <= 286, HDIST <= 30; the code-length code must
 *     be complete; a repeat (16) needs a previous length; repeats must not
 *     overrun HLIT+HDIST; the end-of-block symbol must have a code;
 *   - literal/length and distance codes: over-subscribed is an error,
 *     incomplete is an error unless the code is a single length-1 code;
 *     a distance code with no symbols is accepted until a distance is needed;
 *   - literal/length symbols 286-287 and distance symbols 30-31 are invalid;
 *   - a distance beyond the bytes produced so far is an error;
 *   - running out of input before the final block ends is an error.
 * Decoding is the canonical bit-at-a-time method (count/symbol tables), the
 * simplest form that is obviously the RFC's prefix code.
 *
 * Parity pinning (tests/test_inflate.py): every result is compared with
 * Python zlib.decompress(wbits=-15) on generated streams (all zlib levels and
 * strategies, stored/fixed/dynamic blocks, 32 KiB distances, corrupted
 * streams -> error iff zlib errors), and, when the reference tree is
 * present, on every deflated entry of the reference's own
 * for_the_author_only.zip (CRC-32 and size from its central directory).
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <pthread.h>

/* status codes, shared with include/zcrc.h (ZCRC_INFLATE_*) */
enum {
  INF_OK = 0,
  INF_ERR_BLOCK_TYPE = 1,
  INF_ERR_STORED_LEN = 2,
  INF_ERR_CODES = 3,
  INF_ERR_SYMBOL = 4,
  INF_ERR_DIST = 5,
  INF_ERR_OUTPUT = 6,
  INF_ERR_INPUT = 7,
};

#define MAXBITS 15
#define MAXLCODES 288
#define MAXDCODES 32

typedef struct {
  const uint8_t *in;
  size_t inlen, incnt; /* bytes consumed into the bit buffer */
  uint32_t bitbuf;
  int bitcnt;
  uint8_t *out;
  size_t outcap, outcnt;
  int err;
} state;

/* need <= 16 bits, LSB first (RFC 1951 3.1.1) */
static uint32_t getbits(state *s, int need) {
  while (s->bitcnt < need) {
    if (s->incnt >= s->inlen) {
      if (!s->err) s->err = INF_ERR_INPUT;
      return 0;
    }
    s->bitbuf |= (uint32_t)s->in[s->incnt++] << s->bitcnt;
    s->bitcnt += 8;
  }
  const uint32_t v = s->bitbuf & ((1u << need) - 1u);
  s->bitbuf >>= need;
  s->bitcnt -= need;
  return v;
}

typedef struct {
  short count[MAXBITS + 1];
  short symbol[MAXLCODES];
} huffman;

/* Canonical code from lengths (RFC 1951 3.2.2).  Returns the number of
 * unused codes: 0 complete, > 0 incomplete, < 0 over-subscribed. */
static int construct(huffman *h, const short *length, int n, int *max_len) {
  for (int len = 0; len <= MAXBITS; len++) h->count[len] = 0;
  for (int sym = 0; sym < n; sym++) h->count[length[sym]]++;
  *max_len = 0;
  for (int len = 1; len <= MAXBITS; len++)
    if (h->count[len]) *max_len = len;
  if (h->count[0] == n) return 0; /* no codes */
  int left = 1;
  for (int len = 1; len <= MAXBITS; len++) {
    left <<= 1;
    left -= h->count[len];
    if (left < 0) return left;
  }
  short offs[MAXBITS + 1];
  offs[1] = 0;
  for (int len = 1; len < MAXBITS; len++) offs[len + 1] = offs[len] + h->count[len];
  for (int sym = 0; sym < n; sym++)
    if (length[sym] != 0) h->symbol[offs[length[sym]]++] = (short)sym;
  return left;
}

/* zlib's acceptance of a literal/length or distance code */
static int code_ok(int left, int max_len) { return left == 0 || (left > 0 && max_len == 1) || max_len == 0; }

/* one symbol, canonical decode; -1 if no code matches */
static int decode(state *s, const huffman *h) {
  int code = 0, first = 0, index = 0;
  for (int len = 1; len <= MAXBITS; len++) {
    code |= (int)getbits(s, 1);
    if (s->err) return -1;
    const int count = h->count[len];
    if (code - count < first) return h->symbol[index + (code - first)];
    index += count;
    first += count;
    first <<= 1;
    code <<= 1;
  }
  return -1;
}

static const short kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                   31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const short kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint16_t kDistBase[30] = {1,    2,    3,    4,    5,    7,     9,     13,    17,  25,
                                       33,   49,   65,   97,   129,  193,   257,   385,   513, 769,
                                       1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
static const short kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

static int codes(state *s, const huffman *lencode, const huffman *distcode) {
  for (;;) {
    int sym = decode(s, lencode);
    if (s->err) return s->err;
    if (sym < 0) return INF_ERR_SYMBOL;
    if (sym < 256) {
      if (s->outcnt >= s->outcap) return INF_ERR_OUTPUT;
      s->out[s->outcnt++] = (uint8_t)sym;
    } else if (sym == 256) {
      return INF_OK;
    } else {
      sym -= 257;
      if (sym >= 29) return INF_ERR_SYMBOL; /* 286, 287 */
      const size_t len = (size_t)kLenBase[sym] + getbits(s, kLenExtra[sym]);
      const int dsym = decode(s, distcode);
      if (s->err) return s->err;
      if (dsym < 0 || dsym >= 30) return INF_ERR_SYMBOL;
      const size_t dist = (size_t)kDistBase[dsym] + getbits(s, kDistExtra[dsym]);
      if (s->err) return s->err;
      if (dist > s->outcnt) return INF_ERR_DIST;
      if (len > s->outcap - s->outcnt) return INF_ERR_OUTPUT;
      for (size_t k = 0; k < len; k++, s->outcnt++) s->out[s->outcnt] = s->out[s->outcnt - dist];
    }
  }
}

static int stored(state *s) {
  s->bitbuf = 0; /* drop to a byte boundary (3.2.4) */
  s->bitcnt = 0;
  if (s->inlen - s->incnt < 4) return INF_ERR_INPUT;
  const unsigned len = s->in[s->incnt] | (unsigned)s->in[s->incnt + 1] << 8;
  const unsigned nlen = s->in[s->incnt + 2] | (unsigned)s->in[s->incnt + 3] << 8;
  s->incnt += 4;
  if (len != (~nlen & 0xFFFFu)) return INF_ERR_STORED_LEN;
  if (s->inlen - s->incnt < len) {
    /* zlib copies what it has and then reports the truncation; the output
     * up to that point is not a result anyway */
    return INF_ERR_INPUT;
  }
  if (len > s->outcap - s->outcnt) return INF_ERR_OUTPUT;
  memcpy(s->out + s->outcnt, s->in + s->incnt, len);
  s->outcnt += len;
  s->incnt += len;
  return INF_OK;
}

/* fixed codes (RFC 1951 3.2.6), built once */
static huffman g_fixed_len, g_fixed_dist;
static pthread_once_t g_fixed_once = PTHREAD_ONCE_INIT;

static void build_fixed(void) {
  short lengths[MAXLCODES];
  int max_len;
  int sym = 0;
  for (; sym < 144; sym++) lengths[sym] = 8;
  for (; sym < 256; sym++) lengths[sym] = 9;
  for (; sym < 280; sym++) lengths[sym] = 7;
  for (; sym < MAXLCODES; sym++) lengths[sym] = 8;
  construct(&g_fixed_len, lengths, MAXLCODES, &max_len);
  for (sym = 0; sym < MAXDCODES; sym++) lengths[sym] = 5; /* 30, 31 decode as invalid */
  construct(&g_fixed_dist, lengths, MAXDCODES, &max_len);
}

static int fixed(state *s) {
  pthread_once(&g_fixed_once, build_fixed);
  return codes(s, &g_fixed_len, &g_fixed_dist);
}

static int dynamic(state *s) {
  static const short order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
  short lengths[MAXLCODES + MAXDCODES];
  huffman lencode, distcode;
  int max_len;
  const int nlen = (int)getbits(s, 5) + 257;
  const int ndist = (int)getbits(s, 5) + 1;
  const int ncode = (int)getbits(s, 4) + 4;
  if (s->err) return s->err;
  if (nlen > 286 || ndist > 30) return INF_ERR_CODES;
  int index;
  for (index = 0; index < ncode; index++) lengths[order[index]] = (short)getbits(s, 3);
  for (; index < 19; index++) lengths[order[index]] = 0;
  if (s->err) return s->err;
  if (construct(&lencode, lengths, 19, &max_len) != 0) return INF_ERR_CODES; /* must be complete */
  index = 0;
  while (index < nlen + ndist) {
    int sym = decode(s, &lencode);
    if (s->err) return s->err;
    if (sym < 0) return INF_ERR_CODES;
    if (sym < 16) {
      lengths[index++] = (short)sym;
      continue;
    }
    short len = 0;
    int rep;
    if (sym == 16) {
      if (index == 0) return INF_ERR_CODES;
      len = lengths[index - 1];
      rep = 3 + (int)getbits(s, 2);
    } else if (sym == 17) {
      rep = 3 + (int)getbits(s, 3);
    } else {
      rep = 11 + (int)getbits(s, 7);
    }
    if (s->err) return s->err;
    if (index + rep > nlen + ndist) return INF_ERR_CODES;
    while (rep--) lengths[index++] = len;
  }
  if (lengths[256] == 0) return INF_ERR_CODES;
  int left = construct(&lencode, lengths, nlen, &max_len);
  if (!code_ok(left, max_len)) return INF_ERR_CODES;
  left = construct(&distcode, lengths + nlen, ndist, &max_len);
  if (!code_ok(left, max_len)) return INF_ERR_CODES;
  return codes(s, &lencode, &distcode);
}

/* Inflate one raw DEFLATE stream.  *out_len = bytes produced (valid only on
 * INF_OK), *consumed = input bytes used through the end of the final block. */
int oracle_inflate(const uint8_t *src, size_t src_len, uint8_t *dst, size_t cap, size_t *out_len,
                   size_t *consumed) {
  state s;
  memset(&s, 0, sizeof(s));
  s.in = src;
  s.inlen = src_len;
  s.out = dst;
  s.outcap = cap;
  int last, rc;
  do {
    last = (int)getbits(&s, 1);
    const int type = (int)getbits(&s, 2);
    if (s.err) {
      rc = s.err;
      break;
    }
    if (type == 0)
      rc = stored(&s);
    else if (type == 1)
      rc = fixed(&s);
    else if (type == 2)
      rc = dynamic(&s);
    else
      rc = INF_ERR_BLOCK_TYPE;
  } while (!last && rc == INF_OK);
  if (out_len) *out_len = s.outcnt;
  if (consumed) *consumed = s.incnt;
  return rc;
}

/* ------------------------------------------------- batch (pthread pool) */

typedef struct {
  const uint8_t *const *src;
  const uint64_t *src_len;
  uint8_t *const *dst;
  const uint64_t *cap;
  uint64_t *out_len;
  int32_t *status;
  size_t n;
  int nthreads, tid;
} batch_job;

static void *batch_worker(void *p) {
  batch_job *j = (batch_job *)p;
  for (size_t i = (size_t)j->tid; i < j->n; i += (size_t)j->nthreads) {
    size_t ol = 0;
    j->status[i] = oracle_inflate(j->src[i], j->src_len[i], j->dst[i], j->cap[i], &ol, NULL);
    j->out_len[i] = ol;
  }
  return NULL;
}

int oracle_inflate_batch(const uint8_t *const *src, const uint64_t *src_len, uint8_t *const *dst,
                         const uint64_t *cap, uint64_t *out_len, int32_t *status, size_t n, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  batch_job jobs[256];
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (batch_job){src, src_len, dst, cap, out_len, status, n, nthreads, t};
    if (pthread_create(&th[t], NULL, batch_worker, &jobs[t]) != 0) return -1;
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  return 0;
}
