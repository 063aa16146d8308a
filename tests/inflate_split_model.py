"""CPU model of the block-parallel (speculative) inflate of ONE raw DEFLATE
stream -- TEST INFRASTRUCTURE, the specification the GPU kernels of
zipsfs_amd/csrc/zcrc_inflate_split.hip follow.

Why: ZIPsFS preloads one deflated entry at a time (zip_fread() inside
preloadram_now, src/ZIPsFS_preloadfileram.c:286-306; libzip inflates with
zlib), so the batched inflate -- one wave per stream -- decodes a single large
entry on one wave.  DEFLATE is serial inside a stream, but its blocks start at
bit positions that can be found without decoding what precedes them, and a
block's symbols can be decoded without its 32 KiB history if back-references
into that history are kept as markers.  The algorithm (the two-pass scheme of
pugz / rapidgzip, restated from the published descriptions):

1. **Find.**  The compressed stream is cut into chunks of `chunk_bytes`.  For
   chunk i (i >= 1) the finder returns the first bit position in
   [8 i chunk_bytes, 8 (i+1) chunk_bytes) where a dynamic-Huffman block
   header is valid by zlib 1.2.11's rules (`header_ok`).  Every true dynamic
   block start passes; a false positive only costs work (step 3).  Chunk 0
   starts at bit 0.  Stored and fixed-Huffman blocks are not searched for:
   the chunk before simply decodes through them.
2. **Speculative decode.**  Chunk i decodes from its candidate with an
   unknown history: output elements are bytes (0..255) or markers
   `kMarker + w`, "byte w of the 32 KiB before the chunk's first output"
   (w = 32768 + position, position < 0).  A copy propagates markers.  At
   every block start at or beyond the next candidate c_j (j > i) it stops
   when its position equals c_j (link i -> j); a candidate it steps over was
   a false positive and is skipped.  It also stops at the end of the final
   block, or on an error.
3. **Chain.**  Starting at chunk 0 (a true start), follow the links to the
   chunk that decoded the final block.  Every chunk on the chain started at
   a true block boundary (its predecessor's decode reached it), so its
   elements are the stream's, up to the markers.  Off-chain chunks are
   discarded.  Any error on the chain, a marker reaching before the stream
   start, output beyond `cap` or a chunk's output region overflowing sends
   the stream to the serial decoder, which reports zlib's exact status.
4. **Resolve.**  Output offsets are the prefix sum along the chain.  The
   last 32 KiB of each chain chunk are resolved in chain order (each needs
   only its predecessor's resolved tail); then every chunk's remaining
   markers are resolved in parallel from those tails.

The model returns the bytes and the chain statistics; tests check the bytes
against zlib.decompress and the oracle.
"""
from __future__ import annotations

from dataclasses import dataclass, field

CLEN_ORDER = (16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15)
MARKER = 0x8000  # element >= MARKER: byte (element - MARKER) of the 32 KiB window before the chunk
WINDOW = 32768

OK, ERR_BLOCK_TYPE, ERR_STORED_LEN, ERR_CODES, ERR_SYMBOL, ERR_DIST, ERR_OUTPUT, ERR_INPUT = range(8)


class Bits:
    """LSB-first bit reader at an arbitrary bit position; bits past the end
    read as zero and set `over` (the caller turns it into ERR_INPUT)."""

    def __init__(self, data: bytes, bitpos: int = 0):
        self.d = data
        self.n = len(data)
        self.pos = bitpos

    def peek(self, k: int) -> int:
        p = self.pos
        b0 = p >> 3
        chunk = self.d[b0:b0 + 4 + (k >> 3)]
        v = int.from_bytes(chunk, "little") >> (p & 7)
        return v & ((1 << k) - 1)

    def get(self, k: int) -> int:
        v = self.peek(k)
        self.pos += k
        return v

    @property
    def over(self) -> bool:
        return self.pos > 8 * self.n


def build(lengths, n: int, clen: bool):
    """Canonical code over lengths[0:n] -> (lut dict (len, code) -> symbol,
    max_len) or None where zlib rejects it (over-subscribed; incomplete
    unless a single length-1 code -- never for the code-length code)."""
    count = [0] * 16
    for L in lengths[:n]:
        count[L] += 1
    count[0] = 0
    left = 1
    for L in range(1, 16):
        left = 2 * left - count[L]
        if left < 0:
            return None
    max_len = max((L for L in range(1, 16) if count[L]), default=0)
    if left > 0 and max_len and (clen or max_len != 1):
        return None
    code, first = 0, [0] * 16
    for L in range(1, 16):
        code = (code + count[L - 1]) << 1 if L > 1 else 0
        first[L] = code
    nxt = first[:]
    table = {}
    for s in range(n):
        L = lengths[s]
        if L:
            table[(L, nxt[L])] = s
            nxt[L] += 1
    return table, max_len


def decode_sym(br: Bits, code):
    table, max_len = code
    c = 0
    for L in range(1, max_len + 1):
        c = (c << 1) | br.get(1)
        s = table.get((L, c))
        if s is not None:
            return s
    return -1


FIXED_LL = None
FIXED_D = None


def fixed_codes():
    global FIXED_LL, FIXED_D
    if FIXED_LL is None:
        ll = [8] * 144 + [9] * 112 + [7] * 24 + [8] * 8
        FIXED_LL = build(ll, 288, False)
        FIXED_D = build([5] * 32, 32, False)
    return FIXED_LL, FIXED_D


def read_dynamic(br: Bits):
    """The dynamic header at br.pos (after BFINAL/BTYPE): (status, ll, d)."""
    nlen = br.get(5) + 257
    ndist = br.get(5) + 1
    ncode = br.get(4) + 4
    if nlen > 286 or ndist > 30:
        return ERR_CODES, None, None
    lengths = [0] * 19
    for i in range(ncode):
        lengths[CLEN_ORDER[i]] = br.get(3)
    cl = build(lengths, 19, True)
    if cl is None or cl[1] == 0:
        return ERR_CODES, None, None
    lens = []
    total = nlen + ndist
    while len(lens) < total:
        sym = decode_sym(br, cl)
        if sym < 0:
            return ERR_CODES, None, None
        if sym < 16:
            lens.append(sym)
            continue
        if sym == 16:
            if not lens:
                return ERR_CODES, None, None
            val, rep = lens[-1], 3 + br.get(2)
        elif sym == 17:
            val, rep = 0, 3 + br.get(3)
        else:
            val, rep = 0, 11 + br.get(7)
        if len(lens) + rep > total:
            return ERR_CODES, None, None
        lens.extend([val] * rep)
    if br.over:
        return ERR_INPUT, None, None
    if lens[256] == 0:
        return ERR_CODES, None, None
    ll = build(lens, nlen, False)
    d = build(lens[nlen:], ndist, False)
    if ll is None or d is None:
        return ERR_CODES, None, None
    return OK, ll, d


def header_ok(data: bytes, bitpos: int) -> bool:
    """A valid dynamic block header starts at bitpos (the finder's test)."""
    br = Bits(data, bitpos)
    br.get(1)
    if br.get(2) != 2:
        return False
    st, _, _ = read_dynamic(br)
    return st == OK


def find_candidates(data: bytes, chunk_bytes: int):
    """Candidate block starts, one per chunk (None: none in the chunk)."""
    nchunks = max(1, -(-len(data) // chunk_bytes))
    cand = [0]
    for i in range(1, nchunks):
        lo, hi = 8 * i * chunk_bytes, min(8 * (i + 1) * chunk_bytes, 8 * len(data))
        c = None
        for p in range(lo, hi):
            if header_ok(data, p):
                c = p
                break
        cand.append(c)
    return cand


LEN_BASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195,
            227, 258]
LEN_EXTRA = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DIST_BASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
             4097, 6145, 8193, 12289, 16385, 24577]
DIST_EXTRA = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]


@dataclass
class ChunkResult:
    start: int                 # bit position the chunk decoded from
    status: int = OK
    final: bool = False        # ended with the final block
    link: int = -1             # index of the candidate it stopped at (-1: none)
    out: list = field(default_factory=list)
    reach: int = 0             # furthest marker reach before the chunk start (bytes)
    end_bit: int = 0


def spec_decode(data: bytes, start: int, cand, me: int, spec: bool, limit: int | None = None) -> ChunkResult:
    """Decode from bit `start`; stop at a block start equal to a candidate
    c_j (j > me), at the end of the final block, or on an error.  `spec`:
    the history is unknown (markers); chunk 0 decodes exactly."""
    br = Bits(data, start)
    res = ChunkResult(start=start)
    out = res.out
    j = me + 1
    while True:
        pos = br.pos
        while j < len(cand) and (cand[j] is None or cand[j] < pos):
            j += 1
        if j < len(cand) and cand[j] == pos and me >= 0:
            res.link = j
            break
        last = br.get(1)
        typ = br.get(2)
        if br.over:
            res.status = ERR_INPUT
            break
        st = OK
        if typ == 0:
            br.pos = (br.pos + 7) & ~7
            ln, nln = br.get(16), br.get(16)
            if ln != (~nln & 0xFFFF):
                st = ERR_STORED_LEN
            elif br.pos // 8 + ln > len(data):
                st = ERR_INPUT
            else:
                b = br.pos // 8
                out.extend(data[b:b + ln])
                br.pos += 8 * ln
        elif typ == 3:
            st = ERR_BLOCK_TYPE
        else:
            if typ == 1:
                ll, dd = fixed_codes()
            else:
                st, ll, dd = read_dynamic(br)
            if st == OK:
                st = codes(br, ll, dd, out, res, spec)
        if st == OK and br.over:
            st = ERR_INPUT
        if st != OK:
            res.status = st
            break
        if limit is not None and len(out) > limit:
            res.status = ERR_OUTPUT
            break
        if last:
            res.final = True
            break
    res.end_bit = br.pos
    return res


def codes(br: Bits, ll, dd, out: list, res: ChunkResult, spec: bool) -> int:
    while True:
        sym = decode_sym(br, ll)
        if sym < 0 or br.over:
            return ERR_INPUT if br.over else ERR_SYMBOL
        if sym < 256:
            out.append(sym)
            continue
        if sym == 256:
            return OK
        k = sym - 257
        if k >= 29:
            return ERR_SYMBOL
        length = LEN_BASE[k] + br.get(LEN_EXTRA[k])
        ds = decode_sym(br, dd)
        if ds < 0 or ds >= 30:
            return ERR_INPUT if br.over else ERR_SYMBOL
        dist = DIST_BASE[ds] + br.get(DIST_EXTRA[ds])
        if br.over:
            return ERR_INPUT
        p = len(out)
        if MATCH_HOOK is not None:
            MATCH_HOOK(p, length, dist, spec)
        if dist > p:
            if not spec or dist > p + WINDOW:
                return ERR_DIST
            res.reach = max(res.reach, dist - p)
        for t in range(length):
            s = p - dist + t
            out.append(out[s] if s >= 0 else MARKER + WINDOW + s)


MATCH_HOOK = None  # tests: called with (position, length, distance, spec) per match of codes()


def inflate_split(data: bytes, cap: int, chunk_bytes: int, region=None):
    """The whole scheme.  Returns (status, bytes, stats); status None means
    'fell back to the serial decoder' (stats['fallback'] says why)."""
    cand = find_candidates(data, chunk_bytes)
    results = {}
    for i, c in enumerate(cand):
        if c is None:
            continue
        lim = region(i, cand) if region else None
        results[i] = spec_decode(data, c, cand, i, spec=(i > 0), limit=lim)
    chain, i = [], 0
    stats = {"chunks": len(cand), "candidates": sum(c is not None for c in cand), "fallback": None}
    while True:
        r = results[i]
        chain.append(i)
        if r.status != OK:
            stats["fallback"] = f"chunk {i} status {r.status}"
            return None, None, stats
        if r.final:
            break
        if r.link < 0:
            stats["fallback"] = f"chunk {i} neither final nor linked"
            return None, None, stats
        i = r.link
    stats["chain"] = len(chain)
    if (results[chain[-1]].end_bit + 7) // 8 > len(data):
        stats["fallback"] = "input"
        return None, None, stats
    offs, o = [], 0
    for i in chain:
        offs.append(o)
        if results[i].reach > o:
            stats["fallback"] = "distance before the stream start"
            return None, None, stats
        o += len(results[i].out)
    if o > cap:
        stats["fallback"] = "output"
        return None, None, stats
    dst = bytearray(o)
    # tails in chain order, then the rest (the GPU's two resolve passes)
    for m, i in enumerate(chain):
        el, base = results[i].out, offs[m]
        for t in range(max(0, len(el) - WINDOW), len(el)):
            v = el[t]
            dst[base + t] = v if v < MARKER else dst[base - WINDOW + (v - MARKER)]
    for m, i in enumerate(chain):
        el, base = results[i].out, offs[m]
        for t in range(0, max(0, len(el) - WINDOW)):
            v = el[t]
            dst[base + t] = v if v < MARKER else dst[base - WINDOW + (v - MARKER)]
    return OK, bytes(dst), stats


# ------------------------------------------------------------------ parts
# Round 3, second level: a chunk whose candidate starts a long block is cut
# into `parts` items.  Item (k, j >= 1) starts at b_j, a token boundary found
# by a probe: decode `probe_tokens` tokens of chunk k's first block (tables
# from the header at c_k) from the guess g_j = c_k + j |R_k| / parts and take
# the position after them -- Huffman codes resynchronise, usually within a
# few dozen tokens, so b_j is a true token boundary with high probability.
# It is only trusted once an earlier item lands on it exactly: while inside
# chunk k's first block an item checks every token boundary against the
# later b_m of its chunk (landing -> link to item (k, m)); one it steps over
# is skipped (that item's work is wasted).  Past that block only candidates
# are targets, at block starts, as above.


def probe(data: bytes, c: int, guess: int, ntok: int):
    """Position after ntok tokens decoded from `guess` with the tables of the
    block whose header is at c; None when the decode meets an end of block
    or an invalid code first (the guess is not inside that block's codes)."""
    br = Bits(data, c)
    br.get(3)
    st, ll, dd = read_dynamic(br)
    if st != OK or guess < br.pos:
        return None
    br.pos = guess
    for _ in range(ntok):
        sym = decode_sym(br, ll)
        if sym < 0 or sym == 256 or sym >= 286 or br.over:
            return None
        if sym > 256:
            k = sym - 257
            br.get(LEN_EXTRA[k])
            ds = decode_sym(br, dd)
            if ds < 0 or ds >= 30:
                return None
            br.get(DIST_EXTRA[ds])
        if br.over:
            return None
    return br.pos


def part_decode(data: bytes, start: int, hdr, targets, cand, me_chunk: int, spec: bool):
    """Decode item from `start`: a block header when hdr is None (item j =
    0), else a token boundary inside the block whose header is at hdr.
    targets: [(b_m, m)] of the later items of this chunk, checked at every
    token boundary while in that first block; candidates of later chunks are
    checked at block starts.  Returns (ChunkResult, link), link = ("part", m)
    or ("chunk", k') or None."""
    br = Bits(data, start)
    res = ChunkResult(start=start)
    out = res.out
    ti, j = 0, me_chunk + 1
    in_first = True
    if hdr is not None:
        hb = Bits(data, hdr)
        bfinal = hb.get(1)
        hb.get(2)
        _, ll, dd = read_dynamic(hb)
        st, landed, ti = codes_targets(br, ll, dd, out, res, spec, targets, ti)
        in_first = False
        if st != OK or landed is not None or bfinal:
            res.status = st
            res.final = st == OK and landed is None and bool(bfinal)
            res.end_bit = br.pos
            return res, (("part", landed) if landed is not None else None)
    link = None
    while True:
        pos = br.pos
        while j < len(cand) and (cand[j] is None or cand[j] < pos):
            j += 1
        if j < len(cand) and cand[j] == pos:
            link = ("chunk", j)
            break
        last = br.get(1)
        typ = br.get(2)
        if br.over:
            res.status = ERR_INPUT
            break
        landed = None
        if typ == 0:
            br.pos = (br.pos + 7) & ~7
            ln, nln = br.get(16), br.get(16)
            if ln != (~nln & 0xFFFF):
                res.status = ERR_STORED_LEN
                break
            b = br.pos // 8
            if b + ln > len(data):
                res.status = ERR_INPUT
                break
            out.extend(data[b:b + ln])
            br.pos += 8 * ln
        elif typ == 3:
            res.status = ERR_BLOCK_TYPE
            break
        else:
            if typ == 1:
                ll, dd = fixed_codes()
            else:
                st, ll, dd = read_dynamic(br)
                if st != OK:
                    res.status = st
                    break
            st, landed, ti = codes_targets(br, ll, dd, out, res, spec, targets if in_first else [], ti)
            if st != OK:
                res.status = st
                break
        in_first = False
        if landed is not None:
            link = ("part", landed)
            break
        if br.over:
            res.status = ERR_INPUT
            break
        if last:
            res.final = True
            break
    res.end_bit = br.pos
    return res, link


def codes_targets(br: Bits, ll, dd, out: list, res: ChunkResult, spec: bool, targets, ti: int):
    """codes() with per-token landing checks: (status, landed item index or
    None, next target index)."""
    while True:
        while ti < len(targets) and targets[ti][0] < br.pos:
            ti += 1
        if ti < len(targets) and targets[ti][0] == br.pos:
            return OK, targets[ti][1], ti
        sym = decode_sym(br, ll)
        if sym < 0 or br.over:
            return (ERR_INPUT if br.over else ERR_SYMBOL), None, ti
        if sym < 256:
            out.append(sym)
            continue
        if sym == 256:
            return OK, None, ti
        k = sym - 257
        if k >= 29:
            return ERR_SYMBOL, None, ti
        length = LEN_BASE[k] + br.get(LEN_EXTRA[k])
        ds = decode_sym(br, dd)
        if ds < 0 or ds >= 30:
            return (ERR_INPUT if br.over else ERR_SYMBOL), None, ti
        dist = DIST_BASE[ds] + br.get(DIST_EXTRA[ds])
        if br.over:
            return ERR_INPUT, None, ti
        p = len(out)
        if dist > p:
            if not spec or dist > p + WINDOW:
                return ERR_DIST, None, ti
            res.reach = max(res.reach, dist - p)
        for t in range(length):
            s = p - dist + t
            out.append(out[s] if s >= 0 else MARKER + WINDOW + s)


def inflate_split_parts(data: bytes, cap: int, chunk_bytes: int, parts: int = 8, probe_tokens: int = 64,
                        max_parts: int = 0):
    """The scheme with `parts` items per chunk.  Returns (status, bytes,
    stats) like inflate_split (status None: the serial decoder runs).
    max_parts > parts: a chunk with a candidate borrows the items of the
    candidate-less chunks after it, cutting its block into
    T = min(max_parts, (kn - k) parts) parts (zcrc_inflate_impl.h owner();
    the GPU's max_parts is kMaxParts = 64)."""
    cand = find_candidates(data, chunk_bytes)
    nbits = 8 * len(data)
    max_parts = max(max_parts, parts)
    starts = {}  # (k, j) -> (start, hdr)
    tg = {}      # k -> [(b_m, m)]
    for k, c in enumerate(cand):
        if c is None:
            continue
        kn = next((x for x in range(k + 1, len(cand)) if cand[x] is not None), len(cand))
        nxt = cand[kn] if kn < len(cand) else nbits
        T = min(max_parts, (kn - k) * parts)
        starts[(k, 0)] = (c, None)
        bs = []
        if k > 0 or c == 0:
            last = c
            for m in range(1, T):
                b = probe(data, c, c + m * ((nxt - c) // T), probe_tokens)
                if b is not None and last < b < nxt:
                    bs.append((b, m))
                    starts[(k, m)] = (b, c)
                    last = b
        tg[k] = bs
    results = {}
    for (k, m), (st, hdr) in starts.items():
        targets = [t for t in tg[k] if t[1] > m]
        results[(k, m)] = part_decode(data, st, hdr, targets, cand, k, spec=(k, m) != (0, 0))
    chain, item = [], (0, 0)
    stats = {"chunks": len(cand), "items": len(starts), "fallback": None}
    while True:
        r, link = results[item]
        chain.append(item)
        if r.status != OK:
            stats["fallback"] = f"item {item} status {r.status}"
            return None, None, stats
        if r.final:
            break
        if link is None:
            stats["fallback"] = f"item {item} neither final nor linked"
            return None, None, stats
        item = (item[0], link[1]) if link[0] == "part" else (link[1], 0)
    stats["chain"] = len(chain)
    if (results[chain[-1]][0].end_bit + 7) // 8 > len(data):
        stats["fallback"] = "input"
        return None, None, stats
    out = bytearray()
    for it in chain:
        r = results[it][0]
        if r.reach > len(out):
            stats["fallback"] = "distance before the stream start"
            return None, None, stats
        base = len(out)
        for v in r.out:
            out.append(v if v < MARKER else out[base - WINDOW + (v - MARKER)])
    if len(out) > cap:
        stats["fallback"] = "output"
        return None, None, stats
    return OK, bytes(out), stats
