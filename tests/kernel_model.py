"""CPU model of zcrc_kernels.hip's decomposition (TEST INFRASTRUCTURE).

Re-executes, with numpy over the 64 lanes x 4 dword streams, exactly the
arithmetic the HIP kernel performs -- wave-range partition and boundary
snapping, 16-B aligned 1 KiB blocks with out-of-range zero fill, edge
fix-ups (mask + seed injection), the braided MCT(x^8192) stream update, the
in-lane / cross-lane combine tree, the x^(-8t) alignment shift, split-piece
x^(8d) shifts and xor combine.  Checked against the oracle on CPU so that
decomposition bugs are caught without a GPU; the GPU tests then check the
real kernel against the oracle.
"""
from __future__ import annotations

import numpy as np

POLY = 0xEDB88320
ONE = 0x80000000

# constants mirrored from zcrc_internal.h
K_WAVES = 16
K_MIN_RANGE = 64 << 10
K_SPLIT_GRAIN = 64 << 10
K_SPLIT_MIN = 2 * K_SPLIT_GRAIN
K_MIN_PIECE = 4096
K_DYN_UNIT = 128 << 10
K_DYN_AUTO = 0xFF
K_DYN_SHIFT = K_DYN_AUTO
K_DYN_SMALL_AVG = 512 << 10


def times_x(r: int) -> int:
    return (r >> 1) ^ (POLY if r & 1 else 0)


def times_xinv(r: int) -> int:
    return (((r ^ POLY) << 1) | 1) & 0xFFFFFFFF if r & 0x80000000 else (r << 1) & 0xFFFFFFFF


def gf2_mul(a: int, b: int) -> int:
    p = 0
    for i in range(32):
        if (a >> (31 - i)) & 1:
            p ^= b
        b = times_x(b)
    return p


def xpow8(nbytes: int) -> int:
    acc, v, k = ONE, ONE >> 1, 0
    x2k = [v]
    for _ in range(70):
        v = gf2_mul(v, v)
        x2k.append(v)
    k = 3
    while nbytes:
        if nbytes & 1:
            acc = gf2_mul(acc, x2k[k])
        nbytes >>= 1
        k += 1
    return acc


def x8grain_table() -> list:
    """zcrc_tables.h x8grain[j][m] = x^(8 * 65536 * m * 256^j): base
    x^(2^(19 + 8j)) raised to m (TableBlob; the split-piece shift)."""
    x2k, v = [], ONE >> 1
    for _ in range(51):
        x2k.append(v)
        v = gf2_mul(v, v)
    out = []
    for j in range(4):
        g, row = ONE, []
        for _ in range(256):
            row.append(g)
            g = gf2_mul(g, x2k[19 + 8 * j])
        out.append(row)
    return out


def grain_shift(r: int, nbytes: int, grain=None) -> int:
    """zcrc_batch_kernel.h shift_bytes for nbytes = 65536 m: r times at most
    four x8grain products (byte j of m picks row j)."""
    assert nbytes % 65536 == 0 and nbytes < 1 << 48
    g = grain or x8grain_table()
    m = nbytes >> 16
    r = gf2_mul(g[0][m & 255], r)
    for j in (1, 2, 3):
        if m >> (8 * j):
            r = gf2_mul(g[j][(m >> (8 * j)) & 255], r)
    return r


def xinvpow8(nbytes: int) -> int:
    r = ONE
    for _ in range(8 * nbytes):
        r = times_xinv(r)
    return r


def mct(c: int) -> np.ndarray:
    t = np.zeros((4, 256), dtype=np.uint32)
    # linearity: build from the 32 single-bit products
    bits = [gf2_mul(c, 1 << b) for b in range(32)]
    for j in range(4):
        for v in range(256):
            acc = 0
            for b in range(8):
                if (v >> b) & 1:
                    acc ^= bits[8 * j + b]
            t[j, v] = acc
    return t


def mct_apply(t: np.ndarray, r):
    r = np.asarray(r, dtype=np.uint32)
    return (t[0][r & 0xFF] ^ t[1][(r >> 8) & 0xFF] ^ t[2][(r >> 16) & 0xFF] ^ t[3][r >> 24]).astype(np.uint32)


class Tables:
    def __init__(self):
        self.braid = mct(xpow8(1024))
        self.braid256 = mct(xpow8(256))  # the small-buffer kernel's table
        self.braid128 = mct(xpow8(128))  # its table for 128-B blocks (8 lanes)
        self.comb = [mct(xinvpow8(b)) for b in (4, 8, 16, 32, 64, 128, 256, 512)]
        self.tshift = [mct(xinvpow8(t)) for t in range(16)]
        # r * x^-8 = (r << 8) ^ xinv8[r >> 24] (zcrc_gf2.h build_xinv8_table)
        self.xinv8 = np.zeros(256, dtype=np.uint32)
        std = np.zeros(256, dtype=np.uint32)
        for v in range(256):
            r = v
            for _ in range(8):
                r = times_x(r)
            std[v] = r
        self.stdtab = std
        for v in range(256):
            self.xinv8[int(std[v]) >> 24] = ((int(std[v]) << 8) & 0xFFFFFFFF) | v


_TABLES = None


def tables() -> Tables:
    global _TABLES
    if _TABLES is None:
        _TABLES = Tables()
    return _TABLES


# ------------------------------------------------------------ partition

class Batch:
    """Buffers as (address, length) into one flat numpy 'memory'."""

    def __init__(self, memory: np.ndarray, addrs, lens, seeds=None):
        self.mem = memory
        self.addrs = [int(a) for a in addrs]
        self.lens = [int(n) for n in lens]
        self.seeds = [0] * len(self.lens) if seeds is None else [int(s) & 0xFFFFFFFF for s in seeds]
        self.prefix = np.concatenate([[0], np.cumsum(np.asarray(self.lens, dtype=np.uint64))]).astype(np.uint64)
        self.n = len(self.lens)
        self.total = int(self.prefix[-1])

    def lower_bound(self, t: int) -> int:
        return int(np.searchsorted(self.prefix, np.uint64(t), side="left"))

    def snap(self, t: int) -> int:
        tot = self.total
        if t == 0 or t >= tot:
            return tot if t >= tot else 0
        i = self.lower_bound(t)
        pi = int(self.prefix[i])
        if pi == t:
            return t
        b0 = int(self.prefix[i - 1])
        n, p = pi - b0, t - b0
        if n < K_SPLIT_MIN:
            return pi
        q = n - K_SPLIT_GRAIN * ((n - p) // K_SPLIT_GRAIN)
        if q < K_MIN_PIECE:
            return b0
        return b0 + q


def device_lower_bound(prefix, n: int, t: int):
    """BatchView::lower_bound_ex (zcrc_batch_kernel.h): the wave-wide 64-ary
    search whose last level loads prefix(lo-1 .. lo+62) -> (i, prefix(i),
    prefix(i-1))."""
    lo, hi = 0, n
    while hi - lo > 62:
        step = (hi - lo + 63) // 64
        f = next(l for l in range(64) if int(prefix[min(lo + (l + 1) * step, hi)]) >= t)
        nhi = min(lo + (f + 1) * step, hi)
        lo, hi = (lo if f == 0 else lo + f * step + 1), nhi
    v = [int(prefix[lo + l - 1]) if (lo + l >= 1 and lo + l - 1 <= hi) else None for l in range(64)]
    f = next(l for l in range(1, 64) if v[l] is not None and v[l] >= t)
    r = lo - 1 + f
    return r, v[f], (v[f - 1] if r else 0)


def device_snap(batch: "Batch", t: int):
    """BatchView::snap_at on the device search: (S, lb = lower_bound(S),
    first = the first buffer overlapping [S, ...))."""
    tot, n = batch.total, batch.n
    if t == 0:
        return 0, 0, 0
    if t >= tot:
        x = device_lower_bound(batch.prefix, n, tot)[0]
        return tot, x, x
    i, pi, pim1 = device_lower_bound(batch.prefix, n, t)
    if pi == t:
        return t, i, i
    b0 = pim1
    m, p = pi - b0, t - b0
    if m < K_SPLIT_MIN:
        return pi, i, i
    q = m - K_SPLIT_GRAIN * ((m - p) // K_SPLIT_GRAIN)
    if q < K_MIN_PIECE:
        x = device_lower_bound(batch.prefix, n, b0)[0]
        return b0, x, x
    return b0 + q, i, (i - 1 if q < m else i)


def wave_ranges(batch: Batch, num_cus: int, dyn_shift: int = K_DYN_SHIFT, unit: int = K_DYN_UNIT):
    """Every (s0, s1, last) range the kernel processes: W static wave ranges
    over the first Ts bytes, then the dynamic units of `unit` nominal bytes
    over the last Td = total >> dyn_shift bytes (zcrc_batch_kernel.h,
    crc32_batch_kernel).  Which wave claims a unit does not matter for the
    result, so the model lists them in order."""
    total = batch.total
    want = max(1, (total + K_MIN_RANGE - 1) // K_MIN_RANGE, batch.n)
    W = min(want, num_cus * K_WAVES)
    if dyn_shift == K_DYN_AUTO:
        dyn_shift = 1 if batch.n and total // batch.n < K_DYN_SMALL_AVG else 2
    Td = (total >> dyn_shift) if dyn_shift else 0
    if Td // W < unit:
        Td = 0
    Ts = total - Td
    q, r = divmod(Ts, W)
    out = []
    for w in range(W):
        s0 = batch.snap(q * w + (r * w) // W)
        if w + 1 == W:
            s1 = batch.snap(Ts) if Td else total
        else:
            s1 = batch.snap(q * (w + 1) + (r * (w + 1)) // W)
        out.append((s0, s1, w + 1 == W and not Td))
    units = (Td + unit - 1) // unit if Td else 0
    for u in range(units):
        t0 = Ts + u * unit
        last = u + 1 == units
        s0 = batch.snap(min(t0, total))
        s1 = total if last else batch.snap(min(t0 + unit, total))
        out.append((s0, s1, last))
    return out


def wave_pieces(batch: Batch, s0: int, s1: int, last: bool):
    """(buffer, rel_lo, rel_hi) pieces of one wave, as the kernel walks them."""
    if s0 >= s1 and not last:
        return []
    i = batch.lower_bound(s0)
    if 0 < i <= batch.n and int(batch.prefix[i]) > s0:
        i -= 1
    pieces = []
    while i < batch.n:
        b0, b1 = int(batch.prefix[i]), int(batch.prefix[i + 1])
        if b0 >= s1 and not last:
            break
        n = b1 - b0
        rel_lo = s0 - b0 if s0 > b0 else 0
        rel_hi = n if (b1 < s1 or last) else s1 - b0
        pieces.append((i, rel_lo, rel_hi))
        i += 1
    return pieces


# ------------------------------------------------------------ one piece

def _lowmask(k):
    k = np.asarray(k, dtype=np.int64)
    kk = np.clip(k, 0, 3).astype(np.uint64)
    part = (np.uint64(1) << (np.uint64(8) * kk)) - np.uint64(1)
    return np.where(k <= 0, np.uint64(0), np.where(k >= 4, np.uint64(0xFFFFFFFF), part)).astype(np.uint64)


def _inj_word(inj: int, o):
    """Bits of the 4-byte injection landing in a dword at relative byte offset o."""
    o = np.asarray(o, dtype=np.int64)
    inj = np.uint64(inj)
    shl = (inj << (np.uint64(8) * np.clip(o, 0, 3).astype(np.uint64))) & np.uint64(0xFFFFFFFF)
    shr = inj >> (np.uint64(8) * np.clip(-o, 0, 3).astype(np.uint64))
    return np.where((o >= 0) & (o < 4), shl, np.where((o < 0) & (o > -4), shr, np.uint64(0))).astype(np.uint64)


def crc_piece(mem: np.ndarray, pstart: int, pend: int, inj: int, T: Tables) -> int:
    lanes = np.arange(64, dtype=np.int64)
    astart = pstart & ~15
    aend = (pend + 15) & ~15
    span = aend - astart  # the buffer resource's range: chunks outside read zeros
    agrid = (pend + 127) & ~127  # the block grid ends at the 128-B line after pend
    gspan = agrid - astart
    K = (gspan + 1023) >> 10
    tpad = agrid - pend
    c0 = gspan - 1024 * K + 16 * lanes
    rs, re = pstart - astart, pend - astart
    s = np.zeros((64, 4), dtype=np.uint32)
    for it in range(K):
        c = c0 + 1024 * it
        data = np.zeros((64, 16), dtype=np.uint8)
        ok = (c >= 0) & (c < span)
        for l in np.nonzero(ok)[0]:
            data[l] = mem[astart + c[l]: astart + c[l] + 16]
        words = data.view("<u4").astype(np.uint64)  # (64, 4)
        if it <= 1 or it + 1 == K:
            lo = np.clip(rs - c, -64, 64)
            hi = np.clip(re - c, -64, 64)
            io = lo.copy()
            for q in range(4):
                m = _lowmask(hi - 4 * q) & ~_lowmask(lo - 4 * q) & np.uint64(0xFFFFFFFF)
                words[:, q] = ((words[:, q] & m) ^ _inj_word(inj, io - 4 * q)) & np.uint64(0xFFFFFFFF)
        x = (s.astype(np.uint64) ^ words).astype(np.uint32)
        s = mct_apply(T.braid, x)
    s0, s1, s2, s3 = s[:, 0], s[:, 1], s[:, 2], s[:, 3]
    r = (s0 ^ mct_apply(T.comb[0], s1)) ^ mct_apply(T.comb[1], s2 ^ mct_apply(T.comb[0], s3))
    for j in range(6):
        moved = mct_apply(T.comb[2 + j], r)
        d = 1 << j
        shifted = np.concatenate([moved[d:], moved[64 - d:]])  # shfl_down: out of range keeps own
        shifted[64 - d:] = moved[64 - d:]
        r = r ^ shifted
    r0 = int(r[0])
    if tpad:  # < 128 (the kernel: combine tables of 4..64 bytes, then x^-1 steps)
        r0 = gf2_mul(r0, xinvpow8(tpad))
    return r0


def run_batch(batch: Batch, num_cus: int = 256, dyn_shift: int = K_DYN_SHIFT, unit: int = K_DYN_UNIT) -> np.ndarray:
    """CRCs of every buffer, computed the way the kernel computes them."""
    T = tables()
    out = np.zeros(batch.n, dtype=np.uint32)
    for (s0, s1, last) in wave_ranges(batch, num_cus, dyn_shift, unit):
        for (i, rel_lo, rel_hi) in wave_pieces(batch, s0, s1, last):
            n = batch.lens[i]
            seed = batch.seeds[i]
            whole = rel_lo == 0 and rel_hi == n
            if n < 4:
                r = (~seed) & 0xFFFFFFFF
                for p in range(n):
                    r = (r >> 8) ^ int(T.stdtab[(r ^ int(batch.mem[batch.addrs[i] + p])) & 0xFF])
                out[i] = (~r) & 0xFFFFFFFF
                continue
            inj = (~seed) & 0xFFFFFFFF if rel_lo == 0 else 0
            r = crc_piece(batch.mem, batch.addrs[i] + rel_lo, batch.addrs[i] + rel_hi, inj, T)
            if whole:
                out[i] = (~r) & 0xFFFFFFFF
            else:
                d = n - rel_hi
                contrib = gf2_mul(xpow8(d), r) if d else r ^ 0xFFFFFFFF
                out[i] ^= np.uint32(contrib)
    return out


def run_one_launch(batch: Batch, num_cus: int = 256) -> np.ndarray:
    """The one-launch kernel's round-4 per-buffer mode (zcrc_batch_kernel.h,
    kPB = 4; n <= 16 x CUs): every buffer of at most kPerBufMax bytes is
    checksummed whole by its own wave; when any buffer is longer, the
    in-kernel scan runs over effective lengths (the short buffers count as
    empty) and its walk skips the short buffers (skip_small), so every
    buffer is computed exactly once."""
    assert batch.n <= K_WAVES * num_cus
    T = tables()
    out = np.zeros(batch.n, dtype=np.uint32)
    short = [L <= K_PER_BUF_MAX for L in batch.lens]
    for i in range(batch.n):
        if not short[i]:
            continue
        n, seed = batch.lens[i], batch.seeds[i]
        if n < 4:
            r = (~seed) & 0xFFFFFFFF
            for p in range(n):
                r = (r >> 8) ^ int(T.stdtab[(r ^ int(batch.mem[batch.addrs[i] + p])) & 0xFF])
            out[i] = (~r) & 0xFFFFFFFF
        else:
            out[i] = (~crc_piece(batch.mem, batch.addrs[i], batch.addrs[i] + n, (~seed) & 0xFFFFFFFF, T)) & 0xFFFFFFFF
    if all(short):
        return out
    eff = Batch(batch.mem, batch.addrs, [0 if sh else L for sh, L in zip(short, batch.lens)], batch.seeds)
    for (s0, s1, last) in wave_ranges(eff, num_cus):
        for (i, rel_lo, rel_hi) in wave_pieces(eff, s0, s1, last):
            if short[i]:
                continue  # skip_small
            n, seed = batch.lens[i], batch.seeds[i]
            inj = (~seed) & 0xFFFFFFFF if rel_lo == 0 else 0
            r = crc_piece(batch.mem, batch.addrs[i] + rel_lo, batch.addrs[i] + rel_hi, inj, T)
            if rel_lo == 0 and rel_hi == n:
                out[i] = (~r) & 0xFFFFFFFF
            else:
                d = n - rel_hi
                out[i] ^= np.uint32(gf2_mul(xpow8(d), r) if d else r ^ 0xFFFFFFFF)
    return out


# ------------------------------------------------------------ small-buffer kernel

def crc_small_group(mem: np.ndarray, pstart: int, length: int, seed: int, G: int, T: Tables,
                    extra_blocks: int = 0, blk: int = 256) -> int:
    """zcrc_small_kernel.h small_body for one buffer: G lanes, `blk`-byte
    blocks (256: MCT(x^2048); 128: MCT(x^1024), the product's 8-lane form),
    C = blk/16/G chunks per lane, end-aligned; `extra_blocks` leading blocks
    that load nothing (the wave runs its largest buffer's block count)."""
    if length < 4:
        r = (~seed) & 0xFFFFFFFF
        for p in range(length):
            r = (r >> 8) ^ int(T.stdtab[(r ^ int(mem[pstart + p])) & 0xFF])
        return (~r) & 0xFFFFFFFF
    C = blk // 16 // G
    astart = pstart & ~15
    rs = pstart - astart
    re = rs + length
    span = (re + 15) & ~15
    K = (span + blk - 1) // blk
    kmax = K + extra_blocks
    inj = (~seed) & 0xFFFFFFFF
    lanes = np.arange(G, dtype=np.int64)
    s = np.zeros((G, 4 * C), dtype=np.uint32)
    rel0 = span - blk * kmax + 16 * C * lanes
    for k in range(kmax):
        for c in range(C):
            rel = rel0 + blk * k + 16 * c
            data = np.zeros((G, 16), dtype=np.uint8)
            for l in range(G):
                if rel[l] >= 0:
                    data[l] = mem[astart + rel[l]: astart + rel[l] + 16]
            words = data.view("<u4").astype(np.uint64)
            edge = (rel >= 0) & ((rel < rs + 4) | (rel + 16 > re))
            lo = np.clip(rs - rel, -64, 64)
            hi = np.clip(re - rel, -64, 64)
            for q in range(4):
                m = _lowmask(hi - 4 * q) & ~_lowmask(lo - 4 * q) & np.uint64(0xFFFFFFFF)
                fixed = ((words[:, q] & m) ^ _inj_word(inj, lo - 4 * q)) & np.uint64(0xFFFFFFFF)
                words[:, q] = np.where(edge, fixed, words[:, q])
            x = (s[:, 4 * c:4 * c + 4].astype(np.uint64) ^ words).astype(np.uint32)
            s[:, 4 * c:4 * c + 4] = mct_apply(T.braid256 if blk == 256 else T.braid128, x)
    ns = 4 * C
    v = [s[:, m].copy() for m in range(ns)]
    t = 0
    while (1 << t) < ns:  # in-lane tree: combine tables 0.. (4 B, 8 B, 16 B)
        for m in range(0, ns, 2 << t):
            v[m] = v[m] ^ mct_apply(T.comb[t], v[m + (1 << t)])
        t += 1
    r = v[0]
    j = 0
    while (1 << j) < G:  # cross-lane: 16 C B apart, doubling
        moved = mct_apply(T.comb[t + j], r)
        d = 1 << j
        shifted = moved.copy()
        shifted[:G - d] = moved[d:]
        r = r ^ shifted
        j += 1
    r0 = int(r[0])
    tpad = span - re  # < 16
    for b in (1, 0):
        if tpad >> 2 & (1 << b):
            r0 = int(mct_apply(T.comb[b], np.array([r0], dtype=np.uint32))[0])
    for _ in range(tpad & 3):  # the x^-8 byte table (zcrc_small_kernel.h)
        r0 = ((r0 << 8) & 0xFFFFFFFF) ^ int(T.xinv8[r0 >> 24])
    return (~r0) & 0xFFFFFFFF


K_SMALL_MAX = 8192
K_SIZE_CLASSES = K_SMALL_MAX // 256 + 1
K_SMALL_COST = 14  # zcrc_internal.h kSmallCostDefault (quarters of a batch-kernel byte)
K_BIG_MIN = 1 << 20  # zcrc_internal.h kBigMin
K_SPLIT_MAX_TILES = 256  # zcrc_internal.h kSplitMaxTiles


def split_tile(n: int) -> int:
    """Buffers per split-plan tile (zcrc_internal.h split_per_thread): 1024 x
    the smallest of 1, 2, 4, 8 that keeps the tiles within kSplitMaxTiles."""
    per = 1
    while per < 8 and -(-n // (1024 * per)) > K_SPLIT_MAX_TILES:
        per *= 2
    return 1024 * per


def split_plan(lens, grid: int = 256, force: bool = False, small_cost: int = K_SMALL_COST, direct_ok: bool = True):
    """zcrc_kernels.hip plan_split_scatter's decisions and lists: (split,
    large list -- on a split, buffers below kBigMin first, then the others,
    each in index order -- with its prefix, small list tile by tile (split_tile(n)
    buffers), by size class within a tile and in index order within a class,
    small workgroups, small lanes)."""
    lens = [int(x) for x in lens]
    small = [i for i, L in enumerate(lens) if L <= K_SMALL_MAX]
    large = [i for i, L in enumerate(lens) if L > K_SMALL_MAX]
    as_ = sum(lens[i] for i in small)
    al = sum(lens[i] for i in large)
    ws, wl = small_cost * as_, 4 * al
    wgs = grid
    if large:
        wgs = (grid * ws + ws + wl - 1) // (ws + wl) if ws else 0
    split = bool(small) and (force or wgs >= 2)
    if large:
        wgs = min(max(wgs, 1), grid - 1)
    if not split:
        return dict(split=False, large=list(range(len(lens))), small=[], wgs=wgs, lanes=16)
    tile = split_tile(len(lens))
    by_class = sorted(small, key=lambda i: (i // tile, (lens[i] + 255) >> 8, i))
    lanes = 8 if as_ <= 2048 * len(small) else 16
    if not large and direct_ok:  # mode 2: about equal small buffers, walked in index order without lists
        mean = as_ / len(small)
        if sum(lens[i] * lens[i] for i in small) / len(small) - mean * mean <= 128.0 * 128.0:
            return dict(split=True, direct=True, large=[], small=list(small), wgs=grid, lanes=lanes)
    # round 4: the batch kernel's buffers medium first, then big (>= kBigMin), each in index order
    large = [i for i in large if lens[i] < K_BIG_MIN] + [i for i in large if lens[i] >= K_BIG_MIN]
    return dict(split=True, large=large, small=by_class, wgs=wgs, lanes=lanes)


# ---------------------------------------------------------------- one launch
K_PER_BUF_MAX = K_MIN_RANGE  # zcrc_internal.h kPerBufMax


def braid_lds_loaded() -> np.ndarray:
    """The batch kernel's LDS braid area (32768 words) as the table fill
    writes it from TableBlob::braid (zcrc_batch_kernel.h, load_tables):
    thread t writes the 16-B chunk c = t + 1024 k with 4 copies of
    braid[j][v], j = 2 (o >> 16) + ((o >> 7) & 1), v = (o >> 8) & 255, o = 16 c."""
    T = tables()
    lds = np.zeros(32768, dtype=np.uint32)
    for c in range(8192):
        o = 16 * c
        j = 2 * (o >> 16) + ((o >> 7) & 1)
        v = (o >> 8) & 255
        lds[4 * c:4 * c + 4] = T.braid[j, v]
    return lds


def braid_lds_built() -> np.ndarray:
    """The per-buffer mode's braid (zcrc_batch_kernel.h, braid_gen_lane and
    the ds_bpermute exchange): lane L of wave w builds entry (j = L >> 4,
    v = 4 w + (L & 3) + 64 ((L >> 2) & 3)) from the 32 single-bit products
    q[p] = x^8192 * (1 << p); thread (w, l) then writes chunk 64 w + l +
    1024 k with lane src = (l >> 4) + 4 (k & 3) + 16 (2 (k >> 2) + ((l >> 3) & 1))'s entry."""
    q = [gf2_mul(xpow8(1024), 1 << p) for p in range(32)]
    lds = np.zeros(32768, dtype=np.uint32)
    for w in range(16):
        e = []
        for L in range(64):
            j, v = L >> 4, 4 * w + (L & 3) + 64 * ((L >> 2) & 3)
            acc = 0
            for b in range(8):
                if (v >> b) & 1:
                    acc ^= q[8 * j + b]
            e.append(acc)
        for l in range(64):
            t = 64 * w + l
            for k in range(8):
                src = (l >> 4) + 4 * (k & 3) + 16 * (2 * (k >> 2) + ((l >> 3) & 1))
                c = t + 1024 * k
                lds[4 * c:4 * c + 4] = e[src]
    return lds


def comb_lds_built() -> np.ndarray:
    """The round-4 per-buffer mode's combine area (zcrc_batch_kernel.h,
    comb_gen): thread (w, l) writes chunk 64 w + l of tables 0..3 and chunk
    1024 + 64 w + l of tables 4..7; chunk t holds table c = t >> 8, row j =
    (t >> 6) & 3, entries v = 4 (t & 63) + e, e < 4, each the xor of the
    products q_c[8 j + b] = x^(-8 * 4 * 2^c) * (1 << (8 j + b)) over v's set bits
    (bits 2..7 from the lane, shared by its four entries)."""
    area = np.zeros(8192, dtype=np.uint32)
    for c in range(8):
        q = [gf2_mul(xinvpow8(4 << c), 1 << p) for p in range(32)]
        for w in range(16):
            if (w >> 2) != (c & 3):
                continue
            j = w & 3
            for l in range(64):
                t = (1024 if c >= 4 else 0) + 64 * w + l
                assert t >> 8 == c and (t >> 6) & 3 == j
                base = 0
                for i in range(6):
                    if (l >> i) & 1:
                        base ^= q[8 * j + 2 + i]
                words = [base, base ^ q[8 * j], base ^ q[8 * j + 1], base ^ q[8 * j] ^ q[8 * j + 1]]
                area[4 * t:4 * t + 4] = words
    return area


def per_buffer_plan(lens, num_cus: int = 256):
    """The one-launch kernel's per-buffer mode (zcrc_batch_kernel.h,
    crc32_batch_kernel, kFused): taken when n <= 16 x grid and no length
    exceeds kPerBufMax; then wave slot s of workgroup g checksums buffer
    s * grid + g whole.  Returns {buffer: (g, s)} or None (in-kernel scan)."""
    n = len(lens)
    if n > K_WAVES * num_cus or any(L > K_PER_BUF_MAX for L in lens):
        return None
    out = {}
    for g in range(num_cus):
        for s in range(K_WAVES):
            b = s * num_cus + g
            if b < n:
                out[b] = (g, s)
    return out
