"""A small FLAC encoder written from RFC 9639, used only by the tests to make
streams for the native decoder (csrc/ou_flac.cpp) -- libFLAC / soundfile are
not in this image.  Every subframe type, stereo mode, block-size / sample-size
code and Rice form the decoder handles can be forced per frame."""
import numpy as np


class BitWriter:
    def __init__(self):
        self.bits = []

    def put(self, v, k):
        v = int(v) & ((1 << k) - 1) if k else 0
        for i in range(k - 1, -1, -1):
            self.bits.append((v >> i) & 1)

    def unary(self, q):
        self.bits.extend([0] * q)
        self.bits.append(1)

    def align(self):
        while len(self.bits) % 8:
            self.bits.append(0)

    def bytes(self):
        assert len(self.bits) % 8 == 0
        a = np.packbits(np.array(self.bits, dtype=np.uint8))
        return a.tobytes()


def crc8(data):
    c = 0
    for b in data:
        c ^= b
        for _ in range(8):
            c = ((c << 1) ^ 0x07) & 0xFF if c & 0x80 else (c << 1) & 0xFF
    return c


def crc16(data):
    c = 0
    for b in data:
        c ^= b << 8
        for _ in range(8):
            c = ((c << 1) ^ 0x8005) & 0xFFFF if c & 0x8000 else (c << 1) & 0xFFFF
    return c


def _utf8(n):
    if n < 0x80:
        return bytes([n])
    for nb in range(2, 8):
        if n < (1 << (5 * nb + 1)):
            break
    out = []
    for _ in range(nb - 1):
        out.append(0x80 | (n & 0x3F))
        n >>= 6
    lead = ((0xFF << (8 - nb)) & 0xFF) | n
    return bytes([lead] + out[::-1])


def _residual(w, res, order, bsize, porder=0, method=0, escape=False):
    w.put(method, 2)
    w.put(porder, 4)
    pbits = 4 if method == 0 else 5
    part = bsize >> porder
    i = 0
    for p in range(1 << porder):
        cnt = part - (order if p == 0 else 0)
        chunk = res[i:i + cnt]
        i += cnt
        if escape:
            w.put((1 << pbits) - 1, pbits)
            raw = max(1, max((int(abs(v)).bit_length() + 1 for v in chunk), default=1))
            w.put(raw, 5)
            for v in chunk:
                w.put(v, raw)
            continue
        u = [(2 * int(v)) if v >= 0 else (-2 * int(v) - 1) for v in chunk]
        mean = (sum(u) / len(u)) if u else 0
        k = max(0, min((1 << pbits) - 2, int(mean).bit_length() - 1 if mean >= 1 else 0))
        w.put(k, pbits)
        for x in u:
            w.unary(x >> k)
            w.put(x & ((1 << k) - 1), k)


FIXED = {0: [], 1: [1], 2: [2, -1], 3: [3, -3, 1], 4: [4, -6, 4, -1]}


def _subframe(w, s, bps, kind, wasted=0, lpc=None, porder=0, method=0, escape=False):
    """kind: 'constant' | 'verbatim' | ('fixed', order) | 'lpc' (lpc =
    (coefs, prec, shift))."""
    s = [int(v) for v in s]
    bsize = len(s)
    if wasted:
        assert all(v % (1 << wasted) == 0 for v in s)
        s = [v >> wasted for v in s]
    eb = bps - wasted
    w.put(0, 1)
    if kind == "constant":
        w.put(0, 6)
    elif kind == "verbatim":
        w.put(1, 6)
    elif kind[0] == "fixed":
        w.put(8 + kind[1], 6)
    else:
        w.put(32 + len(lpc[0]) - 1, 6)
    if wasted:
        w.put(1, 1)
        w.unary(wasted - 1)
    else:
        w.put(0, 1)
    if kind == "constant":
        w.put(s[0], eb)
    elif kind == "verbatim":
        for v in s:
            w.put(v, eb)
    elif kind[0] == "fixed":
        order = kind[1]
        for v in s[:order]:
            w.put(v, eb)
        c = FIXED[order]
        res = [s[i] - sum(c[j] * s[i - 1 - j] for j in range(order)) for i in range(order, bsize)]
        _residual(w, res, order, bsize, porder, method, escape)
    else:
        coefs, prec, shift = lpc
        order = len(coefs)
        for v in s[:order]:
            w.put(v, eb)
        w.put(prec - 1, 4)
        w.put(shift, 5)
        for c in coefs:
            w.put(c, prec)
        res = [s[i] - (sum(coefs[j] * s[i - 1 - j] for j in range(order)) >> shift) for i in range(order, bsize)]
        _residual(w, res, order, bsize, porder, method, escape)


BS_CODES = {192: 1, 576: 2, 1152: 3, 2304: 4, 4608: 5, 256: 8, 512: 9, 1024: 10, 2048: 11, 4096: 12,
            8192: 13, 16384: 14, 32768: 15}
SS_CODES = {8: 1, 12: 2, 16: 4, 20: 5, 24: 6, 32: 7}


def encode(x, fs, bps, frames, total_in_streaminfo=True):
    """x: int array [channels][n]; frames: list of dicts with keys
    'n' (block size), 'mode' (0 independent, 8 left/side, 9 side/right,
    10 mid/side), 'sub' (per-channel kwargs for _subframe), optional
    'bs_code' ('table' | 6 | 7) and 'ss_from_streaminfo'."""
    ch, total = x.shape
    out = bytearray(b"fLaC")
    info = BitWriter()
    bmax = max(f["n"] for f in frames)
    info.put(min(f["n"] for f in frames), 16)
    info.put(bmax, 16)
    info.put(0, 24)
    info.put(0, 24)
    info.put(fs, 20)
    info.put(ch - 1, 3)
    info.put(bps - 1, 5)
    info.put(total if total_in_streaminfo else 0, 36)
    info.put(0, 128)
    body = info.bytes()
    out += bytes([0x80 | 0]) + len(body).to_bytes(3, "big") + body
    pos = 0
    for fi, f in enumerate(frames):
        n, mode = f["n"], f.get("mode", 0)
        blk = [np.asarray(x[c, pos:pos + n], dtype=np.int64) for c in range(ch)]
        if mode == 8:
            chans, extra = [blk[0], blk[0] - blk[1]], [0, 1]
        elif mode == 9:
            chans, extra = [blk[0] - blk[1], blk[1]], [1, 0]
        elif mode == 10:
            chans, extra = [(blk[0] + blk[1]) >> 1, blk[0] - blk[1]], [0, 1]
        else:
            chans, extra = blk, [0] * ch
        h = BitWriter()
        h.put(0b11111111111110, 14)
        h.put(0, 1)
        h.put(0, 1)   # fixed-blocksize stream: coded number is the frame number
        bs = f.get("bs_code", "table")
        if bs == "table" and n in BS_CODES:
            h.put(BS_CODES[n], 4)
        else:
            bs = 6 if (bs == 6 or (bs == "table" and n <= 256)) else 7
            h.put(bs, 4)
        h.put(0, 4)   # sample rate from STREAMINFO
        h.put(mode if mode else ch - 1, 4)
        h.put(0 if f.get("ss_from_streaminfo") else SS_CODES[bps], 3)
        h.put(0, 1)
        hb = bytearray(h.bytes()) + _utf8(fi)
        if bs == 6:
            hb += bytes([n - 1])
        elif bs == 7:
            hb += (n - 1).to_bytes(2, "big")
        hb.append(crc8(hb))
        w = BitWriter()
        for c in range(ch):
            _subframe(w, chans[c], bps + extra[c], **f["sub"][c])
        w.align()
        frame = bytes(hb) + w.bytes()
        out += frame + crc16(frame).to_bytes(2, "big")
        pos += n
    assert pos == total
    return bytes(out)
